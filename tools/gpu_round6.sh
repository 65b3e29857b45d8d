#!/bin/bash
# Round-6 evidence on the GPU box, in parts (each part one gpurun call):
#   tools/gpu_round6.sh tests     full -m gpu suite + smoke()
#   tools/gpu_round6.sh bench A   bench lines of c4 c5 c1 c2 c3 (with CPU baseline, parity)
#   tools/gpu_round6.sh bench B   bench lines of c2cli c2low i1 i2 pln pln_is
#   tools/gpu_round6.sh trace CONFIG...  kernel trace + stats per config
#   tools/gpu_round6.sh pmc CONFIG...    FETCH / WRITE / VALU / wait passes per config
# Every GPU step runs under its own timeout; the first failure ends the part.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
part=$1; shift
bargs() {  # per-config bench arguments of the evidence lines
  case $1 in
    c4) echo "--config c4" ;;
    c5|c2cli|c2low|i1) echo "--config $1 --steps 3 --warmup 1" ;;
    pln) echo "--config pln --steps 3 --warmup 2" ;;  # the capture (last warmup) warm
    c2) echo "--config c2 --steps 100 --warmup 5" ;;
    *) echo "--config $1 --steps 20 --warmup 3" ;;
  esac
}
pargs() {  # profiling runs: the batched call alone for the multi-image configs
  case $1 in c3|i2) echo "--config $1 --batch-only" ;; *) echo "--config $1" ;; esac
}
case $part in
  tests)
    timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
      > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
      tail -1 gpurun_out/smoke.log ;;
  bench)
    case $1 in A) cs="c4 c5 c1 c2 c3" ;; B) cs="c2cli c2low i1 i2 pln pln_is" ;; *) cs="$*" ;; esac
    for c in $cs; do
      timeout -k 10 400 python -u bench.py $(bargs $c) > gpurun_out/b_$c.log 2>&1 || exit 1
      tail -1 gpurun_out/b_$c.log | cut -c1-120
    done ;;
  trace)
    for c in "$@"; do
      timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r06_${c}_trace -o run \
        --output-format csv -- python3 bench.py --no-cpu --no-e2e $(pargs $c) --steps 3 --warmup 1 \
        > gpurun_out/prof_r06_${c}_trace.log 2>&1 || exit 1
      echo trace $c ok
    done ;;
  pmc)
    for c in "$@"; do
      B="bench.py --no-cpu --no-e2e $(pargs $c) --steps 1 --warmup 0"
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_r06_${c}_fetch -o run --output-format csv -- python3 $B > gpurun_out/prof_r06_${c}_fetch.log 2>&1 && \
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_r06_${c}_write -o run --output-format csv -- python3 $B > gpurun_out/prof_r06_${c}_write.log 2>&1 && \
      timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/prof_r06_${c}_valu -o run --output-format csv -- python3 $B > gpurun_out/prof_r06_${c}_valu.log 2>&1 && \
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES -d gpurun_out/prof_r06_${c}_wait -o run --output-format csv -- python3 $B > gpurun_out/prof_r06_${c}_wait.log 2>&1 || exit 1
      echo pmc $c ok
    done ;;
  *) echo "unknown part $part"; exit 2 ;;
esac
echo part $part done
