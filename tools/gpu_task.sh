#!/bin/bash
# One parametrised entry point for ad-hoc GPU-box work (replaces the round-3
# one-off gpu_r03*.sh scripts).  Every GPU step runs under its own timeout and
# the first failure ends the script.
#   tools/gpu_task.sh tests                      full -m gpu suite + smoke()
#   tools/gpu_task.sh bench CONFIG[@TAG] [bench args]  one bench line -> gpurun_out/b_CONFIG[_TAG].log
#   tools/gpu_task.sh trace TAG [bench args]     rocprofv3 kernel trace + stats
#   tools/gpu_task.sh pmc TAG SET [bench args]   one PMC set (mem | valu | wait | lds),
#                                                one rocprofv3 pass per counter group
#   tools/gpu_task.sh stress [N]                 CSR + small-path stress sweeps
#   tools/gpu_task.sh variants TAG "V1 V2" [bench args]   tools/variants.sh run -> gpurun_out/v_TAG.log
#   tools/gpu_task.sh stats TAG VARIANT NB D BITS        tools/prune_stats.py on a stats build
#   tools/gpu_task.sh tiles TAG NB D BITS [VARIANT]      tools/tile_times.py on a tile-times build
#   tools/gpu_task.sh decvar "V1 V2"                     decode tests + timing per variant build
#   tools/gpu_task.sh py TAG SCRIPT [args]               a tools/ script -> gpurun_out/py_TAG.log
#   tools/gpu_task.sh timeline TAG [bench args]          kernel + copy trace -> tools/timeline.py
#   tools/gpu_task.sh vtrace TAG "V1 V2" [bench args]    kernel trace + stats per tools/vrun build
#   tools/gpu_task.sh ktimeline TAG WINDOW_MS SCRIPT [args]  kernel-trace timeline of a script
# Several tasks can be chained: tools/gpu_task.sh tests -- pmc c2 wait --config c2
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
prof() {  # prof DIR ARGS... -- python3 bench args
  local d=$1; shift
  timeout -s KILL 180 rocprofv3 "$@" -d gpurun_out/$d -o run --output-format csv -- \
    python3 bench.py --no-cpu --no-e2e $BARGS > gpurun_out/$d.log 2>&1
}
run_one() {
  local task=$1; shift
  case $task in
    tests)
      timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 \
        --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
        > gpurun_out/smoke.log 2>&1 && echo smoke ok ;;
    bench)
      local c=${1%%@*} n=${1/@/_}; shift
      timeout -k 10 600 python -u bench.py --config $c "$@" > gpurun_out/b_$n.log 2>&1 && \
        tail -1 gpurun_out/b_$n.log | cut -c1-200 ;;
    trace)
      local tag=$1; shift
      BARGS="$* --steps 3 --warmup 1" prof prof_${tag}_trace --kernel-trace --stats && \
        echo trace $tag ok ;;
    pmc)
      local tag=$1 set=$2; shift 2
      BARGS="$* --steps 1 --warmup 0"
      case $set in
        mem)  prof prof_${tag}_fetch --pmc FETCH_SIZE && prof prof_${tag}_write --pmc WRITE_SIZE ;;
        valu) prof prof_${tag}_valu --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE ;;
        wait) prof prof_${tag}_wait --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES ;;
        lds)  prof prof_${tag}_lds --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES ;;
        *) echo "unknown PMC set $set"; return 2 ;;
      esac && echo pmc $tag $set ok ;;
    vpmc)  # vpmc TAG VARIANT SET [bench args]: pmc on a tools/vrun build
      local tag=$1 v=$2; shift 2
      ( export CWQ_LIB_PATH=$PWD/tools/vrun/libcwq_$v.so; run_one pmc $tag "$@" ) ;;
    vtrace)  # vtrace TAG "V1 V2" [bench args]: kernel trace + stats per tools/vrun build
      local tag=$1 vs=$2; shift 2
      for v in $vs; do
        ( export CWQ_LIB_PATH=$PWD/tools/vrun/libcwq_$v.so; run_one trace ${tag}_$v "$@" ) || return 1
        python3 tools/kstats.py $v gpurun_out/prof_${tag}_${v}_trace/run_kernel_stats.csv \
          ${KSUBS:-k_small k_encode k_imp_eval k_csr} || return 1
      done ;;
    stress)
      local n=${1:-400}
      timeout -k 10 300 python -u tools/stress_csr.py $n ${STRESS_SEED:-20000} 200 \
        > gpurun_out/stress_csr.log 2>&1 && tail -1 gpurun_out/stress_csr.log && \
      STRESS_BITS=6,11 timeout -k 10 300 python -u tools/stress_csr.py $n ${STRESS_SEED:-20000} 200 \
        > gpurun_out/stress_small.log 2>&1 && tail -1 gpurun_out/stress_small.log && \
      STRESS_SMALL=1 STRESS_BITS=6,11 timeout -k 10 300 python -u tools/stress_csr.py $n ${STRESS_SEED:-20000} 200 \
        > gpurun_out/stress_fused.log 2>&1 && tail -1 gpurun_out/stress_fused.log ;;
    variants)
      local tag=$1 vs=$2; shift 2
      VARIANTS="$vs" BENCH_ARGS="$*" timeout -k 10 900 bash tools/variants.sh run \
        > gpurun_out/v_$tag.log 2>&1 && cat gpurun_out/v_$tag.log ;;
    stats)
      local tag=$1 v=$2 nb=$3 d=$4 bits=$5
      CWQ_LIB_PATH=$PWD/tools/vrun/libcwq_$v.so PS_D=$d PS_BITS=$bits timeout -k 10 300 \
        python -u tools/prune_stats.py $nb > gpurun_out/s_$tag.log 2>&1 && head -3 gpurun_out/s_$tag.log ;;
    c2parts)
      timeout -k 10 300 python -u tools/c2_parts.py > gpurun_out/c2parts.log 2>&1 && cat gpurun_out/c2parts.log && \
      CWQ_LIB_PATH=$PWD/tools/vrun/libcwq_phases.so timeout -k 10 300 python -u bench.py --config c2 \
        --no-cpu --no-e2e --steps 5 > gpurun_out/c2phases.log 2>&1 && grep cwq gpurun_out/c2phases.log | tail -8 && \
      CWQ_LIB_PATH=$PWD/tools/vrun/libcwq_phases.so timeout -k 10 300 python -u bench.py --config c3 \
        --batch-only --no-cpu --no-e2e --steps 3 > gpurun_out/c3phases.log 2>&1 && grep "cwq batch" gpurun_out/c3phases.log | tail -4 ;;
    decvar)  # decode timing per variant, after its decode tests against the oracle
      for v in $1; do
        CWQ_LIB_PATH=$PWD/tools/vrun/libcwq_$v.so timeout -k 10 300 python -u -m pytest \
          tests/test_gpu.py -q -x -k decode --timeout 120 --timeout-method thread \
          > gpurun_out/decvar_$v.log 2>&1 && tail -1 gpurun_out/decvar_$v.log || return 1
      done
      VARIANTS="$1" timeout -k 10 600 bash tools/decode_variants.sh > gpurun_out/decvar.log 2>&1 && \
        cat gpurun_out/decvar.log ;;
    tiles)
      local tag=$1 nb=$2 d=$3 bits=$4 v=${5:-tt}
      CWQ_LIB_PATH=$PWD/tools/vrun/libcwq_$v.so timeout -k 10 300 \
        python -u tools/tile_times.py $nb $d $bits > gpurun_out/tt_$tag.log 2>&1 && head -6 gpurun_out/tt_$tag.log ;;
    py)  # py TAG SCRIPT [args]: a tools/ script -> gpurun_out/py_TAG.log
      local tag=$1; shift
      timeout -k 10 300 python -u "$@" > gpurun_out/py_$tag.log 2>&1 && tail -4 gpurun_out/py_$tag.log ;;
    timeline)  # kernel + copy trace of a bench run, then tools/timeline.py on it
      local tag=$1; shift
      BARGS="$* --steps 3 --warmup 1" prof prof_${tag}_tl --kernel-trace --memory-copy-trace --stats && \
        python3 tools/timeline.py gpurun_out/prof_${tag}_tl ${TL_MS:-12} > gpurun_out/tl_$tag.txt && \
        tail -3 gpurun_out/tl_$tag.txt ;;
    ktimeline)  # ktimeline TAG WINDOW_MS SCRIPT [args]: kernel trace of a tools/ script + timeline.py
      local tag=$1 win=$2; shift 2
      timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_kt -o run \
        --output-format csv -- python3 "$@" > gpurun_out/prof_${tag}_kt.log 2>&1 && \
        python3 tools/timeline.py gpurun_out/prof_${tag}_kt $win > gpurun_out/tl_$tag.txt && \
        tail -n 1 gpurun_out/prof_${tag}_kt.log && tail -n 1 gpurun_out/tl_$tag.txt ;;
    *) echo "unknown task $task"; return 2 ;;
  esac
}
args=()
for a in "$@" --; do
  if [ "$a" = "--" ]; then
    [ ${#args[@]} -gt 0 ] && { run_one "${args[@]}" || exit 1; }
    args=()
  else
    args+=("$a")
  fi
done
echo gpu_task done
