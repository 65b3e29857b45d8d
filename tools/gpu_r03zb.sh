set -o pipefail
# k_small_screen: scalar branch at row ends (base) vs selects (gen):
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
STRESS_BITS=6,11 timeout -k 10 300 python -u tools/stress_csr.py 400 22000 200 > gpurun_out/stress_small.log 2>&1 && tail -1 gpurun_out/stress_small.log && \
for v in base gen; do
  L=""; [ $v != base ] && L=$PWD/tools/vscreen/libcwq_$v.so
  CWQ_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_$v -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --config c2 --steps 4 --warmup 1 > gpurun_out/prof_c2_$v.log 2>&1 || exit 1
  CWQ_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_$v -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --config c3 --batch-only --steps 4 --warmup 1 > gpurun_out/prof_c3_$v.log 2>&1 || exit 1
done && \
echo r03za done
