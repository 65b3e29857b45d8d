set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pln_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_pln.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pln -o run --output-format csv -- python3 -u bench.py --config pln --steps 2 --warmup 1 > gpurun_out/p_pln.log 2>&1
