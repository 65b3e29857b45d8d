set -o pipefail
# PLN codec: GPU tests + bench (run on the GPU box)
timeout -k 10 600 python -u -m pytest tests/test_pln_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_pln.log 2>&1 && \
timeout -k 10 600 python -u bench.py --config pln --steps 2 --warmup 1 > gpurun_out/b_pln.log 2>&1
