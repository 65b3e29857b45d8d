set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_pln_gpu.py -x -q --timeout 300 --timeout-method thread -k "csr or coop or odd_d or grouped or c2_image or codec" > gpurun_out/t_csr.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c2cli --steps 3 --warmup 1 > gpurun_out/b_c2cli.log 2>&1
