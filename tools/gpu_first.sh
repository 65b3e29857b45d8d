set -o pipefail
echo "== default (package sets MIOPEN_FIND_MODE=FAST)" > gpurun_out/first.log
timeout -k 10 300 python -u tools/pln_first_call.py >> gpurun_out/first.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_pln_gpu.py -x -q --timeout 300 --timeout-method thread >> gpurun_out/first.log 2>&1
