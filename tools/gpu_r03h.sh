set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
C3_SPLIT=1 C3_NO_CPROFILE=1 timeout -k 10 120 python -u tools/c3_pyprof.py > gpurun_out/c3_k.log 2>&1 && grep 'ms per call' gpurun_out/c3_k.log && \
timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 > gpurun_out/b_c3.log 2>&1 && tail -1 gpurun_out/b_c3.log | cut -c1-300 && \
timeout -k 10 300 python -u bench.py --config c2 --steps 100 --warmup 5 > gpurun_out/b_c2.log 2>&1 && tail -1 gpurun_out/b_c2.log | cut -c1-300 && \
timeout -k 10 300 python -u bench.py > gpurun_out/b_c4.log 2>&1 && tail -1 gpurun_out/b_c4.log | cut -c1-200
