set -o pipefail
# Round 3, first call: GPU tests + smoke after the ABI 0.2 / record-layout
# changes, and the bench lines of C4, C5, C2, C3 (roofline + cpu_baseline).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
timeout -k 10 300 python -u bench.py > gpurun_out/b_c4.log 2>&1 && tail -1 gpurun_out/b_c4.log && \
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/b_c5.log 2>&1 && tail -1 gpurun_out/b_c5.log && \
timeout -k 10 300 python -u bench.py --config c2 --steps 100 --warmup 5 > gpurun_out/b_c2.log 2>&1 && tail -1 gpurun_out/b_c2.log && \
timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 2 > gpurun_out/b_c3.log 2>&1 && tail -1 gpurun_out/b_c3.log
