set -o pipefail
# full validation at HEAD: GPU tests, smoke(), default bench line (run on the GPU box)
timeout -k 10 1200 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1
