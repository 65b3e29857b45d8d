set -o pipefail
# Round-end evidence (run on the GPU box): full GPU tests, smoke, every bench
# config (gpurun_out/b_<config>.log), and the rocprof/PMC profile of the C4
# headline kernel (tools/profile.sh).  Each GPU step has its own time limit.
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/b_c4.log 2>&1 && \
for c in c5 c1 c2 c2cli c2low c3 i1 i2 pln pln_is; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 > gpurun_out/b_$c.log 2>&1 || exit 1
done && \
bash tools/profile.sh r01_c4_screen --config c4
