set -o pipefail
# Post-change check on the GPU box: full GPU suite, smoke, the CSR stress sweeps
# (pruned vs unpruned on random ragged layouts, at 12-16 bits and at 6-11 bits
# for the screened small-candidate path) and the CSR bench configs.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
timeout -k 10 300 python -u tools/stress_csr.py 400 ${STRESS_SEED:-20000} 200 > gpurun_out/stress_csr.log 2>&1 && tail -1 gpurun_out/stress_csr.log && \
STRESS_BITS=6,11 timeout -k 10 300 python -u tools/stress_csr.py 400 ${STRESS_SEED:-20000} 200 > gpurun_out/stress_small.log 2>&1 && tail -1 gpurun_out/stress_small.log && \
for c in ${CONFIGS:-c2low c2cli pln}; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 > gpurun_out/b_$c.log 2>&1 || exit 1
  tail -1 gpurun_out/b_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['unit'], d['ms_per_step'])"
done
