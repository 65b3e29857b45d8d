set -o pipefail
# full GPU test suite + the grouped / importance benches (run on the GPU box)
timeout -k 10 1200 python -u -m pytest tests -x -q -m gpu > gpurun_out/t_all.log 2>&1 && \
for c in c2cli c2 c3 i1 i2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 > gpurun_out/b_$c.log 2>&1 || exit 1
done
