set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_pln_gpu.py -x -q --timeout 300 --timeout-method thread -k "importance or codec" > gpurun_out/t_imp.log 2>&1 && \
for c in i1 i2 pln_is; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 > gpurun_out/b_$c.log 2>&1 || exit 1
done
