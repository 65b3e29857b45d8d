set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_pln_gpu.py -x -q --timeout 300 --timeout-method thread -k "csr or coop or odd_d or grouped or c2_image or codec or vs_oracle or golden or capi" > gpurun_out/t_split.log 2>&1 && \
for c in c2cli c2low pln c2 c3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 > gpurun_out/b_$c.log 2>&1 || exit 1
done
