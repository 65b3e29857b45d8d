set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_shards_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_shards.log 2>&1 && tail -1 gpurun_out/t_shards.log && \
VARIANTS="base dtm dcomp base dtm dcomp" bash tools/decode_variants.sh > gpurun_out/decode_var.log 2>&1; cat gpurun_out/decode_var.log
