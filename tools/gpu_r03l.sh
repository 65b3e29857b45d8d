set -o pipefail
# Round 3: CSR scoring loops without past-the-end masks (pad unit) and with
# the lane-invariant round-2 product when block indices stay below 2^32.
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh && \
VARIANTS="prepad base prepad base" BENCH_ARGS="--config c2low" bash tools/variants.sh run > gpurun_out/pad_c2low.log 2>&1 && grep -v amdgpu.ids gpurun_out/pad_c2low.log && \
VARIANTS="prepad base prepad base" BENCH_ARGS="--config c2cli" bash tools/variants.sh run > gpurun_out/pad_c2cli.log 2>&1 && grep -v amdgpu.ids gpurun_out/pad_c2cli.log
