set -o pipefail
# Round 3: Philox rounds 0-2 with the stream's uniform terms folded into four
# scalars (philox10_lo) in the uniform, CSR and importance screening loops,
# vs the previous build (head2).
export TMPDIR=/tmp
mkdir -p gpurun_out
CONFIGS="c2low c2cli" bash tools/gpu_check.sh && \
timeout -k 10 300 python -u tools/stress_imp.py 100 > gpurun_out/stress_imp.log 2>&1 && tail -1 gpurun_out/stress_imp.log && \
VARIANTS="head2 base head2 base" BENCH_ARGS="--steps 10 --warmup 2" bash tools/variants.sh run > gpurun_out/plo_c4.log 2>&1 && grep -v amdgpu.ids gpurun_out/plo_c4.log && \
VARIANTS="head2 base head2 base" BENCH_ARGS="--config c5 --steps 3 --warmup 1" bash tools/variants.sh run > gpurun_out/plo_c5.log 2>&1 && grep -v amdgpu.ids gpurun_out/plo_c5.log && \
VARIANTS="head2 base head2 base" BENCH_ARGS="--config c2cli" bash tools/variants.sh run > gpurun_out/plo_c2cli.log 2>&1 && grep -v amdgpu.ids gpurun_out/plo_c2cli.log && \
VARIANTS="head2 base head2 base" BENCH_ARGS="--config i1" bash tools/variants.sh run > gpurun_out/plo_i1.log 2>&1 && grep -v amdgpu.ids gpurun_out/plo_i1.log
