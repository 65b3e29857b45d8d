set -o pipefail
# Round 3: the tau-sharing wave max as six v_max_f32_dpp (inline asm) vs the
# builtin form (nowma).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
timeout -k 10 300 python -u tools/stress_csr.py 200 > gpurun_out/stress_csr.log 2>&1 && tail -1 gpurun_out/stress_csr.log && \
VARIANTS="nowma base nowma base nowma base" BENCH_ARGS="--steps 5 --warmup 1" bash tools/variants.sh run > gpurun_out/wma_c4.log 2>&1 && grep -v amdgpu.ids gpurun_out/wma_c4.log && \
VARIANTS="nowma base nowma base" BENCH_ARGS="--config c5 --steps 3 --warmup 1" bash tools/variants.sh run > gpurun_out/wma_c5.log 2>&1 && grep -v amdgpu.ids gpurun_out/wma_c5.log && \
VARIANTS="nowma base nowma base" BENCH_ARGS="--config c2cli" bash tools/variants.sh run > gpurun_out/wma_c2cli.log 2>&1 && grep -v amdgpu.ids gpurun_out/wma_c2cli.log
