set -o pipefail
# Round 3: importance screen with 32-bit block indices (normal4_screen<true>) vs the previous build.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "importance or imp or pln" --timeout 300 --timeout-method thread > gpurun_out/t_imp.log 2>&1 && tail -1 gpurun_out/t_imp.log && \
timeout -k 10 300 python -u tools/stress_imp.py 200 > gpurun_out/stress_imp.log 2>&1 && tail -1 gpurun_out/stress_imp.log && \
VARIANTS="head1 base head1 base" BENCH_ARGS="--config i1" bash tools/variants.sh run > gpurun_out/lo32_i1.log 2>&1 && grep -v amdgpu.ids gpurun_out/lo32_i1.log && \
VARIANTS="head1 base head1 base" BENCH_ARGS="--config i2" bash tools/variants.sh run > gpurun_out/lo32_i2.log 2>&1 && grep -v amdgpu.ids gpurun_out/lo32_i2.log
