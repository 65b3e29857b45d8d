set -o pipefail
# Round 3: uniform loop with 32-bit candidate counters, an activity compare per
# iteration and the finished-lane mask from the compares (base) vs HEAD (head3).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
timeout -k 10 300 python -u tools/stress_modes.py 300 > gpurun_out/stress_modes.log 2>&1 && tail -1 gpurun_out/stress_modes.log && \
VARIANTS="head3 base head3 base head3 base" BENCH_ARGS="--steps 5 --warmup 1" bash tools/variants.sh run > gpurun_out/c32_c4.log 2>&1 && grep -v amdgpu.ids gpurun_out/c32_c4.log && \
VARIANTS="head3 base head3 base" BENCH_ARGS="--config c5 --steps 3 --warmup 1" bash tools/variants.sh run > gpurun_out/c32_c5.log 2>&1 && grep -v amdgpu.ids gpurun_out/c32_c5.log
