set -o pipefail
# Round 3: a one-class cooperative tile's visit-order records staged in LDS
# (base) vs reading them through the vector-memory path (head4).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
timeout -k 10 300 python -u tools/stress_csr.py 300 41000 200 > gpurun_out/stress_csr.log 2>&1 && tail -1 gpurun_out/stress_csr.log && \
VARIANTS="head4 base head4 base head4 base" BENCH_ARGS="--config c2low" bash tools/variants.sh run > gpurun_out/rl_c2low.log 2>&1 && grep -v amdgpu.ids gpurun_out/rl_c2low.log && \
VARIANTS="head4 base head4 base" BENCH_ARGS="--config pln" bash tools/variants.sh run > gpurun_out/rl_pln.log 2>&1 && grep -v "amdgpu.ids\|cudnn\|MIOpen\|_benchmark_limit" gpurun_out/rl_pln.log && \
VARIANTS="head4 base" BENCH_ARGS="--config c2cli" bash tools/variants.sh run > gpurun_out/rl_c2cli.log 2>&1 && grep -v amdgpu.ids gpurun_out/rl_c2cli.log
