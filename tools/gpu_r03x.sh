set -o pipefail
# Round 3: LDS-staged records in conflict-free split halves (base) vs HEAD (head4).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "csr or coop or grouped or wide or pln" --timeout 300 --timeout-method thread > gpurun_out/t_rl2.log 2>&1 && tail -1 gpurun_out/t_rl2.log && \
timeout -k 10 300 python -u tools/stress_csr.py 200 43000 200 > gpurun_out/stress_csr.log 2>&1 && tail -1 gpurun_out/stress_csr.log && \
VARIANTS="head4 base head4 base head4 base" BENCH_ARGS="--config c2low" bash tools/variants.sh run > gpurun_out/rl2_c2low.log 2>&1 && grep -v amdgpu.ids gpurun_out/rl2_c2low.log && \
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_base.so bash tools/gpu_pmc_mem.sh c2low c2low_rl2 && echo pmc ok
