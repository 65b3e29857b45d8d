set -o pipefail
# Round 3: one alignment class per cooperative workgroup (CWQ_COOP_CLASS_TILES)
export TMPDIR=/tmp
mkdir -p gpurun_out
export CT=$PWD/tools/variants/libcwq_ctile.so
CWQ_LIB_PATH=$CT timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "csr or coop or grouped or wide or pln or stress" --timeout 300 --timeout-method thread > gpurun_out/t_ct.log 2>&1 && tail -1 gpurun_out/t_ct.log && \
CWQ_LIB_PATH=$CT timeout -k 10 300 python -u tools/stress_csr.py 300 31000 200 > gpurun_out/stress_ct.log 2>&1 && tail -1 gpurun_out/stress_ct.log && \
VARIANTS="base ctile base ctile base ctile" BENCH_ARGS="--config c2low" bash tools/variants.sh run > gpurun_out/ct_c2low.log 2>&1 && grep -v amdgpu.ids gpurun_out/ct_c2low.log && \
VARIANTS="base ctile base ctile" BENCH_ARGS="--config pln" bash tools/variants.sh run > gpurun_out/ct_pln.log 2>&1 && grep -v "amdgpu.ids\|cudnn\|MIOpen\|_benchmark_limit" gpurun_out/ct_pln.log
