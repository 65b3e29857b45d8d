set -o pipefail
# Round 3: XCD-aware tile mapping of the general pruned kernel (CWQ_CSR_XCD_MAP).
export TMPDIR=/tmp
mkdir -p gpurun_out
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_xcd2.so timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "csr or coop or grouped or wide" --timeout 200 --timeout-method thread > gpurun_out/t_xcd.log 2>&1 && tail -1 gpurun_out/t_xcd.log && \
VARIANTS="base xcd xcd2 base xcd xcd2" BENCH_ARGS="--config c2low" bash tools/variants.sh run > gpurun_out/xcd_c2low.log 2>&1 && grep -v amdgpu.ids gpurun_out/xcd_c2low.log && \
VARIANTS="base xcd2 base xcd2" BENCH_ARGS="--config c2cli" bash tools/variants.sh run > gpurun_out/xcd_c2cli.log 2>&1 && grep -v amdgpu.ids gpurun_out/xcd_c2cli.log && \
VARIANTS="base xcd xcd2" BENCH_ARGS="--config pln" bash tools/variants.sh run > gpurun_out/xcd_pln.log 2>&1 && grep -v amdgpu.ids gpurun_out/xcd_pln.log
