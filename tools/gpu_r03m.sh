set -o pipefail
# Round 3: cooperative loop loads issued in unit order (CWQ_COOP_LOAD_ORDER) vs HEAD.
export TMPDIR=/tmp
mkdir -p gpurun_out
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_lord.so timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "csr or coop or grouped" --timeout 200 --timeout-method thread > gpurun_out/t_lord.log 2>&1 && tail -1 gpurun_out/t_lord.log && \
VARIANTS="base lord base lord base lord" BENCH_ARGS="--config c2low" bash tools/variants.sh run > gpurun_out/lord_c2low.log 2>&1 && grep -v amdgpu.ids gpurun_out/lord_c2low.log
