set -o pipefail
# Round 3: Philox chains round-interleaved across a cooperative / per-lane
# iteration's units (CWQ_COOP_ILP / CWQ_RUN_ILP variants), c2low and c2cli.
export TMPDIR=/tmp
mkdir -p gpurun_out
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_cilp4w3.so timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "csr or coop or grouped" --timeout 200 --timeout-method thread > gpurun_out/t_ilp4.log 2>&1 && tail -1 gpurun_out/t_ilp4.log && \
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_rilp.so timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "csr or coop or grouped" --timeout 200 --timeout-method thread > gpurun_out/t_rilp.log 2>&1 && tail -1 gpurun_out/t_rilp.log && \
VARIANTS="base cilp2w3 cilp4w3 cilp2w4 base cilp2w3 cilp4w3 cilp2w4" BENCH_ARGS="--config c2low" bash tools/variants.sh run > gpurun_out/ilp_c2low.log 2>&1 && cat gpurun_out/ilp_c2low.log && \
VARIANTS="base rilp rilpw5 cilp4w3 base rilp rilpw5 cilp4w3" BENCH_ARGS="--config c2cli" bash tools/variants.sh run > gpurun_out/ilp_c2cli.log 2>&1 && cat gpurun_out/ilp_c2cli.log
