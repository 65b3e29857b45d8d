set -o pipefail
# Round 3: rocprof kernel stats + FETCH/WRITE/VALU PMC for C5, C2, C3 (batched
# call only) and C4 (incl. the decode kernel), and C5 pruning statistics.
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile.sh r03_c5 --config c5 && \
bash tools/profile.sh r03_c2 --config c2 && \
bash tools/profile.sh r03_c3 --config c3 --batch-only && \
bash tools/profile.sh r03_c4 --config c4 && \
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_stats.so PS_D=16 PS_BITS=24 PS_CONFIG=c5 timeout -k 10 300 python -u tools/prune_stats.py 1024 2 --json gpurun_out/prune_stats_c5.json > gpurun_out/ps_c5.log 2>&1 && cat gpurun_out/ps_c5.log
