set -o pipefail
# Rate dependence of the uniform pruned encoder: units
# evaluated per candidate (-DCWQ_PRUNE_STATS build, tools/prune_stats.py) and
# candidates/s (product library, tools/rate_sweep.py) for d = 16 and 32 at
# 12-24 bits, ~2^30 candidates per stats point and ~2^32 per timed point.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/rate_units.log
for d in 16 32; do
  for b in 12 14 16 18 20 22 24; do
    nb=$(( (1 << 30) >> b )); [ $nb -lt 64 ] && nb=64
    echo "== d=$d bits=$b nb=$nb" >> gpurun_out/rate_units.log
    CWQ_LIB_PATH=$PWD/tools/variants/libcwq_stats.so PS_D=$d PS_BITS=$b timeout -k 10 120 \
      python -u tools/prune_stats.py $nb 2 >> gpurun_out/rate_units.log 2>&1 || exit 1
  done
done && grep -E "^==|units/candidate" gpurun_out/rate_units.log && \
S="" && for d in 16 32; do for b in 12 14 16 18 20 22 24; do
  nb=$(( (1 << 32) >> b )); S="$S $d:$b:$nb"; done; done && \
timeout -k 10 300 python -u tools/rate_sweep.py $S > gpurun_out/rate_time.log 2>&1 && cat gpurun_out/rate_time.log && \
echo r03zc done
