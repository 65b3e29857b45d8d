#!/bin/bash
# rocprofv3 evidence for bench.py's dominant kernel (run on the GPU box).
# Usage: tools/profile.sh TAG [bench args...]   e.g. tools/profile.sh r01_c4 --config c4
# Writes gpurun_out/prof_TAG/*.csv; tools/collect_profile.py turns them into
# profiles/TAG_kernel_stats.csv, profiles/TAG_pmc_*.csv and profiles/traffic_<config>.json.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="bench.py --no-cpu --no-e2e $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $B --steps 3 --warmup 1 > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $B --steps 1 --warmup 0 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $B --steps 1 --warmup 0 > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT/valu -o run --output-format csv -- python3 $B --steps 1 --warmup 0 > $OUT/valu.log 2>&1
echo done
