set -o pipefail
# Round evidence, part 2 (GPU box): rocprof kernel stats + FETCH/WRITE/VALU PMC
# of C4, C5, C2 and C3 (the batched call), the C3 device timeline, the C5
# pruning statistics (-DCWQ_PRUNE_STATS build) and the decode clock series.
export TMPDIR=/tmp
R=${R:-r03}
mkdir -p gpurun_out
bash tools/profile.sh ${R}_c4 --config c4 && \
bash tools/profile.sh ${R}_c5 --config c5 && \
bash tools/profile.sh ${R}_c2 --config c2 && \
bash tools/profile.sh ${R}_c3 --config c3 --batch-only && \
C3_CALLS=6 C3_NO_CPROFILE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R}_c3tl -o run --output-format csv -- python3 tools/c3_pyprof.py > gpurun_out/c3_tl.log 2>&1 && \
python tools/timeline.py gpurun_out/prof_${R}_c3tl 15 > gpurun_out/${R}_c3_timeline.txt && tail -1 gpurun_out/${R}_c3_timeline.txt && \
CWQ_LIB_PATH=$PWD/tools/vrun/libcwq_stats.so PS_D=16 PS_BITS=24 PS_CONFIG=c5 timeout -k 10 170 python -u tools/prune_stats.py 1024 2 --json gpurun_out/prune_stats_c5.json > gpurun_out/ps_c5.log 2>&1 && \
timeout -k 10 120 python -u tools/decode_clock.py > gpurun_out/decode_clock.log 2>&1 && cat gpurun_out/decode_clock.log && \
BATCHES=4 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R}_decode -o run --output-format csv -- python3 tools/decode_clock.py > gpurun_out/decode_trace.log 2>&1 && \
BATCHES=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_${R}_decode_fetch -o run --output-format csv -- python3 tools/decode_clock.py > gpurun_out/decode_fetch.log 2>&1 && \
BATCHES=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_${R}_decode_write -o run --output-format csv -- python3 tools/decode_clock.py > gpurun_out/decode_write.log 2>&1 && \
echo round-evidence-2 done
