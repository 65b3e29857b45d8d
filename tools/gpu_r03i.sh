set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "grouped or c3 or batch" --timeout 300 --timeout-method thread > gpurun_out/t_grp.log 2>&1 && tail -1 gpurun_out/t_grp.log && \
for k in 5 6 7 8; do
  CWQ_BATCH_CHUNKS=$k C3_SPLIT=1 C3_NO_CPROFILE=1 timeout -k 10 120 python -u tools/c3_pyprof.py > gpurun_out/c3_k$k.log 2>&1 || exit 1
  echo "chunks $k: $(grep 'ms per call' gpurun_out/c3_k$k.log | tr '\n' ' ')"
done && \
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_phases.so C3_CALLS=3 C3_NO_CPROFILE=1 timeout -k 10 120 python -u tools/c3_pyprof.py > gpurun_out/c3_phases.log 2>&1 && \
C3_CALLS=6 C3_NO_CPROFILE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3tl -o run --output-format csv -- python3 tools/c3_pyprof.py > gpurun_out/c3_tl.log 2>&1 && \
python tools/timeline.py gpurun_out/prof_c3tl 15 > gpurun_out/c3_timeline.txt && tail -1 gpurun_out/c3_timeline.txt
