set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "grouped or c3 or batch" --timeout 300 --timeout-method thread > gpurun_out/t_grp.log 2>&1 && tail -1 gpurun_out/t_grp.log && \
for k in 4 6 8; do
  CWQ_BATCH_CHUNKS=$k timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --batch-only --no-cpu > gpurun_out/b_c3_k$k.log 2>&1 || exit 1
  echo "chunks $k: $(tail -1 gpurun_out/b_c3_k$k.log | cut -c1-200)"
done && \
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_phases.so timeout -k 10 120 python -u bench.py --config c3 --steps 2 --warmup 1 --batch-only --no-cpu > gpurun_out/b_c3_phases.log 2>&1 && \
timeout -k 10 200 python -u tools/c3_pyprof.py > gpurun_out/c3_pyprof.log 2>&1 && head -45 gpurun_out/c3_pyprof.log
