set -o pipefail
# Round 3: pipelined batch coder (C3) + multi-GPU tests + C5 stats / 1/8 shard.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
for k in 1 2 4 6 8 12; do
  CWQ_BATCH_CHUNKS=$k timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --batch-only --no-cpu > gpurun_out/b_c3_k$k.log 2>&1 || exit 1
  echo "chunks $k: $(tail -1 gpurun_out/b_c3_k$k.log | cut -c1-200)"
done && \
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_phases.so timeout -k 10 120 python -u bench.py --config c3 --steps 2 --warmup 1 --batch-only --no-cpu > gpurun_out/b_c3_phases.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 > gpurun_out/b_c3.log 2>&1 && tail -1 gpurun_out/b_c3.log | cut -c1-400 && \
timeout -k 10 300 python -u bench.py --config c2 --steps 100 --warmup 5 > gpurun_out/b_c2.log 2>&1 && tail -1 gpurun_out/b_c2.log | cut -c1-300 && \
timeout -k 10 300 python -u bench.py --config c5 --blocks 128 --steps 3 --warmup 1 > gpurun_out/b_c5_shard8.log 2>&1 && tail -1 gpurun_out/b_c5_shard8.log | cut -c1-300 && \
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_stats.so PS_D=16 PS_BITS=24 PS_CONFIG=c5 timeout -k 10 170 python -u tools/prune_stats.py 1024 2 --json gpurun_out/prune_stats_c5.json > gpurun_out/ps_c5.log 2>&1 ; cat gpurun_out/ps_c5.log
