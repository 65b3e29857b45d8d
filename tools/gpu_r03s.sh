set -o pipefail
# Round 3: the grouped single call in two halves (cwq_code_grouped_greedy_begin
# / _end): the group-start list is built while the device codes.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config c2 --steps 100 --warmup 5 > gpurun_out/b_c2_$r.log 2>&1 || exit 1
  tail -1 gpurun_out/b_c2_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity']['index_mismatches'])"
done && \
timeout -k 10 300 python -u bench.py --config c2cli --steps 3 --warmup 1 --no-cpu > gpurun_out/b_c2cli_s.log 2>&1 && tail -1 gpurun_out/b_c2cli_s.log | cut -c1-220
