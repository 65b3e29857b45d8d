set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config c3 --no-cpu --steps 100 > gpurun_out/bench_c3_defer100.json 2> gpurun_out/bench_c3_defer100.err &&
C3_DEFER=1 C3_WARMUP=5 timeout -k 10 120 python -u tools/c3_loop.py 20 2>&1 | tail -1 | sed "s/^/defer w5 n20: /" &&
C3_WARMUP=5 timeout -k 10 120 python -u tools/c3_loop.py 20 2>&1 | tail -1 | sed "s/^/sync w5 n20: /"
