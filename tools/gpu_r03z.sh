set -o pipefail
# Small-candidate screen without global atomics for one-tile blocks, one wave
# max per 4-row span, folded Philox below 2^32: GPU suite, the screened
# small-path stress sweep, C2/C3 bench lines and a C3 kernel trace.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
STRESS_BITS=6,11 timeout -k 10 300 python -u tools/stress_csr.py 400 21000 200 > gpurun_out/stress_small.log 2>&1 && tail -1 gpurun_out/stress_small.log && \
timeout -k 10 300 python -u bench.py --config c2 --steps 100 --warmup 5 > gpurun_out/b_c2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 2 > gpurun_out/b_c3.log 2>&1 && \
for c in c2 c3; do tail -1 gpurun_out/b_$c.log | cut -c1-200; done && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3z -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --config c3 --steps 4 --warmup 1 > gpurun_out/prof_c3z.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2z -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --config c2 --steps 4 --warmup 1 > gpurun_out/prof_c2z.log 2>&1 && \
echo r03z done
