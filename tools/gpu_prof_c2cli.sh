set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2cli -o run -- python3 -u bench.py --config c2cli --steps 2 --warmup 1 > gpurun_out/p_c2cli.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config c2cli --steps 2 --warmup 1 --prune-mode 0 > gpurun_out/b_c2cli_m0.log 2>&1
