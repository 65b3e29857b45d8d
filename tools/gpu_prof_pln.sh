set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pln -o run --output-format csv -- python3 -u bench.py --config pln --steps 2 --warmup 1 > gpurun_out/p_pln.log 2>&1
