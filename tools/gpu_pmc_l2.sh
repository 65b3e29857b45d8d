set -o pipefail
export TMPDIR=/tmp
C=${1:-c2low}
B="bench.py --config $C --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2_$C -o run --output-format csv -- python3 $B > gpurun_out/pmc_l2_$C.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_l1_$C -o run --output-format csv -- python3 $B > gpurun_out/pmc_l1_$C.log 2>&1
