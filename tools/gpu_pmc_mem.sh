set -o pipefail
# Vector-memory pipeline PMC passes for the general pruned kernel (GPU box):
# texture addresser / data busy, SQ stalls on the TA FIFOs, L1 and L2 behaviour.
# Usage: tools/gpu_pmc_mem.sh CONFIG TAG   (CWQ_LIB_PATH selects a variant build)
export TMPDIR=/tmp
C=${1:-c2low}
T=${2:-$C}
B="bench.py --no-cpu --no-e2e --config $C --steps 1 --warmup 0"
O=gpurun_out/pmcm_$T
p() { timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$1 -o run --output-format csv -- python3 $B > $O.$1.log 2>&1; }
mkdir -p $O
p TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE && \
p TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE && \
p SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE && \
p TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum && \
p TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum && \
echo pmc-mem done
