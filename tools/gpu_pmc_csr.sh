set -o pipefail
# PMC passes for the general pruned kernel (run on the GPU box).
# Usage: tools/gpu_pmc_csr.sh CONFIG [TAG]   (CWQ_LIB_PATH selects a variant build)
export TMPDIR=/tmp
C=${1:-c2low}
T=${2:-$C}
B="bench.py --no-cpu --no-e2e --config $C --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_$T/t -o run --output-format csv -- python3 $B > gpurun_out/pmc_${T}_t.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d gpurun_out/pmc_$T/a -o run --output-format csv -- python3 $B > gpurun_out/pmc_${T}_a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d gpurun_out/pmc_$T/b -o run --output-format csv -- python3 $B > gpurun_out/pmc_${T}_b.log 2>&1
