set -o pipefail
export TMPDIR=/tmp
C=${1:-i1}
B="bench.py --config $C --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_$C/t -o run --output-format csv -- python3 $B > gpurun_out/pmc_${C}_t.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d gpurun_out/pmc_$C/a -o run --output-format csv -- python3 $B > gpurun_out/pmc_${C}_a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d gpurun_out/pmc_$C/b -o run --output-format csv -- python3 $B > gpurun_out/pmc_${C}_b.log 2>&1
