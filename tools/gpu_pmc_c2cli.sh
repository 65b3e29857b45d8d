set -o pipefail
export TMPDIR=/tmp
B="bench.py --no-cpu --no-e2e --config c2cli --steps 1 --warmup 0"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_c2cli/a -o run --output-format csv -- python3 $B > gpurun_out/pmc_a.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU -d gpurun_out/pmc_c2cli/b -o run --output-format csv -- python3 $B > gpurun_out/pmc_b.log 2>&1
