set -o pipefail
# Round 3: cooperative occupancy with records through the vector-memory path
# (g*: CWQ_COOP_REC_LDS_POS=0, UPL units per lane, w waves/SIMD) vs LDS records (base).
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="base g4w4 g2w6 g2w5 g4w5 g3w5 base g4w4 g2w6 g2w5 g4w5 g3w5" BENCH_ARGS="--config c2low" bash tools/variants.sh run > gpurun_out/occ_c2low.log 2>&1 && grep -v amdgpu.ids gpurun_out/occ_c2low.log
