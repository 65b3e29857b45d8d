#!/bin/bash
# Build compile-time tuning variants of libcwq.so into tools/vrun/ (built here just before a GPU call, removed after it; never shipped otherwise) and
# time each on a bench config (run on the GPU box).
# Usage: tools/variants.sh build | [VARIANTS="base t512"] [BENCH_ARGS="--config c2cli"] tools/variants.sh run
set -e
cd "$(dirname "$0")/.."
CSRC=compression_without_quantization_amd/csrc
OUT=${VOUT:-tools/vrun}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared"
declare -A V=(
  [base]=""
  [stats]="-DCWQ_PRUNE_STATS"
  [phases]="-DCWQ_PHASE_TIMES"
  [nocoop]="-DCWQ_CSR_COOP_ROWS_PER_LANE=0"
  [coop64]="-DCWQ_CSR_COOP_ROWS_PER_LANE=64"
  [t64]="-DCWQ_CSR_COOP_TILE=64 -DCWQ_CSR_COOP_TILES=12288"
  [t256]="-DCWQ_CSR_COOP_TILE=256 -DCWQ_CSR_COOP_TILES=3072"
  [mind128]="-DCWQ_CSR_COOP_MIN_D=128 -DCWQ_CSR_COOP_ROWS_PER_LANE=64"
  [gs16]="-DCWQ_CSR_GTAU_SHARE=1 -DCWQ_CSR_GTAU_MASK=15u -DCWQ_CSR_GTAU_STRIDE=32"
  [gs64]="-DCWQ_CSR_GTAU_SHARE=1 -DCWQ_CSR_GTAU_MASK=63u -DCWQ_CSR_GTAU_STRIDE=32"
  [gs16n]="-DCWQ_CSR_GTAU_SHARE=1 -DCWQ_CSR_GTAU_MASK=15u"
  [t512]="-DCWQ_CSR_TILE=512 -DCWQ_CSR_TILES=16384"
  [t256b]="-DCWQ_CSR_TILE=256 -DCWQ_CSR_TILES=32768"
  [t2048]="-DCWQ_CSR_TILE=2048 -DCWQ_CSR_TILES=4096"
  [idyn]="-DCWQ_IMP_DYNAMIC_MIN_GROUPS=0"
  [cw]="-DCWQ_CSR_COOP_CLASS_WAVES=1"
  [lds4096]="-DCWQ_CSR_LDS_DIMS=4096"
  [lds2048]="-DCWQ_CSR_LDS_DIMS=2048"
  [iw6]="-DCWQ_IMP_MIN_WAVES=6"
  [iw8]="-DCWQ_IMP_MIN_WAVES=8"
  [mask7]="-DCWQ_TAU_SHARE_MASK=7u"
  [mask31]="-DCWQ_TAU_SHARE_MASK=31u"
  [cap512]="-DCWQ_SURVIVOR_CAP=512"
  [w7]="-DCWQ_PRUNE_MIN_WAVES=7"
  [w5]="-DCWQ_PRUNE_MIN_WAVES=5"
  [w8]="-DCWQ_PRUNE_MIN_WAVES=8"
  [upl2]="-DCWQ_COOP_UPL=2"
  [upl2w5]="-DCWQ_COOP_UPL=2 -DCWQ_CSR_COOP_MIN_WAVES=5"
  [head]=prebuilt
  [noint]="-DCWQ_TILE_INTERLEAVE=0"
  [pg1536]="-DCWQ_PRUNE_GRID=1536"
  [pg12k]="-DCWQ_PRUNE_GRID=12288"
  [pg98k]="-DCWQ_PRUNE_GRID=98304"
  [pg1m]="-DCWQ_PRUNE_GRID=1048576"
  [psplit0]="-DCWQ_PREP_SPLIT_MAX_NB=0"
  [noperm]="-DCWQ_IMP_PERMUTE=0"
  [ig0]="-DCWQ_IMP_GTAU_MASK=0u"
  [ig255]="-DCWQ_IMP_GTAU_MASK=255u"
  [dw6]="-DCWQ_DECODE_MIN_WAVES=6"
  [dw8]="-DCWQ_DECODE_MIN_WAVES=8"
  [sf2]="-DCWQ_SPLIT_FEW=2"
  [sf4]="-DCWQ_SPLIT_FEW=4 -DCWQ_ENCODE_SPLIT=4"
  [ct3k]="-DCWQ_CSR_COOP_TILES=3072"
  [ct12k]="-DCWQ_CSR_COOP_TILES=12288"
  [ct256]="-DCWQ_CSR_COOP_TILE=256"
  [r3w5]="-DCWQ_RUN_UPL=3 -DCWQ_CSR_RUN_MIN_WAVES=5"
  [r4w4]="-DCWQ_RUN_UPL=4 -DCWQ_CSR_RUN_MIN_WAVES=4"
  [r2w5]="-DCWQ_RUN_UPL=2 -DCWQ_CSR_RUN_MIN_WAVES=5"
  [split1]="-DCWQ_ENCODE_SPLIT=1"
  [c4r2]="-DCWQ_COOP_UPL=4 -DCWQ_CSR_COOP_MIN_WAVES=4 -DCWQ_RUN_UPL=2"
  [c4r1]="-DCWQ_COOP_UPL=4 -DCWQ_CSR_COOP_MIN_WAVES=4"
  [c4r2m3]="-DCWQ_COOP_UPL=4 -DCWQ_CSR_COOP_MIN_WAVES=4 -DCWQ_RUN_UPL=2 -DCWQ_TAU_SHARE_MASK=7u"
  [upl2w4]="-DCWQ_COOP_UPL=2 -DCWQ_CSR_COOP_MIN_WAVES=4"
  [upl3w4]="-DCWQ_COOP_UPL=3 -DCWQ_CSR_COOP_MIN_WAVES=4"
  [upl4w4]="-DCWQ_COOP_UPL=4 -DCWQ_CSR_COOP_MIN_WAVES=4"
  [upl2w5m7]="-DCWQ_COOP_UPL=2 -DCWQ_CSR_COOP_MIN_WAVES=5 -DCWQ_TAU_SHARE_MASK=7u"
  [u6w4]="-DCWQ_COOP_UPL=6 -DCWQ_CSR_COOP_MIN_WAVES=4"
  [dnt]="-DCWQ_DECODE_NT=1"
  [dtm]="-DCWQ_DECODE_PROBE=1"
  [dcomp]="-DCWQ_DECODE_PROBE=2"
  [dw4]="-DCWQ_DECODE_MIN_WAVES=4"
  [u4w3]="-DCWQ_COOP_UPL=4 -DCWQ_CSR_COOP_MIN_WAVES=3"
  [u4w5]="-DCWQ_COOP_UPL=4 -DCWQ_CSR_COOP_MIN_WAVES=5"
  [u8w3]="-DCWQ_COOP_UPL=8 -DCWQ_CSR_COOP_MIN_WAVES=3"
  [prepad]=prebuilt
  [lord]="-DCWQ_COOP_LOAD_ORDER=1"
  [nowma]="-DCWQ_WAVE_MAX_ASM=0"
  [noctile]="-DCWQ_COOP_CLASS_TILES=0"
  [seed0]="-DCWQ_SEED_LOG2=0"
  [seed14]="-DCWQ_SEED_LOG2=14"
  [seed18]="-DCWQ_SEED_LOG2=18"
  [seed20]="-DCWQ_SEED_LOG2=20"
  [stats0]="-DCWQ_PRUNE_STATS -DCWQ_SEED_LOG2=0"
  [fw7]="-DCWQ_FUSED_WAVES=7"
  [cw5]="-DCWQ_CSR_COOP_MIN_WAVES=5"
  [rw7]="-DCWQ_CSR_RUN_MIN_WAVES=7"
  [pnofin]="-DCWQ_PROBE_NOFIN"
  [pnoex]="-DCWQ_PROBE_NOEXACT"
  [pnoboth]="-DCWQ_PROBE_NOFIN -DCWQ_PROBE_NOEXACT"
  [fw6]="-DCWQ_FUSED_WAVES=6"
  [nofuse]="-DCWQ_SMALL_FUSED=0"
  [ni0]="-DCWQ_FUSED_NOINLINE=0"
  [tt8k]="-DCWQ_TARGET_TILES=8192"
  [tt32k]="-DCWQ_TARGET_TILES=32768"
  [tt64k]="-DCWQ_TARGET_TILES=65536"
  [tauold]="-DCWQ_TAU_FROM_KEYS=0"
  [seed16]="-DCWQ_SEED_LOG2=16"
  [tt]="-DCWQ_TILE_TIMES"
  [qt]="-DCWQ_QUAD_TIMES"
  [pipe0]="-DCWQ_SMALL_PIPE=0"
  [lpt0]="-DCWQ_SMALL_LPT=0"
  [tt0]="-DCWQ_TILE_TIMES -DCWQ_XCD_BALANCE=0"
  [xcd0]="-DCWQ_XCD_BALANCE=0"
  [tail1]="-DCWQ_TAIL_SPLIT=1"
  [q0]="-DCWQ_TILE_QUEUE=0"
  [qg3k]="-DCWQ_QUEUE_GRID=3072"
  [qg6k]="-DCWQ_QUEUE_GRID=6144"
  [qtail1]="-DCWQ_TAIL_SPLIT=1"
  [tail2]="-DCWQ_TAIL_SPLIT=2"
  [tail8]="-DCWQ_TAIL_SPLIT=8"
  [glds0]="-DCWQ_DECODE_GLDS=0"
  [eni0]="-DCWQ_EXACT_NOINLINE=0"
  [eni0fw6]="-DCWQ_EXACT_NOINLINE=0 -DCWQ_FUSED_WAVES=6"
  [fw6]="-DCWQ_FUSED_WAVES=6"
  [glds3]="-DCWQ_GLDS_SLOTS=3 -DCWQ_GLDS_MIN_WAVES=5"
  [fw7ni0]="-DCWQ_FUSED_WAVES=7 -DCWQ_FUSED_NOINLINE=0"
)
if [ "$1" = build ]; then
  mkdir -p $OUT
  for k in ${VARIANTS:-"${!V[@]}"}; do
    [ "${V[$k]}" = prebuilt ] && continue  # built by hand from an older commit
    hipcc $FLAGS ${V[$k]} -o $OUT/libcwq_$k.so $CSRC/cwq_kernels.hip $CSRC/cwq_importance.hip $CSRC/cwq_pln.hip $CSRC/cwq_partition.hip $CSRC/cwq_capi.hip $CSRC/cwq_ac.cpp &
  done
  wait
else
  # VARIANTS="base t512" selects variants; BENCH_ARGS="--config c2cli" the workload
  for k in ${VARIANTS:-$(echo "${!V[@]}" | tr ' ' '\n' | sort)}; do
    [ "$k" = stats ] && continue  # counters only: tools/prune_stats.py
    [ "$k" = phases ] && continue  # host phase timings only
    echo "== $k ${V[$k]}"
    lp=$PWD/$OUT/libcwq_$k.so
    [ "$k" = main ] && lp=$PWD/compression_without_quantization_amd/libcwq.so  # the in-tree build
    CWQ_LIB_PATH=$lp timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --steps 2 --warmup 1 $BENCH_ARGS | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('roofline', {}).get('kernel_ms'))"
  done
fi
