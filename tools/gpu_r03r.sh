set -o pipefail
# Round 3: INTER tiles (several per block) share tau through keys[g] inside the
# loop (CWQ_INTER_KEY_SHARE), C5 and its N = 8 shard, vs the build without.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
timeout -k 10 300 python -u tools/stress_modes.py 300 > gpurun_out/stress_modes.log 2>&1 && tail -1 gpurun_out/stress_modes.log && \
VARIANTS="nokey base key15 nokey base key15" BENCH_ARGS="--config c5 --steps 3 --warmup 1" bash tools/variants.sh run > gpurun_out/key_c5.log 2>&1 && grep -v amdgpu.ids gpurun_out/key_c5.log && \
VARIANTS="nokey base key15 nokey base key15" BENCH_ARGS="--config c5 --blocks 128 --steps 3 --warmup 1" bash tools/variants.sh run > gpurun_out/key_c5s.log 2>&1 && grep -v amdgpu.ids gpurun_out/key_c5s.log && \
for v in nokey base; do CWQ_LIB_PATH=$PWD/tools/variants/libcwq_$v.so timeout -k 10 300 python -u tools/rate_sweep.py 16:20:4096 32:22:256 64:20:512 8:24:256 > gpurun_out/key_rs_$v.log 2>&1 || exit 1; echo "== $v"; grep -v amdgpu.ids gpurun_out/key_rs_$v.log; done
