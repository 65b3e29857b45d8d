set -o pipefail
# Round evidence, part 1 (run on the GPU box): full GPU tests, smoke, every
# bench config (gpurun_out/b_<config>.log) and the driver's multi-rank launch
# rehearsed at N=2 (torch.distributed.run, two ranks sharing the box's GPU).
# Part 2 (profiles) is tools/gpu_profiles.sh.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
timeout -k 10 600 python -u bench.py > gpurun_out/b_c4.log 2>&1 && tail -1 gpurun_out/b_c4.log | cut -c1-160 && \
for c in c5 c2cli c2low i1 pln; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 > gpurun_out/b_$c.log 2>&1 || exit 1
done && \
for c in c1 c3 i2 pln_is; do  # short steps: more of them (host and launch jitter)
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 2 > gpurun_out/b_$c.log 2>&1 || exit 1
done && \
timeout -k 10 300 python -u bench.py --config c2 --steps 100 --warmup 5 > gpurun_out/b_c2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --blocks 128 --steps 20 --warmup 2 > gpurun_out/b_c5_shard8.log 2>&1 && \
timeout -k 10 300 python -u bench.py --blocks 125000 --steps 3 --warmup 1 --no-cpu > gpurun_out/b_c4_shard8.log 2>&1 && \
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --blocks 65536 > gpurun_out/b_torchrun2.log 2>&1 && tail -1 gpurun_out/b_torchrun2.log | cut -c1-160 && \
echo round-evidence-1 done
