"""Decode timing vs GPU clock ramp (GPU box): C4 decode (10^6 x d=32 blocks)
run back to back in batches of 20 launches, each batch timed with HIP events
on the launch stream; prints the per-launch time of every batch.  Short kernels
that follow an idle period may run before the clock has ramped up."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
from compression_without_quantization_amd.synthetic import make_blocks_range  # noqa: E402

nb, d, bits = 1_000_000, 32, 16
h = make_blocks_range(0, nb, d, bits)
dev = torch.device("cuda", 0)
pl = torch.from_numpy(h["prior_loc"].reshape(-1)).to(dev)
ps = torch.from_numpy(h["prior_scale"].reshape(-1)).to(dev)
idx = torch.from_numpy(np.random.default_rng(0).integers(0, 1 << bits, (nb, 1)).astype(np.int32)).to(dev)
out = torch.empty(nb * d, dtype=torch.float32, device=dev)
C.decode_blocks(idx, pl, ps, bits, 1, 42, block_dim=d, out_sample=out)
torch.cuda.synchronize()
time.sleep(float(os.environ.get("IDLE_S", "0.5")))  # let the clock drop, as in bench.py
res = []
for b in range(int(os.environ.get("BATCHES", "12"))):
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        C.decode_blocks(idx, pl, ps, bits, 1, 42, block_dim=d, out_sample=out)
    e.record()
    torch.cuda.synchronize()
    res.append(a.elapsed_time(e) / 20 * 1e3)
print("decode us per launch by batch of 20:", " ".join(f"{x:.1f}" for x in res))
print("GB/s at the best batch:", nb * (12 * d + 4) / (min(res) * 1e-6) / 1e9)
