"""Do host<->device copies overlap a running encode on MI355X?  (GPU box)

Times, for one 65,536-block C4 chunk (33.5 MB of inputs): a numpy copy into
pinned memory, H2D from pageable and from pinned memory alone, the encode
alone, and the encode with each kind of H2D issued on a second stream while it
runs.  Usage: python tools/copy_overlap.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
from compression_without_quantization_amd.synthetic import make_blocks_range  # noqa: E402

dev = torch.device("cuda", 0)
nb, d = 65536, 32
host = make_blocks_range(0, nb, d, 16)
arrs = [np.ascontiguousarray(host[k].reshape(-1)) for k in
        ("post_loc", "post_scale", "prior_loc", "prior_scale")]
src = np.concatenate(arrs)
pin = torch.empty(src.size, dtype=torch.float32, pin_memory=True)
dst = torch.empty(src.size, dtype=torch.float32, device=dev)
x = [torch.from_numpy(a).to(dev) for a in arrs]
out_i = torch.empty((nb, 1), dtype=torch.int32, device=dev)
out_s = torch.empty(nb * d, dtype=torch.float32, device=dev)
ws = torch.empty(C.encode_workspace_bytes(nb, nb * d, block_dim=d), dtype=torch.uint8,
                 device=dev)
side = torch.cuda.Stream(dev)


def encode():
    C.encode_blocks(*x, 16, 1, 42, block_dim=d, out_idx=out_i, out_sample=out_s, workspace=ws)


def timed(f, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


def h2d_pageable():
    dst.copy_(torch.from_numpy(src), non_blocking=True)


def h2d_pinned():
    dst.copy_(pin, non_blocking=True)


def both(copy):
    def f():
        encode()
        with torch.cuda.stream(side):
            copy()
    return f


encode()
print(f"numpy -> pinned copy  {timed(lambda: pin.numpy().__setitem__(slice(None), src)):8.2f} ms "
      f"({src.nbytes / 1e6:.1f} MB)", flush=True)
print(f"H2D pageable          {timed(h2d_pageable):8.2f} ms", flush=True)
print(f"H2D pinned            {timed(h2d_pinned):8.2f} ms", flush=True)
print(f"encode                {timed(encode):8.2f} ms", flush=True)
print(f"encode + H2D pageable {timed(both(h2d_pageable)):8.2f} ms", flush=True)
print(f"encode + H2D pinned   {timed(both(h2d_pinned)):8.2f} ms", flush=True)
