"""cProfile of one I1 image through code_grouped_importance_sample (GPU box):
where the ~3 ms of host time per image around the 8.4 ms scoring goes."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
import compression_without_quantization_amd.coded_importance_sampler as I  # noqa: E402
from compression_without_quantization_amd.synthetic import make_latents  # noqa: E402

I.VERBOSE = False
dev = torch.device("cuda", 0)
q_loc, q_scale, p_loc, p_scale = make_latents(196608, bits_per_dim=1.1, seed=0)
t = C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev))
p = C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev))


def call():
    return C.code_grouped_importance_sample(None, t, p, 42, 20, 4, 16)


for _ in range(3):
    call()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    call()
torch.cuda.synchronize()
print(f"{(time.perf_counter() - t0) / 10 * 1e3:.3f} ms per call", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    call()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(15)
