"""cProfile of the PLN codec's compress on the GPU box (bench.py --config pln_is's
workload: one 512x768 image, importance level 1), to see where the host time
goes.  Prints the top functions by cumulative time.

  python tools/pln_prof.py [greedy|importance] [calls]"""
import cProfile
import os
import pstats
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd.coded_greedy_sampler as S  # noqa: E402
import compression_without_quantization_amd.coded_importance_sampler as I  # noqa: E402
from compression_without_quantization_amd import pln as P  # noqa: E402

level1 = sys.argv[1] if len(sys.argv) > 1 else "importance"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
S.VERBOSE = I.VERBOSE = False
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
torch.backends.cudnn.benchmark = False
torch.backends.cudnn.deterministic = True
model = P.ProbabilisticLadderNetwork().to(dev).eval()
H, W = 512, 768
rng = np.random.default_rng(0)
yy, xx = np.mgrid[0:H, 0:W] / max(H, W)
base = np.stack([np.sin(6 * xx + c) * np.cos(4 * yy - c) for c in range(3)], -1)
img = np.clip(0.5 + 0.35 * base + 0.05 * rng.standard_normal((H, W, 3)), 0, 1).astype(
    np.float32)[None]
kw = dict(n_steps=30, n_bits_per_step=14, greedy_max_group_size_bits=12,
          use_importance_sampling=(level1 == "importance"),
          second_level_n_bits_per_group=20, second_level_max_group_size_bits=2,
          second_level_dim_kl_bit_limit=16, first_level_n_bits_per_group=20,
          first_level_max_group_size_bits=4, first_level_dim_kl_bit_limit=16)
path = os.path.join(tempfile.mkdtemp(), "img.miracle")
for _ in range(3):
    model.code_image_greedy(None, img, 42, comp_file_path=path, **kw)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    model.code_image_greedy(None, img, 42, comp_file_path=path, **kw)
torch.cuda.synchronize()
print(f"compress {(time.perf_counter() - t0) / n * 1e3:.2f} ms per image")
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    model.code_image_greedy(None, img, 42, comp_file_path=path, **kw)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
