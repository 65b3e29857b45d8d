"""Encode time of uniform block shapes across KL rates (GPU box).

Times one encode_blocks call (prune mode 2, device-resident synthetic blocks)
per "d:bits:nb" shape given on the command line, best of 3 after a warmup;
prints ms, blocks/s and candidates/s.  With CWQ_LIB_PATH set to a variant
build (tools/variants.sh) it compares launch policies such as
CWQ_PRE_MIN_CAND across rates.  Usage: python tools/rate_sweep.py 16:20:4096 ...
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
from compression_without_quantization_amd.synthetic import make_blocks  # noqa: E402

dev = torch.device("cuda", 0)
for spec in sys.argv[1:]:
    d, bits, nb = (int(v) for v in spec.split(":"))
    b = make_blocks(nb, d, bits)
    x = [torch.from_numpy(b[k].reshape(-1)).to(dev)
         for k in ("post_loc", "post_scale", "prior_loc", "prior_scale")]
    C.encode_blocks(*x, bits, 1, 42, block_dim=d)
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        C.encode_blocks(*x, bits, 1, 42, block_dim=d)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    print(f"d={d:3d} bits={bits:2d} nb={nb:7d}  {best * 1e3:9.2f} ms  {nb / best:11.4e} blocks/s  "
          f"{nb * 2.0 ** bits / best:11.4e} cand/s", flush=True)
