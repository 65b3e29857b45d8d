"""Which blocks / steps of a small-candidate CSR encode differ from the oracle
(the test_small_path_adversarial inputs, kind "normal"), for the library
selected by CWQ_LIB_PATH.  Usage: python tools/debug_small.py [BITS] [N_STEPS]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
from oracle import oracle as O  # noqa: E402

bits = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rng = np.random.default_rng(sum(map(ord, "normal")) + bits)
sizes = [3, 20, 1, 45, 0, 7, 64, 33, 64, 2, 0, 0, 5]
off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
D = int(off[-1])
pl = (0.2 * rng.standard_normal(D)).astype(np.float32)
ps = rng.uniform(0.5, 2.0, D).astype(np.float32)
tl = (pl + ps * rng.standard_normal(D) * 0.8).astype(np.float32)
ts = (ps * rng.uniform(0.3, 1.0, D)).astype(np.float32)
wi, ws = O.greedy_encode(tl, ts, pl, ps, off, bits, n_steps, 5)
for mode in (0, 2):
    gi, gs = C.encode_blocks(tl, ts, pl, ps, bits, n_steps, 5, block_off=off, prune_mode=mode)
    torch.cuda.synchronize()
    gi, gs = gi.cpu().numpy(), gs.cpu().numpy()
    for b in range(len(sizes)):
        sl = slice(off[b], off[b + 1])
        ok_i = np.array_equal(gi[b], wi[b])
        ok_s = np.array_equal(gs[sl].view(np.uint32), ws[sl].view(np.uint32))
        if not (ok_i and ok_s):
            print(f"mode {mode} block {b} d={sizes[b]}: gpu {gi[b].tolist()} oracle {wi[b].tolist()}"
                  f" sample_equal={ok_s}")
    print(f"mode {mode}: {int((gi != wi).sum())} index mismatches", flush=True)
