"""Ad-hoc sweep (GPU box): random shapes/inputs, encoder modes 0/1/2 must agree.
Usage: python tools/stress_modes.py [trials] [first_seed]"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C
from compression_without_quantization_amd import _lib

lib = _lib.load()
trials = int(sys.argv[1]) if len(sys.argv) > 1 else 200
first = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
bad = 0
for t in range(first, first + trials):
    rng = np.random.default_rng(t)
    d = int(rng.choice([8, 16, 24, 32, 40, 48, 56, 64]))
    bits = int(rng.integers(1, 21))
    n_steps = int(rng.integers(1, 4))
    nb = int(rng.integers(1, 17))
    rho = float(rng.choice([1.0, 0.5, 0.9, 1.5]))
    seed = int(rng.integers(-2 ** 31, 2 ** 31 - 1))
    n = nb * d
    kind = t % 4
    scale = np.exp(rng.uniform(-6, 6, n)) if kind == 0 else np.ones(n)
    pl = (rng.standard_cauchy(n) * scale).astype(np.float32)
    ps = (scale * rng.uniform(0.3, 3.0, n)).astype(np.float32)
    tl = (pl + ps * rng.standard_normal(n) * rng.uniform(0, 3)).astype(np.float32)
    ts = (ps * np.exp(rng.uniform(-4, 1, n))).astype(np.float32)
    if kind == 2:
        tl = pl.copy(); ts = ps.copy()
    if kind == 3:
        ts = (ps * np.exp(rng.uniform(-9, -6, n))).astype(np.float32)
    outs = []
    for mode in (0, 1, 2):
        i, s = C.encode_blocks(tl, ts, pl, ps, bits, n_steps, seed, rho=rho, block_dim=d,
                               prune_mode=mode)
        torch.cuda.synchronize()
        outs.append((i.cpu().numpy(), s.cpu().numpy().view(np.uint32)))
    ok = all(np.array_equal(outs[0][0], o[0]) and np.array_equal(outs[0][1], o[1]) for o in outs[1:])
    if not ok:
        bad += 1
        print("MISMATCH trial", t, d, bits, n_steps, nb, rho, kind, flush=True)
print(f"{trials} trials, {bad} mismatches", flush=True)
