"""Ad-hoc sweep (GPU box): random group layouts through the importance encoder,
screened (mode 2) against exact (mode 0), plus the decode round trip.

Covers what the fixed tests do not: thousands of groups (the dynamic tile
hand-out starts at 4096), sample counts from 1 to 2^18, group sizes past the
screening LDS limit.  Prints one line per trial; exits 1 on a mismatch.

Usage: python tools/stress_imp.py [trials] [first_seed] [max_seconds]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
from compression_without_quantization_amd import _lib  # noqa: E402


def inputs(rng, n, kind):
    pl = np.zeros(n, np.float32)
    ps = np.ones(n, np.float32)
    tl = (rng.standard_normal(n) * 0.7).astype(np.float32)
    ts = rng.uniform(0.3, 0.95, n).astype(np.float32)
    if kind == "heavy":
        scale = np.exp(rng.uniform(-3, 3, n))
        pl = (rng.standard_cauchy(n) * scale).astype(np.float32)
        ps = (scale * rng.uniform(0.5, 2.0, n)).astype(np.float32)
        tl = (pl + ps * rng.standard_normal(n) * rng.uniform(0, 2)).astype(np.float32)
        ts = (ps * np.exp(rng.uniform(-2, 0.5, n))).astype(np.float32)
    elif kind == "wide":
        ts = rng.uniform(1.0, 3.0, n).astype(np.float32)
    return tl, ts, pl, ps


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 40000
    budget = float(sys.argv[3]) if len(sys.argv) > 3 else 240.0
    lib = _lib.load()
    t_end = time.time() + budget
    bad = done = 0
    for t in range(first, first + trials):
        if time.time() > t_end:
            break
        rng = np.random.default_rng(t)
        shape = t % 3
        if shape == 0:    # many small groups (dynamic tile hand-out)
            nb = int(rng.integers(3000, 7000))
            sizes = rng.integers(1, 17, nb)
            ns = np.minimum(2 ** rng.uniform(0, 12, nb), 4096).astype(np.int64)
        elif shape == 1:  # few groups, many samples
            nb = int(rng.integers(1, 40))
            sizes = rng.integers(1, 17, nb)
            ns = (2 ** rng.uniform(0, 18, nb)).astype(np.int64)
        else:             # long groups, some beyond the screening LDS limit
            nb = int(rng.integers(1, 12))
            sizes = rng.integers(16, 400, nb)
            ns = (2 ** rng.uniform(0, 16, nb)).astype(np.int64)
        ns = np.maximum(ns, 1)
        off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        D = int(off[-1])
        kind = ["normal", "heavy", "wide"][int(rng.integers(0, 3))]
        tl, ts, pl, ps = inputs(rng, D, kind)
        seed = int(rng.integers(-2 ** 31, 2 ** 31 - 1))
        out = []
        for mode in (0, 2):
            i, s = C.importance_encode_blocks(tl, ts, pl, ps, off, ns, seed, prune_mode=mode)
            torch.cuda.synchronize()
            out.append((i.cpu().numpy(), s.cpu().numpy().view(np.uint32)))
        dec = C.importance_decode_blocks(out[1][0], pl, ps, off, seed)
        dec = dec.cpu().numpy().view(np.uint32)
        ok = (np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
              and np.array_equal(dec, out[1][1]))
        done += 1
        bad += not ok
        print(f"trial {t} {'ok ' if ok else 'BAD'} nb={nb} D={D} max_d={int(sizes.max())} "
              f"max_n={int(ns.max())} {kind}", flush=True)
    print(f"{done} trials, {bad} mismatches", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
