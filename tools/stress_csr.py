"""Ad-hoc sweep (GPU box): random ragged group layouts through the general pruned
kernel (k_encode_prune_csr), pruned (mode 2) against unpruned exact (mode 0).

Wider than tests/test_gpu.py::test_csr_random_stress: group sizes up to a few
thousand dims, so it reaches the cooperative 16-lane rows (d >= 256), the
constants read from global memory (d > 1024), the 2- and 3-stream step splits,
near-tie (low-rate) inputs, per-lane rows of long groups (constants in global
memory) and groups past the sorted-order limit (8189 dims).  Prints one line per trial; exits 1 on a mismatch.

Usage: [STRESS_BITS=lo,hi] python tools/stress_csr.py [trials] [first_seed] [max_seconds]
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
    if kind == "heavy":
        scale = np.exp(rng.uniform(-3, 3, n))
        pl = (rng.standard_cauchy(n) * scale).astype(np.float32)
        ps = (scale * rng.uniform(0.5, 2.0, n)).astype(np.float32)
        tl = (pl + ps * rng.standard_normal(n) * rng.uniform(0, 2)).astype(np.float32)
        ts = (ps * np.exp(rng.uniform(-2, 0.5, n))).astype(np.float32)
    elif kind == "lowrate":  # posterior close to the prior: many near-ties
        pl = (0.1 * rng.standard_normal(n)).astype(np.float32)
        ps = rng.uniform(0.8, 1.2, n).astype(np.float32)
        tl = (pl + 0.05 * ps * rng.standard_normal(n)).astype(np.float32)
        ts = (ps * rng.uniform(0.9, 1.0, n)).astype(np.float32)
    else:
        tl = rng.standard_normal(n).astype(np.float32)
        ts = rng.uniform(0.2, 1.0, n).astype(np.float32)
        pl = (0.1 * rng.standard_normal(n)).astype(np.float32)
        ps = rng.uniform(0.8, 1.2, n).astype(np.float32)
    return tl, ts, pl, ps


VERBOSE = bool(os.environ.get("STRESS_VERBOSE"))
# bits per step drawn from [BITS_LO, BITS_HI]: 12-16 reach the general pruned
# kernel (>= 4096 candidates); STRESS_BITS=6,11 the screened small-candidate path
BITS_LO, BITS_HI = (int(v) for v in os.environ.get("STRESS_BITS", "12,16").split(","))
# STRESS_SMALL=1: short groups only (d <= 128; all <= 64 in a third of the trials:
# the small pipeline k_small_prep1 / k_small_one / k_small_finalize with
# STRESS_BITS=6,11)
SMALL = bool(os.environ.get("STRESS_SMALL"))


def encode(lib, tl, ts, pl, ps, off, bits, n_steps, seed, rho, mode):
    if VERBOSE:
        print(f"  mode {mode} ...", flush=True)
    i, s = C.encode_blocks(tl, ts, pl, ps, bits, n_steps, seed, rho=rho, block_off=off,
                           prune_mode=mode)
    torch.cuda.synchronize()
    return i.cpu().numpy(), s.cpu().numpy().view(np.uint32)


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 9000
    budget = float(sys.argv[3]) if len(sys.argv) > 3 else 240.0
    lib = _lib.load()
    t_end = time.time() + budget
    bad = done = 0
    for t in range(first, first + trials):
        if time.time() > t_end:
            break
        rng = np.random.default_rng(t)
        nb = int(rng.integers(1, 9))
        shape = t % 6
        if shape == 4:    # many long groups: per-lane rows reading constants from global
            nb = int(rng.integers(50, 120))
            sizes = rng.integers(900, 3000, nb)
        elif shape == 5:  # one huge group: unsorted (natural) visit order
            sizes = np.array([int(rng.integers(8200, 20000))] + list(rng.integers(0, 50, nb - 1)))
        elif shape == 0:    # a few long groups: cooperative rows, some beyond LDS
            sizes = rng.integers(200, 4000, nb)
        elif shape == 1:  # mixed short and long in one launch
            sizes = np.where(rng.random(nb) < 0.5, rng.integers(0, 200, nb),
                             rng.integers(256, 2500, nb))
        elif shape == 2:  # many short groups: per-lane rows, multi-stream split
            nb = int(rng.integers(16, 200))
            sizes = rng.integers(0, 300, nb)
        else:             # uniform long groups
            sizes = np.full(nb, int(rng.choice([256, 300, 1024, 1025, 2048, 3001])))
        if SMALL:  # the fused small-candidate kernel's blocks (d <= 128), many of them
            nb = int(rng.integers(1, 3000))
            sizes = rng.integers(0, int(rng.choice([3, 8, 33, 65, 65, 129])), nb)  # 65: max 64 (fused)
        sizes = [int(x) for x in sizes]
        if sum(sizes) == 0:
            sizes[0] = 1
        off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        D = int(off[-1])
        bits = int(rng.integers(BITS_LO, BITS_HI + 1))
        n_steps = int(rng.integers(1, 4))
        rho = float(rng.choice([1.0, 0.7, 1.3]))
        seed = int(rng.integers(-2 ** 31, 2 ** 31 - 1))
        kind = ["normal", "heavy", "lowrate"][int(rng.integers(0, 3))]
        tl, ts, pl, ps = inputs(rng, D, kind)
        i0, s0 = encode(lib, tl, ts, pl, ps, off, bits, n_steps, seed, rho, 0)
        i2, s2 = encode(lib, tl, ts, pl, ps, off, bits, n_steps, seed, rho, 2)
        ok = np.array_equal(i0, i2) and np.array_equal(s0, s2)
        done += 1
        bad += not ok
        print(f"trial {t} {'ok ' if ok else 'BAD'} nb={nb} D={D} max_d={max(sizes)} "
              f"bits={bits} steps={n_steps} rho={rho} {kind}", flush=True)
    print(f"{done} trials, {bad} mismatches", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
