"""How many greedy-coder indices depend on the one undeclarable numeric choice
of the per-dim normaliser c_j = fl32(0.9189385f + log sigma_j) (SURVEY.md A.5,
DESIGN.md 2).  The oracle declares glibc logf for log sigma; TF's CPU kernel
would use Eigen's plog for full 8-wide packets (dims below 8 floor(d / 8)) and
std::log for the tail, and either may differ by one ulp.  Re-encodes C4 blocks
(the bench's first N, d = 32, 16 bits) and one C2 image (196,608 PLN-like
latents, grouped at 8 bits) with log sigma replaced by:

  plog      Eigen 3.3 plog<Packet8f> (non-fused mul + add: a plain -mavx build)
            on the full packets, logf on the tail
  plog_fma  the same with fused multiply-adds (an -mfma build)
  up / down logf + 1 ulp / - 1 ulp on every dim
  random    logf +- 1 ulp per dim (seeded signs)

and counts the indices that change.  CPU only (the oracle).  Writes
profiles/normaliser_sensitivity.json.

Usage: python tools/normaliser_sensitivity.py [--c4-blocks 10000] [--threads N]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import oracle as O  # noqa: E402
from compression_without_quantization_amd.synthetic import (DEFAULT_SEED, make_blocks_range,  # noqa
                                                            make_latents)
from compression_without_quantization_amd.coded_greedy_sampler import group_size_threshold  # noqa


def packet_plog(ts, block_off, fma):
    """log sigma as TF's Eigen unary op would give it per block: plog on the
    first 8 floor(d / 8) dims of each block's [d] vector, logf on the rest."""
    out = O.logf_table(ts)
    pl = O.eigen_plog(ts, fma)
    for g in range(block_off.size - 1):
        a, b = int(block_off[g]), int(block_off[g + 1])
        v = a + (b - a) // 8 * 8
        out[a:v] = pl[a:v]
    return out


def variants(ts, block_off, rng):
    lf = O.logf_table(ts)
    sgn = rng.integers(0, 2, ts.size) * 2 - 1
    return {
        "plog": packet_plog(ts, block_off, False),
        "plog_fma": packet_plog(ts, block_off, True),
        "up": np.nextafter(lf, np.float32(np.inf)),
        "down": np.nextafter(lf, np.float32(-np.inf)),
        "random": np.where(sgn > 0, np.nextafter(lf, np.float32(np.inf)),
                           np.nextafter(lf, np.float32(-np.inf))).astype(np.float32),
    }


def run(name, tl, ts, pl, ps, off, bits, n_steps, thr):
    base_idx, base_s = O.greedy_encode(tl, ts, pl, ps, off, bits, n_steps, 42, 1.0, 0, thr)
    lf = O.logf_table(ts)
    same_idx, same_s, gap = O.greedy_encode_lsig(tl, ts, pl, ps, off, bits, n_steps, 42, lf, 1.0,
                                                 0, thr, gaps=True)
    assert np.array_equal(same_idx, base_idx) and np.array_equal(same_s.view(np.uint32),
                                                                   base_s.view(np.uint32))
    out = {"indices": int(base_idx.size), "blocks": int(off.size - 1), "n_bits": bits}
    # a changed normaliser moves every row by nearly the same amount: only rows
    # within the summation's rounding noise (~1e-5 nats for these rows) of the
    # winner can trade places, so the best - second-best gaps bound the rate
    g = gap.reshape(-1)
    out["best_second_gap"] = {
        "min": float(g.min()), "median": float(np.median(g)),
        "frac_below_1e-4": float((g < 1e-4).mean()), "frac_below_1e-5": float((g < 1e-5).mean()),
        "frac_below_1e-6": float((g < 1e-6).mean()),
        "frac_below_1e-2_per_nat": float((g < 1e-2).mean() / 1e-2)}
    half = np.float32(0.5 * np.log(2.0 * np.pi))
    c_base = half + lf
    for vname, ls in variants(ts, off, np.random.default_rng(7)).items():
        t0 = time.perf_counter()
        vi, vs = O.greedy_encode_lsig(tl, ts, pl, ps, off, bits, n_steps, 42, ls, 1.0, 0, thr)
        flips = int((vi != base_idx).sum())
        nb_flip = int((vi != base_idx).any(axis=1).sum())
        out[vname] = {
            "log_sigma_changed_frac": float((ls != lf).mean()),
            "normaliser_changed_frac": float(((half + ls) != c_base).mean()),
            "index_flips": flips, "index_flip_rate": flips / base_idx.size,
            "blocks_changed": nb_flip, "seconds": round(time.perf_counter() - t0, 2)}
        print(name, vname, out[vname], flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c4-blocks", type=int, default=10000)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "normaliser_sensitivity.json"))
    a = ap.parse_args()
    res = {"method": __doc__.strip().split("\n\n")[0] + " (tools/normaliser_sensitivity.py)",
           "eigen_plog_source": "[ext] Eigen 3.3 plog<Packet8f> restated from its published "
                                "Cephes coefficients (oracle/cwq_oracle.c cwqo_eigen_plog); "
                                "unpinned, like the rest of SURVEY.md A.2-A.6"}
    # plog vs glibc logf over a dense sample of the sigma range the inputs use
    x = np.random.default_rng(1).uniform(0.05, 4.0, 4_000_000).astype(np.float32)
    d = O.eigen_plog(x).view(np.int32).astype(np.int64) - O.logf_table(x).view(np.int32)
    res["plog_vs_logf"] = {"sample": "4e6 uniform floats in [0.05, 4)",
                           "differ_frac": float((d != 0).mean()), "max_ulp": int(np.abs(d).max())}
    h = make_blocks_range(0, a.c4_blocks, 32, 16, seed=DEFAULT_SEED)
    off = np.arange(a.c4_blocks + 1, dtype=np.int64) * 32
    res["c4"] = run("c4", h["post_loc"].reshape(-1), h["post_scale"].reshape(-1),
                    h["prior_loc"].reshape(-1), h["prior_scale"].reshape(-1), off, 16, 1,
                    a.threads)
    # C2: one image's level-1 latents, standardised, grouped at 8 bits
    ql, qs, pl, ps = make_latents(32 * 48 * 128, bits_per_dim=1.1, seed=0)
    tl, ts = O.standardise(ql, qs, pl, ps)
    kl = O.kl_normal_normal(ql, qs, pl, ps)
    st = np.asarray(O.group_starts(kl, 8, group_size_threshold(12)), dtype=np.int64)
    D = tl.size
    res["c2"] = run("c2", tl, ts, np.zeros(D, np.float32), np.ones(D, np.float32), st, 8, 1,
                    a.threads)
    res["c2"]["groups_with_full_packets"] = int((np.diff(st) >= 8).sum())
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("plog_vs_logf",)}))


if __name__ == "__main__":
    main()
