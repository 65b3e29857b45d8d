"""How many greedy-coder indices depend on the per-candidate numeric choices
that TF/TFP/Eigen cannot pin here.

The oracle declares TFP <= 0.7's Normal.log_prob, -0.5*((x-mu)/sigma)^2 - c,
and Eigen 3.3's AVX (Packet8f) inner-dim sum order.  A TF build could have
computed each candidate row with another log-prob form or sum order; unlike the
per-dim normaliser (tools/normaliser_sensitivity.py) these change every
candidate's value by a different rounding, so they are the choices that can
move an argmax.  The oracle scores every candidate under all
2 forms x 6 orders (oracle.sem_variant_names()):

  forms   tfp07  (declared)  -0.5 * square((x - mu) / sigma) - c
          tfp08  TFP >= 0.8  -0.5 * squared_difference(x / sigma, mu / sigma) - c
  orders  avx8   (declared)  Eigen 3.3 Packet8f partials, predux, scalar tail
          sse4               Packet4f (an SSE-only build)
          avx8x2             two Packet8f accumulators (Eigen 3.4 style)
          avx512             Packet16f folded to Packet8f (AVX512DQ predux)
          seq                a scalar build: left to right
          tree               pairwise halving (a GPU tree reduction, representative)

and, for the RNG's transcendentals, 4 generator variants on the
declared form and order:

  rng     ulp_hash           every Box-Muller output one ulp off glibc's, up or
                             down by a hash of (stream, index): a libm (TF-GPU,
                             Eigen numext, another C library) whose logf /
                             sincosf differ in the last place
          ulp_up, ulp_down   every output one ulp toward +inf / -inf
          v1_f32             the angle in float, (2.0f * (float)M_PI) * U, not
                             TF's double 2.0f * M_PI

and records, per variant, how many indices differ from the declared encoder's
given the same history (multi-step groups follow the declared chain), with the
declared best - second-best gap of every index and of every flipped one.
CPU only (the oracle).  Writes profiles/semantics_sensitivity.json.

Workloads (bench.py's synthetic generators, the bench's own seeds):
  c4     the first --c4-blocks C4 blocks (d=32, 16 bits)
  c2     one C2 image (196,608 latents, grouped at 8 bits)
  c5     the first --c5-blocks C5 blocks (d=16, 24 bits)
  c2cli  --cli-groups evenly spaced groups of the C2 image at the CLI's
         greedy defaults (30 steps x 14 bits, ~376 dims per group)
  c2low  the low-rate C2 image's groups (30 x 14 bits, groups up to 4095
         dims): all of them by default (--low-groups N: N evenly spaced)

Usage: python tools/semantics_sensitivity.py [--c4-blocks 10000] [--c5-blocks 32]
           [--cli-groups 48] [--low-groups 0] [--threads N] [--only c4,c2]
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

GAP_EDGES = [0.0, 1e-7, 1e-6, 1e-5, 1e-4, 1e-3, 1e-2, 1e-1, 1.0, np.inf]


def gap_hist(g):
    h, _ = np.histogram(g, bins=GAP_EDGES)
    return {f"[{a:g},{b:g})": int(c) for a, b, c in zip(GAP_EDGES[:-1], GAP_EDGES[1:], h)}


def summarise(vidx, gap, dev, blocks_note):
    """vidx [nb, ns, V] (v = 0 declared), gap [nb, ns], dev [nb, ns, V].

    Besides the observed flips, a model estimate of the rate: variant v swaps
    the declared best and second-best rows iff their deviations differ by more
    than the gap.  With the gap density near 0 rho0 (per nat, from the nonzero
    gaps below 0.1) and the two rows' deviations independent like the best
    row's, the rate is about rho0 * E|dev_1 - dev_2| ~ rho0 * sqrt(2) * rms(dev).
    Exact ties (gap 0) are counted apart: they are rows on the log-density's
    plateau (-0.5 z^2 below half an ulp of the normaliser, e.g. the 1-dim last
    group of a grouped latent), equal under every variant and resolved by the
    lowest index (A.7)."""
    names = O.sem_variant_names()
    nb, ns, nv = vidx.shape
    base = vidx[..., 0]
    n = base.size
    g = gap.reshape(-1)
    ties = g == 0.0
    rho0 = float(((g > 0.0) & (g < 0.1)).sum() / max(int((~ties).sum()), 1) / 0.1)
    out = {"indices": int(n), "blocks": int(nb), "steps_per_block": int(ns),
           "sample": blocks_note,
           "best_second_gap": {"min": float(g.min()), "median": float(np.median(g)),
                               "frac_below_1e-5": float((g < 1e-5).mean()),
                               "frac_below_1e-6": float((g < 1e-6).mean()),
                               "exact_ties": int(ties.sum()),
                               "density_near_0_per_nat": rho0,
                               "histogram_nats": gap_hist(g)},
           "variants": {}}
    est_max = 0.0
    worst = 0
    for v in range(1, nv):
        fl = vidx[..., v] != base
        k = int(fl.sum())
        worst = max(worst, k)
        dv = np.abs(dev[..., v].astype(np.float64)).reshape(-1)
        rms = float(np.sqrt((dv ** 2).mean()))
        est = rho0 * np.sqrt(2.0) * rms
        est_max = max(est_max, est)
        out["variants"][names[v]] = {
            "index_flips": k, "index_flip_rate": k / n,
            "best_row_deviation_nats": {"rms": rms, "max": float(dv.max()),
                                        "frac_rows_changed": float((dv > 0).mean())},
            "model_flip_rate": est,
            "flip_rate_95pct_upper": (3.0 / n if k == 0 else None),
            "blocks_with_a_flip": int(fl.any(axis=1).sum()),
            "flipped_gaps_max": float(gap[fl].max()) if k else None,
            "flipped_gap_histogram_nats": gap_hist(gap[fl]) if k else None}
    out["max_flips_over_variants"] = worst
    out["max_flip_rate_over_variants"] = worst / n
    out["max_model_flip_rate_over_variants"] = est_max
    return out


def run(name, tl, ts, pl, ps, off, bits, n_steps, thr, note):
    t0 = time.perf_counter()
    vidx, _, gap, dev = O.greedy_encode_semvar(tl, ts, pl, ps, off, bits, n_steps, 42, 1.0, 0,
                                               thr)
    r = summarise(vidx, gap, dev, note)
    r["n_bits"], r["seconds"] = bits, round(time.perf_counter() - t0, 1)
    print(name, json.dumps({k: r[k] for k in ("indices", "max_flips_over_variants",
                                              "max_model_flip_rate_over_variants", "seconds")}),
          {v: x["index_flips"] for v, x in r["variants"].items()}, flush=True)
    return r


def uniform(nb, d, bits):
    h = make_blocks_range(0, nb, d, bits, seed=DEFAULT_SEED)
    return ([h[k].reshape(-1) for k in ("post_loc", "post_scale", "prior_loc", "prior_scale")],
            np.arange(nb + 1, dtype=np.int64) * d)


def grouped(bpd, bits, n_steps, n_groups):
    """Image 0's latents (bench.py grouped_main: seed 0), standardised and
    partitioned as the grouped coder does; n_groups evenly spaced groups (all
    if None).  Returns the standardised CSR slice and a note."""
    ql, qs, pl, ps = make_latents(32 * 48 * 128, bits_per_dim=bpd, seed=0)
    tl, ts = O.standardise(ql, qs, pl, ps)
    kl = O.kl_normal_normal(ql, qs, pl, ps)
    st = np.asarray(O.group_starts(kl, bits * n_steps, group_size_threshold(12)), np.int64)
    G = st.size - 1
    pick = np.arange(G) if n_groups is None or n_groups >= G else \
        np.unique(np.linspace(0, G - 1, n_groups).round().astype(np.int64))
    a, b = st[pick], st[pick + 1]
    sel = np.concatenate([np.arange(x, y) for x, y in zip(a, b)])
    off = np.concatenate([[0], np.cumsum(b - a)]).astype(np.int64)
    D = sel.size
    note = (f"{pick.size} of the image's {G} groups ({D} dims; sizes {int((b - a).min())}-"
            f"{int((b - a).max())})")
    return (tl[sel], ts[sel], np.zeros(D, np.float32), np.ones(D, np.float32)), off, note


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c4-blocks", type=int, default=10000)
    ap.add_argument("--c5-blocks", type=int, default=32)
    ap.add_argument("--cli-groups", type=int, default=48)
    ap.add_argument("--low-groups", type=int, default=0, help="0: every group")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--only", default="c4,c2,c5,c2cli,c2low")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "semantics_sensitivity.json"))
    a = ap.parse_args()
    only = set(a.only.split(","))
    res = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            res = json.load(f)
    res["method"] = (__doc__.strip().split("\n\n")[0] + " (tools/semantics_sensitivity.py)")
    res["variants"] = O.sem_variant_names()[1:]
    res["declared"] = O.sem_variant_names()[0]
    res["source"] = ("[ext] TFP 0.8 Normal._log_prob and Eigen 3.3/3.4 reducer packet orders "
                     "recalled from their public sources, and proxies for a non-glibc "
                     "logf/sincosf and a float 2*pi (oracle/cwq_oracle.c "
                     "cwqo_greedy_encode_semvar); unpinned, like SURVEY.md A.4-A.6")
    if "c4" in only:
        (tl, ts, pl, ps), off = uniform(a.c4_blocks, 32, 16)
        res["c4"] = run("c4", tl, ts, pl, ps, off, 16, 1, a.threads,
                        f"first {a.c4_blocks} C4 blocks")
    if "c5" in only:
        (tl, ts, pl, ps), off = uniform(a.c5_blocks, 16, 24)
        res["c5"] = run("c5", tl, ts, pl, ps, off, 24, 1, a.threads,
                        f"first {a.c5_blocks} C5 blocks (2^24 candidates each)")
    if "c2" in only:
        (tl, ts, pl, ps), off, note = grouped(1.1, 8, 1, None)
        res["c2"] = run("c2", tl, ts, pl, ps, off, 8, 1, a.threads, "C2 image 0: " + note)
    if "c2cli" in only:
        (tl, ts, pl, ps), off, note = grouped(1.1, 14, 30, a.cli_groups)
        res["c2cli"] = run("c2cli", tl, ts, pl, ps, off, 14, 30, a.threads,
                           "C2 image 0 at 30 x 14 bits: " + note)
    if "c2low" in only:
        (tl, ts, pl, ps), off, note = grouped(0.06, 14, 30, a.low_groups or None)
        res["c2low"] = run("c2low", tl, ts, pl, ps, off, 14, 30, a.threads,
                           "low-rate C2 image 0 at 30 x 14 bits: " + note)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
