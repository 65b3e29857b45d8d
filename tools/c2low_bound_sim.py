"""Simulation behind DESIGN.md 9c (c2low): does a reachable-range bound for the
unvisited dims (|z| <= 5.68, the Box-Muller output range) drop rows earlier than
the zero-deficit bound the CSR kernel uses?  Largest c2low group, 30 shard steps
of 2^14 candidates, exact f64 deficits, each step's final best known in advance
(the ideal drop test).  Prints per step the fraction of dims visited: A = zero-
deficit bound, B = reachable bound, same order, Bo = reachable bound visiting by
expected deficit minus the bound.  CPU only; ~10 min."""
import sys, numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from compression_without_quantization_amd.synthetic import make_latents
import compression_without_quantization_amd.coded_greedy_sampler as S
q, qs, p, ps = make_latents(196608, bits_per_dim=0.06)
tl, ts = (q - p) / ps, qs / ps  # standardised target (f64 is enough here)
kl = (np.log(ps / qs) + (qs ** 2 + (q - p) ** 2) / (2 * ps ** 2) - 0.5).astype(np.float32)
st = S.group_starts(kl, 14 * 30, 12)
sz = np.diff(st)
print("groups", len(sz), "sizes max", sz.max(), "mean", sz.mean())
gi = int(sys.argv[1]) if len(sys.argv) > 1 else int(np.argmax(sz))
a0, a1 = st[gi], st[gi + 1]
mu = tl[a0:a1].astype(np.float64); sg = ts[a0:a1].astype(np.float64)
d = mu.size
nst = 30; b = 1 / np.sqrt(nst); Z = 5.68
rng = np.random.default_rng(1)
Sacc = np.zeros(d)
tot = {"A": 0, "B": 0, "Bo": 0}; full = 0
for step in range(nst):
    a = Sacc - mu
    ed = 0.5 * (a * a + b * b) / sg**2
    m = 0.5 * (np.maximum(0, np.abs(a) - Z * b) / sg) ** 2
    orders = {"A": np.argsort(-ed), "B": np.argsort(-ed), "Bo": np.argsort(-(ed - m))}
    Zs = rng.standard_normal((16384, d), dtype=np.float32)
    best = None
    dall = []
    for c in range(0, 16384, 2048):
        x = a[None, :] + b * Zs[c:c + 2048].astype(np.float64)
        dd = 0.5 * (x / sg) ** 2
        dall.append(dd)
    D = np.concatenate(dall)
    tot_d = D.sum(1)
    ib = int(np.argmin(tot_d)); Db = tot_d[ib]
    for k, o in orders.items():
        mm = m[o] if k != "A" else np.zeros(d)
        rest = np.concatenate([np.cumsum(mm[::-1])[::-1][1:], [0.0]])  # bound of dims after position
        vis = 0
        for c in range(0, 16384, 2048):
            cs = np.cumsum(D[c:c + 2048][:, o], axis=1) + rest[None, :]
            drop = cs > Db * (1 + 1e-12)
            first = np.where(drop.any(1), drop.argmax(1) + 1, d)
            vis += first.sum()
        tot[k] += vis
    full += 16384 * d
    Sacc = Sacc + b * Zs[ib].astype(np.float64)
    print(step, {k: round(v / full, 4) for k, v in tot.items()}, "K/Db", round(m.sum() / Db, 3), flush=True)
