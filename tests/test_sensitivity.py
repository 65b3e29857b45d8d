"""CPU: the normaliser sensitivity machinery (tools/normaliser_sensitivity.py,
DESIGN.md 2).  The per-dim normaliser 0.9189385f + log sigma_j is the one
declared numeric choice TF cannot pin here (glibc logf vs Eigen plog, SURVEY.md
A.5): the oracle's override path must reproduce the declared encoder exactly,
the Eigen plog restatement must stay within one ulp of logf, and a +-1 ulp
change of every log sigma must (almost) never move an index."""
import json
import os

import numpy as np

from conftest import REPO
from oracle import oracle as O
from compression_without_quantization_amd.synthetic import DEFAULT_SEED, make_blocks_range


def _c4(nb):
    h = make_blocks_range(0, nb, 32, 16, seed=DEFAULT_SEED)
    return ([h[k].reshape(-1) for k in ("post_loc", "post_scale", "prior_loc", "prior_scale")],
            np.arange(nb + 1, dtype=np.int64) * 32)


def test_override_with_logf_is_the_declared_encoder():
    (tl, ts, pl, ps), off = _c4(24)
    bits = 10
    wi, ws = O.greedy_encode(tl, ts, pl, ps, off, bits, 2, 42)
    for ls in (None, O.logf_table(ts)):
        gi, gs, gap = O.greedy_encode_lsig(tl, ts, pl, ps, off, bits, 2, 42, ls, gaps=True)
        assert np.array_equal(gi, wi) and np.array_equal(gs.view(np.uint32), ws.view(np.uint32))
        assert (gap >= 0).all() and gap.shape == (24, 2)


def test_eigen_plog_within_one_ulp_of_logf():
    x = np.random.default_rng(3).uniform(1e-3, 50.0, 200_000).astype(np.float32)
    lf = O.logf_table(x).view(np.int32).astype(np.int64)
    for fma in (False, True):
        d = O.eigen_plog(x, fma).view(np.int32).astype(np.int64) - lf
        assert np.abs(d).max() <= 1
        assert 0.01 < (d != 0).mean() < 0.3  # it is a different algorithm
    sp = O.eigen_plog(np.array([1.0, 0.0, -1.0, np.inf], np.float32))
    assert sp[0] == 0.0 and sp[1] == -np.inf and np.isnan(sp[2])


def test_one_ulp_normaliser_change_moves_no_index():
    (tl, ts, pl, ps), off = _c4(64)
    bits = 12
    base, _ = O.greedy_encode(tl, ts, pl, ps, off, bits, 1, 42)
    lf = O.logf_table(ts)
    flips = 0
    for ls in (np.nextafter(lf, np.float32(np.inf)), np.nextafter(lf, np.float32(-np.inf)),
               O.eigen_plog(ts)):
        vi, _ = O.greedy_encode_lsig(tl, ts, pl, ps, off, bits, 1, 42, ls)
        flips += int((vi != base).sum())
    assert flips <= 1


def test_committed_sensitivity_record():
    with open(os.path.join(REPO, "profiles", "normaliser_sensitivity.json")) as f:
        r = json.load(f)
    for cfg in ("c4", "c2"):
        for v in ("plog", "plog_fma", "up", "down", "random"):
            assert r[cfg][v]["index_flips"] == 0, (cfg, v)
    assert r["c4"]["blocks"] == 10000 and r["plog_vs_logf"]["max_ulp"] == 1


# ---------------------------------------------------------------------------
# Per-candidate semantics (tools/semantics_sensitivity.py): the
# TFP >= 0.8 log-prob form and other Eigen sum orders.
# ---------------------------------------------------------------------------
def _np_orders(x):
    """The six row-sum orders of cwqo_sem_rowsum restated in numpy float32."""
    f = np.float32
    d = x.size

    def packets(w, nacc):
        vec = d // w * w
        p = [np.zeros(w, f), np.zeros(w, f)]
        np_ = vec // w
        pairs = np_ // 2 * 2 if nacc == 2 else 0
        for k in range(np_):
            a = (k % 2) if k < pairs else 0
            p[a] = (p[a] + x[k * w:(k + 1) * w]).astype(f)
        q = (p[0] + p[1]).astype(f) if nacc == 2 else p[0]
        t = f(0)
        for j in range(vec, d):
            t = f(t + x[j])
        if w == 16:
            q = (q[:8] + q[8:]).astype(f)
        if w >= 8:
            q = (q[:4] + q[4:]).astype(f)
        return f(t + f(f(q[0] + q[2]) + f(q[1] + q[3])))

    def seq():
        s = f(0)
        for v in x:
            s = f(s + v)
        return s

    def tree(a):
        if a.size == 0:
            return f(0)
        if a.size == 1:
            return a[0]
        h = a.size // 2
        return f(tree(a[:h]) + tree(a[h:]))
    return [packets(8, 1), packets(4, 1), packets(8, 2), packets(16, 1), seq(), tree(x)]


def test_sem_rowsum_orders_match_numpy_restatement():
    rng = np.random.default_rng(11)
    for d in list(range(0, 70)) + [127, 376, 1000, 4095]:
        x = (rng.standard_normal(d) * 10.0 ** rng.uniform(-3, 3, d)).astype(np.float32)
        want = _np_orders(x)
        got = [O.sem_rowsum(x, o) for o in range(6)]
        assert [np.float32(g) for g in got] == want, d
        assert got[0] == O.eigen_rowsum(x)


def test_semvar_declared_variant_is_the_encoder():
    (tl, ts, pl, ps), off = _c4(16)
    for bits, ns in ((9, 3), (12, 1)):
        vi, vs, gap, dev = O.greedy_encode_semvar(tl, ts, pl, ps, off, bits, ns, 42)
        wi, ws = O.greedy_encode(tl, ts, pl, ps, off, bits, ns, 42)
        assert vi.shape == (16, ns, len(O.sem_variant_names()))
        assert np.array_equal(vi[..., 0], wi)
        assert np.array_equal(vs.view(np.uint32), ws.view(np.uint32))
        assert (dev[..., 0] == 0).all() and (gap >= 0).all()
        # the variants move rows by rounding only: far below the gaps here
        assert np.abs(dev).max() < 1e-4


def test_semvar_flip_detection_on_a_constructed_tie():
    """Two dims whose rows tie under one sum order only: the machinery must
    see a flip when the values differ by less than a rounding."""
    x = np.array([1e8, 1.0, -1e8, 1.0], np.float32)
    o = [O.sem_rowsum(x, k) for k in range(6)]
    assert len(set(o)) > 1  # the orders round differently on this row


def test_committed_semantics_record():
    with open(os.path.join(REPO, "profiles", "semantics_sensitivity.json")) as f:
        r = json.load(f)
    names = O.sem_variant_names()[1:]
    assert r["variants"] == names
    for cfg, n_min in (("c4", 10000), ("c2", 40000), ("c5", 32), ("c2cli", 1000),
                       ("c2low", 100)):
        assert r[cfg]["indices"] >= n_min, cfg
        assert set(r[cfg]["variants"]) == set(names), cfg
        for v in names:
            rec = r[cfg]["variants"][v]
            # the committed flips are what the parity claim carries; any flip
            # must sit at a best - second-best gap of the rows' rounding size:
            # <= 64-dim rows (c4, c5, c2) 1e-4 nats; the CLI configs' rows sum
            # up to 4,095 float terms of a few nats each (|row| ~ 10^3-10^4,
            # an ulp ~ 10^-4..10^-3 and a d-term sum's rounding up to ~d ulps)
            lim = 1e-4 if cfg in ("c4", "c5", "c2") else 1e-2
            assert rec["index_flips"] == 0 or rec["flipped_gaps_max"] < lim, (cfg, v)
    # the RNG-transcendental variants are part of the record
    assert {"rng/ulp_hash", "rng/ulp_up", "rng/ulp_down", "rng/v1_f32"} <= set(names)
    assert r["c2low"]["blocks"] == 50 and r["c2low"]["indices"] == 1500  # every group
