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
