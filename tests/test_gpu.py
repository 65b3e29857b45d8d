"""GPU parity tests: libcwq.so (gfx950 kernels) against the CPU oracle.

Bar: bit-exact.  Indices are compared as integers; samples as float32 bit
patterns (the north star allows 1e-5 on samples; we require equality).
The oracle itself is pinned as described in oracle/cwq_oracle.c (Random123
KATs, glibc libm, reference bit-string examples); parity against TensorFlow
is unpinned (the reference cannot run here).
"""
import hashlib
import json
import os
import warnings

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

N23 = 1 << 23


@pytest.fixture(scope="module")
def cwq(cwqlib):
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import compression_without_quantization_amd as C
    return C


def _u32(a):
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


def _assert_bits_equal(got, want, what):
    g, w = _u32(got), _u32(want)
    bad = np.nonzero(g != w)[0]
    assert bad.size == 0, f"{what}: {bad.size} of {w.size} differ, first at {bad[:8]}"


# ---------------------------------------------------------------------------
# transcendentals: device restatement vs host glibc, full 2^23 domains
# ---------------------------------------------------------------------------
def test_device_box_muller_exhaustive(cwq, cwqlib, oracle):
    dev = torch.device("cuda")
    rad = torch.empty(N23, dtype=torch.float32, device=dev)
    sn = torch.empty_like(rad)
    cs = torch.empty_like(rad)
    rc = cwqlib.cwq_selftest_bm_tables(0, N23, rad.data_ptr(), sn.data_ptr(), cs.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    _assert_bits_equal(rad.cpu().numpy(), oracle.bm_radius_table(0, N23), "radius")
    ws, wc = oracle.bm_sincos_table(0, N23)
    _assert_bits_equal(sn.cpu().numpy(), ws, "sin")
    _assert_bits_equal(cs.cpu().numpy(), wc, "cos")
    t = json.load(open(os.path.join(GOLDEN, "bm_tables.json")))
    assert hashlib.sha256(rad.cpu().numpy().tobytes()).hexdigest() == t["radius_sha256"]


def test_device_logf_all_positive_floats_strided(cwq, cwqlib, oracle):
    # every 61st positive float (35M values incl. subnormals) + specials
    bits = np.arange(0, 0x7f800001, 61, dtype=np.uint32)
    x = np.concatenate([bits.view(np.float32),
                        np.array([0, 1, np.inf, -1, -0.0, np.nan, 1e-45], np.float32)])
    want = oracle.logf_table(x)
    xd = torch.from_numpy(x).cuda()
    out = torch.empty_like(xd)
    assert cwqlib.cwq_selftest_logf(xd.data_ptr(), x.size, out.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream) == 0
    got = out.cpu().numpy()
    nan = np.isnan(want) & np.isnan(got)
    _assert_bits_equal(got[~nan], want[~nan], "logf")


# ---------------------------------------------------------------------------
# RNG (misc.py:3-17)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("d,n,seed", [(1, 33, 42000), (7, 1001, -5), (32, 65536, 123457),
                                      (13, 4097, 2147483647)])
def test_stateless_normal_sample(cwq, oracle, d, n, seed):
    rng = np.random.default_rng(d)
    loc = rng.standard_normal(d).astype(np.float32)
    scale = rng.uniform(0.1, 3, d).astype(np.float32)
    got = cwq.stateless_normal_sample(loc, scale, n, seed)
    want = oracle.stateless_normal_sample(loc, scale, n, seed)
    _assert_bits_equal(got, want, "stateless_normal_sample")


# ---------------------------------------------------------------------------
# coder vs golden fixtures
# ---------------------------------------------------------------------------
GOLDEN_CASES = ["oracle_c1.npz", "oracle_c4_slice.npz", "oracle_multistep.npz",
                "oracle_odd_d.npz", "oracle_c5_slice.npz"]


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_encode_decode_golden(cwq, golden, name):
    g = golden(name)
    off = g["block_off"]
    args = (int(g["n_bits"]), int(g["n_steps"]), int(g["seed"]))
    kw = dict(rho=float(g["rho"]), block_id_base=int(g["block_id_base"]))
    idx, sample = cwq.encode_blocks(g["t_loc"], g["t_scale"], g["p_loc"], g["p_scale"], *args,
                                    block_off=off, **kw)
    assert np.array_equal(idx.cpu().numpy(), g["idx"])
    _assert_bits_equal(sample.cpu().numpy(), g["sample"], name + " sample")
    d = np.diff(off)
    if (d == d[0]).all():  # uniform entry point too
        idx2, sample2 = cwq.encode_blocks(g["t_loc"], g["t_scale"], g["p_loc"], g["p_scale"],
                                          *args, block_dim=int(d[0]), **kw)
        assert np.array_equal(idx2.cpu().numpy(), g["idx"])
        _assert_bits_equal(sample2.cpu().numpy(), g["sample"], name + " uniform")
    dec = cwq.decode_blocks(g["idx"], g["p_loc"], g["p_scale"], *args, block_off=off, **kw)
    _assert_bits_equal(dec.cpu().numpy(), g["sample"], name + " decode")


# ---------------------------------------------------------------------------
# coder vs oracle on random configurations (edge cases of the reference)
# ---------------------------------------------------------------------------
CASES = [
    # nb, d, bits, n_steps, rho, seed, base
    (5, 1, 0, 1, 1.0, 42, 0),        # 2^0 = one candidate
    (9, 3, 1, 2, 1.0, -3, 7),        # odd d, tiny N, negative seed
    (4, 8, 4, 1, 1.0, 42, 0),        # C1 shape
    (3, 5, 10, 4, 0.7, 99, 2),       # multi-step, rho
    (17, 32, 8, 1, 1.0, 2147483, 0),  # 1000*seed wraps int32
    (2, 33, 12, 2, 1.3, 5, 0),       # d > 32, Eigen tail, split tiles
    (6, 12, 9, 1, 1.0, 0, 123),
    (1, 64, 14, 1, 1.0, 42, 0),
]


@pytest.mark.parametrize("case", CASES)
def test_encode_vs_oracle(cwq, oracle, case):
    nb, d, bits, n_steps, rho, seed, base = case
    from compression_without_quantization_amd.synthetic import make_blocks
    b = make_blocks(nb, d, max(bits, 2), seed=1000 + nb * d + bits)
    tl, ts, pl, ps = (b[k].reshape(-1) for k in ("post_loc", "post_scale", "prior_loc",
                                                 "prior_scale"))
    off = np.arange(nb + 1) * d
    wi, ws = oracle.greedy_encode(tl, ts, pl, ps, off, bits, n_steps, seed, rho, base)
    gi, gs = cwq.encode_blocks(tl, ts, pl, ps, bits, n_steps, seed, rho=rho, block_off=off,
                               block_id_base=base)
    assert np.array_equal(gi.cpu().numpy(), wi)
    _assert_bits_equal(gs.cpu().numpy(), ws, f"sample {case}")
    dec = cwq.decode_blocks(wi, pl, ps, bits, n_steps, seed, rho=rho, block_off=off,
                            block_id_base=base)
    _assert_bits_equal(dec.cpu().numpy(), ws, f"decode {case}")


def test_ragged_blocks_with_empty_groups(cwq, oracle):
    rng = np.random.default_rng(4)
    sizes = [0, 3, 1, 0, 17, 8, 5, 0, 40, 2]
    off = np.concatenate([[0], np.cumsum(sizes)])
    D = int(off[-1])
    tl = rng.standard_normal(D).astype(np.float32)
    ts = rng.uniform(0.2, 1.0, D).astype(np.float32)
    pl = np.zeros(D, np.float32)
    ps = np.ones(D, np.float32)
    wi, ws = oracle.greedy_encode(tl, ts, pl, ps, off, 8, 1, 42)
    gi, gs = cwq.encode_blocks(tl, ts, pl, ps, 8, 1, 42, block_off=off)
    assert np.array_equal(gi.cpu().numpy(), wi)
    assert (wi[np.array(sizes) == 0] == 0).all()  # empty group -> index 0
    _assert_bits_equal(gs.cpu().numpy(), ws, "ragged")


# ---------------------------------------------------------------------------
# reference surface
# ---------------------------------------------------------------------------
def test_code_greedy_sample_api(cwq, oracle):
    rng = np.random.default_rng(8)
    d = 11
    t_loc = rng.standard_normal(d).astype(np.float32)
    t_scale = rng.uniform(0.3, 0.9, d).astype(np.float32)
    p_loc = (0.1 * rng.standard_normal(d)).astype(np.float32)
    p_scale = rng.uniform(0.8, 1.2, d).astype(np.float32)
    best, code = cwq.code_greedy_sample(t_loc, t_scale, p_loc, p_scale, 7, 3, 17)
    wi, ws = oracle.code_greedy_sample(t_loc, t_scale, p_loc, p_scale, 7, 3, 17)
    assert code == ''.join(cwq.to_bit_string(int(i), 7) for i in wi)
    _assert_bits_equal(best, ws, "code_greedy_sample")
    dec = cwq.decode_greedy_sample(code, p_loc, p_scale, 7, 3, 17)
    _assert_bits_equal(dec, ws, "decode_greedy_sample")
    # torch in -> torch out, same values
    tb, tcode = cwq.code_greedy_sample(*(torch.from_numpy(a).cuda() for a in
                                         (t_loc, t_scale, p_loc, p_scale)), 7, 3, 17)
    assert isinstance(tb, torch.Tensor) and tb.is_cuda and tcode == code


def test_encode_decode_convenience(cwq, oracle):
    from compression_without_quantization_amd.synthetic import make_blocks
    b = make_blocks(20, 16, 10)
    idx, samp = cwq.encode(b["prior_loc"], b["prior_scale"], b["post_loc"], b["post_scale"],
                           42, 10)
    assert idx.shape == (20,) and samp.shape == (20, 16)
    off = np.arange(21) * 16
    wi, ws = oracle.greedy_encode(b["post_loc"], b["post_scale"], b["prior_loc"],
                                  b["prior_scale"], off, 10, 1, 42)
    assert np.array_equal(idx, wi[:, 0])
    _assert_bits_equal(samp.reshape(-1), ws, "encode()")
    bitcode = cwq.indices_to_bitcode(idx, 10)
    for arg in (idx, bitcode):
        dec = cwq.decode(arg, b["prior_loc"], b["prior_scale"], 42, 10)
        _assert_bits_equal(dec.reshape(-1), ws, "decode()")


def test_grouped_golden(cwq, golden):
    g = golden("oracle_grouped.npz")
    cwq.coded_greedy_sampler.VERBOSE = False
    target = cwq.Normal(g["q_loc"], g["q_scale"])
    proposal = cwq.Normal(g["p_loc"], g["p_scale"])
    sample, bitcode, starts = cwq.code_grouped_greedy_sample(None, target, proposal, 1, 8, 42)
    assert starts == [int(v) for v in g["starts"]]
    assert bitcode == cwq.indices_to_bitcode(g["idx"], 8)
    _assert_bits_equal(sample, g["sample"], "grouped sample")
    dec = cwq.decode_grouped_greedy_sample(None, bitcode, starts, proposal, 8, 1, 42)
    _assert_bits_equal(dec, g["sample"], "grouped decode")
    assert starts[-1] == g["p_loc"].size  # caller's list not mutated


def test_grouped_dtype_errors(cwq):
    t = cwq.Normal(np.zeros(4, np.float64), np.ones(4, np.float64))
    p = cwq.Normal(np.zeros(4, np.float32), np.ones(4, np.float32))
    with pytest.raises(Exception, match="Target datatype must be float32!"):
        cwq.code_grouped_greedy_sample(None, t, p, 1, 8, 42)
    with pytest.raises(Exception, match="Proposal datatype must be float32!"):
        cwq.code_grouped_greedy_sample(None, p, t, 1, 8, 42)
    with pytest.raises(Exception, match="Proposal datatype must be float32!"):
        cwq.decode_grouped_greedy_sample(None, "0" * 8, [0], t, 8, 1, 42)


# ---------------------------------------------------------------------------
# full-size configurations: oracle on a sample + size-independent properties
# ---------------------------------------------------------------------------
def test_c2_image_grouped_full(cwq, oracle):
    """C2: one 512x768 image's level-1 latents (196,608 dims) at 8 bits/group."""
    from compression_without_quantization_amd.synthetic import make_latents
    q_loc, q_scale, p_loc, p_scale = make_latents(32 * 48 * 128, seed=5)
    cwq.coded_greedy_sampler.VERBOSE = False
    sample, bitcode, starts = cwq.code_grouped_greedy_sample(
        None, cwq.Normal(q_loc, q_scale), cwq.Normal(p_loc, p_scale), 1, 8, 42)
    ws, wi, wst = oracle.code_grouped_greedy_sample(q_loc, q_scale, p_loc, p_scale, 1, 8, 42,
                                                    cwq.group_size_threshold(12))
    assert starts == wst
    assert bitcode == cwq.indices_to_bitcode(wi, 8)
    _assert_bits_equal(sample, ws, "C2 sample")
    dec = cwq.decode_grouped_greedy_sample(None, bitcode, starts, cwq.Normal(p_loc, p_scale),
                                           8, 1, 42)
    _assert_bits_equal(dec, ws, "C2 decode")


def test_c4_full_size_roundtrip_and_sample(cwq, oracle):
    """C4: 10^6 blocks x d=32 at 16 bits.  Round trip on all blocks; oracle on 48."""
    from compression_without_quantization_amd.synthetic import make_blocks
    nb, d, bits = 1_000_000, 32, 16
    b = make_blocks(nb, d, bits)
    dev = torch.device("cuda")
    t = {k: torch.from_numpy(v.reshape(-1)).to(dev) for k, v in b.items()}
    idx, sample = cwq.encode_blocks(t["post_loc"], t["post_scale"], t["prior_loc"],
                                    t["prior_scale"], bits, 1, 42, block_dim=d)
    dec = cwq.decode_blocks(idx, t["prior_loc"], t["prior_scale"], bits, 1, 42, block_dim=d)
    assert torch.equal(dec.view(torch.int32), sample.view(torch.int32))
    idx_h = idx.cpu().numpy().reshape(-1)
    assert idx_h.min() >= 0 and idx_h.max() < (1 << bits)
    pick = np.random.default_rng(0).choice(nb, 48, replace=False)
    for g in pick:
        s = slice(g * d, (g + 1) * d)
        wi, ws = oracle.code_greedy_sample(b["post_loc"][g], b["post_scale"][g],
                                           b["prior_loc"][g], b["prior_scale"][g], bits, 1,
                                           42 + int(g))
        assert wi[0] == idx_h[g], f"block {g}"
        _assert_bits_equal(sample[s].cpu().numpy(), ws, f"block {g}")


# ---------------------------------------------------------------------------
# pruned encoder (uniform d % 8 == 0): same results as the unpruned kernel and
# the oracle, including adversarial inputs where the bound is tight or useless
# ---------------------------------------------------------------------------
def _uniform_encode(cwq, cwqlib, tl, ts, pl, ps, d, bits, n_steps, seed, rho, mode):
    """mode: 0 unpruned, 1 pruning on exact values, 2 pruning with screening
    (cwq_options.prune_mode of this call only)."""
    i, s = cwq.encode_blocks(tl, ts, pl, ps, bits, n_steps, seed, rho=rho, block_dim=d,
                             prune_mode=int(mode))
    torch.cuda.synchronize()
    return i.cpu().numpy(), s.cpu().numpy()


@pytest.mark.parametrize("d,bits,n_steps,nb,rho", [
    (8, 4, 1, 64, 1.0), (8, 12, 1, 16, 1.0), (16, 14, 1, 8, 1.0), (24, 10, 2, 12, 1.0),
    (32, 16, 1, 6, 1.0), (32, 9, 3, 10, 0.8), (40, 11, 1, 8, 1.0), (64, 13, 1, 4, 1.0),
    # 2^20+ candidates (many tiles per block, tau close to the best row):
    # multi-step (best carried), rho, group counts G = d / 4 from 2 to 16
    (16, 20, 1, 1, 1.0), (8, 20, 1, 3, 1.0), (16, 21, 2, 2, 0.9), (24, 20, 1, 2, 1.0),
    (32, 20, 3, 2, 1.0), (64, 20, 1, 1, 1.0), (16, 22, 1, 2, 1.0),
    # the tile queue (tiles of >= 4096 candidates, more tiles than the resident
    # grid): one tile per block (C4's shape), and block-interleaved tiles with
    # the tail split (C5's shape), two steps
    (16, 12, 1, 16384, 1.0), (16, 20, 2, 64, 1.0)])
def test_pruned_matches_unpruned_and_oracle(cwq, cwqlib, oracle, d, bits, n_steps, nb, rho):
    from compression_without_quantization_amd.synthetic import make_blocks
    b = make_blocks(nb, d, bits, seed=77 + d + bits)
    tl, ts, pl, ps = (b[k].reshape(-1) for k in ("post_loc", "post_scale", "prior_loc",
                                                 "prior_scale"))
    i0, s0 = _uniform_encode(cwq, cwqlib, tl, ts, pl, ps, d, bits, n_steps, 42, rho, 0)
    for mode in (1, 2):
        i1, s1 = _uniform_encode(cwq, cwqlib, tl, ts, pl, ps, d, bits, n_steps, 42, rho, mode)
        assert np.array_equal(i1, i0), f"mode {mode}"
        _assert_bits_equal(s1, s0, f"pruned (mode {mode}) vs unpruned")
    if (1 << bits) * d * nb <= (1 << 22):
        wi, ws = oracle.greedy_encode(tl, ts, pl, ps, np.arange(nb + 1) * d, bits, n_steps, 42,
                                      rho)
        assert np.array_equal(i1, wi)
        _assert_bits_equal(s1, ws, "pruned vs oracle")


@pytest.mark.parametrize("kind", ["posterior_is_prior", "tiny_scales", "huge_scales",
                                  "inf_scale", "zero_scale", "mixed_sign_norm", "nan_scale",
                                  "nan_loc_one_dim", "far_locs", "huge_locs", "tiny_locs"])
@pytest.mark.parametrize("mode", [1, 2])
def test_pruned_adversarial(cwq, cwqlib, oracle, kind, mode):
    nb, d, bits = 6, 16, 10
    tl, ts, pl, ps = _adversarial_inputs(kind, nb, d)
    i1, s1 = _uniform_encode(cwq, cwqlib, tl, ts, pl, ps, d, bits, 1, 42, 1.0, mode)
    wi, ws = oracle.greedy_encode(tl, ts, pl, ps, np.arange(nb + 1) * d, bits, 1, 42)
    assert np.array_equal(i1, wi)
    _assert_bits_equal(s1, ws, kind)


@pytest.mark.parametrize("kind", ["posterior_is_prior", "tiny_scales", "huge_scales",
                                  "inf_scale", "zero_scale", "mixed_sign_norm", "nan_scale",
                                  "nan_loc_one_dim", "far_locs", "huge_locs", "tiny_locs"])
def test_pruned_adversarial_high_rate(cwq, cwqlib, kind):
    """The same inputs with 2^20 candidates (16 tiles per block; the
    survivor list overflows on the near-tie inputs): the screened pass equals
    the unpruned kernel, which the 10-bit test above pins to the oracle."""
    nb, d, bits = 3, 16, 20
    tl, ts, pl, ps = _adversarial_inputs(kind, nb, d)
    i0, s0 = _uniform_encode(cwq, cwqlib, tl, ts, pl, ps, d, bits, 1, 42, 1.0, 0)
    i2, s2 = _uniform_encode(cwq, cwqlib, tl, ts, pl, ps, d, bits, 1, 42, 1.0, 2)
    assert np.array_equal(i2, i0)
    _assert_bits_equal(s2, s0, kind)


def _adversarial_inputs(kind, nb, d):
    rng = np.random.default_rng(sum(map(ord, kind)))
    pl = rng.standard_normal(nb * d).astype(np.float32)
    ps = rng.uniform(0.5, 2, nb * d).astype(np.float32)
    tl = pl.copy()
    ts = ps.copy()
    if kind == "tiny_scales":      # huge deficits, normaliser M_j >> 0
        ts = (ps * 1e-6).astype(np.float32)
        tl = (pl + 0.1 * ps * rng.standard_normal(nb * d)).astype(np.float32)
    elif kind == "huge_scales":    # flat target: everything is a near-tie
        ts = (ps * 1e6).astype(np.float32)
    elif kind == "inf_scale":
        ts[3] = np.inf
    elif kind == "zero_scale":
        ts[5] = 0.0
        tl[5] = pl[5]
    elif kind == "nan_scale":      # every candidate's value is NaN -> index 0
        ts[:] = np.nan
    elif kind == "nan_loc_one_dim":  # NaN in one dim of every other block
        tl[7::32] = np.nan
    elif kind == "mixed_sign_norm":  # some c_j < 0 (M_j > 0), some > 0
        ts = np.where(rng.uniform(size=nb * d) < 0.5, 0.05, 3.0).astype(np.float32)
    elif kind == "far_locs":       # |loc| >> scale: the float rounding of loc + scale z dominates
        pl = (3.0e4 + pl).astype(np.float32)
        tl = (pl + 0.3 * ps * rng.standard_normal(nb * d)).astype(np.float32)
        ts = (0.01 * ps).astype(np.float32)
    elif kind == "huge_locs":      # outside the screening gate: exact pruning for these tiles
        pl = (1.0e35 * np.sign(pl)).astype(np.float32)
        tl = pl.copy()
        ts = (ps * 1e33).astype(np.float32)
        ps = (ps * 1e33).astype(np.float32)
    elif kind == "tiny_locs":      # values near zero: subnormal-range differences
        pl = (pl * 1e-30).astype(np.float32)
        ps = (ps * 1e-30).astype(np.float32)
        tl = (pl + 0.5 * ps * rng.standard_normal(nb * d)).astype(np.float32)
        ts = (0.7 * ps).astype(np.float32)
    return tl, ts, pl, ps


def test_screen_tables_within_bounds(cwq, cwqlib):
    """The screening pass's Box-Muller approximations (hardware v_log/v_sqrt/
    v_sin/v_cos) stay within the constants its bounds are built on
    (kScreenEr, kScreenEs, kScreenRmax in csrc/cwq_kernels.hip), over all 2^23
    inputs of each."""
    k_er, k_es, k_rmax = 1.0e-6, 6.0e-7, 5.68
    dev = torch.device("cuda")
    t = [torch.empty(N23, dtype=torch.float32, device=dev) for _ in range(6)]
    st = torch.cuda.current_stream().cuda_stream
    assert cwqlib.cwq_selftest_bm_tables(0, N23, t[0].data_ptr(), t[1].data_ptr(),
                                         t[2].data_ptr(), st) == 0
    assert cwqlib.cwq_selftest_screen_tables(0, N23, t[3].data_ptr(), t[4].data_ptr(),
                                             t[5].data_ptr(), st) == 0
    torch.cuda.synchronize()
    a = [x.cpu().numpy().astype(np.float64) for x in t]
    assert np.isfinite(a[3]).all() and np.isfinite(a[4]).all() and np.isfinite(a[5]).all()
    a[3] = a[3] * np.sqrt(2.0 * np.log(2.0))    # the table holds r~ / sqrt(2 ln 2)
    assert np.abs(a[3] - a[0]).max() <= k_er
    assert np.abs(a[4] - a[1]).max() <= k_es
    assert np.abs(a[5] - a[2]).max() <= k_es
    assert a[0].max() <= k_rmax and a[3].max() <= k_rmax


def test_device_wave_max(cwq, cwqlib):
    """The DPP wave-wide max (tau sharing in the pruned kernel) on random waves,
    with -inf, ties and the maximum in every lane position."""
    rng = np.random.default_rng(5)
    nw = 4096
    x = rng.standard_normal((nw, 64)).astype(np.float32)
    x[:64, :] = -np.inf
    for w in range(64):
        x[64 + w, w] = 100.0                 # max in lane w
        x[128 + w, :] = -np.inf
        x[128 + w, w] = -5.0                 # single finite lane
    x[300, :] = 3.0                          # all equal
    xd = torch.from_numpy(x).cuda()
    out = torch.empty(nw, dtype=torch.float32, device="cuda")
    assert cwqlib.cwq_selftest_wave_max(xd.data_ptr(), nw, out.data_ptr(),
                                        torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), x.max(axis=1))


def test_device_fast_division_correctly_rounded(cwq, cwqlib):
    """The 5-op quotient used by the pruned kernel equals IEEE a/b on its
    documented domain: 2^-60 <= |a| <= 2^60 (or 0), 2^-60 <= b <= 2^60."""
    rng = np.random.default_rng(11)
    n = 1 << 24
    parts = []
    for _ in range(6):
        # random significands, exponents spread over the whole domain
        a = (rng.uniform(1, 2, n) * np.exp2(rng.integers(-60, 60, n))).astype(np.float32)
        a *= np.where(rng.uniform(size=n) < 0.5, -1, 1).astype(np.float32)
        b = (rng.uniform(1, 2, n) * np.exp2(rng.integers(-60, 60, n))).astype(np.float32)
        parts.append((a, b))
    # adversarial: b = 1 +- k ulp, a = near multiples of b; b = powers of two
    k = rng.integers(1, 1 << 20, n)
    b = (np.float32(1) + k.astype(np.float32) * np.float32(2 ** -23)).astype(np.float32)
    m = rng.integers(1, 1 << 24, n).astype(np.float64)
    a = (m * b.astype(np.float64) * (1 + rng.integers(-3, 4, n) * 2.0 ** -24)).astype(np.float32)
    parts.append((a, b))
    parts.append((rng.uniform(-4, 4, n).astype(np.float32),
                  np.exp2(rng.integers(-60, 61, n)).astype(np.float32)))
    parts.append((np.zeros(1024, np.float32), rng.uniform(0.1, 9, 1024).astype(np.float32)))
    for a, b in parts:
        ad = torch.from_numpy(a).cuda()
        bd = torch.from_numpy(b).cuda()
        out = torch.empty_like(ad)
        assert cwqlib.cwq_selftest_div(ad.data_ptr(), bd.data_ptr(), a.size, out.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream) == 0
        want = (a / b).astype(np.float32)
        got = out.cpu().numpy()
        got = np.where(a == 0, np.abs(got), got)  # sign of a zero quotient is irrelevant
        want = np.where(a == 0, np.abs(want), want)
        _assert_bits_equal(got, want, "fast division")


# ---------------------------------------------------------------------------
# importance sampler (code/coded_importance_sampler.py)
# ---------------------------------------------------------------------------
def test_importance_encode_vs_oracle(cwq, oracle):
    from compression_without_quantization_amd.coded_importance_sampler import num_samples_plan
    rng = np.random.default_rng(21)
    sizes = [1, 4, 3, 16, 7, 2, 9, 16, 5, 1, 12]
    off = np.concatenate([[0], np.cumsum(sizes)])
    D = int(off[-1])
    tl = (rng.standard_normal(D) * 0.8).astype(np.float32)
    ts = rng.uniform(0.25, 0.95, D).astype(np.float32)
    pl = np.zeros(D, np.float32)
    ps = np.ones(D, np.float32)
    kl = oracle.kl_normal_normal(tl, ts, pl, ps)
    ns = num_samples_plan(kl, off)
    assert np.array_equal(ns, oracle.importance_plan(kl, off))
    assert ns.max() > 1000
    wi, ws = oracle.importance_encode(tl, ts, pl, ps, off, ns, 1234, 3)
    gi, gs = cwq.importance_encode_blocks(tl, ts, pl, ps, off, ns, 1234, block_id_base=3)
    assert np.array_equal(gi.cpu().numpy(), wi)
    _assert_bits_equal(gs.cpu().numpy(), ws, "importance sample")
    dec = cwq.importance_decode_blocks(wi, pl, ps, off, 1234, block_id_base=3)
    _assert_bits_equal(dec.cpu().numpy(), ws, "importance decode")


@pytest.mark.parametrize("kind", ["random", "ties"])
def test_importance_small_group_threshold(cwq, oracle, kind):
    """Groups of at most 128 candidates are coded by k_imp_small (one wave,
    exact rows), larger ones by k_imp_eval's tiles: counts either side of the
    threshold (and 1, 64, 65) give the oracle's indices and samples."""
    rng = np.random.default_rng(31 if kind == "random" else 32)
    counts = [1, 2, 63, 64, 65, 127, 128, 129, 130, 255, 256, 257, 1000, 5000]
    ns = np.array(counts * 3, dtype=np.int64)
    rng.shuffle(ns)
    sizes = rng.integers(1, 17, ns.size)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D = int(off[-1])
    tl = (rng.standard_normal(D) * 0.8).astype(np.float32)
    ts = rng.uniform(0.25, 0.95, D).astype(np.float32)
    if kind == "ties":  # every score 0: the lowest index wins in both kernels
        tl[:], ts[:] = 0.0, 1.0
    pl = np.zeros(D, np.float32)
    ps = np.ones(D, np.float32)
    wi, ws = oracle.importance_encode(tl, ts, pl, ps, off, ns, 4321, 5)
    gi, gs = cwq.importance_encode_blocks(tl, ts, pl, ps, off, ns, 4321, block_id_base=5)
    assert np.array_equal(gi.cpu().numpy(), wi)
    _assert_bits_equal(gs.cpu().numpy(), ws, f"importance small/large groups ({kind})")


def test_importance_single_block_api(cwq, oracle):
    rng = np.random.default_rng(22)
    d = 6
    tl = rng.standard_normal(d).astype(np.float32)
    ts = rng.uniform(0.3, 0.9, d).astype(np.float32)
    pl = (0.2 * rng.standard_normal(d)).astype(np.float32)
    ps = rng.uniform(0.8, 1.3, d).astype(np.float32)
    best, code = cwq.code_importance_sample(tl, ts, pl, ps, 20, 99)
    n = oracle.importance_num_samples(tl, ts, pl, ps)
    wi, ws = oracle.importance_encode(tl, ts, pl, ps, [0, d], [n], 99)
    assert code == cwq.elias_delta_code(int(wi[0]) + 1)
    _assert_bits_equal(best.reshape(-1), ws, "code_importance_sample")
    b2, ind = cwq.code_importance_sample(tl, ts, pl, ps, 20, 99, return_index_only=True)
    assert ind == int(wi[0]) + 1
    last, clen, index, samples = cwq.decode_importance_sample(code.encode(), pl, ps, 99)
    assert clen == len(code) and index == int(wi[0]) and samples.shape == (index + 1, d)
    _assert_bits_equal(last.reshape(-1), ws, "decode_importance_sample")
    _assert_bits_equal(cwq.decode_importance_sample(ind, pl, ps, 99, use_index=True).reshape(-1),
                       ws, "decode_importance_sample(use_index)")


def test_importance_grouped_golden(cwq, golden):
    g = golden("oracle_importance.npz")
    import compression_without_quantization_amd.coded_importance_sampler as I
    I.VERBOSE = False
    target = cwq.Normal(g["q_loc"], g["q_scale"])
    proposal = cwq.Normal(g["p_loc"], g["p_scale"])
    sample, bitcode, starts, (oi, oq) = cwq.code_grouped_importance_sample(
        None, target, proposal, int(g["seed"]), int(g["n_bits_per_group"]),
        max_group_size_bits=int(g["max_group_size_bits"]),
        dim_kl_bit_limit=int(g["dim_kl_bit_limit"]))
    assert list(starts) == list(g["starts"])
    assert np.array_equal(oi, g["outlier_indices"]) and np.array_equal(oq, g["outlier_q"])
    assert bitcode == ''.join(cwq.elias_delta_code(int(i)) for i in g["indices"])
    _assert_bits_equal(sample, g["sample"], "grouped importance sample")
    # decode: the group starts travel without the trailing D (:294)
    dec = cwq.decode_grouped_importance_sample(None, bitcode, list(starts[:-1]), proposal,
                                               int(g["n_bits_per_group"]), int(g["seed"]),
                                               oi, oq)
    keep = np.ones(sample.size, bool)
    keep[oi] = False
    _assert_bits_equal(dec[keep], sample[keep], "grouped importance decode")
    # outliers travel as quint16 over [-30, 30] (:156): clamped, one step of 60/65535
    assert np.allclose(dec[~keep], np.clip(sample[~keep], -30, 30), atol=60 / 65535)
    # index form
    _, indices, _, _ = cwq.code_grouped_importance_sample(
        None, target, proposal, int(g["seed"]), int(g["n_bits_per_group"]),
        max_group_size_bits=int(g["max_group_size_bits"]),
        dim_kl_bit_limit=int(g["dim_kl_bit_limit"]), return_indices=True)
    assert list(indices) == list(g["indices"])
    dec2 = cwq.decode_grouped_importance_sample(None, list(indices), list(starts[:-1]),
                                                proposal, 20, int(g["seed"]), oi, oq,
                                                use_indices=True)
    _assert_bits_equal(dec2, dec, "use_indices decode")


def test_importance_batch_equals_single_calls(cwq, oracle):
    """code_grouped_importance_sample_batch (one native call for every item)
    returns exactly what one code_grouped_importance_sample per item returns,
    item i with its own seed: I2's shape (24 level-2 latent sets of 2,304 dims,
    20 bits/group, groups <= 3 dims) plus an empty item, a 1-dim item, an item
    with outliers and a NaN dim, and a wrapped seed; item 0 also against the
    oracle's whole pipeline."""
    import compression_without_quantization_amd.coded_importance_sampler as I
    from compression_without_quantization_amd.synthetic import make_latents
    I.VERBOSE = False
    lat, seeds = [], []
    for i in range(24):
        lat.append(make_latents(8 * 12 * 24, seed=5000 + i))
        seeds.append(42 + 3 * i)
    for D, kind in ((0, "empty"), (1, "one"), (500, "outliers")):
        q_loc, q_scale, p_loc, p_scale = make_latents(max(D, 1), bits_per_dim=1.5, seed=77 + D)
        q_loc, q_scale, p_loc, p_scale = q_loc[:D], q_scale[:D], p_loc[:D], p_scale[:D]
        if kind == "outliers":
            q_loc[::40] = p_loc[::40] + 40 * p_scale[::40]
            q_loc[7] = np.nan
        lat.append((q_loc, q_scale, p_loc, p_scale))
        seeds.append(2 ** 31 - 2 if kind == "outliers" else -5)
    dev = torch.device("cuda", 0)
    ts = [cwq.Normal(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)) for a, b, _, _ in lat]
    ps = [cwq.Normal(torch.from_numpy(c).to(dev), torch.from_numpy(d).to(dev)) for _, _, c, d in lat]
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        batch = I.code_grouped_importance_sample_batch(None, ts, ps, seeds, 20,
                                                       max_group_size_bits=2,
                                                       dim_kl_bit_limit=16)
    assert len(batch) == len(lat)
    for i, (t, p, s) in enumerate(zip(ts, ps, seeds)):
        one = I.code_grouped_importance_sample(None, t, p, s, 20, max_group_size_bits=2,
                                               dim_kl_bit_limit=16)
        b = batch[i]
        _assert_bits_equal(b[0], one[0], f"batch sample, item {i}")
        assert b[1] == one[1], i
        assert np.array_equal(np.asarray(b[2]), np.asarray(one[2])), i
        assert np.array_equal(b[3][0], one[3][0]) and np.array_equal(b[3][1], one[3][1]), i
    assert batch[24][1] == "" and list(batch[24][2]) == [0]
    assert batch[26][3][0].size >= 12
    # index form, and item 0 against the oracle's pipeline
    idx = I.code_grouped_importance_sample_batch(None, ts[:1], ps[:1], seeds[:1], 20,
                                                 max_group_size_bits=2, dim_kl_bit_limit=16,
                                                 return_indices=True)[0]
    ql, qs, pl, pls = lat[0]
    wsm, wi, wst, (oi, oq) = oracle.code_grouped_importance_sample(ql, qs, pl, pls, seeds[0], 20,
                                                                   2, 16)
    assert list(idx[1]) == list(wi)
    assert np.array_equal(np.asarray(idx[2]), np.asarray(wst))
    assert np.array_equal(idx[3][0], oi) and np.array_equal(idx[3][1], oq)
    _assert_bits_equal(idx[0], wsm, "batch item 0 vs oracle")


def test_importance_instantiations_agree_on_large_groups(cwq):
    """Launches large enough for the largest tile size (>= 2^25 candidates):
    the batched call (per-group seeds, tile size known on the host), the fused
    single call (seed + g, tile size known on the host) and the step-by-step
    path (cwq_importance_encode: tile size chosen on the device) run the three
    k_imp_eval instantiations over the same groups; all must agree bit for bit."""
    import compression_without_quantization_amd.coded_importance_sampler as I
    from compression_without_quantization_amd.synthetic import make_latents
    I.VERBOSE = False
    lat = [make_latents(6000, bits_per_dim=1.6, seed=900 + i) for i in range(2)]
    dev = torch.device("cuda", 0)
    ts = [cwq.Normal(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)) for a, b, _, _ in lat]
    ps = [cwq.Normal(torch.from_numpy(c).to(dev), torch.from_numpy(d).to(dev)) for _, _, c, d in lat]
    batch = I.code_grouped_importance_sample_batch(None, ts, ps, [11, 12], 20)
    old = I.USE_FUSED
    try:
        for i, (t, p) in enumerate(zip(ts, ps)):
            want = {}
            for fused in (True, False):
                I.USE_FUSED = fused
                want[fused] = I.code_grouped_importance_sample(None, t, p, 11 + i, 20)
            n = I.num_samples_plan(
                I._kl(dev, *(x.reshape(-1) for x in (*_std_target(t, p), torch.zeros(6000, device=dev),
                                                      torch.ones(6000, device=dev)))).cpu().numpy(),
                np.asarray(want[True][2]))
            assert int(np.maximum(n, 1).sum()) >= 1 << 25, "not a largest-tile launch"
            for w in want.values():
                _assert_bits_equal(batch[i][0], w[0], f"large groups, item {i}")
                assert batch[i][1] == w[1]
                assert np.array_equal(np.asarray(batch[i][2]), np.asarray(w[2]))
    finally:
        I.USE_FUSED = old


def _std_target(t, p):
    """The standardised target (coded_importance_sampler.py:137-138) of a latent
    with no outliers (the test's latents have none above 16 bits)."""
    return (t.loc - p.loc) / p.scale, t.scale / p.scale


# ---------------------------------------------------------------------------
# importance sampler screening pass: the screened encoder must
# give the same indices and samples as the exact one, also where the bound is
# loose (tiny target scales), useless (all ties) or gated off (huge values)
# ---------------------------------------------------------------------------
def _importance_modes(cwq, cwqlib, tl, ts, pl, ps, off, ns, seed):
    out = []
    for mode in (0, 2):
        i, s = cwq.importance_encode_blocks(tl, ts, pl, ps, off, ns, seed, prune_mode=mode)
        torch.cuda.synchronize()
        out.append((i.cpu().numpy(), s.cpu().numpy()))
    return out


@pytest.mark.parametrize("kind", ["pln_like", "tiny_target", "wide_target", "ties",
                                  "huge_values", "far_means", "long_rows"])
def test_importance_screening_matches_exact(cwq, cwqlib, oracle, kind):
    rng = np.random.default_rng(sum(map(ord, kind)))
    sizes = [15, 3, 1, 7, 15, 4, 12, 2, 9, 15]
    if kind == "long_rows":
        sizes = [64, 200, 33, 256, 300]   # 300 > the screening LDS limit: exact fallback
    off = np.concatenate([[0], np.cumsum(sizes)])
    D = int(off[-1])
    tl = (rng.standard_normal(D) * 0.7).astype(np.float32)
    ts = rng.uniform(0.3, 0.95, D).astype(np.float32)
    pl = np.zeros(D, np.float32)
    ps = np.ones(D, np.float32)
    if kind == "tiny_target":
        ts = rng.uniform(1e-4, 1e-3, D).astype(np.float32)
        tl = (rng.standard_normal(D) * 1e-3).astype(np.float32)
    elif kind == "wide_target":     # sigma_q > sigma_p: the log ratio is convex in z
        ts = rng.uniform(1.0, 3.0, D).astype(np.float32)
    elif kind == "ties":            # target == proposal: every score is 0, index 0 wins
        tl[:] = 0.0
        ts[:] = 1.0
    elif kind == "huge_values":
        pl = (rng.standard_normal(D) * 1e20).astype(np.float32)
        ps = rng.uniform(1e18, 1e19, D).astype(np.float32)
        tl = pl.copy()
        ts = (ps * 0.5).astype(np.float32)
    elif kind == "far_means":
        pl = (3.0e4 + rng.standard_normal(D)).astype(np.float32)
        ps = rng.uniform(0.5, 2.0, D).astype(np.float32)
        tl = (pl + 0.5 * ps * rng.standard_normal(D)).astype(np.float32)
        ts = (ps * rng.uniform(0.3, 0.9, D)).astype(np.float32)
    ns = np.array([min(int(x), 50_000) for x in
                   rng.integers(1, 60_000, len(sizes))], dtype=np.int64)
    ns[2] = 1
    (i0, s0), (i2, s2) = _importance_modes(cwq, cwqlib, tl, ts, pl, ps, off, ns, 77)
    assert np.array_equal(i0, i2), kind
    _assert_bits_equal(s2, s0, f"importance screened vs exact ({kind})")
    if kind in ("pln_like", "ties", "wide_target"):
        wi, ws = oracle.importance_encode(tl, ts, pl, ps, off, ns, 77)
        assert np.array_equal(i2, wi)
        _assert_bits_equal(s2, ws, f"importance vs oracle ({kind})")


@pytest.mark.parametrize("trial", range(12))
def test_pruned_random_stress(cwq, cwqlib, trial):
    """Random shapes, budgets, step counts, rho, seeds and heavy-tailed
    inputs: the three encoder modes must agree bit for bit."""
    rng = np.random.default_rng(1000 + trial)
    d = int(rng.choice([8, 16, 24, 32, 40, 48, 56, 64]))
    bits = int(rng.integers(1, 19))
    n_steps = int(rng.integers(1, 4))
    nb = int(rng.integers(1, 9))
    rho = float(rng.choice([1.0, 0.7, 1.3]))
    seed = int(rng.integers(-2 ** 31, 2 ** 31 - 1))
    n = nb * d
    scale = np.exp(rng.uniform(-3, 3, n))
    pl = (rng.standard_cauchy(n) * scale).astype(np.float32)
    ps = (scale * rng.uniform(0.5, 2.0, n)).astype(np.float32)
    tl = (pl + ps * rng.standard_normal(n) * rng.uniform(0, 2)).astype(np.float32)
    ts = (ps * np.exp(rng.uniform(-2, 0.5, n))).astype(np.float32)
    i0, s0 = _uniform_encode(cwq, cwqlib, tl, ts, pl, ps, d, bits, n_steps, seed, rho, 0)
    for mode in (1, 2):
        i1, s1 = _uniform_encode(cwq, cwqlib, tl, ts, pl, ps, d, bits, n_steps, seed, rho, mode)
        assert np.array_equal(i1, i0), (trial, mode, d, bits, n_steps)
        _assert_bits_equal(s1, s0, f"stress trial {trial} mode {mode}")


# ---------------------------------------------------------------------------
# general pruned kernel (k_encode_prune_csr): ragged groups and uniform d the
# fast kernel does not take, >= 4096 candidates
# ---------------------------------------------------------------------------
def _csr_encode(cwq, cwqlib, tl, ts, pl, ps, off, bits, n_steps, seed, rho, mode):
    i, s = cwq.encode_blocks(tl, ts, pl, ps, bits, n_steps, seed, rho=rho, block_off=off,
                             prune_mode=int(mode))
    torch.cuda.synchronize()
    return i.cpu().numpy(), s.cpu().numpy()


def _heavy_inputs(rng, n):
    scale = np.exp(rng.uniform(-3, 3, n))
    pl = (rng.standard_cauchy(n) * scale).astype(np.float32)
    ps = (scale * rng.uniform(0.5, 2.0, n)).astype(np.float32)
    tl = (pl + ps * rng.standard_normal(n) * rng.uniform(0, 2)).astype(np.float32)
    ts = (ps * np.exp(rng.uniform(-2, 0.5, n))).astype(np.float32)
    return tl, ts, pl, ps


@pytest.mark.parametrize("sizes,bits,n_steps,rho", [
    ([0, 3, 1, 0, 17, 8, 5, 0, 40, 2, 9, 130], 12, 1, 1.0),
    ([5] * 9, 13, 2, 1.0),
    ([7, 33, 301, 1, 12], 14, 1, 0.9),
    ([100, 100, 100], 12, 3, 1.0),
    ([1100, 40, 600], 12, 2, 1.0),
])
def test_csr_pruned_vs_oracle(cwq, cwqlib, oracle, sizes, bits, n_steps, rho):
    rng = np.random.default_rng(sum(sizes) + bits)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D = int(off[-1])
    tl = rng.standard_normal(D).astype(np.float32)
    ts = rng.uniform(0.2, 1.0, D).astype(np.float32)
    pl = (0.1 * rng.standard_normal(D)).astype(np.float32)
    ps = rng.uniform(0.8, 1.2, D).astype(np.float32)
    wi, ws = oracle.greedy_encode(tl, ts, pl, ps, off, bits, n_steps, 42, rho)
    for mode in (0, 1, 2):
        gi, gs = _csr_encode(cwq, cwqlib, tl, ts, pl, ps, off, bits, n_steps, 42, rho, mode)
        assert np.array_equal(gi, wi), (mode, gi.reshape(-1)[:8], wi.reshape(-1)[:8])
        _assert_bits_equal(gs, ws, f"csr mode {mode}")


@pytest.mark.parametrize("kind", ["far_locs", "huge_locs", "tiny_locs", "flat"])
def test_csr_pruned_adversarial(cwq, cwqlib, oracle, kind):
    rng = np.random.default_rng(7)
    sizes = [3, 20, 1, 45]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D = int(off[-1])
    pl = np.zeros(D, np.float32)
    ps = np.ones(D, np.float32)
    ts = rng.uniform(0.3, 1.0, D).astype(np.float32)
    if kind == "far_locs":
        tl = (rng.standard_normal(D) * 40).astype(np.float32)
    elif kind == "huge_locs":
        tl = (rng.standard_normal(D) * 1e30).astype(np.float32)
        pl = (rng.standard_normal(D) * 1e30).astype(np.float32)
    elif kind == "tiny_locs":
        ts = (rng.uniform(0.3, 1.0, D) * 1e-20).astype(np.float32)
        tl = (rng.standard_normal(D) * 1e-20).astype(np.float32)
    else:  # near-ties everywhere: the survivor list overflows, tiles are redone
        ts = np.full(D, 1e3, np.float32)
        tl = np.zeros(D, np.float32)
    wi, ws = oracle.greedy_encode(tl, ts, pl, ps, off, 12, 1, 5)
    for mode in (0, 2):
        gi, gs = _csr_encode(cwq, cwqlib, tl, ts, pl, ps, off, 12, 1, 5, 1.0, mode)
        assert np.array_equal(gi, wi), (kind, mode)
        _assert_bits_equal(gs, ws, f"csr {kind} mode {mode}")


@pytest.mark.parametrize("kind", ["normal", "far_locs", "huge_locs", "tiny_locs", "flat",
                                  "posterior_is_prior", "inf_scale", "zero_scale", "nan_scale",
                                  "nan_loc_one_dim"])
@pytest.mark.parametrize("bits,n_steps", [(6, 1), (8, 2), (11, 1)])
@pytest.mark.parametrize("path", ["pipeline", "three_kernel"])
def test_small_path_adversarial(cwq, cwqlib, oracle, kind, bits, n_steps, path):
    """The screened small-candidate paths (64 <= 2^b < 4096) on
    ragged groups (an empty one included): near-ties everywhere overflow the
    survivor list (exact fallback), non-finite or out-of-range constants fail
    the gate (exact fallback); every mode equals the oracle.  "pipeline": every
    block <= 64 dims, so the small pipeline takes the launch (k_small_prep1,
    k_small_one, k_small_finalize); "three_kernel": a 130-dim block sends it to
    k_small_prep/screen/survivors."""
    rng = np.random.default_rng(sum(map(ord, kind)) + bits)
    sizes = [3, 20, 1, 45, 0, 7, 64, 130] if path == "three_kernel" else \
        [3, 20, 1, 45, 0, 7, 64, 33, 64, 2, 0, 0, 5]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D = int(off[-1])
    pl = (0.2 * rng.standard_normal(D)).astype(np.float32)
    ps = rng.uniform(0.5, 2.0, D).astype(np.float32)
    tl = (pl + ps * rng.standard_normal(D) * 0.8).astype(np.float32)
    ts = (ps * rng.uniform(0.3, 1.0, D)).astype(np.float32)
    if kind == "far_locs":
        tl = (rng.standard_normal(D) * 40).astype(np.float32)
    elif kind == "huge_locs":
        tl = (rng.standard_normal(D) * 1e30).astype(np.float32)
        pl = (rng.standard_normal(D) * 1e30).astype(np.float32)
    elif kind == "tiny_locs":
        ts = (rng.uniform(0.3, 1.0, D) * 1e-20).astype(np.float32)
        tl = (rng.standard_normal(D) * 1e-20).astype(np.float32)
    elif kind == "flat":
        ts = np.full(D, 1e3, np.float32)
        tl = np.zeros(D, np.float32)
    elif kind == "posterior_is_prior":
        tl, ts = pl.copy(), ps.copy()
    elif kind == "inf_scale":
        ts[5] = np.inf
    elif kind == "zero_scale":
        ts[30] = 0.0
        tl[30] = pl[30]
    elif kind == "nan_scale":
        ts[:] = np.nan
    elif kind == "nan_loc_one_dim":
        tl[40] = np.nan
    wi, ws = oracle.greedy_encode(tl, ts, pl, ps, off, bits, n_steps, 5)
    for mode in (0, 2):
        gi, gs = _csr_encode(cwq, cwqlib, tl, ts, pl, ps, off, bits, n_steps, 5, 1.0, mode)
        assert np.array_equal(gi, wi), (kind, bits, mode)
        _assert_bits_equal(gs, ws, f"small path {kind} bits {bits} mode {mode}")


@pytest.mark.parametrize("trial", range(12))
def test_csr_random_stress(cwq, cwqlib, trial):
    """Random ragged layouts (empty groups included) and odd uniform d, heavy-
    tailed inputs: modes 0 and 2 agree bit for bit."""
    rng = np.random.default_rng(5000 + trial)
    nb = int(rng.integers(1, 7))
    if trial % 3 == 2:
        sizes = [int(rng.choice([1, 3, 5, 7, 9, 12, 20, 72, 100]))] * nb
    else:
        sizes = [int(x) for x in rng.integers(0, 160, nb)]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D = int(off[-1])
    if D == 0:
        sizes[0] = 1
        off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        D = 1
    bits = int(rng.integers(12, 17))
    n_steps = int(rng.integers(1, 4))
    rho = float(rng.choice([1.0, 0.7, 1.3]))
    seed = int(rng.integers(-2 ** 31, 2 ** 31 - 1))
    tl, ts, pl, ps = _heavy_inputs(rng, D)
    i0, s0 = _csr_encode(cwq, cwqlib, tl, ts, pl, ps, off, bits, n_steps, seed, rho, 0)
    i2, s2 = _csr_encode(cwq, cwqlib, tl, ts, pl, ps, off, bits, n_steps, seed, rho, 2)
    assert np.array_equal(i2, i0), (trial, sizes, bits, n_steps)
    _assert_bits_equal(s2, s0, f"csr stress trial {trial}")


@pytest.mark.parametrize("d,bits,nb", [(5, 13, 7), (12, 12, 4), (100, 14, 2), (72, 12, 3)])
def test_uniform_odd_d_general_pruned(cwq, cwqlib, oracle, d, bits, nb):
    rng = np.random.default_rng(d * bits)
    tl, ts, pl, ps = _heavy_inputs(rng, nb * d)
    off = np.arange(nb + 1, dtype=np.int64) * d
    wi, ws = oracle.greedy_encode(tl, ts, pl, ps, off, bits, 2, 11)
    for mode in (0, 2):
        gi, gs = _uniform_encode(cwq, cwqlib, tl, ts, pl, ps, d, bits, 2, 11, 1.0, mode)
        assert np.array_equal(gi, wi), (d, mode)
        _assert_bits_equal(gs, ws, f"uniform d={d} mode {mode}")


@pytest.mark.parametrize("sizes,bits,n_steps,kind", [
    ([4095, 2000, 300, 257], 14, 2, "normal"),   # few long rows: cooperative 16-lane rows
    ([1500, 255, 256, 40], 13, 3, "normal"),     # coop and per-lane rows in one launch
    ([600] * 3, 14, 1, "flat"),                  # near-ties: survivor overflow, redo, exact
    ([700, 900], 12, 2, "heavy"),
    # row lengths around the loops' unit strides (4 units per lane of a 16-lane
    # slot: 64 units per iteration; 2 units per iteration of a per-lane row)
    # and the LDS / visit-order-record boundary at 1024 dims
    ([256, 257, 259, 255, 1021, 1024, 1025, 1027], 12, 2, "normal"),
    ([1087, 1089, 4093, 513, 511, 7, 3, 1], 12, 2, "heavy"),
])
def test_csr_cooperative_rows_vs_oracle(cwq, cwqlib, oracle, sizes, bits, n_steps, kind):
    rng = np.random.default_rng(sum(sizes) * bits)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D = int(off[-1])
    if kind == "heavy":
        tl, ts, pl, ps = _heavy_inputs(rng, D)
    else:
        tl = rng.standard_normal(D).astype(np.float32)
        ts = rng.uniform(0.2, 1.0, D).astype(np.float32)
        pl = (0.1 * rng.standard_normal(D)).astype(np.float32)
        ps = rng.uniform(0.8, 1.2, D).astype(np.float32)
        if kind == "flat":
            ts = np.full(D, 1e3, np.float32)
            tl = np.zeros(D, np.float32)
    wi, ws = oracle.greedy_encode(tl, ts, pl, ps, off, bits, n_steps, 42, 1.0)
    for mode in (0, 2):
        gi, gs = _csr_encode(cwq, cwqlib, tl, ts, pl, ps, off, bits, n_steps, 42, 1.0, mode)
        assert np.array_equal(gi, wi), (kind, mode, gi.reshape(-1)[:8], wi.reshape(-1)[:8])
        _assert_bits_equal(gs, ws, f"coop {kind} mode {mode}")


@pytest.mark.parametrize("d,bits", [
    (1100, 24),   # per-lane rows, visit-order records: n_cand d = 1.06 * 2^34
    (1024, 24),   # constants in LDS, n_cand d = 2^34 exactly: the last 32-bit launch
    (8200, 21),   # cooperative rows, natural order: n_cand d = 1.0009 * 2^34
])
def test_csr_wide_counters_vs_oracle(cwq, cwqlib, oracle, d, bits):
    """The general pruned kernel drops counter word 1 from its Philox rounds
    (HI0) only when every block index (n d + j) / 4 of the launch is below
    2^32, i.e. n_cand d <= 2^34.  One block on either side of that limit,
    against the oracle's full scan (its rows split over threads)."""
    rng = np.random.default_rng(d * bits)
    tl = rng.standard_normal(d).astype(np.float32)
    ts = rng.uniform(0.2, 1.0, d).astype(np.float32)
    pl = (0.1 * rng.standard_normal(d)).astype(np.float32)
    ps = rng.uniform(0.8, 1.2, d).astype(np.float32)
    off = np.array([0, d], np.int64)
    wi, ws = oracle.code_greedy_sample_rows(tl, ts, pl, ps, bits, 42)
    gi, gs = _csr_encode(cwq, cwqlib, tl, ts, pl, ps, off, bits, 1, 42, 1.0, 2)
    assert int(gi.reshape(-1)[0]) == int(wi[0]), (d, bits, gi.reshape(-1), wi)
    _assert_bits_equal(gs, ws, f"wide counters d={d} bits={bits}")


@pytest.mark.parametrize("sizes,bits,n_steps", [
    ([300, 40] * 7, 16, 1),    # 14 groups: 439 tiles/group asked, 437 hold candidates
    ([260] * 3 + [20] * 36, 16, 2),  # three stream parts of 13 groups: 473 asked, 472 used
])
def test_csr_tiling_leaves_no_empty_tile(cwq, cwqlib, oracle, sizes, bits, n_steps):
    """Tile counts that do not divide the candidates evenly (found by
    tools/stress_csr.py): the launcher must not create tiles past the last
    candidate, whose negative row ranges would never drain."""
    rng = np.random.default_rng(len(sizes) * bits)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    tl, ts, pl, ps = _heavy_inputs(rng, int(off[-1]))
    wi, ws = oracle.greedy_encode(tl, ts, pl, ps, off, bits, n_steps, 7, 1.0)
    gi, gs = _csr_encode(cwq, cwqlib, tl, ts, pl, ps, off, bits, n_steps, 7, 1.0, 2)
    assert np.array_equal(gi, wi)
    _assert_bits_equal(gs, ws, "uneven csr tiling")


@pytest.mark.parametrize("kind", ["pln_like", "outliers", "nan_dim", "single"])
def test_importance_grouped_fused_matches_stepwise(cwq, kind):
    """cwq_code_grouped_importance (one native call) returns exactly what the
    step-by-step host pipeline returns: sample bits, bitcode, starts, outliers."""
    import compression_without_quantization_amd.coded_importance_sampler as I
    from compression_without_quantization_amd.synthetic import make_latents
    D = {"pln_like": 4000, "outliers": 777, "nan_dim": 300, "single": 1}[kind]
    q_loc, q_scale, p_loc, p_scale = make_latents(D, bits_per_dim=1.5, seed=D)
    if kind == "outliers":
        q_loc[::50] = p_loc[::50] + 40 * p_scale[::50]   # KL far above the limit
    if kind == "nan_dim":
        q_loc[17] = np.nan
    t, p = cwq.Normal(q_loc, q_scale), cwq.Normal(p_loc, p_scale)
    old = (I.USE_FUSED, I.VERBOSE)
    try:
        I.VERBOSE = False
        res = {}
        for fused in (True, False):
            I.USE_FUSED = fused
            with warnings.catch_warnings():
                warnings.simplefilter("error", RuntimeWarning)  # no undefined NaN cast
                res[fused] = I.code_grouped_importance_sample(None, t, p, 42, 16,
                                                              max_group_size_bits=3,
                                                              dim_kl_bit_limit=12)
    finally:
        I.USE_FUSED, I.VERBOSE = old
    a, b = res[True], res[False]
    _assert_bits_equal(a[0], b[0], f"fused sample ({kind})")
    assert a[1] == b[1]
    assert np.array_equal(np.asarray(a[2]), np.asarray(b[2]))
    assert np.array_equal(a[3][0], b[3][0]) and np.array_equal(a[3][1], b[3][1])
    if kind == "outliers":
        assert a[3][0].size >= 15
    if kind == "nan_dim":  # a NaN outlier draw is coded as 0 (quantize_quint16)
        k = list(a[3][0]).index(17)
        assert a[3][1][k] == 0 and np.isnan(a[0][17])


def test_capi_from_plain_c(cwq):
    """examples/capi_demo (plain C over include/cwq.h, built by `make`) encodes
    and decodes on the device; its indices equal the Python API's on the same
    inputs and its decode round trip is bit-exact."""
    import subprocess
    from conftest import REPO
    exe = os.path.join(REPO, "examples", "capi_demo")
    assert os.path.exists(exe), "build it with `make` (__graft_entry__.build does)"
    nb, d, bits, seed = 300, 20, 12, -7
    out = subprocess.run([exe, str(nb), str(d), str(bits), str(seed)], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    f = dict(zip(out.stdout.split()[::2], out.stdout.split()[1::2]))
    n = nb * d
    k = np.arange(2 * n, dtype=np.uint64)
    u = ((k * np.uint64(2654435761)) & np.uint64(0xFFFFFFFF)).astype(np.float32) * \
        np.float32(1.0 / 4294967296.0)
    tl = (u[:n] - np.float32(0.5)).astype(np.float32)
    ts = (np.float32(0.3) + np.float32(0.6) * u[n:]).astype(np.float32)
    idx, _ = cwq.encode_blocks(tl, ts, np.zeros(n, np.float32), np.ones(n, np.float32), bits, 1,
                               seed, block_dim=d)
    idx = idx.cpu().numpy().reshape(-1)
    s = 0
    for v in idx:
        s = (s * 1000003 + int(np.uint32(v))) % (1 << 64)
    assert int(f["idx0"]) == int(idx[0]) and int(f["checksum"]) == s
    assert int(f["roundtrip_mismatch"]) == 0


def test_philox_counter_crosses_2_32(cwq, oracle):
    """Rows whose flat normal index n*d passes 4 * 2^32 (Philox block index
    above 2^32: TF's 128-bit counter carries into its second word): decoding
    rows on both sides of the carry matches the oracle, and the encoder's
    winner row round trips (d=136, 2^27 candidates, one block)."""
    d, bits, seed = 136, 27, 11
    rng = np.random.default_rng(9)
    tl = rng.standard_normal(d).astype(np.float32) * 0.3
    ts = rng.uniform(0.5, 1.0, d).astype(np.float32)
    pl = np.zeros(d, np.float32)
    ps = np.ones(d, np.float32)
    off = np.array([0, d], np.int64)
    cross = (1 << 34) // d                      # first row whose block index is >= 2^32
    for n in (0, cross - 1, cross, cross + 1, (1 << bits) - 1):
        want = oracle.greedy_decode(np.array([[n]], np.int32), pl, ps, off, bits, 1, seed)
        got = cwq.decode_blocks(np.array([[n]], np.int32), pl, ps, bits, 1, seed, block_off=off)
        _assert_bits_equal(got.cpu().numpy(), want, f"decode row {n}")
    idx, sample = cwq.encode_blocks(tl, ts, pl, ps, bits, 1, seed, block_off=off)
    i = idx.cpu().numpy().reshape(-1)
    want = oracle.greedy_decode(i.reshape(1, 1).astype(np.int32), pl, ps, off, bits, 1, seed)
    _assert_bits_equal(sample.cpu().numpy(), want, "encoder winner row")


def test_encode_captured_in_hip_graph(cwq, cwqlib):
    """The C ABI is stream-ordered and capturable (include/cwq.h): a multi-step
    CSR encode, which forks onto the library's streams and joins back, and a
    uniform encode are captured into one HIP graph; replays reproduce the eager
    results bit for bit."""
    rng = np.random.default_rng(21)
    sizes = [300, 17, 450, 5, 260, 33, 1]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D = int(off[-1])
    dev = torch.device("cuda")
    f = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)
    tl = f(rng.standard_normal(D))
    ts = f(rng.uniform(0.3, 1.0, D))
    z, o = torch.zeros(D, device=dev), torch.ones(D, device=dev)
    offs = torch.from_numpy(off).to(dev)
    nb, steps, bits = len(sizes), 3, 12
    idx = torch.zeros((nb, steps), dtype=torch.int32, device=dev)
    smp = torch.zeros(D, dtype=torch.float32, device=dev)
    ws = torch.empty(cwqlib.cwq_greedy_encode_workspace_size(nb, D, max(sizes)),
                     dtype=torch.uint8, device=dev)
    ub, ud = 64, 32                                    # uniform C4-shaped blocks
    utl = f(rng.standard_normal(ub * ud) * 0.5)
    uts = f(rng.uniform(0.3, 0.9, ub * ud))
    uz, uo = torch.zeros(ub * ud, device=dev), torch.ones(ub * ud, device=dev)
    uidx = torch.zeros((ub, 1), dtype=torch.int32, device=dev)
    usmp = torch.zeros(ub * ud, dtype=torch.float32, device=dev)
    uws = torch.empty(cwqlib.cwq_greedy_encode_uniform_workspace_size(ub, ud), dtype=torch.uint8,
                      device=dev)

    def run():
        st = torch.cuda.current_stream().cuda_stream
        assert cwqlib.cwq_greedy_encode(
            tl.data_ptr(), ts.data_ptr(), z.data_ptr(), o.data_ptr(), offs.data_ptr(), nb, D,
            max(sizes), bits, steps, 42, 1.0, 0, idx.data_ptr(), smp.data_ptr(), ws.data_ptr(),
            ws.numel(), None, st) == 0
        assert cwqlib.cwq_greedy_encode_uniform(
            utl.data_ptr(), uts.data_ptr(), uz.data_ptr(), uo.data_ptr(), ub, ud, 14, 1, 7, 1.0,
            0, uidx.data_ptr(), usmp.data_ptr(), uws.data_ptr(), uws.numel(), None, st) == 0

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        run()                                          # eager (creates the library streams)
    torch.cuda.synchronize()
    want = [t.clone() for t in (idx, smp, uidx, usmp)]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="relaxed"):
        run()
    for _ in range(2):
        for t in (idx, smp, uidx, usmp):
            t.zero_()
        g.replay()
        torch.cuda.synchronize()
        for got, w in zip((idx, smp, uidx, usmp), want):
            assert torch.equal(got.view(torch.int32), w.view(torch.int32))
