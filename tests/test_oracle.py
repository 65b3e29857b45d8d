"""CPU tests: the oracle against its pins (KATs, reference bit-string examples,
golden fixtures) and the host-side pieces of the product (grouping, bit strings)."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, REPO
from compression_without_quantization_amd import binary_io as B
from compression_without_quantization_amd.coded_greedy_sampler import group_size_threshold


def _json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_philox_random123_kat(oracle, mathcheck):
    for v in _json("philox_kat.json")["vectors"]:
        ctr = np.array([int(x, 16) for x in v["ctr"]], np.uint32)
        key = np.array([int(x, 16) for x in v["key"]], np.uint32)
        want = [int(x, 16) for x in v["out"]]
        assert list(oracle.philox(ctr, key)) == want
        out = np.zeros(4, np.uint32)
        mathcheck.mc_philox(ctr.ctypes.data_as(ctypes.c_void_p),
                            key.ctypes.data_as(ctypes.c_void_p),
                            out.ctypes.data_as(ctypes.c_void_p))
        assert list(out) == want  # the product header's Philox


def test_philox_three_implementations_agree(oracle, mathcheck):
    """SURVEY.md 8(c) pin 1: the oracle's Philox4x32-10, the product header's
    (csrc/cwq_math.h) and ROCm's own rocRAND engine
    (/opt/rocm/include/rocrand/rocrand_philox4x32_10.h:270-302, compiled for the
    host by tests/native/rocrand_pin.cpp) on 10^6 random (counter, key) pairs,
    plus the edge words 0 and 0xffffffff."""
    import subprocess
    subprocess.check_call(["make", "-C", REPO, "tests/native/librocrand_pin.so"],
                          stdout=subprocess.DEVNULL)
    rr = ctypes.CDLL(os.path.join(REPO, "tests", "native", "librocrand_pin.so"))
    vp = ctypes.c_void_p
    for f in (rr.rr_philox_many, oracle.lib().cwqo_philox4x32_10_many, mathcheck.mc_philox_many):
        f.argtypes = [vp, vp, ctypes.c_int64, vp]
        f.restype = None
    rng = np.random.default_rng(123)
    n = 1_000_000
    ctr = rng.integers(0, 1 << 32, (n, 4), dtype=np.uint64).astype(np.uint32)
    key = rng.integers(0, 1 << 32, (n, 2), dtype=np.uint64).astype(np.uint32)
    ctr[:16] = np.array([0, 0xffffffff], np.uint32)[(np.arange(64).reshape(16, 4) >> 1) & 1]
    key[:16] = np.array([0, 0xffffffff], np.uint32)[np.arange(32).reshape(16, 2) & 1]
    outs = []
    for f in (rr.rr_philox_many, oracle.lib().cwqo_philox4x32_10_many, mathcheck.mc_philox_many):
        o = np.zeros((n, 4), np.uint32)
        f(ctr.ctypes.data, key.ctypes.data, n, o.ctypes.data)
        outs.append(o)
    assert np.array_equal(outs[0], outs[1]), "rocRAND vs oracle"
    assert np.array_equal(outs[0], outs[2]), "rocRAND vs product header"
    kat = _json("philox_kat.json")["vectors"][0]  # ctr 0, key 0
    assert [int(x, 16) for x in kat["ctr"]] == [0, 0, 0, 0]
    o = np.zeros(4, np.uint32)
    z = np.zeros(4, np.uint32)
    rr.rr_philox_many(z.ctypes.data, z.ctypes.data, 1, o.ctypes.data)
    assert list(o) == [int(x, 16) for x in kat["out"]]


def test_stateless_normal_fixture(oracle):
    sn = _json("stateless_normal.json")
    for s0 in ("42000", "-7", "2147483647", "0"):
        z = oracle.stateless_normal(int(s0), 42, 4099)
        assert [float(v).hex() for v in z[:16]] == sn[s0]["head"]
        assert hashlib.sha256(z.tobytes()).hexdigest() == sn[s0]["sha256_4099"]
    key, ctr = oracle.generate_key(42000, 42)
    assert [int(v) for v in key] == sn["generate_key_42000_42"]["key"]
    assert [int(v) for v in ctr] == sn["generate_key_42000_42"]["ctr"]


def test_stateless_normal_layout(oracle):
    # A.3: element k of the flat [N, d] output is word k%4 of Philox block k//4;
    # a longer draw extends a shorter one (same counter stream).
    a = oracle.stateless_normal(123, 42, 37)
    b = oracle.stateless_normal(123, 42, 1000)
    assert np.array_equal(a.view(np.uint32), b[:37].view(np.uint32))
    # normal-ish statistics
    z = oracle.stateless_normal(5, 42, 200000)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01


def test_stateless_normal_sample_misc(oracle):
    # misc.py:14-15 scale*z then loc+ (two roundings)
    loc = np.array([0.5, -1.25, 3.0], np.float32)
    scale = np.array([2.0, 0.3, 1e-3], np.float32)
    out = oracle.stateless_normal_sample(loc, scale, 5, 77)
    z = oracle.stateless_normal(77, 42, 15).reshape(5, 3)
    want = loc[None, :] + (scale[None, :] * z)
    assert np.array_equal(out.view(np.uint32), want.astype(np.float32).view(np.uint32))


def test_bm_tables_fixture(oracle):
    t = _json("bm_tables.json")
    n = 1 << 23
    rad = oracle.bm_radius_table(0, n)
    s, c = oracle.bm_sincos_table(0, n)
    assert hashlib.sha256(rad.tobytes()).hexdigest() == t["radius_sha256"]
    assert hashlib.sha256(s.tobytes()).hexdigest() == t["sin_sha256"]
    assert hashlib.sha256(c.tobytes()).hexdigest() == t["cos_sha256"]


def test_bitstring_reference_examples():
    bs = _json("bitstring.json")
    for num, nb, want in bs["to_bit_string"]:
        assert B.to_bit_string(num, nb) == want
    for code, want in bs["from_bit_string"]:
        assert B.from_bit_string(code) == want
        assert B.from_bit_string(code.encode()) == want
    for num, nb in bs["overflow"]:
        with pytest.raises(Exception, match="bigger than what we can encode"):
            B.to_bit_string(num, nb)


def test_bitcode_vectorised_matches_scalar():
    rng = np.random.default_rng(0)
    for nbits in (1, 4, 8, 16, 24):
        idx = rng.integers(0, 1 << nbits, size=257)
        code = B.indices_to_bitcode(idx, nbits)
        assert code == ''.join(B.to_bit_string(int(i), nbits) for i in idx)
        back = B.bitcode_to_indices(code, nbits, idx.size)
        assert np.array_equal(back, idx)
    with pytest.raises(Exception, match="bigger than what we can encode"):
        B.indices_to_bitcode([3, 16], 4)
    # short trailing slice reads missing bits as 0 (tf.strings.substr clamp)
    assert list(B.bitcode_to_indices("1011", 3, 2)) == [5, 1]


def test_bitcode_parse_native_matches_scalar():
    """cwq_bitcode_to_indices (the native parse behind bitcode_to_indices for
    widths <= 30) against from_bit_string of each LSB-first slice, on every
    width, truncated strings (missing chars read '0') and chars other than '1'."""
    rng = np.random.default_rng(1)
    for nbits in range(0, 31):
        for count in (0, 1, 7, 64, 129):
            idx = rng.integers(0, 1 << nbits, size=count) if nbits else np.zeros(count, np.int64)
            code = B.indices_to_bitcode(idx, nbits)
            for cut in sorted({len(code), max(len(code) - 5, 0), len(code) // 3}):
                s = code[:cut]
                want = [B.from_bit_string(s[i * nbits:(i + 1) * nbits]) for i in range(count)]
                got = B.bitcode_to_indices(s, nbits, count)
                assert got.dtype == np.int64 and list(got) == want, (nbits, count, cut)
                assert list(B.bitcode_to_indices(s.encode(), nbits, count, dtype=np.int32)) == want
    assert list(B.bitcode_to_indices("1x21" * 3, 2, 6)) == [1, 2, 1, 2, 1, 2]
    with pytest.raises(Exception):
        B.bitcode_to_indices("0101", 3, -1)


def _eigen_sum_py(x):
    x = np.asarray(x, np.float32)
    d = x.size
    vec = (d // 8) * 8
    p = np.zeros(8, np.float32)
    for j in range(0, vec, 8):
        p = (p + x[j:j + 8]).astype(np.float32)
    t = np.float32(0)
    for j in range(vec, d):
        t = np.float32(t + x[j])
    q = (p[:4] + p[4:]).astype(np.float32)
    r = np.float32(np.float32(q[0] + q[2]) + np.float32(q[1] + q[3]))
    return np.float32(t + r)


def test_eigen_rowsum_order(oracle):
    rng = np.random.default_rng(1)
    for d in (0, 1, 5, 8, 9, 16, 31, 32, 33, 100):
        for _ in range(20):
            x = (rng.standard_normal(d) * 10 ** rng.uniform(-3, 6, d)).astype(np.float32)
            assert np.float32(oracle.eigen_rowsum(x)) == _eigen_sum_py(x)
    # the order is observable: sequential summation differs on this vector
    x = np.array([1e8, 1, -1e8, 1, 1, 1, 1, 1, 3], np.float32)
    assert np.float32(oracle.eigen_rowsum(x)) == _eigen_sum_py(x)


def test_log_prob_tfp_form(oracle):
    # A.5: -0.5*((x-mu)/s)^2 - (0.9189385f + logf(s)), float32 ops
    for x, mu, s in [(0.3, -0.2, 0.7), (5.0, 0.0, 1.0), (-1e-3, 2.0, 3.5)]:
        x, mu, s = np.float32(x), np.float32(mu), np.float32(s)
        z = np.float32(np.float32(x - mu) / s)
        u = np.float32(np.float32(-0.5) * np.float32(z * z))
        c = np.float32(np.float32(0.9189385332046727) + np.float32(oracle.logf_table([s])[0]))
        assert np.float32(oracle.lib().cwqo_normal_log_prob(x, mu, s)) == np.float32(u - c)


@pytest.mark.parametrize("name", ["oracle_c1.npz", "oracle_c4_slice.npz",
                                  "oracle_multistep.npz", "oracle_odd_d.npz"])
def test_oracle_reproduces_golden(oracle, golden, name):
    g = golden(name)
    idx, sample = oracle.greedy_encode(g["t_loc"], g["t_scale"], g["p_loc"], g["p_scale"],
                                       g["block_off"], int(g["n_bits"]), int(g["n_steps"]),
                                       int(g["seed"]), float(g["rho"]), int(g["block_id_base"]))
    assert np.array_equal(idx, g["idx"])
    assert np.array_equal(sample.view(np.uint32), g["sample"].view(np.uint32))
    dec = oracle.greedy_decode(idx, g["p_loc"], g["p_scale"], g["block_off"], int(g["n_bits"]),
                               int(g["n_steps"]), int(g["seed"]), float(g["rho"]),
                               int(g["block_id_base"]))
    assert np.array_equal(dec.view(np.uint32), sample.view(np.uint32))


def test_oracle_single_block_equals_batched(oracle, golden):
    g = golden("oracle_multistep.npz")
    off = g["block_off"]
    for b in range(off.size - 1):
        s = slice(off[b], off[b + 1])
        idx, sample = oracle.code_greedy_sample(
            g["t_loc"][s], g["t_scale"][s], g["p_loc"][s], g["p_scale"][s], int(g["n_bits"]),
            int(g["n_steps"]), int(g["seed"]) + int(g["block_id_base"]) + b, float(g["rho"]))
        assert np.array_equal(idx, g["idx"][b])
        assert np.array_equal(sample.view(np.uint32), g["sample"][s].view(np.uint32))


@pytest.mark.parametrize("d,bits,kind", [(40, 6, "normal"), (9, 12, "normal"),
                                         (33, 11, "flat"), (5, 10, "ties")])
def test_oracle_rows_split_equals_serial(oracle, d, bits, kind):
    """cwqo_code_greedy_sample_rows (rows over threads, the wide-counter GPU
    tests' checker) returns the serial scan's first maximal row and sample."""
    rng = np.random.default_rng(d * bits)
    tl = rng.standard_normal(d).astype(np.float32)
    ts = rng.uniform(0.2, 1, d).astype(np.float32)
    pl = (0.1 * rng.standard_normal(d)).astype(np.float32)
    ps = rng.uniform(0.8, 1.2, d).astype(np.float32)
    if kind == "flat":     # near-ties everywhere
        tl, ts = np.zeros(d, np.float32), np.full(d, 1e3, np.float32)
    if kind == "ties":     # every row has the same value: row 0 must win
        tl, ts = np.zeros(d, np.float32), np.full(d, np.inf, np.float32)
    for nthreads in (1, 3, 0):
        want = oracle.code_greedy_sample(tl, ts, pl, ps, bits, 1, 77)
        got = oracle.code_greedy_sample_rows(tl, ts, pl, ps, bits, 77, nthreads=nthreads)
        assert int(got[0][0]) == int(want[0][0]), (kind, nthreads, got[0], want[0])
        assert np.array_equal(got[1].view(np.uint32), want[1].view(np.uint32))


def test_oracle_argmax_is_best(oracle):
    # brute force: argmax of the row sums over the materialised candidates
    rng = np.random.default_rng(5)
    d, bits, seed = 6, 7, 1234
    tl = rng.standard_normal(d).astype(np.float32)
    ts = rng.uniform(0.2, 1, d).astype(np.float32)
    pl = np.zeros(d, np.float32)
    ps = np.ones(d, np.float32)
    idx, sample = oracle.code_greedy_sample(tl, ts, pl, ps, bits, 1, seed)
    cand = oracle.stateless_normal_sample(pl, ps, 1 << bits, 1000 * seed)
    lp = np.array([[oracle.lib().cwqo_normal_log_prob(float(v), float(m), float(s))
                    for v, m, s in zip(row, tl, ts)] for row in cand], np.float32)
    sums = np.array([_eigen_sum_py(r) for r in lp])
    assert idx[0] == int(np.argmax(sums))
    assert np.array_equal(sample, (np.float32(0) + cand[idx[0]]).astype(np.float32))


def _group_starts_py(kl_divs, n_bits_per_group, max_group_size_bits):
    """Transcription of coded_greedy_sampler.py:207-252 (numpy scalar semantics)."""
    group_start_indices = [0]
    current_group_size = 0
    current_group_kl = 0
    n_nats_per_group = n_bits_per_group * np.log(2) - 1
    D = len(kl_divs)
    for idx in range(D):
        group_bits = np.log(current_group_size + 1) / np.log(2)
        if group_bits >= max_group_size_bits or \
           current_group_kl + kl_divs[idx] >= n_nats_per_group or \
           idx == D - 1:
            group_start_indices.append(idx)
            current_group_size = 1
            current_group_kl = kl_divs[idx]
        else:
            current_group_kl += kl_divs[idx]
            current_group_size += 1
    group_start_indices += [D]
    return group_start_indices


@pytest.mark.parametrize("case", range(8))
def test_grouping_matches_reference_loop(oracle, cwqlib, case):
    from compression_without_quantization_amd.coded_greedy_sampler import group_starts
    rng = np.random.default_rng(100 + case)
    D = [1, 2, 50, 3000, 20000, 9000, 7, 5000][case]
    bits, maxbits = [(8, 12), (8, 12), (4, 3), (8, 12), (16, 12), (8, 5), (2, 1), (8, 12)][case]
    kl = rng.gamma(0.7, 1.0, D).astype(np.float32)
    if case == 3:
        kl[:] = 1e-5          # many near-zero dims: size cap binds (4095)
    if case == 7:
        kl[0] = 100.0         # kl[0] >= n_nats: duplicate leading 0 (empty group)
    want = _group_starts_py(kl, bits, maxbits)
    assert group_starts(kl, bits, maxbits) == want
    assert oracle.group_starts(kl, bits, group_size_threshold(maxbits)) == want


def test_group_size_threshold():
    for bits in range(1, 16):
        s = group_size_threshold(bits)
        assert np.log(s + 1) / np.log(2) >= bits
        assert s == 0 or not (np.log(s) / np.log(2) >= bits)


def test_kl_and_standardise_float32(oracle):
    rng = np.random.default_rng(9)
    n = 1000
    ql, pl = rng.standard_normal((2, n)).astype(np.float32)
    qs, ps = rng.uniform(0.1, 3, (2, n)).astype(np.float32)
    kl = oracle.kl_normal_normal(ql, qs, pl, ps)
    exact = (np.log(ps.astype(np.float64) / qs) + (qs.astype(np.float64) ** 2 +
             (ql.astype(np.float64) - pl) ** 2) / (2 * ps.astype(np.float64) ** 2) - 0.5)
    assert np.allclose(kl, exact, rtol=1e-4, atol=1e-5)
    tl, ts = oracle.standardise(ql, qs, pl, ps)
    assert np.array_equal(tl, ((ql - pl) / ps).astype(np.float32))
    assert np.array_equal(ts, (qs / ps).astype(np.float32))


@pytest.mark.parametrize("strict", [False, True])
def test_grouping_exact_threshold_ties(cwqlib, strict):
    """Running sums landing exactly on the float32 neighbours of n_nats: the
    native scan's float32 threshold must agree with the reference's float64
    comparison (>= for the greedy coder, > for the importance coder)."""
    from compression_without_quantization_amd.coded_greedy_sampler import (
        group_size_threshold, group_starts)
    from compression_without_quantization_amd.coded_importance_sampler import (
        importance_group_size_threshold, importance_group_starts)
    bits = 8 if not strict else 20
    n_nats = bits * np.log(2) - 1
    up = np.float32(n_nats)
    while float(up) < n_nats:
        up = np.nextafter(up, np.float32(np.inf))
    cands = [up, np.nextafter(up, np.float32(0)), np.nextafter(up, np.float32(np.inf))]
    if float(up) == n_nats:
        cands.append(up)
    kl = []
    for c in cands * 5:
        kl += [np.float32(c - np.float32(2.0)), np.float32(2.0), np.float32(0.25)]
    kl = np.asarray(kl, np.float32)
    if not strict:
        want = _group_starts_py(kl, bits, 12)
        assert group_starts(kl, bits, 12) == want
    else:
        # transcription of coded_importance_sampler.py:178-203 (strict >)
        thr = importance_group_size_threshold(4)
        starts, cur_size, cur_kl = [0], 0, np.float32(0)
        for i in range(kl.size):
            s = np.float32(cur_kl + kl[i])
            if cur_size >= thr or float(s) > n_nats or i == kl.size - 1:
                starts.append(i)
                cur_size, cur_kl = 1, kl[i]
            else:
                cur_kl, cur_size = s, cur_size + 1
        starts.append(kl.size)
        got = importance_group_starts(kl, bits, 4)
        assert list(got) == starts


@pytest.mark.parametrize("kind", range(5))
def test_grouping_chunked_scan_matches_reference_loop(cwqlib, kind):
    """Inputs past 8K dims take the 8-chunk speculative scan with sequential
    fix-up; it must reproduce the reference loop exactly, also when the size
    cap binds everywhere or every dim is its own group."""
    from compression_without_quantization_amd.coded_greedy_sampler import group_starts
    from compression_without_quantization_amd.synthetic import make_latents
    rng = np.random.default_rng(40 + kind)
    D = [30011, 50000, 9000, 65537, 20000][kind]
    if kind == 0:
        kl = rng.gamma(0.7, 1.0, D)
    elif kind == 1:
        kl = np.full(D, 1e-5)                  # only the 4095-dim cap closes groups
    elif kind == 2:
        kl = rng.uniform(3, 10, D)             # every dim over the budget
    elif kind == 3:
        kl = np.where(rng.uniform(size=D) < 0.5, 1e-4, rng.gamma(2, 2, D))
    else:
        q, qs, p, ps = make_latents(D, seed=kind)
        t, s = (q - p) / ps, qs / ps
        kl = 0.5 * (s ** 2 + t ** 2 - 1 - 2 * np.log(s))
    kl = kl.astype(np.float32)
    bits, maxbits = [(8, 12), (8, 12), (4, 3), (16, 12), (8, 5)][kind]
    assert group_starts(kl, bits, maxbits) == _group_starts_py(kl, bits, maxbits)
