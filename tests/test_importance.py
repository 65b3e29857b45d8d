"""CPU tests for the importance sampler's host pieces (code/coded_importance_sampler.py,
code/binary_io.py:7-39) and its oracle."""
import numpy as np
import pytest

from compression_without_quantization_amd import binary_io as B
from compression_without_quantization_amd.coded_importance_sampler import (
    dequantize_quint16, importance_group_size_threshold, importance_group_starts,
    num_samples_plan, quantize_quint16)


def _elias_ref(x):
    """Transcription of binary_io.py:7-21."""
    lg2 = np.log(2)
    n = np.floor(np.log(x) / lg2).astype(np.int32)
    l = np.floor(np.log(n + 1) / lg2).astype(np.int32)
    length_length_code = ''.join(["0"] * l)
    length_code = B.to_bit_string(n + 1, l + 1)[::-1]
    num_code = B.to_bit_string(x, n + 1)[::-1][1:]
    return length_length_code + length_code + num_code


def test_elias_delta_known_vectors():
    # standard Elias-delta codes
    known = {1: "1", 2: "0100", 3: "0101", 4: "01100", 7: "01111", 8: "00100000",
             17: "001010001"}
    for x, c in known.items():
        assert B.elias_delta_code(x) == c
    rng = np.random.default_rng(0)
    # x < 2^30: above that the reference's own to_bit_string(x, n + 1) overflows
    # (2 ** np.int32(31)), a latent bug its ~2^19 importance indices never reach
    xs = list(range(1, 3000)) + list(rng.integers(1, 2 ** 30, 3000)) + \
        [2 ** k for k in range(30)] + [2 ** k - 1 for k in range(1, 31)]
    for x in xs:
        c = B.elias_delta_code(int(x))
        assert c == _elias_ref(int(x))
        # exact integer form of the float64 formula below 2^31
        n = int(x).bit_length() - 1
        assert len(c) == 2 * ((n + 1).bit_length() - 1) + n + 1
        num, ln = B.elias_delta_decode(c + "0110")
        assert (num, ln) == (int(x), len(c))


def test_elias_concatenation_parses_sequentially():
    rng = np.random.default_rng(1)
    xs = [int(v) for v in rng.integers(1, 400000, 500)]
    code = (''.join(B.elias_delta_code(x) for x in xs)).encode()
    out = []
    while code:
        num, ln = B.elias_delta_decode(code)
        out.append(num)
        code = code[ln:]
    assert out == xs


def test_quint16_matches_oracle(oracle):
    rng = np.random.default_rng(2)
    x = np.concatenate([rng.uniform(-40, 40, 100000), [-30, 30, 0, -31, 31, 29.99999]])
    x = x.astype(np.float32)
    q = quantize_quint16(x)
    assert np.array_equal(q, oracle.quantize_quint16(x))
    d = dequantize_quint16(q)
    assert np.array_equal(d.view(np.uint32), oracle.dequantize_quint16(q).view(np.uint32))
    inside = np.abs(x) <= 30
    assert np.max(np.abs(d[inside] - x[inside])) <= 60 / 65535 / 2 * 1.01


def test_quint16_nan_is_zero(oracle):
    """A NaN outlier draw has a defined code: 0 (the code of -30), in the
    product and the oracle, without NumPy's undefined float -> uint16 cast."""
    import warnings
    x = np.array([np.nan, -np.nan, 1.0, np.inf, -np.inf], dtype=np.float32)
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        q = quantize_quint16(x)
    assert q.tolist() == [0, 0, 33860, 65535, 0]
    assert np.array_equal(q, oracle.quantize_quint16(x))


@pytest.mark.parametrize("case", range(5))
def test_importance_grouping_matches_transcription(oracle, cwqlib, case):
    rng = np.random.default_rng(40 + case)
    D = [1, 20, 3000, 5000, 100][case]
    bits, maxbits = [(20, 4), (20, 2), (20, 4), (8, 3), (20, 0)][case]
    kl = rng.gamma(0.8, 2.0, D).astype(np.float32)
    if case == 3:
        kl[0] = 50.0
    want = oracle.importance_group_starts(kl, bits, maxbits)
    assert importance_group_starts(kl, bits, maxbits) == want


def test_importance_size_threshold():
    for bits in range(0, 10):
        s = importance_group_size_threshold(bits)
        assert np.log(s + 1) / np.log(2) > bits
        assert s == 0 or not (np.log(s) / np.log(2) > bits)


def test_num_samples_plan_matches_oracle(oracle, cwqlib):
    rng = np.random.default_rng(3)
    for _ in range(20):
        d = int(rng.integers(1, 17))
        tl = rng.standard_normal(d).astype(np.float32)
        ts = rng.uniform(0.3, 1.0, d).astype(np.float32)
        pl = np.zeros(d, np.float32)
        ps = np.ones(d, np.float32)
        kl = oracle.kl_normal_normal(tl, ts, pl, ps)
        n = num_samples_plan(kl, [0, d])[0]
        assert n == oracle.importance_num_samples(tl, ts, pl, ps)
        assert n == int(np.ceil(np.exp(np.float64(kl.sum())))) or abs(
            n - np.exp(np.float64(kl.sum()))) < 1e-3 * n + 2


def test_oracle_importance_argmax_brute_force(oracle):
    rng = np.random.default_rng(4)
    d, seed = 5, 77
    tl = rng.standard_normal(d).astype(np.float32) * 0.5
    ts = rng.uniform(0.4, 0.9, d).astype(np.float32)
    pl = np.zeros(d, np.float32)
    ps = np.ones(d, np.float32)
    n = oracle.importance_num_samples(tl, ts, pl, ps)
    idx, sample = oracle.importance_encode(tl, ts, pl, ps, [0, d], [n], seed)
    cand = oracle.stateless_normal_sample(pl, ps, n, seed)
    lp = lambda x, m, s: oracle.lib().cwqo_normal_log_prob(float(x), float(m), float(s))
    w = np.array([[np.float32(lp(v, m, s)) - np.float32(lp(v, 0, 1))
                   for v, m, s in zip(row, tl, ts)] for row in cand], np.float32)
    from test_oracle import _eigen_sum_py
    sums = np.array([_eigen_sum_py(r) for r in w])
    assert idx[0] == int(np.argmax(sums))
    assert np.array_equal(sample, cand[idx[0]])
    assert np.array_equal(oracle.importance_decode_block(idx[0], pl, ps, seed), sample)


def test_elias_many_matches_per_value(cwqlib):
    """The native batch coder (cwq_elias_delta_encode/decode) equals the
    per-value restatement of binary_io.py:7-39 and parses its own output."""
    from compression_without_quantization_amd.binary_io import (
        elias_delta_code, elias_delta_code_many, elias_delta_decode_many)
    rng = np.random.default_rng(8)
    xs = np.concatenate([np.arange(1, 5000), rng.integers(1, 2 ** 30, 5000),
                         [2 ** k for k in range(30)], [2 ** k - 1 for k in range(1, 31)]])
    want = ''.join(elias_delta_code(int(v)) for v in xs)
    got = elias_delta_code_many(xs)
    assert got == want
    back, used = elias_delta_decode_many(got + "0101", xs.size)
    assert used == len(got) and np.array_equal(back, xs)
    # values past 2^30 take the per-value path
    big = [2 ** 30, 2 ** 30 + 5, 7]
    assert elias_delta_code_many(big) == ''.join(elias_delta_code(v) for v in big)
    with pytest.raises(ValueError):
        elias_delta_decode_many(got[:-3], xs.size)
    assert elias_delta_code_many([]) == ''
