"""CPU: the product's device-math restatement (csrc/cwq_math.h, compiled for the
host) equals the host glibc 2.35 libm on the FULL Box-Muller input domains
(every transcendental input has only 2^23 distinct values)."""
import ctypes

import numpy as np

N = 1 << 23


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def test_radius_exhaustive(oracle, mathcheck):
    want = oracle.bm_radius_table(0, N)
    got = np.empty(N, np.float32)
    mathcheck.mc_bm_radius_table(ctypes.c_uint32(0), ctypes.c_int64(N), _p(got))
    bad = np.nonzero(want.view(np.uint32) != got.view(np.uint32))[0]
    assert bad.size == 0, f"{bad.size} mismatches, first m={bad[:5]}"


def test_sincos_exhaustive(oracle, mathcheck):
    ws, wc = oracle.bm_sincos_table(0, N)
    gs = np.empty(N, np.float32)
    gc = np.empty(N, np.float32)
    mathcheck.mc_bm_sincos_table(ctypes.c_uint32(0), ctypes.c_int64(N), _p(gs), _p(gc))
    assert np.array_equal(ws.view(np.uint32), gs.view(np.uint32))
    assert np.array_equal(wc.view(np.uint32), gc.view(np.uint32))


def test_logf_random_and_special(oracle, mathcheck):
    rng = np.random.default_rng(0)
    x = rng.integers(0, 0x7f800000, size=1 << 22, dtype=np.uint32).view(np.float32)
    x = np.concatenate([x, np.array([0.0, 1.0, np.inf, -1.0, np.nan, 1e-45, 1.1754942e-38,
                                     1.0000001, 0.99999994, 3.4028235e38], np.float32)])
    want = oracle.logf_table(x)
    got = np.empty_like(x)
    mathcheck.mc_logf_table(_p(x), ctypes.c_int64(x.size), _p(got))
    both_nan = np.isnan(want) & np.isnan(got)
    assert np.array_equal(want.view(np.uint32)[~both_nan], got.view(np.uint32)[~both_nan])
