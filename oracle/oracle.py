"""ctypes wrapper of the CPU oracle (oracle/cwq_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / the reported CPU baseline.  The
product package never imports this module.  Parity vs the TF reference is
unpinned beyond the pins listed in cwq_oracle.c's header.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libcwq_oracle.so")

_lib = None


def build(force=False):
    src = os.path.join(HERE, "cwq_oracle.c")
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-C", REPO, "oracle/libcwq_oracle.so"],
                              stdout=subprocess.DEVNULL)
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        vp, i64, i32, f32, f64, ci = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_float, ctypes.c_double, ctypes.c_int)
        sig = {
            "cwqo_philox4x32_10": (None, [vp, vp, vp]),
            "cwqo_generate_key": (None, [i32, i32, vp, vp]),
            "cwqo_stateless_normal": (None, [i32, i32, i64, vp]),
            "cwqo_stateless_normal_sample": (None, [vp, vp, i64, i64, i32, vp]),
            "cwqo_bm_radius": (f32, [ctypes.c_uint32]),
            "cwqo_bm_radius_table": (None, [ctypes.c_uint32, i64, vp]),
            "cwqo_bm_sincos_table": (None, [ctypes.c_uint32, i64, vp, vp]),
            "cwqo_logf_table": (None, [vp, i64, vp]),
            "cwqo_log_normalization": (f32, [f32]),
            "cwqo_normal_log_prob": (f32, [f32, f32, f32]),
            "cwqo_eigen_rowsum": (f32, [vp, i64]),
            "cwqo_code_greedy_sample": (ci, [vp, vp, vp, vp, i64, ci, ci, i32, f32, vp, vp]),
            "cwqo_decode_greedy_sample": (ci, [vp, vp, vp, i64, ci, ci, i32, f32, vp]),
            "cwqo_code_greedy_sample_rows": (ci, [vp, vp, vp, vp, i64, ci, i32, f32, vp, vp, ci]),
            "cwqo_greedy_encode": (ci, [vp, vp, vp, vp, vp, i64, ci, ci, i32, f32, i64, vp, vp,
                                        ci]),
            "cwqo_greedy_decode": (ci, [vp, vp, vp, vp, i64, ci, ci, i32, f32, i64, vp, ci]),
            "cwqo_greedy_encode_lsig": (ci, [vp, vp, vp, vp, vp, i64, ci, ci, i32, f32, i64, vp,
                                             vp, vp, vp, ci]),
            "cwqo_greedy_encode_semvar": (ci, [vp, vp, vp, vp, vp, i64, ci, ci, i32, f32, i64,
                                               vp, vp, vp, vp, ci]),
            "cwqo_sem_num_variants": (ci, []),
            "cwqo_sem_rowsum": (f32, [vp, i64, ci]),
            "cwqo_eigen_plog": (f32, [f32, ci]),
            "cwqo_eigen_plog_table": (None, [vp, i64, ci, vp]),
            "cwqo_standardise": (None, [vp, vp, vp, vp, i64, vp, vp]),
            "cwqo_kl_normal_normal": (None, [vp, vp, vp, vp, i64, vp]),
            "cwqo_group_starts": (i64, [vp, i64, i64, f64, vp, i64]),
            "cwqo_destandardise": (None, [vp, vp, vp, i64, vp]),
            "cwqo_num_threads": (ci, []),
            "cwqo_importance_num_samples": (i64, [vp, vp, vp, vp, i64]),
            "cwqo_importance_plan": (None, [vp, vp, i64, vp]),
            "cwqo_importance_encode_block": (ci, [vp, vp, vp, vp, i64, i32, i64, vp, vp]),
            "cwqo_importance_decode_block": (None, [i64, vp, vp, i64, i32, vp]),
            "cwqo_importance_encode": (ci, [vp, vp, vp, vp, vp, i64, vp, i32, i64, vp, vp, ci]),
            "cwqo_quantize_quint16": (None, [vp, i64, f32, f32, vp]),
            "cwqo_dequantize_quint16": (None, [vp, i64, f32, f32, vp]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None and a.size else None


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1))


def philox(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().cwqo_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def generate_key(s0, s1):
    key = np.zeros(2, dtype=np.uint32)
    ctr = np.zeros(4, dtype=np.uint32)
    lib().cwqo_generate_key(int(s0), int(s1), _p(key), _p(ctr))
    return key, ctr


def stateless_normal(s0, s1, n):
    out = np.empty(int(n), dtype=np.float32)
    lib().cwqo_stateless_normal(int(s0), int(s1), int(n), _p(out))
    return out


def stateless_normal_sample(loc, scale, num_samples, seed):
    l, s = _f32(loc), _f32(scale)
    out = np.empty(int(num_samples) * l.size, dtype=np.float32)
    lib().cwqo_stateless_normal_sample(_p(l), _p(s), l.size, int(num_samples), int(seed),
                                       _p(out))
    return out.reshape(int(num_samples), l.size)


def bm_radius_table(m0, count):
    out = np.empty(int(count), dtype=np.float32)
    lib().cwqo_bm_radius_table(int(m0), int(count), _p(out))
    return out


def bm_sincos_table(m0, count):
    s = np.empty(int(count), dtype=np.float32)
    c = np.empty(int(count), dtype=np.float32)
    lib().cwqo_bm_sincos_table(int(m0), int(count), _p(s), _p(c))
    return s, c


def logf_table(x):
    x = _f32(x)
    out = np.empty_like(x)
    lib().cwqo_logf_table(_p(x), x.size, _p(out))
    return out


def eigen_rowsum(x):
    x = _f32(x)
    return float(lib().cwqo_eigen_rowsum(_p(x), x.size))


def code_greedy_sample(t_loc, t_scale, p_loc, p_scale, n_bits_per_step, n_steps, seed, rho=1.):
    tl, ts, pl, ps = map(_f32, (t_loc, t_scale, p_loc, p_scale))
    idx = np.zeros(int(n_steps), dtype=np.int32)
    sample = np.zeros(tl.size, dtype=np.float32)
    rc = lib().cwqo_code_greedy_sample(_p(tl), _p(ts), _p(pl), _p(ps), tl.size,
                                       int(n_bits_per_step), int(n_steps), int(seed),
                                       float(rho), _p(idx), _p(sample))
    assert rc == 0, rc
    return idx, sample


def code_greedy_sample_rows(t_loc, t_scale, p_loc, p_scale, n_bits, seed, rho=1., nthreads=0):
    """code_greedy_sample for one block and one step with the candidate rows
    split over OpenMP threads (same argmax as the serial scan): blocks too large
    for one core."""
    tl, ts, pl, ps = map(_f32, (t_loc, t_scale, p_loc, p_scale))
    idx = np.zeros(1, dtype=np.int32)
    sample = np.zeros(tl.size, dtype=np.float32)
    rc = lib().cwqo_code_greedy_sample_rows(_p(tl), _p(ts), _p(pl), _p(ps), tl.size, int(n_bits),
                                            int(seed), float(rho), _p(idx), _p(sample),
                                            int(nthreads))
    assert rc == 0, rc
    return idx, sample


def decode_greedy_sample(idx, p_loc, p_scale, n_bits_per_step, n_steps, seed, rho=1.):
    pl, ps = _f32(p_loc), _f32(p_scale)
    ix = np.ascontiguousarray(np.asarray(idx, dtype=np.int32).reshape(-1))
    out = np.zeros(pl.size, dtype=np.float32)
    rc = lib().cwqo_decode_greedy_sample(_p(ix), _p(pl), _p(ps), pl.size, int(n_bits_per_step),
                                         int(n_steps), int(seed), float(rho), _p(out))
    assert rc == 0, rc
    return out


def greedy_encode(t_loc, t_scale, p_loc, p_scale, block_off, n_bits_per_step, n_steps, seed,
                  rho=1., block_id_base=0, nthreads=0):
    tl, ts, pl, ps = map(_f32, (t_loc, t_scale, p_loc, p_scale))
    off = np.ascontiguousarray(np.asarray(block_off, dtype=np.int64))
    nb = off.size - 1
    idx = np.zeros(nb * int(n_steps), dtype=np.int32)
    sample = np.zeros(tl.size, dtype=np.float32)
    rc = lib().cwqo_greedy_encode(_p(tl), _p(ts), _p(pl), _p(ps), _p(off), nb,
                                  int(n_bits_per_step), int(n_steps), int(seed), float(rho),
                                  int(block_id_base), _p(idx), _p(sample), int(nthreads))
    assert rc == 0, rc
    return idx.reshape(nb, int(n_steps)), sample


def greedy_encode_lsig(t_loc, t_scale, p_loc, p_scale, block_off, n_bits_per_step, n_steps,
                       seed, log_scale, rho=1., block_id_base=0, nthreads=0, gaps=False):
    """greedy_encode with log(sigma_j) supplied per dim (the per-dim normaliser
    0.9189385f + log sigma_j of SURVEY.md A.5; None = logf): normaliser
    sensitivity only.  gaps=True also returns the best - second-best row value
    of every step (float64 [nb, n_steps])."""
    tl, ts, pl, ps = map(_f32, (t_loc, t_scale, p_loc, p_scale))
    ls = None if log_scale is None else _f32(log_scale)
    off = np.ascontiguousarray(np.asarray(block_off, dtype=np.int64))
    nb = off.size - 1
    idx = np.zeros(nb * int(n_steps), dtype=np.int32)
    sample = np.zeros(tl.size, dtype=np.float32)
    gap = np.zeros(nb * int(n_steps), dtype=np.float64) if gaps else None
    rc = lib().cwqo_greedy_encode_lsig(_p(tl), _p(ts), _p(pl), _p(ps), _p(off), nb,
                                       int(n_bits_per_step), int(n_steps), int(seed), float(rho),
                                       int(block_id_base), _p(ls), _p(idx), _p(sample), _p(gap),
                                       int(nthreads))
    assert rc == 0, rc
    if gaps:
        return idx.reshape(nb, int(n_steps)), sample, gap.reshape(nb, int(n_steps))
    return idx.reshape(nb, int(n_steps)), sample


SEM_FORMS = ("tfp07", "tfp08")
SEM_ORDERS = ("avx8", "sse4", "avx8x2", "avx512", "seq", "tree")
SEM_RNG = ("ulp_hash", "ulp_up", "ulp_down", "v1_f32")


def sem_variant_names():
    """Names of the per-candidate semantics variants, in the oracle's order
    v = form * len(SEM_ORDERS) + order, then the RNG-transcendental variants
    (declared form and order on other normals, cwq_oracle.c SEM_NRNG);
    v = 0 ('tfp07/avx8') is declared."""
    return [f + "/" + o for f in SEM_FORMS for o in SEM_ORDERS] + ["rng/" + r for r in SEM_RNG]


def sem_rowsum(x, order):
    a = _f32(x)
    return float(lib().cwqo_sem_rowsum(_p(a), a.size, int(order)))


def greedy_encode_semvar(t_loc, t_scale, p_loc, p_scale, block_off, n_bits_per_step, n_steps,
                         seed, rho=1., block_id_base=0, nthreads=0):
    """The declared encoder with every candidate row also scored under each
    per-candidate semantics variant (sem_variant_names()).  Returns
    (vidx int32 [nb, n_steps, V], sample [D] of the declared chain, gap float64
    [nb, n_steps] = declared best - second-best, dev float32 [nb, n_steps, V] =
    variant v's value of the declared best row minus the declared value).
    vidx[..., v] is the index variant v would emit at that step given the
    declared history."""
    tl, ts, pl, ps = map(_f32, (t_loc, t_scale, p_loc, p_scale))
    off = np.ascontiguousarray(np.asarray(block_off, dtype=np.int64))
    nb, ns = off.size - 1, int(n_steps)
    nv = lib().cwqo_sem_num_variants()
    vidx = np.zeros(nb * ns * nv, dtype=np.int32)
    sample = np.zeros(tl.size, dtype=np.float32)
    gap = np.zeros(nb * ns, dtype=np.float64)
    dev = np.zeros(nb * ns * nv, dtype=np.float32)
    rc = lib().cwqo_greedy_encode_semvar(_p(tl), _p(ts), _p(pl), _p(ps), _p(off), nb,
                                         int(n_bits_per_step), ns, int(seed), float(rho),
                                         int(block_id_base), _p(vidx), _p(sample), _p(gap),
                                         _p(dev), int(nthreads))
    assert rc == 0, rc
    return vidx.reshape(nb, ns, nv), sample, gap.reshape(nb, ns), dev.reshape(nb, ns, nv)


def eigen_plog(x, fma=False):
    """Eigen 3.3 plog<Packet8f> per lane ([ext] restatement, cwq_oracle.c)."""
    a = _f32(x)
    out = np.empty_like(a)
    lib().cwqo_eigen_plog_table(_p(a), a.size, 1 if fma else 0, _p(out))
    return out


def greedy_decode(idx, p_loc, p_scale, block_off, n_bits_per_step, n_steps, seed, rho=1.,
                  block_id_base=0, nthreads=0):
    pl, ps = _f32(p_loc), _f32(p_scale)
    off = np.ascontiguousarray(np.asarray(block_off, dtype=np.int64))
    ix = np.ascontiguousarray(np.asarray(idx, dtype=np.int32).reshape(-1))
    nb = off.size - 1
    out = np.zeros(pl.size, dtype=np.float32)
    rc = lib().cwqo_greedy_decode(_p(ix), _p(pl), _p(ps), _p(off), nb, int(n_bits_per_step),
                                  int(n_steps), int(seed), float(rho), int(block_id_base),
                                  _p(out), int(nthreads))
    assert rc == 0, rc
    return out


def standardise(q_loc, q_scale, p_loc, p_scale):
    ql, qs, pl, ps = map(_f32, (q_loc, q_scale, p_loc, p_scale))
    tl, ts = np.empty_like(ql), np.empty_like(ql)
    lib().cwqo_standardise(_p(ql), _p(qs), _p(pl), _p(ps), ql.size, _p(tl), _p(ts))
    return tl, ts


def kl_normal_normal(q_loc, q_scale, p_loc, p_scale):
    ql, qs, pl, ps = map(_f32, (q_loc, q_scale, p_loc, p_scale))
    out = np.empty_like(ql)
    lib().cwqo_kl_normal_normal(_p(ql), _p(qs), _p(pl), _p(ps), ql.size, _p(out))
    return out


def group_starts(kl, n_bits_per_group, size_threshold):
    k = _f32(kl)
    cap = k.size + 2
    st = np.empty(cap, dtype=np.int64)
    n = lib().cwqo_group_starts(_p(k), k.size, int(size_threshold),
                                float(n_bits_per_group * np.log(2) - 1), _p(st), cap)
    assert n > 0
    return [int(v) for v in st[:n]]


def destandardise(sample, p_loc, p_scale):
    s, pl, ps = map(_f32, (sample, p_loc, p_scale))
    out = np.empty_like(s)
    lib().cwqo_destandardise(_p(s), _p(pl), _p(ps), s.size, _p(out))
    return out


def code_grouped_greedy_sample(q_loc, q_scale, p_loc, p_scale, n_steps, n_bits_per_step, seed,
                               size_threshold, rho=1., nthreads=0):
    """Whole grouped pipeline (coded_greedy_sampler.py:170-296) on the CPU.

    Returns (sample [D], indices [G, n_steps], starts list).
    """
    tl, ts = standardise(q_loc, q_scale, p_loc, p_scale)
    kl = kl_normal_normal(q_loc, q_scale, p_loc, p_scale)
    starts = group_starts(kl, n_bits_per_step * n_steps, size_threshold)
    D = tl.size
    idx, samp = greedy_encode(tl, ts, np.zeros(D, np.float32), np.ones(D, np.float32), starts,
                              n_bits_per_step, n_steps, seed, rho, 0, nthreads)
    return destandardise(samp, p_loc, p_scale), idx, starts


# --------------------------------------------------------------------------
# importance sampler (code/coded_importance_sampler.py)
# --------------------------------------------------------------------------
def importance_num_samples(t_loc, t_scale, p_loc, p_scale):
    tl, ts, pl, ps = map(_f32, (t_loc, t_scale, p_loc, p_scale))
    return int(lib().cwqo_importance_num_samples(_p(tl), _p(ts), _p(pl), _p(ps), tl.size))


def importance_plan(kl, starts):
    k = _f32(kl)
    st = np.ascontiguousarray(np.asarray(starts, dtype=np.int64))
    out = np.zeros(max(st.size - 1, 1), dtype=np.int64)
    lib().cwqo_importance_plan(_p(k), _p(st), st.size - 1, _p(out))
    return out[:st.size - 1]


def importance_encode(t_loc, t_scale, p_loc, p_scale, block_off, n_samples, seed,
                      block_id_base=0, nthreads=0):
    tl, ts, pl, ps = map(_f32, (t_loc, t_scale, p_loc, p_scale))
    off = np.ascontiguousarray(np.asarray(block_off, dtype=np.int64))
    ns = np.ascontiguousarray(np.asarray(n_samples, dtype=np.int64))
    nb = off.size - 1
    idx = np.zeros(max(nb, 1), dtype=np.int64)
    sample = np.zeros(tl.size, dtype=np.float32)
    rc = lib().cwqo_importance_encode(_p(tl), _p(ts), _p(pl), _p(ps), _p(off), nb, _p(ns),
                                      int(seed), int(block_id_base), _p(idx), _p(sample),
                                      int(nthreads))
    assert rc == 0, rc
    return idx[:nb], sample


def importance_decode_block(index, p_loc, p_scale, seed):
    pl, ps = _f32(p_loc), _f32(p_scale)
    out = np.zeros(pl.size, dtype=np.float32)
    lib().cwqo_importance_decode_block(int(index), _p(pl), _p(ps), pl.size, int(seed), _p(out))
    return out


def quantize_quint16(x, mn=-30.0, mx=30.0):
    v = _f32(x)
    out = np.zeros(v.size, dtype=np.uint16)
    lib().cwqo_quantize_quint16(_p(v), v.size, float(mn), float(mx), _p(out))
    return out


def dequantize_quint16(q, mn=-30.0, mx=30.0):
    qq = np.ascontiguousarray(np.asarray(q, dtype=np.uint16))
    out = np.zeros(qq.size, dtype=np.float32)
    lib().cwqo_dequantize_quint16(_p(qq), qq.size, float(mn), float(mx), _p(out))
    return out


def importance_group_starts(kl, n_bits_per_group, max_group_size_bits):
    """coded_importance_sampler.py:178-203, transcribed (strict comparisons)."""
    kl = np.asarray(kl, np.float32)
    starts = [0]
    cur_size = 0
    cur_kl = 0
    n_nats = n_bits_per_group * np.log(2) - 1
    D = kl.size
    for idx in range(D):
        group_bits = np.log(cur_size + 1) / np.log(2)
        if group_bits > max_group_size_bits or cur_kl + kl[idx] > n_nats or idx == D - 1:
            starts.append(idx)
            cur_size = 1
            cur_kl = kl[idx]
        else:
            cur_kl += kl[idx]
            cur_size += 1
    return starts + [D]


def code_grouped_importance_sample(q_loc, q_scale, p_loc, p_scale, seed, n_bits_per_group,
                                   max_group_size_bits=4, dim_kl_bit_limit=12, nthreads=0):
    """Whole grouped importance pipeline (:112-274) on the CPU, with the same
    deterministic outlier draw as the product (stateless seed [seed-1, 42]).
    Returns (sample [D], indices (index+1) list, starts list, (outlier idx, quint16))."""
    ql, qs, pl, ps = map(_f32, (q_loc, q_scale, p_loc, p_scale))
    D = ql.size
    tl, ts = standardise(ql, qs, pl, ps)
    kl_bits = kl_normal_normal(ql, qs, pl, ps) / np.float32(np.log(2))
    keep = kl_bits <= dim_kl_bit_limit
    tl = np.where(keep, tl, np.float32(0)).astype(np.float32)
    ts = np.where(keep, ts, np.float32(1)).astype(np.float32)
    out_idx = np.nonzero(~keep)[0].astype(np.int64)
    s1 = int(np.int32(np.uint32((int(seed) - 1) & 0xFFFFFFFF)))
    target_samples = stateless_normal_sample(ql, qs, 1, s1).reshape(-1)
    out_q = quantize_quint16(target_samples[out_idx])
    zeros, ones = np.zeros(D, np.float32), np.ones(D, np.float32)
    kl_divs = kl_normal_normal(tl, ts, zeros, ones)
    starts = importance_group_starts(kl_divs, n_bits_per_group, max_group_size_bits)
    ns = importance_plan(kl_divs, starts)
    idx, samp = importance_encode(tl, ts, zeros, ones, starts, ns, seed, 0, nthreads)
    sample = np.where(keep, destandardise(samp, pl, ps), target_samples).astype(np.float32)
    return sample, [int(i) + 1 for i in idx], starts, (out_idx, out_q)


# --------------------------------------------------------------------------
# PLN latent plumbing (code/pln.py), numpy float32 -- each op is one IEEE
# operation, so numpy's results are the reference's float32 values
# --------------------------------------------------------------------------
def pln_posterior(lik_loc, lik_scale, prior_loc, prior_scale, eps=1e-12):
    """pln.py:165-185 in the reference's operation order."""
    ll, ls, pl, ps = map(lambda a: np.asarray(a, np.float32), (lik_loc, lik_scale, prior_loc,
                                                               prior_scale))
    e = np.float32(eps)
    lv = ls * ls
    pv = ps * ps
    lp = np.float32(1) / (lv + e)
    pp = np.float32(1) / (pv + e)
    cv = np.float32(1) / (lp + pp)
    cs = np.sqrt(cv)
    cl = ll * pp
    cl = cl + pl * lp
    cl = cl * cv
    return cl.astype(np.float32), cs.astype(np.float32)


def pln_permutations(seed, n1, n2):
    """pln.py:304-313: np.random.seed(seed); permutation(n1); permutation(n2)."""
    state = np.random.get_state()
    try:
        np.random.seed(seed)
        p1 = np.random.permutation(n1).astype("int32")
        p2 = np.random.permutation(n2).astype("int32")
    finally:
        np.random.set_state(state)
    return p1, p2


def nhwc_permute_flatten(x_nchw, perm):
    """tf.reshape(x_nhwc, [-1]) then tfp Permute.forward: y[i] = x[perm[i]]."""
    flat = np.ascontiguousarray(np.transpose(np.asarray(x_nchw, np.float32), (0, 2, 3, 1)))
    return flat.reshape(-1)[np.asarray(perm, np.int64)]


def unpermute_to_nchw(v, perm, shape_nchw):
    """Permute.inverse, reshape to NHWC, returned NCHW."""
    n, c, h, w = shape_nchw
    flat = np.empty(n * c * h * w, np.float32)
    flat[np.asarray(perm, np.int64)] = np.asarray(v, np.float32).reshape(-1)
    return np.ascontiguousarray(np.transpose(flat.reshape(n, h, w, c), (0, 3, 1, 2)))
