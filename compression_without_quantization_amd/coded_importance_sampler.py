"""Coded importance sampler -- code/coded_importance_sampler.py on the gfx950 kernels.

  code_importance_sample            (:29-79)
  decode_importance_sample          (:82-109)
  code_grouped_importance_sample    (:112-274)
  decode_grouped_importance_sample  (:277-363)

Candidate scoring runs in libcwq.so (cwq_importance_encode).  Host code keeps
only the reference's per-group bookkeeping: the sequential partition
(cwq_importance_group_starts), the per-group candidate count
ceil(exp(sum KL)) (cwq_importance_plan), Elias-delta strings and the
quint16 outlier packing.

Deliberate differences from the TF1 reference:
  * the reference draws the outlier dims' target sample with an unseeded
    `target.sample()` (:150, non-deterministic); here it
    is the stateless draw x = q_loc + q_scale * z, z ~ stateless_normal([D],
    seed=[seed - 1, 42]) (seed - 1 is never a group's seed), so encoding is
    reproducible;
  * decode_grouped_importance_sample does not append to the caller's list
    (:294 mutates it);
  * results are concrete values; `sess` is accepted and ignored.
"""
import ctypes
import functools

import numpy as np
import torch

from . import _lib
from .binary_io import (elias_delta_code, elias_delta_code_many, elias_delta_decode,
                        elias_delta_decode_many)
from .coded_greedy_sampler import _device_of, _f32, _is_float32, _like_input, _ptr

VERBOSE = True
USE_FUSED = True   # code_grouped_importance_sample in one native call (tests compare both paths)
QUANT_MIN, QUANT_MAX = -30.0, 30.0


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


@functools.lru_cache(maxsize=64)
def importance_group_size_threshold(max_group_size_bits):
    """Smallest s with np.log(s + 1) / np.log(2) > max_group_size_bits (:185-187)."""
    bits = max_group_size_bits
    s = max(int(2 ** bits) - 3, 0)
    while s > 0 and np.log(s + 1) / np.log(2) > bits:
        s -= 1
    while not (np.log(s + 1) / np.log(2) > bits):
        s += 1
    return s


def importance_group_starts(kl_divs, n_bits_per_group, max_group_size_bits=4):
    """coded_importance_sampler.py:164-203 -> group start list with D appended."""
    kl = np.ascontiguousarray(np.asarray(kl_divs, dtype=np.float32).reshape(-1))
    D = kl.size
    n_nats = n_bits_per_group * np.log(2) - 1
    cap = D + 2
    starts = np.empty(cap, dtype=np.int64)
    n = _lib.load().cwq_importance_group_starts(
        kl.ctypes.data if D else None, D, importance_group_size_threshold(max_group_size_bits),
        float(n_nats), starts.ctypes.data, cap)
    _lib.check(n, "cwq_importance_group_starts")
    return [int(v) for v in starts[:n]]


def num_samples_plan(kl_divs, starts):
    """:48-51 per group: int32(ceil(exp(reduce_sum(kl)))) (host bookkeeping)."""
    kl = np.ascontiguousarray(np.asarray(kl_divs, dtype=np.float32).reshape(-1))
    st = np.ascontiguousarray(np.asarray(starts, dtype=np.int64).reshape(-1))
    ng = st.size - 1
    out = np.empty(max(ng, 1), dtype=np.int64)
    _lib.check(_lib.load().cwq_importance_plan(kl.ctypes.data if kl.size else None,
                                               st.ctypes.data, ng, out.ctypes.data),
               "cwq_importance_plan")
    return out[:ng]


def _kl(dev, a_loc, a_scale, b_loc, b_scale):
    n = a_loc.numel()
    out = torch.empty(n, dtype=torch.float32, device=dev)
    _lib.check(_lib.load().cwq_kl_normal_normal(_ptr(a_loc), _ptr(a_scale), _ptr(b_loc),
                                                _ptr(b_scale), n, _ptr(out), _stream(dev)),
               "cwq_kl_normal_normal")
    return out


def importance_encode_blocks(t_loc, t_scale, p_loc, p_scale, block_off, n_samples, seed,
                             block_id_base=0, prune_mode=None):
    """cwq_importance_encode over CSR groups.  Returns (index int64 [nb], sample f32 [D]).
    ``prune_mode`` 2 (default) screens candidates, 0/1 score them all exactly
    (cwq_options); results never depend on it."""
    lib = _lib.load()
    dev = _device_of(t_loc, t_scale, p_loc, p_scale)
    tl, ts, pl, ps = (_f32(x, dev, w) for x, w in ((t_loc, "t_loc"), (t_scale, "t_scale"),
                                                   (p_loc, "p_loc"), (p_scale, "p_scale")))
    D = tl.numel()
    offs = torch.as_tensor(np.asarray(block_off, dtype=np.int64)).to(dev)
    nb = offs.numel() - 1
    ns = torch.as_tensor(np.asarray(n_samples, dtype=np.int64)).to(dev)
    idx = torch.empty(max(nb, 0), dtype=torch.int64, device=dev)
    sample = torch.empty(D, dtype=torch.float32, device=dev)
    need = int(lib.cwq_importance_workspace_size(nb, D))
    ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
    seed32 = int(np.int32(np.uint32(int(seed) & 0xFFFFFFFF)))
    with torch.cuda.device(dev):
        _lib.check(lib.cwq_importance_encode(
            _ptr(tl), _ptr(ts), _ptr(pl), _ptr(ps), offs.data_ptr(), _ptr(ns), nb, D, seed32,
            int(block_id_base), _ptr(idx), _ptr(sample), ws.data_ptr(), ws.numel(),
            _lib.options(prune_mode), _stream(dev)), "cwq_importance_encode")
    return idx, sample


def importance_decode_blocks(index, p_loc, p_scale, block_off, seed, block_id_base=0):
    """cwq_importance_decode over CSR groups.  Returns sample f32 [D]."""
    lib = _lib.load()
    dev = _device_of(index, p_loc, p_scale)
    pl, ps = _f32(p_loc, dev, "p_loc"), _f32(p_scale, dev, "p_scale")
    D = pl.numel()
    offs = torch.as_tensor(np.asarray(block_off, dtype=np.int64)).to(dev)
    nb = offs.numel() - 1
    ix = torch.as_tensor(np.asarray(index.cpu() if isinstance(index, torch.Tensor) else index,
                                    dtype=np.int64)).to(dev)
    out = torch.empty(D, dtype=torch.float32, device=dev)
    seed32 = int(np.int32(np.uint32(int(seed) & 0xFFFFFFFF)))
    with torch.cuda.device(dev):
        _lib.check(lib.cwq_importance_decode(_ptr(ix), _ptr(pl), _ptr(ps), offs.data_ptr(), nb,
                                             D, seed32, int(block_id_base), _ptr(out),
                                             _stream(dev)), "cwq_importance_decode")
    return out


# ---------------------------------------------------------------------------
# reference surface
# ---------------------------------------------------------------------------
def code_importance_sample(t_loc, t_scale, p_loc, p_scale, n_coding_bits, seed,
                           return_index_only=False):
    """:29-79.  Returns (best_sample [1, d], index + 1) or (best_sample, Elias code)."""
    dev = _device_of(t_loc, t_scale, p_loc, p_scale)
    tl, ts, pl, ps = (_f32(x, dev, "input") for x in (t_loc, t_scale, p_loc, p_scale))
    d = tl.numel()
    kl = _kl(dev, tl, ts, pl, ps).cpu().numpy()
    n = num_samples_plan(kl, [0, d])
    idx, sample = importance_encode_blocks(tl, ts, pl, ps, [0, d], n, seed)
    index = int(idx[0].item())
    best = _like_input(sample.reshape(1, d), t_loc)
    if return_index_only:
        return best, index + 1
    return best, elias_delta_code(index + 1)


def decode_importance_sample(sample_index, p_loc, p_scale, seed, use_index=False):
    """:82-109.  use_index: sample_index is index + 1 -> samples[-1:].  Otherwise
    sample_index is an Elias-delta string/bytes -> (samples[-1:], code_length,
    index, samples) with samples the index + 1 candidates."""
    from .misc import stateless_normal_sample
    dev = _device_of(p_loc, p_scale)
    pl, ps = _f32(p_loc, dev, "p_loc"), _f32(p_scale, dev, "p_scale")
    d = pl.numel()
    if use_index:
        index = int(sample_index) - 1
        row = importance_decode_blocks([index], pl, ps, [0, d], seed)
        return _like_input(row.reshape(1, d), p_loc)
    num, code_length = elias_delta_decode(sample_index)
    index = num - 1
    samples = stateless_normal_sample(pl, ps, index + 1, seed)
    return (_like_input(samples[-1:].reshape(1, d), p_loc), code_length, index,
            _like_input(samples.reshape(index + 1, d), p_loc))


def quantize_quint16(x, mn=QUANT_MIN, mx=QUANT_MAX):
    """tf.quantization.quantize(x, mn, mx, tf.quint16) (MIN_COMBINED, float32):
    uint16((clamp(x) - mn) * float32(65535 / (mx - mn)) + 0.5f).

    NaN (a NaN outlier draw) is coded as 0, the code of ``mn``: the value an
    x86 truncating conversion gives (cvttss2si returns the integer-indefinite
    0x80000000, whose low 16 bits are 0).  The reference's float -> quint16
    cast of NaN (:156) is unspecified; this build fixes it instead of leaving
    it to NumPy's undefined cast."""
    x = np.asarray(x, dtype=np.float32)
    scale = np.float32((65535.0 - 0.0) / (float(mx) - float(mn)))
    v = np.maximum(np.minimum(x, np.float32(mx)), np.float32(mn))
    t = (v - np.float32(mn)) * scale
    t = t + np.float32(0.5)
    t = np.where(np.isnan(t), np.float32(0.0), t)
    return t.astype(np.uint16)


def dequantize_quint16(q, mn=QUANT_MIN, mx=QUANT_MAX):
    """tf.quantization.dequantize(q, mn, mx) for quint16 (MIN_COMBINED, float32)."""
    sf = np.float32((np.float32(mx) - np.float32(mn)) / np.float32(65535.0))
    return (np.asarray(q, dtype=np.uint16).astype(np.float32) * sf + np.float32(mn)).astype(
        np.float32)


def _outlier_target_draw(dev, q_loc, q_scale, seed):
    from .misc import stateless_normal_sample
    s = int(np.int32(np.uint32((int(seed) - 1) & 0xFFFFFFFF)))
    return stateless_normal_sample(q_loc, q_scale, 1, s).reshape(-1)


def code_grouped_importance_sample(sess, target, proposal, seed, n_bits_per_group,
                                   max_group_size_bits=4, dim_kl_bit_limit=12,
                                   return_group_indices_only=False, return_indices=False,
                                   return_indices_only=False, *, prune_mode=None,
                                   eval_ms_out=None):
    """:112-274.  Returns (sample np.float32 [D], bitcode str | indices,
    group_start_indices np.ndarray, outlier_extras (indices int64, quint16)).
    ``prune_mode`` (keyword only, not in the reference): cwq_options.prune_mode
    of the encoder; results never depend on it.  ``eval_ms_out`` (keyword
    only): a ctypes.c_float the fused call writes its candidate-scoring
    launches' milliseconds to (bench.py's kernel timer)."""
    if not _is_float32(target.loc) or not _is_float32(target.scale):
        raise Exception("Target datatype must be float32!")
    if not _is_float32(proposal.loc) or not _is_float32(proposal.scale):
        raise Exception("Proposal datatype must be float32!")
    dev = _device_of(target.loc, target.scale, proposal.loc, proposal.scale)
    with torch.cuda.device(dev):
        return _code_grouped_importance_on(dev, target, proposal, seed, n_bits_per_group,
                                           max_group_size_bits, dim_kl_bit_limit,
                                           return_group_indices_only, return_indices,
                                           return_indices_only, prune_mode, eval_ms_out)


def _code_grouped_importance_on(dev, target, proposal, seed, n_bits_per_group,
                                max_group_size_bits, dim_kl_bit_limit, return_group_indices_only,
                                return_indices, return_indices_only, prune_mode,
                                eval_ms_out=None):
    lib = _lib.load()
    q_loc, q_scale = _f32(target.loc, dev, "target.loc"), _f32(target.scale, dev, "target.scale")
    p_loc, p_scale = _f32(proposal.loc, dev, "proposal.loc"), _f32(proposal.scale, dev,
                                                                   "proposal.scale")
    D = p_loc.numel()
    if USE_FUSED and not (return_group_indices_only or return_indices_only):
        return _code_grouped_fused(lib, dev, q_loc, q_scale, p_loc, p_scale, D, seed,
                                   n_bits_per_group, max_group_size_bits, dim_kl_bit_limit,
                                   return_indices, prune_mode, eval_ms_out)
    zeros = torch.zeros(D, dtype=torch.float32, device=dev)
    ones = torch.ones(D, dtype=torch.float32, device=dev)
    # :137-138 standardise
    t_loc = torch.empty(D, dtype=torch.float32, device=dev)
    t_scale = torch.empty(D, dtype=torch.float32, device=dev)
    _lib.check(lib.cwq_standardise(_ptr(q_loc), _ptr(q_scale), _ptr(p_loc), _ptr(p_scale), D,
                                   _ptr(t_loc), _ptr(t_scale), _stream(dev)), "cwq_standardise")
    # :142 kl_bits = KL(target || proposal) / ln 2 (float32)
    kl_bits = _kl(dev, q_loc, q_scale, p_loc, p_scale).cpu().numpy() / np.float32(np.log(2))
    keep = kl_bits <= dim_kl_bit_limit
    keep_d = torch.from_numpy(keep).to(dev)
    t_loc = torch.where(keep_d, t_loc, zeros)                      # :144
    t_scale = torch.where(keep_d, t_scale, ones)                   # :145
    outlier_indices = np.nonzero(~keep)[0].astype(np.int64)       # :148
    target_samples = _outlier_target_draw(dev, q_loc, q_scale, seed)  # :150 (see docstring)
    outlier_samples = quantize_quint16(
        target_samples.cpu().numpy()[outlier_indices])           # :153-156
    outlier_extras = (outlier_indices, outlier_samples)
    # :160-163 KL of the standardised target vs N(0, 1)
    kl_divs = _kl(dev, t_loc, t_scale, zeros, ones).cpu().numpy()
    if VERBOSE:
        total_kl_bits = np.sum(kl_divs) / np.log(2)
        print("Total KL to split up: {:.2f} bits, "
              "maximum bits per group: {}, "
              "estimated number of groups: {},"
              "coding {} dimensions".format(total_kl_bits, n_bits_per_group,
                                            total_kl_bits // n_bits_per_group + 1, D))
    starts = importance_group_starts(kl_divs, n_bits_per_group, max_group_size_bits)
    group_start_indices = np.array(starts)
    if return_group_indices_only:
        return group_start_indices, _group_kls(kl_divs, starts)
    n_samples = num_samples_plan(kl_divs, starts)
    idx, sample = importance_encode_blocks(t_loc, t_scale, zeros, ones, starts, n_samples, seed,
                                           prune_mode=prune_mode)
    indices = tuple((idx.cpu().numpy() + 1).tolist())
    if return_indices_only:
        return indices
    out = torch.empty(D, dtype=torch.float32, device=dev)         # :265 rescale
    _lib.check(lib.cwq_destandardise(_ptr(sample), _ptr(p_loc), _ptr(p_scale), D, _ptr(out),
                                     _stream(dev)), "cwq_destandardise")
    sample_h = np.where(keep, out.cpu().numpy(), target_samples.cpu().numpy())  # :267
    sample_h = sample_h.astype(np.float32)
    if return_indices:
        return sample_h, indices, group_start_indices, outlier_extras
    bitcode = elias_delta_code_many(indices)
    return sample_h, bitcode, group_start_indices, outlier_extras


def _code_grouped_fused(lib, dev, q_loc, q_scale, p_loc, p_scale, D, seed, n_bits_per_group,
                        max_group_size_bits, dim_kl_bit_limit, return_indices, prune_mode=None,
                        eval_ms_out=None):
    """The common path of code_grouped_importance_sample in one native call
    (cwq_code_grouped_importance); same results as the step-by-step path."""
    need = int(lib.cwq_code_grouped_importance_workspace_size(D))
    ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
    sample_h = np.empty(max(D, 1), dtype=np.float32)
    index_h = np.empty(D + 2, dtype=np.int64)
    starts_h = np.empty(D + 2, dtype=np.int64)
    out_i = np.empty(max(D, 1), dtype=np.int64)
    out_v = np.empty(max(D, 1), dtype=np.float32)
    n_out = np.zeros(1, dtype=np.int64)
    kl_sum = ctypes.c_double(0.0)
    seed32 = int(np.int32(np.uint32(int(seed) & 0xFFFFFFFF)))
    G = _lib.check(lib.cwq_code_grouped_importance(
        _ptr(q_loc), _ptr(q_scale), _ptr(p_loc), _ptr(p_scale), D, seed32,
        float(np.float32(dim_kl_bit_limit)), importance_group_size_threshold(max_group_size_bits),
        float(n_bits_per_group * np.log(2) - 1), sample_h.ctypes.data, index_h.ctypes.data,
        starts_h.ctypes.data, starts_h.size, out_i.ctypes.data, out_v.ctypes.data,
        n_out.ctypes.data, ctypes.byref(kl_sum) if VERBOSE else None, ws.data_ptr(), ws.numel(),
        _lib.options(prune_mode, eval_ms_out=eval_ms_out), _stream(dev)),
        "cwq_code_grouped_importance")
    if VERBOSE:
        total_kl_bits = kl_sum.value / np.log(2)
        print("Total KL to split up: {:.2f} bits, "
              "maximum bits per group: {}, "
              "estimated number of groups: {},"
              "coding {} dimensions".format(total_kl_bits, n_bits_per_group,
                                            total_kl_bits // n_bits_per_group + 1, D))
    # views of this call's buffers; the indices + 1 coded straight from the array
    no = int(n_out[0])
    outlier_extras = (out_i[:no], quantize_quint16(out_v[:no]))
    group_start_indices = starts_h[:G + 1]
    vals = index_h[:G] + 1
    sample_h = sample_h[:D]
    if return_indices:
        return sample_h, tuple(vals.tolist()), group_start_indices, outlier_extras
    return sample_h, elias_delta_code_many(vals), group_start_indices, outlier_extras


def code_grouped_importance_sample_batch(sess, targets, proposals, seeds, n_bits_per_group,
                                         max_group_size_bits=4, dim_kl_bit_limit=12,
                                         return_indices=False, *, prune_mode=None,
                                         eval_ms_out=None):
    """code_grouped_importance_sample (coded_importance_sampler.py:112-274) for a
    batch of independent items (the level-2 latents of a dataset's images,
    pln.py:350-359) in one native call (cwq_code_grouped_importance_batch): one
    preparation launch and one encode launch over every item's groups.

    ``targets`` / ``proposals``: sequences of distributions (``.loc`` /
    ``.scale``), item i coded with seed ``seeds[i]`` (an int: the same seed for
    every item).  Returns a list with one (sample, bitcode | indices,
    group_start_indices, outlier_extras) per item, each equal to
    code_grouped_importance_sample on that item alone.  Not in the reference
    (an extension for throughput)."""
    lib = _lib.load()
    targets, proposals = list(targets), list(proposals)
    if len(targets) != len(proposals):
        raise ValueError("targets and proposals must have the same length")
    n_items = len(targets)
    if n_items == 0:
        return []
    if np.ndim(seeds) == 0:
        seeds = [int(seeds)] * n_items
    seeds = [int(x) for x in seeds]
    if len(seeds) != n_items:
        raise ValueError("one seed per item")
    seeds32 = np.array([int(np.int32(np.uint32(s & 0xFFFFFFFF))) for s in seeds], dtype=np.int32)
    raw = ([t.loc for t in targets], [t.scale for t in targets], [p.loc for p in proposals],
           [p.scale for p in proposals])
    f32 = torch.float32
    # the common case (float32 CUDA tensors on one device): the checks and the
    # concatenation without per-array wrapper calls (24 items: ~0.3 ms less)
    fast = all(type(a) is torch.Tensor and a.dtype is f32 and a.is_cuda for c in raw for a in c)
    if fast:
        dev = raw[0][0].device
        fast = all(a.device == dev for c in raw for a in c)
    if not fast:
        for t, p in zip(targets, proposals):
            if not _is_float32(t.loc) or not _is_float32(t.scale):
                raise Exception("Target datatype must be float32!")   # :126-129
            if not _is_float32(p.loc) or not _is_float32(p.scale):
                raise Exception("Proposal datatype must be float32!")
        dev = _device_of(*[a for c in raw for a in c])
    with torch.cuda.device(dev):
        cols = raw if fast else [[_f32(a, dev, n) for a in c]
                                 for c, n in zip(raw, ("target.loc", "target.scale",
                                                       "proposal.loc", "proposal.scale"))]
        sz = [a.numel() for a in cols[0]]
        if any([a.numel() for a in c] != sz for c in cols[1:]):
            raise ValueError("target and proposal of an item must have the same size")
        sizes = np.array(sz, dtype=np.int64)
        # the four concatenated inputs as four quarters of one buffer (one cat;
        # along dim 0 of equal trailing shapes it is the concatenation of the
        # flattened arrays, 1-D latents always; else each array flattened first,
        # which cost 65 us for I2's 96 arrays)
        item_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        D = int(item_off[-1])
        flat = [a for c in cols for a in c]
        try:
            big = torch.cat(flat).reshape(-1)
        except RuntimeError:
            big = None
        if big is None or big.numel() != 4 * D:
            big = torch.cat([a.reshape(-1) for a in flat])
        cat = [big[k * D:(k + 1) * D] for k in range(4)]
        need = int(lib.cwq_code_grouped_importance_batch_workspace_size(D, n_items))
        ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        sample_h = np.empty(max(D, 1), dtype=np.float32)
        index_h = np.empty(D + n_items, dtype=np.int64)
        starts_h = np.empty(D + 2 * n_items, dtype=np.int64)
        n_starts = np.zeros(n_items, dtype=np.int64)
        out_i = np.empty(max(D, 1), dtype=np.int64)
        out_v = np.zeros(max(D, 1), dtype=np.float32)  # quantised whole below
        n_out = np.zeros(n_items, dtype=np.int64)
        kl_sum = np.zeros(n_items, dtype=np.float64)
        _lib.check(lib.cwq_code_grouped_importance_batch(
            n_items, item_off.ctypes.data, _ptr(cat[0]), _ptr(cat[1]), _ptr(cat[2]), _ptr(cat[3]),
            seeds32.ctypes.data, float(np.float32(dim_kl_bit_limit)),
            importance_group_size_threshold(max_group_size_bits),
            float(n_bits_per_group * np.log(2) - 1), sample_h.ctypes.data, index_h.ctypes.data,
            starts_h.ctypes.data, starts_h.size, n_starts.ctypes.data, out_i.ctypes.data,
            out_v.ctypes.data, n_out.ctypes.data, kl_sum.ctypes.data, ws.data_ptr(), ws.numel(),
            _lib.options(prune_mode, eval_ms_out=eval_ms_out), _stream(dev)),
            "cwq_code_grouped_importance_batch")
    # every item's index + 1 values, outlier codes and bit strings in one pass
    # each (one native Elias-delta call, one quint16 pass over the outliers
    # only; per-item calls cost ~20 us apiece), then split per item.  The
    # per-item arrays are views of this call's buffers (disjoint slices).
    ns_all = n_starts.astype(np.int64)
    G = np.maximum(ns_all - 1, 0)
    goff = np.concatenate([[0], np.cumsum(G)])
    # item i's indices sit at index_h[item_off[i] + i + g], g < G_i
    src = np.arange(goff[-1], dtype=np.int64) + np.repeat(
        item_off[:-1] + np.arange(n_items, dtype=np.int64) - goff[:-1], G)
    vals = index_h[src] + 1
    # item i's outliers sit at out_i / out_v[item_off[i] : item_off[i] + n_out[i]]
    ooff = np.concatenate([[0], np.cumsum(n_out)])
    osrc = np.arange(ooff[-1], dtype=np.int64) + np.repeat(item_off[:-1] - ooff[:-1], n_out)
    o_idx = out_i[osrc]
    o_q = quantize_quint16(out_v[osrc])
    if return_indices:
        vals_l = vals.tolist()
    else:
        codes = elias_delta_code_many(vals)
        if vals.size:  # code lengths: 2 floor(log2(n + 1)) + n + 1, n = floor(log2 x)
            nb_ = np.frexp(vals)[1] - 1
            coff = np.concatenate([[0], np.cumsum(_ELIAS_LEN[nb_])])[goff]
        else:
            coff = np.zeros(n_items + 1, np.int64)
    res = []
    for i in range(n_items):
        a, b = int(item_off[i]), int(item_off[i + 1])
        if VERBOSE and b > a:
            total_kl_bits = kl_sum[i] / np.log(2)
            print("Total KL to split up: {:.2f} bits, "
                  "maximum bits per group: {}, "
                  "estimated number of groups: {},"
                  "coding {} dimensions".format(total_kl_bits, n_bits_per_group,
                                                total_kl_bits // n_bits_per_group + 1, b - a))
        o0, o1 = int(ooff[i]), int(ooff[i + 1])
        gs = starts_h[a + 2 * i:a + 2 * i + int(ns_all[i])]
        code = (tuple(vals_l[goff[i]:goff[i + 1]]) if return_indices
                else codes[coff[i]:coff[i + 1]])
        res.append((sample_h[a:b], code, gs, (o_idx[o0:o1], o_q[o0:o1])))
    return res


# Elias-delta code length by n = floor(log2 x): n + 2 floor(log2(n + 1)) + 1
_ELIAS_LEN = np.array([n + 2 * (int(n + 1).bit_length() - 1) + 1 for n in range(64)], np.int64)


def _group_kls(kl_divs, starts):
    """The reference's group_kls list (:192): the running group KL in bits at
    every boundary (print-only in the coder)."""
    out = []
    cur = np.float32(0)
    for a, b in zip(starts[:-1], starts[1:]):
        out.append(cur / np.log(2))
        cur = np.float32(0)
        for v in np.asarray(kl_divs, np.float32)[a:b]:
            cur = np.float32(cur + v)
    return out


def decode_grouped_importance_sample(sess, bitcode, group_start_indices, proposal,
                                     n_bits_per_group, seed, outlier_indices, outlier_samples,
                                     use_indices=False):
    """:277-363.  group_start_indices WITHOUT the trailing D (the reference
    appends it, :294).  Returns np.float32 [D]."""
    if not _is_float32(proposal.loc) or not _is_float32(proposal.scale):
        raise Exception("Proposal datatype must be float32!")
    lib = _lib.load()
    dev = _device_of(proposal.loc, proposal.scale)
    p_loc, p_scale = _f32(proposal.loc, dev, "proposal.loc"), _f32(proposal.scale, dev,
                                                                   "proposal.scale")
    D = p_loc.numel()
    starts = [int(s) for s in np.asarray(group_start_indices).reshape(-1)] + [D]
    G = len(starts) - 1
    if use_indices:
        index = [int(bitcode[i]) - 1 for i in range(G)]
    else:
        nums, _ = elias_delta_decode_many(bitcode, G)               # :325-336
        index = [int(v) - 1 for v in nums]
    zeros = torch.zeros(D, dtype=torch.float32, device=dev)
    ones = torch.ones(D, dtype=torch.float32, device=dev)
    sample = importance_decode_blocks(index, zeros, ones, starts, seed)
    out = torch.empty(D, dtype=torch.float32, device=dev)          # :347 rescale
    _lib.check(lib.cwq_destandardise(_ptr(sample), _ptr(p_loc), _ptr(p_scale), D, _ptr(out),
                                     _stream(dev)), "cwq_destandardise")
    sample_h = out.cpu().numpy()
    # :351-361 dequantise outliers and put them back where the update is non-zero
    deq = dequantize_quint16(outlier_samples)
    updates = np.zeros(D, dtype=np.float32)
    updates[np.asarray(outlier_indices, dtype=np.int64).reshape(-1)] = deq
    return np.where(updates == 0, sample_h, updates).astype(np.float32)
