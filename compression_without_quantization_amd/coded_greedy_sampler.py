"""Greedy coded sampler -- the reference's API on the gfx950 kernels.

Mirrors code/coded_greedy_sampler.py of the reference function for function:

  code_greedy_sample            (:29-89)
  decode_greedy_sample          (:93-167)
  code_grouped_greedy_sample    (:170-296)
  decode_grouped_greedy_sample  (:299-364)

plus the batched block API the north star asks for:

  encode(prior_loc, prior_scale, post_loc, post_scale, seed, kl_bits)
  decode(indices_or_bitcode, prior_loc, prior_scale, seed, kl_bits)
  encode_blocks / decode_blocks   (CSR or uniform blocks, explicit n_steps)

Differences from the TF1 reference (deliberate, documented in DESIGN.md):
  * functions return concrete values instead of graph tensors; ``sess`` is
    accepted and ignored;
  * decode_grouped_greedy_sample does not append to the caller's
    ``group_start_indices`` list (the reference mutates it, :323); the decoded
    groups are the same;
  * ``adaptive``, ``backfitting_steps`` and ``use_log_prob`` are accepted and
    ignored, exactly as in the reference.

All arithmetic runs in libcwq.so; nothing here computes samples on the CPU.
"""
import array
import concurrent.futures
import ctypes
import functools
import threading
import warnings
import weakref
import time

import numpy as np
import torch

from . import _lib
from .binary_io import bitcode_to_indices, indices_to_bitcode

VERBOSE = True


# ---------------------------------------------------------------------------
# tensor plumbing
# ---------------------------------------------------------------------------
def _device_of(*xs):
    for x in xs:
        if isinstance(x, torch.Tensor) and x.is_cuda:
            return x.device
    if not torch.cuda.is_available():
        raise RuntimeError("compression_without_quantization_amd needs a ROCm GPU "
                           "(torch.cuda.is_available() is False); there is no CPU path")
    return torch.device("cuda", torch.cuda.current_device())


def _is_float32(x):
    if isinstance(x, torch.Tensor):
        return x.dtype == torch.float32
    return np.asarray(x).dtype == np.float32


def _f32(x, device, what):
    if isinstance(x, torch.Tensor):
        if x.device == device and x.dtype == torch.float32 and x.is_contiguous():
            return x.view(-1)  # the common case, without three no-op torch calls
        t = x
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(x)))
    if t.dtype != torch.float32:
        raise TypeError(f"{what} must be float32, got {t.dtype}")
    return t.to(device=device).contiguous().reshape(-1)


def _ptr(t):
    return t.data_ptr() if t is not None and t.numel() > 0 else None


def _like_input(t, ref):
    """Return ``t`` (a cuda tensor) as the caller's array type."""
    if isinstance(ref, torch.Tensor):
        return t
    return t.cpu().numpy()


class Normal:
    """Minimal stand-in for tfd.Normal: anything with .loc/.scale/.dtype works."""

    def __init__(self, loc, scale):
        self.loc = loc
        self.scale = scale

    @property
    def dtype(self):
        return self.loc.dtype


# ---------------------------------------------------------------------------
# batched block API (C ABI: cwq_greedy_encode[_uniform], cwq_greedy_decode[_uniform])
# ---------------------------------------------------------------------------
def encode_workspace_bytes(nb, total_dims, block_dim=None, max_block_dim=None):
    """Workspace bytes of encode_blocks: CSR blocks (nb, total_dims, none
    longer than ``max_block_dim``, default total_dims), or uniform blocks of
    ``block_dim`` (cwq_greedy_encode[_uniform]_workspace_size)."""
    lib = _lib.load()
    if block_dim is not None:
        return int(lib.cwq_greedy_encode_uniform_workspace_size(int(nb), int(block_dim)))
    mbd = int(total_dims if max_block_dim is None else max_block_dim)
    return int(lib.cwq_greedy_encode_workspace_size(int(nb), int(total_dims), mbd))


def encode_blocks(t_loc, t_scale, p_loc, p_scale, n_bits_per_step, n_steps, seed, rho=1.,
                  block_dim=None, block_off=None, max_block_dim=None, block_id_base=0,
                  out_idx=None, out_sample=None, workspace=None, prune_mode=None,
                  eval_events=None):
    """code_greedy_sample over many blocks at once.

    Blocks are either uniform (``block_dim``) or CSR (``block_off``, nb+1
    offsets).  Block g is coded with seed ``seed + block_id_base + g``
    (coded_greedy_sampler.py:282).  Returns (idx int32 [nb, n_steps],
    sample f32 [D]) as cuda tensors.  ``prune_mode`` (0/1/2, default 2) and
    ``eval_events`` ((start, stop) hipEvent_t handles) are this call's
    cwq_options (include/cwq.h); results never depend on the mode.
    """
    lib = _lib.load()
    dev = _device_of(t_loc, t_scale, p_loc, p_scale)
    tl = _f32(t_loc, dev, "t_loc")
    ts = _f32(t_scale, dev, "t_scale")
    pl = _f32(p_loc, dev, "p_loc")
    ps = _f32(p_scale, dev, "p_scale")
    D = tl.numel()
    if not (ts.numel() == pl.numel() == ps.numel() == D):
        raise ValueError("t_loc, t_scale, p_loc, p_scale must have the same size")
    if (block_dim is None) == (block_off is None):
        raise ValueError("give exactly one of block_dim / block_off")
    if block_dim is not None:
        block_dim = int(block_dim)
        if block_dim < 0 or (block_dim == 0 and D != 0) or (block_dim and D % block_dim):
            raise ValueError(f"D={D} is not a multiple of block_dim={block_dim}")
        nb = D // block_dim if block_dim else 0
        offs = None
    else:
        offs_h = np.asarray(block_off.cpu() if isinstance(block_off, torch.Tensor)
                            else block_off, dtype=np.int64).reshape(-1)
        nb = offs_h.size - 1
        if nb < 0 or offs_h[0] != 0 or offs_h[-1] != D or (np.diff(offs_h) < 0).any():
            raise ValueError("block_off must be non-decreasing from 0 to D")
        if max_block_dim is None:
            max_block_dim = int(np.diff(offs_h).max()) if nb > 0 else 0
        offs = torch.from_numpy(offs_h).to(dev)
    n_steps = int(n_steps)
    if out_idx is None:
        out_idx = torch.empty((nb, n_steps), dtype=torch.int32, device=dev)
    if out_sample is None:
        out_sample = torch.empty(D, dtype=torch.float32, device=dev)
    need = encode_workspace_bytes(nb, D, block_dim if offs is None else None,
                                  None if offs is None else max_block_dim)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
    opts = _lib.options(prune_mode, eval_events)
    seed32 = int(np.int32(np.uint32(int(seed) & 0xFFFFFFFF)))
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        if offs is None:
            rc = lib.cwq_greedy_encode_uniform(
                _ptr(tl), _ptr(ts), _ptr(pl), _ptr(ps), nb, block_dim, int(n_bits_per_step),
                n_steps, seed32, float(rho), int(block_id_base), _ptr(out_idx),
                _ptr(out_sample), workspace.data_ptr(), workspace.numel(), opts, stream)
        else:
            rc = lib.cwq_greedy_encode(
                _ptr(tl), _ptr(ts), _ptr(pl), _ptr(ps), offs.data_ptr(), nb, D,
                int(max_block_dim), int(n_bits_per_step), n_steps, seed32, float(rho),
                int(block_id_base), _ptr(out_idx), _ptr(out_sample), workspace.data_ptr(),
                workspace.numel(), opts, stream)
    _lib.check(rc, "cwq_greedy_encode")
    return out_idx, out_sample


def decode_blocks(idx, p_loc, p_scale, n_bits_per_step, n_steps, seed, rho=1.,
                  block_dim=None, block_off=None, block_id_base=0, out_sample=None):
    """decode_greedy_sample over many blocks (inverse of encode_blocks)."""
    lib = _lib.load()
    dev = _device_of(idx, p_loc, p_scale)
    pl = _f32(p_loc, dev, "p_loc")
    ps = _f32(p_scale, dev, "p_scale")
    D = pl.numel()
    if ps.numel() != D:
        raise ValueError("p_loc and p_scale must have the same size")
    it = idx if isinstance(idx, torch.Tensor) else torch.from_numpy(np.asarray(idx))
    it = it.to(device=dev, dtype=torch.int32).contiguous().reshape(-1)
    n_steps = int(n_steps)
    if out_sample is None:
        out_sample = torch.empty(D, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    seed32 = int(np.int32(np.uint32(int(seed) & 0xFFFFFFFF)))
    if (block_dim is None) == (block_off is None):
        raise ValueError("give exactly one of block_dim / block_off")
    with torch.cuda.device(dev):
        return _decode_blocks_on(lib, it, pl, ps, D, n_steps, n_bits_per_step, seed32, rho,
                                 block_dim, block_off, block_id_base, out_sample, dev, stream)


def _decode_blocks_on(lib, it, pl, ps, D, n_steps, n_bits_per_step, seed32, rho, block_dim,
                      block_off, block_id_base, out_sample, dev, stream):
    if block_dim is not None:
        block_dim = int(block_dim)
        nb = D // block_dim if block_dim else 0
        if it.numel() != nb * n_steps:
            raise ValueError("idx must hold nb * n_steps entries")
        rc = lib.cwq_greedy_decode_uniform(
            _ptr(it), _ptr(pl), _ptr(ps), nb, block_dim, int(n_bits_per_step), n_steps, seed32,
            float(rho), int(block_id_base), _ptr(out_sample), stream)
    else:
        offs_h = np.asarray(block_off.cpu() if isinstance(block_off, torch.Tensor)
                            else block_off, dtype=np.int64).reshape(-1)
        nb = offs_h.size - 1
        if nb < 0 or offs_h[0] != 0 or offs_h[-1] != D or (np.diff(offs_h) < 0).any():
            raise ValueError("block_off must be non-decreasing from 0 to D")
        if it.numel() != nb * n_steps:
            raise ValueError("idx must hold nb * n_steps entries")
        offs = torch.from_numpy(offs_h).to(dev)
        mbd = int(np.diff(offs_h).max()) if nb > 0 else 0
        rc = lib.cwq_greedy_decode(
            _ptr(it), _ptr(pl), _ptr(ps), offs.data_ptr(), nb, D, mbd, int(n_bits_per_step),
            n_steps, seed32, float(rho), int(block_id_base), _ptr(out_sample), stream)
    _lib.check(rc, "cwq_greedy_decode")
    return out_sample


# ---------------------------------------------------------------------------
# north-star convenience surface
# ---------------------------------------------------------------------------
def encode(prior_loc, prior_scale, post_loc, post_scale, seed, kl_bits, block_id_base=0):
    """Code every block (row) of [nb, d] (or one [d] block) at ``kl_bits`` bits.

    = code_greedy_sample(t=post, p=prior, n_bits_per_step=kl_bits, n_steps=1,
    seed=seed + block_id_base + g) for each row g.  Returns (indices int32 [nb],
    samples f32 [nb, d]) in the input's array type.
    """
    shape = tuple(np.shape(prior_loc)) if not isinstance(prior_loc, torch.Tensor) \
        else tuple(prior_loc.shape)
    d = shape[-1] if len(shape) else 1
    idx, sample = encode_blocks(post_loc, post_scale, prior_loc, prior_scale, kl_bits, 1, seed,
                                block_dim=d, block_id_base=block_id_base)
    return _like_input(idx.reshape(shape[:-1]), prior_loc), \
        _like_input(sample.reshape(shape), prior_loc)


def decode(indices_or_bitcode, prior_loc, prior_scale, seed, kl_bits, block_id_base=0):
    """Inverse of encode: indices (int [nb]) or the LSB-first bitcode str."""
    shape = tuple(np.shape(prior_loc)) if not isinstance(prior_loc, torch.Tensor) \
        else tuple(prior_loc.shape)
    d = shape[-1] if len(shape) else 1
    nb = int(np.prod(shape[:-1])) if len(shape) > 1 else 1
    if isinstance(indices_or_bitcode, (str, bytes)):
        indices_or_bitcode = bitcode_to_indices(indices_or_bitcode, int(kl_bits), nb)
    sample = decode_blocks(indices_or_bitcode, prior_loc, prior_scale, kl_bits, 1, seed,
                           block_dim=d, block_id_base=block_id_base)
    return _like_input(sample.reshape(shape), prior_loc)


# ---------------------------------------------------------------------------
# reference surface
# ---------------------------------------------------------------------------
def code_greedy_sample(t_loc, t_scale, p_loc, p_scale, n_bits_per_step, n_steps, seed, rho=1.):
    """coded_greedy_sampler.py:29-89 for one block.

    Returns (best_sample [d] f32, sample_index str of n_bits_per_step*n_steps
    LSB-first bits), best_sample in the caller's array type.
    """
    d = int(np.prod(np.shape(t_loc))) if not isinstance(t_loc, torch.Tensor) else t_loc.numel()
    idx, sample = encode_blocks(t_loc, t_scale, p_loc, p_scale, n_bits_per_step, n_steps, seed,
                                rho=rho, block_off=[0, d])
    bits = indices_to_bitcode(idx.cpu().numpy(), int(n_bits_per_step))
    return _like_input(sample, t_loc), bits


def decode_greedy_sample(sample_index, p_loc, p_scale, n_bits_per_step, n_steps, seed, rho=1.):
    """coded_greedy_sampler.py:93-167 for one block."""
    d = int(np.prod(np.shape(p_loc))) if not isinstance(p_loc, torch.Tensor) else p_loc.numel()
    if isinstance(sample_index, (str, bytes)):
        idx = bitcode_to_indices(sample_index, int(n_bits_per_step), int(n_steps))
    else:
        idx = np.asarray(sample_index, dtype=np.int64).reshape(-1)
    sample = decode_blocks(idx.astype(np.int32), p_loc, p_scale, n_bits_per_step, n_steps, seed,
                           rho=rho, block_off=[0, d])
    return _like_input(sample, p_loc)


@functools.lru_cache(maxsize=64)
def group_size_threshold(max_group_size_bits):
    """Smallest s with np.log(s + 1) / np.log(2) >= max_group_size_bits (:230-232)."""
    bits = max_group_size_bits
    s = max(int(2 ** bits) - 3, 0)
    while np.log(s + 1) / np.log(2) >= bits and s > 0:
        s -= 1
    while not (np.log(s + 1) / np.log(2) >= bits):
        s += 1
    return s


def group_starts(kl_divs, n_bits_per_group, max_group_size_bits=12):
    """coded_greedy_sampler.py:207-252 -> group_start_indices (a list, with D appended)."""
    return _group_starts_array(kl_divs, n_bits_per_group, max_group_size_bits).tolist()


def _group_starts_array(kl_divs, n_bits_per_group, max_group_size_bits=12):
    kl = np.ascontiguousarray(np.asarray(kl_divs, dtype=np.float32).reshape(-1))
    D = kl.size
    n_nats = n_bits_per_group * np.log(2) - 1
    cap = D + 2
    starts = np.empty(cap, dtype=np.int64)
    lib = _lib.load()
    n = lib.cwq_group_starts(kl.ctypes.data if D else None, D,
                             group_size_threshold(max_group_size_bits), float(n_nats),
                             starts.ctypes.data, cap)
    _lib.check(n, "cwq_group_starts")
    return starts[:n]


def _dist_parts(dist, dev, what):
    if not _is_float32(dist.loc) or not _is_float32(dist.scale):
        raise Exception(f"{what} datatype must be float32!")
    return _f32(dist.loc, dev, what + ".loc"), _f32(dist.scale, dev, what + ".scale")


def code_grouped_greedy_sample(sess, target, proposal, n_steps, n_bits_per_step, seed,
                               max_group_size_bits=12, adaptive=True, backfitting_steps=0,
                               use_log_prob=False, rho=1., *, prune_mode=None,
                               eval_events=None, eval_ms_out=None):
    """coded_greedy_sampler.py:170-296.

    Returns (sample np.float32 [D], bitcode str, group_start_indices list).
    ``prune_mode`` (keyword only, not in the reference): the encoder's
    cwq_options.prune_mode; results never depend on it.  ``eval_events``
    (keyword only): (start, stop) hipEvent_t handles recorded around the
    candidate-scoring launches (bench.py's kernel timer).
    """
    lib = _lib.load()
    dev = _device_of(target.loc, target.scale, proposal.loc, proposal.scale)
    # :183-187
    if not _is_float32(target.loc) or not _is_float32(target.scale):
        raise Exception("Target datatype must be float32!")
    if not _is_float32(proposal.loc) or not _is_float32(proposal.scale):
        raise Exception("Proposal datatype must be float32!")
    q_loc, q_scale = _dist_parts(target, dev, "Target")
    p_loc, p_scale = _dist_parts(proposal, dev, "Proposal")
    D = p_loc.numel()
    n_steps, n_bits_per_step = int(n_steps), int(n_bits_per_step)
    n_bits_per_group = n_bits_per_step * n_steps
    stream = torch.cuda.current_stream(dev).cuda_stream
    # one native call: standardise + KL (:193-210), host grouping (:207-252),
    # one coder per group with seed + g (:273-284), destandardise (:292) and
    # the LSB-first bitcode (:81-87, :288)
    need = int(lib.cwq_code_grouped_greedy_workspace_size(D, n_steps))
    ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
    bits_h = _scratch_bytes(max((D + 1) * n_bits_per_group, 1))  # <= D + 1 groups
    kl_sum = ctypes.c_double(0.0)
    n_nats = n_bits_per_group * np.log(2) - 1
    seed32 = int(np.int32(np.uint32(int(seed) & 0xFFFFFFFF)))
    args = (_ptr(q_loc), _ptr(q_scale), _ptr(p_loc), _ptr(p_scale), D, n_steps, n_bits_per_step,
            seed32, float(rho), group_size_threshold(max_group_size_bits), float(n_nats))
    opts = _lib.options(prune_mode, eval_events, eval_ms_out)
    kls = ctypes.byref(kl_sum) if VERBOSE else None
    with torch.cuda.device(dev):
        if eval_ms_out is not None:  # the library times the encode: the one-shot call
            sample_h = np.empty(D, dtype=np.float32)
            starts_h = np.empty(D + 2, dtype=np.int64)
            G = _lib.check(lib.cwq_code_grouped_greedy(
                *args, sample_h.ctypes.data, bits_h.ctypes.data, bits_h.size,
                starts_h.ctypes.data, starts_h.size, kls, ws.data_ptr(), ws.numel(), opts, stream),
                "cwq_code_grouped_greedy")
            starts = starts_h[:G + 1].tolist()
        else:
            # two halves: the ~D/5-element Python list of group starts (~0.3 ms
            # for a Kodak image's 41k groups) is built while the device codes;
            # the sample comes back into page-locked memory it keeps alive
            # the group starts and the sample share one page-locked block (the
            # starts arrive by DMA while the encode runs; the sample view keeps
            # the block alive for the caller)
            blk = torch.empty((D + 2) * 8 + max(D, 1) * 4, dtype=torch.uint8,
                              pin_memory=True).numpy()
            starts_h = blk[:(D + 2) * 8].view(np.int64)
            sample_h = blk[(D + 2) * 8:].view(np.float32)[:D]
            idx_h = _pinned_scratch((D + 1) * n_steps * 4)
            G = _lib.check(lib.cwq_code_grouped_greedy_begin(
                *args, sample_h.ctypes.data, idx_h.data_ptr(), (D + 1) * n_steps,
                starts_h.ctypes.data, starts_h.size, kls, ws.data_ptr(), ws.numel(), opts, stream),
                "cwq_code_grouped_greedy_begin")
            starts = starts_h[:G + 1].tolist()
            _lib.check(lib.cwq_code_grouped_greedy_end(idx_h.data_ptr(), G, n_steps,
                                                       n_bits_per_step, bits_h.ctypes.data,
                                                       bits_h.size, stream),
                       "cwq_code_grouped_greedy_end")
    if VERBOSE:
        total_kl_bits = kl_sum.value / np.log(2)
        print("Total KL to split up: {:.2f} bits, "
              "maximum bits per group: {}, "
              "estimated number of groups: {},"
              "coding {} dimensions".format(total_kl_bits, n_bits_per_group,
                                            total_kl_bits // n_bits_per_group + 1, D))
    bitcode = str(memoryview(bits_h)[:G * n_bits_per_group], 'ascii')
    return sample_h, bitcode, starts


def code_grouped_greedy_sample_batch(sess, targets, proposals, n_steps, n_bits_per_step, seeds,
                                     max_group_size_bits=12, adaptive=True, backfitting_steps=0,
                                     use_log_prob=False, rho=1., *, prune_mode=None,
                                     eval_events=None, eval_ms_out=None, defer=False):
    """code_grouped_greedy_sample (coded_greedy_sampler.py:170-296) for a batch
    of independent items (the images of a dataset, the ladder levels of several
    images) in one native call (cwq_code_grouped_greedy_batch).

    ``targets`` / ``proposals``: sequences of distributions (``.loc`` /
    ``.scale``), item i coded with seed ``seeds[i]`` (an int: the same seed for
    every item, as miracle.py codes each image with the run's seed).  Returns a
    list with one (sample, bitcode, group_start_indices) per item, each equal to
    code_grouped_greedy_sample on that item alone, except that the group starts
    are an np.int64 array rather than a list (building a Python list of a Kodak
    image's ~41k starts costs ~0.5 ms, as much as coding it).  Not in the
    reference (an extension for throughput: one encode launch over every item's
    groups).

    ``defer=True`` (keyword only): return at once a handle whose ``result()``
    gives that list.  The call is queued behind the ones before it (one host
    thread runs them in order on the current stream), so a caller that queues
    batch k + 1 before collecting batch k overlaps k + 1's argument pass and
    k's bitcode strings with the device work instead of leaving the device idle
    between calls.  The results are the same either way.
    """
    lib = _lib.load()
    targets, proposals = list(targets), list(proposals)
    if len(targets) != len(proposals):
        raise ValueError("targets and proposals must have the same length")
    n_items = len(targets)
    if n_items == 0:
        return _Done([]) if defer else []
    if np.ndim(seeds) == 0:
        seeds64 = np.full(n_items, int(seeds), dtype=object)
    else:
        seeds64 = np.array([int(x) for x in seeds], dtype=object)
    if seeds64.size != n_items:
        raise ValueError("one seed per item")
    # int32 wrap of each seed (TF int32 arithmetic), as the single call's seed32
    seeds32 = (seeds64 & 0xFFFFFFFF).astype(np.uint64).astype(np.uint32).view(np.int32)
    cols = ([t.loc for t in targets], [t.scale for t in targets], [p.loc for p in proposals],
            [p.scale for p in proposals])
    f32 = torch.float32
    # the common case (float32 CUDA tensors): few attribute reads per array
    # (48 items: ~0.1 ms instead of ~0.25 ms); torch.cat itself refuses mixed
    # devices, and the concatenations' device is checked once
    fast = all(type(a) is torch.Tensor and a.dtype is f32 and a.is_cuda for c in cols for a in c)
    cat = None
    if fast:
        sz = [a.numel() for a in cols[0]]
        if any([a.numel() for a in c] != sz for c in cols[1:]):
            raise ValueError("target and proposal of an item must have the same size")
        sizes = np.array(sz, dtype=np.int64)
        D0 = int(sizes.sum())
        try:
            # concatenation along dim 0 of equal trailing shapes is the concatenation
            # of the flattened arrays (1-D latents: always); the four columns as
            # the four quarters of one buffer (one cat of 4 n_items tensors)
            big = torch.cat([a for c in cols for a in c]).reshape(-1)
            cat = [big[k * D0:(k + 1) * D0] for k in range(4)] if big.numel() == 4 * D0 else None
        except RuntimeError:
            cat = None
        if cat is not None:
            dev = cat[0].device
            if any(x.device != dev for x in cat[1:]):
                cat = None
    if cat is None:
        dev = _device_of(*[a for c in cols for a in c])
        parts = []
        for t, p in zip(targets, proposals):
            if not _is_float32(t.loc) or not _is_float32(t.scale):
                raise Exception("Target datatype must be float32!")  # :183-187
            if not _is_float32(p.loc) or not _is_float32(p.scale):
                raise Exception("Proposal datatype must be float32!")
            q_loc, q_scale = _dist_parts(t, dev, "Target")
            p_loc, p_scale = _dist_parts(p, dev, "Proposal")
            if not (q_scale.numel() == p_loc.numel() == p_scale.numel() == q_loc.numel()):
                raise ValueError("target and proposal of an item must have the same size")
            parts.append((q_loc, q_scale, p_loc, p_scale))
        sizes = np.array([pt[0].numel() for pt in parts], dtype=np.int64)
        cat = [torch.cat([pt[k] for pt in parts]) for k in range(4)]
    item_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D = int(item_off[-1])
    cat = [x.contiguous() for x in cat]
    n_steps, n_bits_per_step = int(n_steps), int(n_bits_per_step)
    n_bits_per_group = n_bits_per_step * n_steps
    need = int(lib.cwq_code_grouped_greedy_batch_workspace_size(D, n_items, n_steps))
    ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
    # page-locked host memory (asynchronous DMA copies, no page faults): the
    # staging the library copies through is this thread's cached buffer; the
    # sample and starts this call returns share one block of torch's caching
    # host allocator (the arrays keep it alive)
    hneed = int(lib.cwq_code_grouped_greedy_batch_host_workspace_size(D, n_items, n_steps))
    # a deferred call runs while this thread may make other calls that use its
    # cached staging (a single-item batch, code_grouped_greedy_sample): it takes
    # its own page-locked block from a pool until the call has ended
    hws = _pinned_take(hneed) if defer else _pinned_scratch(hneed)
    n_out = D + 2 * n_items
    out_t = torch.empty(max(D, 1) * 4 + n_out * 8, dtype=torch.uint8, pin_memory=True)
    out_np = out_t.numpy()
    starts_h = out_np[:n_out * 8].view(np.int64)
    sample_h = out_np[n_out * 8:].view(np.float32)
    bits_cap = (D + n_items) * n_bits_per_group
    # consumed into str below: reusable (a deferred call's until its result())
    bits_h = _bits_take(bits_cap) if defer else _scratch_bytes(bits_cap)
    bits_off = np.empty(n_items + 1, dtype=np.int64)
    n_starts = np.empty(n_items, dtype=np.int64)
    n_nats = n_bits_per_group * np.log(2) - 1
    stream = torch.cuda.current_stream(dev).cuda_stream
    # With several items the call runs on a helper thread (ctypes releases the
    # GIL) and raises item i's flag once its outputs are final: this thread
    # turns the finished items' bitcodes into str while later chunks code.
    ready = np.zeros(n_items, dtype=np.int32) if n_items > 1 or defer else None

    def call():
        with torch.cuda.device(dev):
            opts = _lib.options(prune_mode, eval_events, eval_ms_out,
                                None if ready is None else ready.ctypes.data)
            _lib.check(lib.cwq_code_grouped_greedy_batch(
                n_items, item_off.ctypes.data, _ptr(cat[0]), _ptr(cat[1]), _ptr(cat[2]),
                _ptr(cat[3]), n_steps, n_bits_per_step, seeds32.ctypes.data, float(rho),
                group_size_threshold(max_group_size_bits), float(n_nats), sample_h.ctypes.data,
                bits_h.ctypes.data, bits_cap, bits_off.ctypes.data, starts_h.ctypes.data,
                starts_h.size, n_starts.ctypes.data, ws.data_ptr(), ws.numel(), hws.data_ptr(),
                hneed, opts, stream), "cwq_code_grouped_greedy_batch")

    mv = memoryview(bits_h)

    def item(i):
        a, b = int(item_off[i]), int(item_off[i + 1])
        bitcode = str(mv[bits_off[i]:bits_off[i + 1]], 'ascii')
        s0 = a + 2 * i  # item i's starts region (cwq_code_grouped_greedy_batch)
        return sample_h[a:b], bitcode, starts_h[s0:s0 + n_starts[i]]

    if ready is None:
        call()
        return [item(i) for i in range(n_items)]
    fut = _batch_thread().submit(call)
    fin = None  # a deferred handle's finalizer (returns the buffers if result() never runs)

    def release():  # the call has ended: a deferred call's buffers go back to their pools
        _bits_give(bits_h)
        _pinned_give(hws)

    def finish():
        out = []
        try:
            for i in range(n_items):
                spins = 0
                while not ready[i] and not fut.done():
                    # yield the GIL (the call needs it only to return); after a
                    # short spin back off, so this thread does not hold a whole
                    # CPU of the quota the native host threads partition on
                    spins += 1
                    time.sleep(0 if spins < 32 else 5e-5)
                if not ready[i]:
                    break  # the call ended early: its error is raised below
                out.append(item(i))
            fut.result()
            out.extend(item(i) for i in range(len(out), n_items))
        finally:
            if defer:
                fut.exception()  # (waits) the buffers are free once the call has ended
                if fin is not None and fin.detach() is not None:
                    release()
        return out

    if not defer:
        return finish()
    h = _Deferred(finish)
    fin = weakref.finalize(h, _abandoned, fut, release)
    return h


def _abandoned(fut, release):
    """A deferred batch handle collected without result(): once its call has
    ended, its buffers return to the pools and an error it raised is reported
    (nobody else will see it)."""
    def done(f):
        e = f.exception()
        if e is not None:
            warnings.warn(f"code_grouped_greedy_sample_batch(defer=True): the call failed and "
                          f"its result() was never requested: {e!r}", RuntimeWarning)
        release()
    fut.add_done_callback(done)


class _Done:
    """A deferred batch call's handle whose result is already known."""

    def __init__(self, value):
        self._value = value

    def result(self):
        return self._value


class _Deferred:
    """code_grouped_greedy_sample_batch(..., defer=True)'s handle: result()
    waits for the call, builds the per-item results once and returns them."""

    def __init__(self, finish):
        self._finish = finish
        self._value = self._error = None
        self._lock = threading.Lock()

    def result(self):
        with self._lock:
            if self._finish is not None:
                f, self._finish = self._finish, None
                try:
                    self._value = f()
                except BaseException as e:  # raised again by every later result()
                    self._error = e
            if self._error is not None:
                raise self._error
            return self._value


_bits_free = []
_bits_lock = threading.Lock()


def _bits_take(n):
    """A bitcode buffer of at least n bytes for a deferred batch call (its
    pages stay mapped between calls: a fresh one costs its page faults)."""
    with _bits_lock:
        for k, b in enumerate(_bits_free):
            if b.size >= n:
                return _bits_free.pop(k)
    return np.empty(max(int(n), 1), dtype=np.uint8)


def _bits_give(b):
    with _bits_lock:
        if len(_bits_free) < 4:
            _bits_free.append(b)


_pinned_free = []


def _pinned_take(n):
    """A page-locked host staging block of at least n bytes for a deferred
    batch call (a torch pinned tensor; returned by _pinned_give)."""
    with _bits_lock:
        for k, b in enumerate(_pinned_free):
            if b.numel() >= n:
                return _pinned_free.pop(k)
    return torch.empty(max(int(n), 1), dtype=torch.uint8, pin_memory=True)


def _pinned_give(b):
    with _bits_lock:
        if len(_pinned_free) < 4:
            _pinned_free.append(b)


_batch_pool = None
_batch_pool_lock = threading.Lock()


def _batch_thread():
    """The helper thread code_grouped_greedy_sample_batch runs the native call
    on (one, created on first use; calls from several threads queue on it)."""
    global _batch_pool
    with _batch_pool_lock:
        if _batch_pool is None:
            _batch_pool = concurrent.futures.ThreadPoolExecutor(
                max_workers=1, thread_name_prefix="cwq-batch")
        return _batch_pool


_scratch = threading.local()


def _pinned_scratch(n):
    """This thread's reusable page-locked host buffer of at least n bytes (a
    torch pinned tensor; the library's staging, never returned to callers)."""
    buf = getattr(_scratch, "pinned", None)
    if buf is None or buf.numel() < n:
        buf = torch.empty(max(int(n), 1), dtype=torch.uint8, pin_memory=True)
        _scratch.pinned = buf
    return buf


def _scratch_bytes(n):
    """A per-thread reusable uint8 buffer of at least n bytes (its pages stay
    mapped between calls)."""
    buf = getattr(_scratch, "buf", None)
    if buf is None or buf.size < n:
        buf = np.empty(max(int(n), 1), dtype=np.uint8)
        _scratch.buf = buf
    return buf


def _int64_array(x):
    """A flat np.int64 copy of ``x``; a Python list of ints (the encoder's
    group_start_indices) goes through array.array, ~2x faster than np.asarray."""
    if isinstance(x, list):
        try:
            return np.frombuffer(array.array('q', x), dtype=np.int64)
        except (TypeError, OverflowError):
            pass
    return np.asarray(x, dtype=np.int64).reshape(-1)


def decode_grouped_greedy_sample(sess, bitcode, group_start_indices, proposal, n_bits_per_step,
                                 n_steps, seed, adaptive=True, rho=1.):
    """coded_greedy_sampler.py:299-364.  Returns np.float32 [D]."""
    lib = _lib.load()
    dev = _device_of(proposal.loc, proposal.scale)
    if not _is_float32(proposal.loc) or not _is_float32(proposal.scale):
        raise Exception("Proposal datatype must be float32!")
    p_loc, p_scale = _dist_parts(proposal, dev, "Proposal")
    D = p_loc.numel()
    n_bits_per_group = n_bits_per_step * n_steps
    starts = np.append(_int64_array(group_start_indices), D)  # :323
    n_listed = len(starts) - 1
    # :345-347 decode group i while its bit slice is non-empty
    n_avail = -(-len(bitcode) // n_bits_per_group) if n_bits_per_group else n_listed
    G = min(n_listed, n_avail)
    idx = bitcode_to_indices(bitcode, int(n_bits_per_step), G * int(n_steps), dtype=np.int32)
    offs = np.asarray(starts[:G + 1], dtype=np.int64)
    if G == 0 or offs[-1] != D:
        raise ValueError(f"decoded groups cover {int(offs[-1]) if G else 0} of {D} dims")
    zeros = torch.zeros(D, dtype=torch.float32, device=dev)
    ones = torch.ones(D, dtype=torch.float32, device=dev)
    sample = decode_blocks(idx, zeros, ones, n_bits_per_step, n_steps, seed,
                           rho=rho, block_off=offs)
    out = torch.empty(D, dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(lib.cwq_destandardise(_ptr(sample), _ptr(p_loc), _ptr(p_scale), D, _ptr(out),
                                         stream), "cwq_destandardise")
    return out.cpu().numpy()
