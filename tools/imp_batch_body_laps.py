"""The body of code_grouped_importance_sample_batch (fast path) on I2's
batch, re-run with a lap after each piece (GPU box): argument checks and
concatenation, host buffers, the native call, then the wrapper's result
work (index gather, quint16 of the outliers, Elias-delta, code lengths, the
per-item views).  Host wall time, averaged.

  python tools/imp_batch_body_laps.py [calls]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
import compression_without_quantization_amd.coded_importance_sampler as I  # noqa: E402
from compression_without_quantization_amd import _lib  # noqa: E402
from compression_without_quantization_amd.binary_io import elias_delta_code_many  # noqa: E402
from compression_without_quantization_amd.synthetic import make_latents  # noqa: E402

I.VERBOSE = False
N = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
lib = _lib.load()
T, P = [], []
for i in range(24):
    q_loc, q_scale, p_loc, p_scale = make_latents(8 * 12 * 24, seed=5000 + i)
    T.append(C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev)))
    P.append(C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev)))

names = ["checks+cat", "host bufs", "native", "gather", "quint16", "elias", "lengths",
         "items"]
acc = np.zeros(len(names))
for it in range(N + 20):
    ts = [time.perf_counter()]
    n_items = len(T)
    seeds32 = np.full(n_items, 42, dtype=np.int32)
    raw = ([t.loc for t in T], [t.scale for t in T], [p.loc for p in P], [p.scale for p in P])
    sz = [a.numel() for a in raw[0]]
    bad = any([a.numel() for a in c] != sz for c in raw[1:])
    sizes = np.array(sz, dtype=np.int64)
    item_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D = int(item_off[-1])
    big = torch.cat([a for c in raw for a in c]).reshape(-1)
    cat = [big[k * D:(k + 1) * D] for k in range(4)]
    ts.append(time.perf_counter())
    need = int(lib.cwq_code_grouped_importance_batch_workspace_size(D, n_items))
    ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
    sample_h = np.empty(max(D, 1), dtype=np.float32)
    index_h = np.empty(D + n_items, dtype=np.int64)
    starts_h = np.empty(D + 2 * n_items, dtype=np.int64)
    n_starts = np.zeros(n_items, dtype=np.int64)
    out_i = np.empty(max(D, 1), dtype=np.int64)
    out_v = np.zeros(max(D, 1), dtype=np.float32)
    n_out = np.zeros(n_items, dtype=np.int64)
    kl_sum = np.zeros(n_items, dtype=np.float64)
    ts.append(time.perf_counter())
    _lib.check(lib.cwq_code_grouped_importance_batch(
        n_items, item_off.ctypes.data, I._ptr(cat[0]), I._ptr(cat[1]), I._ptr(cat[2]),
        I._ptr(cat[3]), seeds32.ctypes.data, float(np.float32(16)),
        I.importance_group_size_threshold(2), float(20 * np.log(2) - 1), sample_h.ctypes.data,
        index_h.ctypes.data, starts_h.ctypes.data, starts_h.size, n_starts.ctypes.data,
        out_i.ctypes.data, out_v.ctypes.data, n_out.ctypes.data, kl_sum.ctypes.data,
        ws.data_ptr(), ws.numel(), _lib.options(None), I._stream(dev)), "batch")
    ts.append(time.perf_counter())
    ns_all = n_starts.astype(np.int64)
    G = np.maximum(ns_all - 1, 0)
    goff = np.concatenate([[0], np.cumsum(G)])
    src = np.arange(goff[-1], dtype=np.int64) + np.repeat(
        item_off[:-1] + np.arange(n_items, dtype=np.int64) - goff[:-1], G)
    vals = index_h[src] + 1
    ts.append(time.perf_counter())
    ooff = np.concatenate([[0], np.cumsum(n_out)])
    osrc = np.arange(ooff[-1], dtype=np.int64) + np.repeat(item_off[:-1] - ooff[:-1], n_out)
    o_idx = out_i[osrc]
    o_q = I.quantize_quint16(out_v[osrc])
    ts.append(time.perf_counter())
    codes = elias_delta_code_many(vals)
    ts.append(time.perf_counter())
    nb_ = np.frexp(vals)[1] - 1
    coff = np.concatenate([[0], np.cumsum(I._ELIAS_LEN[nb_])])[goff]
    ts.append(time.perf_counter())
    res = []
    for i in range(n_items):
        a, b = int(item_off[i]), int(item_off[i + 1])
        o0, o1 = int(ooff[i]), int(ooff[i + 1])
        gs = starts_h[a + 2 * i:a + 2 * i + int(ns_all[i])]
        res.append((sample_h[a:b], codes[coff[i]:coff[i + 1]], gs, (o_idx[o0:o1], o_q[o0:o1])))
    ts.append(time.perf_counter())
    if it >= 20:
        acc += np.diff(ts)
acc = acc / N * 1e6
print("I2 batch body (us): " + ", ".join(f"{k} {v:.1f}" for k, v in zip(names, acc)) +
      f"; sum {acc.sum():.1f}", flush=True)
