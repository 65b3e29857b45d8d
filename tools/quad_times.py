"""Per-block timeline of one k_small_one launch (C2-shaped grouped encode; run
on the GPU box with a -DCWQ_QUAD_TIMES build selected through CWQ_LIB_PATH).
Usage: CWQ_LIB_PATH=tools/vrun/libcwq_qt.so python tools/quad_times.py [BITS] [D] [--one]
Each wave (block) records its start, the end of its screen and its end
(s_memrealtime).  Prints the launch span, the start-time percentiles, how many
waves run at once over time, per-XCD / per-SIMD spread and durations by block
length.  (--one is the only layout since round 5; round 4's four-block
k_small_fused quads are gone, and the flag is kept for old command lines.)"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
from compression_without_quantization_amd import _lib  # noqa: E402
from compression_without_quantization_amd.synthetic import make_latents  # noqa: E402

ONE = True  # a wave per block (k_small_one)
argv = [a for a in sys.argv if a != "--one"]
bits = int(argv[1]) if len(argv) > 1 else 8
D = int(argv[2]) if len(argv) > 2 else 32 * 48 * 128
lib = _lib.load()
dev = torch.device("cuda", 0)
q_loc, q_scale, p_loc, p_scale = (torch.from_numpy(a).to(dev) for a in make_latents(D, seed=0))
tgt, prop = C.Normal(q_loc, q_scale), C.Normal(p_loc, p_scale)
for _ in range(3):  # the last launch is recorded (warm clocks)
    res = C.code_grouped_greedy_sample(None, tgt, prop, 1, bits, 42)
    torch.cuda.synchronize()
G = len(res[2]) - 1
nq = G if ONE else (G + 3) // 4
n = 1 << 16
t = np.zeros((n, 6), np.uint64)
info = np.zeros((n, 4), np.uint32)
got = lib.cwq_debug_quad_times(t.ctypes.data_as(ctypes.c_void_p),
                               info.ctypes.data_as(ctypes.c_void_p), n)
assert got > 0, "not a CWQ_QUAD_TIMES build"
nq = min(nq, got)
t, info = t[:nq].astype(np.int64), info[:nq]
assert (t[:, 5] > 0).all(), "some quads not recorded"
base = t[:, 0].min()
us = (t - base) / 100.0  # s_memrealtime: 100 MHz
span = us[:, 5].max()
dur = us[:, 5] - us[:, 0]
ph = np.diff(us, axis=1)  # constants, screen, exact rows, exact blocks, finalize
print(f"{G} groups, {nq} {'blocks' if ONE else 'quads'} (waves), span {span:.1f} us")
print(f"quad duration us: mean {dur.mean():.2f} med {np.median(dur):.2f} p10 "
      f"{np.percentile(dur, 10):.2f} p90 {np.percentile(dur, 90):.2f} max {dur.max():.2f}")
names = (("screen", "exact", "-", "-", "-") if ONE else
         ("constants", "screen", "exact rows", "exact blocks", "finalize"))
for i, nm in enumerate(names):
    print(f"  {nm:13s}: mean {ph[:, i].mean():6.2f} us ({ph[:, i].sum() / dur.sum():.1%})")
st = us[:, 0]
order = np.argsort(st)
print("start times: " + " ".join(f"p{p}={np.percentile(st, p):.1f}" for p in (0, 50, 75, 79, 80, 85, 90, 99, 100)))
first = st <= np.percentile(st, 1) + 1.0
print(f"quads started within 1 us of the first: {int(first.sum())}; their mean duration "
      f"{dur[first].mean():.2f} us; later quads' mean {dur[~first].mean() if (~first).any() else 0:.2f} us")
late = st > span * 0.5
print(f"quads starting after half the span: {int(late.sum())}")
edges = np.linspace(0, span, 21)
for lo, hi in zip(edges[:-1], edges[1:]):
    busy = (np.minimum(us[:, 5], hi) - np.maximum(us[:, 0], lo)).clip(min=0).sum() / (hi - lo)
    print(f"  {lo:7.1f}-{hi:7.1f} us: {busy:8.1f} waves running")
xcc = info[:, 1] & 0xf
for x in range(8):
    sel = xcc == x
    if sel.any():
        print(f"  XCD {x}: {int(sel.sum())} quads, last end {us[sel, 5].max():.1f} us, "
              f"busy {dur[sel].sum() / 1e3:.2f} ms")
hw = info[:, 0]
simd = (hw >> 4) & 3
cu = (hw >> 8) & 0xf
se = (hw >> 13) & 7
key = ((xcc.astype(np.int64) * 8 + se) * 16 + cu) * 4 + simd
u, cnt = np.unique(key, return_counts=True)
print(f"SIMDs used {u.size}; quads per SIMD: min {cnt.min()} mean {cnt.mean():.2f} max {cnt.max()}")
used = info[:, 2]
ne = info[:, 3] & 0xff
sd = info[:, 3] >> 8
print(f"listed rows scored exactly per quad: mean {used.mean():.2f}, quads with none "
      f"{(used == 0).mean():.1%}; exact blocks {int(ne.sum())}; dims per quad mean {sd.mean():.2f}")
for lo, hi in ((0, 12), (12, 18), (18, 24), (24, 32), (32, 300)):
    sel = (sd >= lo) & (sd < hi)
    if sel.any():
        print(f"  quad dims [{lo},{hi}): {int(sel.sum())} quads, mean dur {dur[sel].mean():.2f} us, "
              f"screen {ph[sel, 1].mean():.2f}, exact {ph[sel, 2].mean():.2f}, fin {ph[sel, 4].mean():.2f}")
