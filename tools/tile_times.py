"""Per-tile timeline of one pruned-encoder launch (run on the GPU box with a
-DCWQ_TILE_TIMES build selected through CWQ_LIB_PATH).
Usage: CWQ_LIB_PATH=tools/vrun/libcwq_tt.so python tools/tile_times.py NB D BITS
Prints the launch span, how many tiles run at once over time, the tile
durations of the first resident round against the later ones, and the drain
at the end of the launch (the time from the last tile start to the last end)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
from compression_without_quantization_amd import _lib  # noqa: E402
from compression_without_quantization_amd.synthetic import make_blocks  # noqa: E402

nb, d, bits = (int(sys.argv[i]) for i in (1, 2, 3))
lib = _lib.load()
h = make_blocks(nb, d, bits, seed=20261015)
t = {k: torch.from_numpy(v.reshape(-1)).cuda() for k, v in h.items()}
for _ in range(2):  # the second launch is timed (warm clocks)
    C.encode_blocks(t["post_loc"], t["post_scale"], t["prior_loc"], t["prior_scale"], bits, 1, 42,
                    block_dim=d)
    torch.cuda.synchronize()
n = 1 << 18
t0 = np.zeros(n, np.uint64)
t1 = np.zeros(n, np.uint64)
wg = np.zeros(n, np.uint32)
got = lib.cwq_debug_tile_times(t0.ctypes.data_as(ctypes.c_void_p), t1.ctypes.data_as(ctypes.c_void_p),
                               wg.ctypes.data_as(ctypes.c_void_p), n)
assert got > 0, "not a CWQ_TILE_TIMES build"
m = t1 > 0
ntile = int(m.sum())
a, b = t0[m].astype(np.int64), t1[m].astype(np.int64)
base = a.min()
a, b = (a - base) / 100.0, (b - base) / 100.0  # microseconds
span = b.max()
dur = b - a
order = np.argsort(a)
first = order[:1536]
rest = order[1536:]
print(f"nb {nb} d {d} bits {bits}: {ntile} tiles, span {span:.1f} us")
print(f"tile duration us: all mean {dur.mean():.1f} med {np.median(dur):.1f} "
      f"p10 {np.percentile(dur, 10):.1f} p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f}")
print(f"  first 1536 started: mean {dur[first].mean():.1f}; later: mean "
      f"{dur[rest].mean() if rest.size else 0:.1f}")
print(f"last start {a.max():.1f} us, drain {span - a.max():.1f} us; "
      f"sum of tile time / (1536 x span) = {dur.sum() / (1536 * span):.3f}")
# concurrency over time
edges = np.linspace(0, span, 21)
for lo, hi in zip(edges[:-1], edges[1:]):
    busy = (np.minimum(b, hi) - np.maximum(a, lo)).clip(min=0).sum() / (hi - lo)
    print(f"  {lo:8.1f}-{hi:8.1f} us: {busy:7.1f} tiles running")
# per XCD (HW_REG_XCC_ID): tiles, busy time and when its last tile ended
xcc = (wg[m] >> 24) & 0xf
for x in range(8):
    sel = xcc == x
    if sel.any():
        print(f"  XCD {x}: {int(sel.sum())} tiles, tile time {dur[sel].sum() / 1e3:.1f} ms, "
              f"last end {b[sel].max():.1f} us")
# tile index (interleaved: block t % nb, tile t // nb) against duration
tt = np.nonzero(m)[0] // nb
for q in range(0, int(tt.max()) + 1, max(1, (int(tt.max()) + 1) // 8)):
    sel = tt == q
    print(f"  tile-of-block {q:4d}: mean duration {dur[sel].mean():.1f} us")
