"""Where one code_grouped_greedy_sample call on C2 spends its time (GPU box):
the whole call, the Python pieces around the native halves, and the halves
themselves (begin: standardise + KL round trip + host partition + enqueue;
the start list; end: wait + bitcode)."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
import compression_without_quantization_amd.coded_greedy_sampler as S  # noqa: E402
from compression_without_quantization_amd import _lib  # noqa: E402
from compression_without_quantization_amd.synthetic import make_latents  # noqa: E402

S.VERBOSE = False
dev = torch.device("cuda", 0)
q_loc, q_scale, p_loc, p_scale = make_latents(196608, bits_per_dim=1.1, seed=0)
tg = C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev))
pr = C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev))
N = 200


def tm(f, n=N):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        r = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3, r


dcall, res = tm(lambda: C.code_grouped_greedy_sample(None, tg, pr, 1, 8, 42))
G = len(res[2]) - 1
lib = _lib.load()
D = 196608
stream = torch.cuda.current_stream(dev).cuda_stream
ws = torch.empty(int(lib.cwq_code_grouped_greedy_workspace_size(D, 1)), dtype=torch.uint8,
                 device=dev)
sample = torch.empty(D, dtype=torch.float32, pin_memory=True).numpy()
idx = torch.empty((D + 1) * 4, dtype=torch.uint8, pin_memory=True)
starts = np.empty(D + 2, np.int64)
bits = np.empty((D + 1) * 8, np.uint8)
ql, qs, pl, ps = (S._ptr(x) for x in (tg.loc, tg.scale, pr.loc, pr.scale))
thr = S.group_size_threshold(12)
nn = float(8 * np.log(2) - 1)


def begin():
    return lib.cwq_code_grouped_greedy_begin(ql, qs, pl, ps, D, 1, 8, 42, 1.0, thr, nn,
                                             sample.ctypes.data, idx.data_ptr(), D + 1,
                                             starts.ctypes.data, D + 2, None, ws.data_ptr(),
                                             ws.numel(), None, stream)


def end():
    return lib.cwq_code_grouped_greedy_end(idx.data_ptr(), G, 1, 8, bits.ctypes.data, bits.size,
                                           stream)


dhalves, _ = tm(lambda: (begin(), end()))
dbegin_sync, _ = tm(lambda: (begin(), torch.cuda.synchronize()))
dlist, _ = tm(lambda: starts[:G + 1].tolist())
dstr, _ = tm(lambda: str(memoryview(bits)[:G * 8], 'ascii'))
dparts, _ = tm(lambda: (S._dist_parts(tg, dev, "T"), S._dist_parts(pr, dev, "P")))
dpin, _ = tm(lambda: torch.empty(D, dtype=torch.float32, pin_memory=True).numpy())
dws, _ = tm(lambda: torch.empty(ws.numel(), dtype=torch.uint8, device=dev))
ev = torch.cuda.Event(enable_timing=True)
ev2 = torch.cuda.Event(enable_timing=True)


def begin_dev():
    ev.record()
    begin()
    ev2.record()


dbd, _ = tm(lambda: (begin_dev(), end()))
print(f"C2 call {dcall:.3f} ms ({G} groups); native begin+end {dhalves:.3f}; begin+sync "
      f"{dbegin_sync:.3f}; list {dlist:.3f}; bitcode str {dstr:.3f}; dist_parts {dparts:.3f}; "
      f"pinned sample {dpin:.3f}; workspace alloc {dws:.3f}; device span of begin's work "
      f"{ev.elapsed_time(ev2):.3f} ms")
