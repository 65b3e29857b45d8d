"""Per-phase host time of code_grouped_greedy_sample_batch's Python wrapper on
C3 (GPU box): the argument pass, the four concatenations, the allocations, and
the call itself, each averaged over back-to-back calls."""
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
T, P = [], []
for i in range(24):
    for li, D in enumerate((32 * 48 * 128, 8 * 12 * 24)):
        q_loc, q_scale, p_loc, p_scale = make_latents(D, bits_per_dim=1.1, seed=1000 * i + li)
        T.append(C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev)))
        P.append(C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev)))
N = 30


def tm(f):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(N):
        r = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / N * 1e3, r


f32 = torch.float32
cols = ([t.loc for t in T], [t.scale for t in T], [p.loc for p in P], [p.scale for p in P])
lib = _lib.load()
Dt = sum(int(t.loc.numel()) for t in T)
res = {}
res["call"], _ = tm(lambda: C.code_grouped_greedy_sample_batch(None, T, P, 1, 8, 42))
res["cols"], _ = tm(lambda: ([t.loc for t in T], [t.scale for t in T], [p.loc for p in P],
                             [p.scale for p in P]))
res["fast_check"], _ = tm(lambda: all(type(a) is torch.Tensor and a.dtype is f32 and a.is_cuda
                                      for c in cols for a in c))
res["sizes"], _ = tm(lambda: [[a.numel() for a in c] for c in cols])
res["cat4"], _ = tm(lambda: [torch.cat(c).reshape(-1) for c in cols])
need = int(lib.cwq_code_grouped_greedy_batch_workspace_size(Dt, len(T), 1))
res["ws_alloc"], _ = tm(lambda: torch.empty(need, dtype=torch.uint8, device=dev))
n_out = Dt + 2 * len(T)
res["pinned_out"], _ = tm(lambda: torch.empty(Dt * 4 + n_out * 8, dtype=torch.uint8,
                                              pin_memory=True).numpy())
res["ws_size_calls"], _ = tm(lambda: (lib.cwq_code_grouped_greedy_batch_workspace_size(Dt, 48, 1),
                                      lib.cwq_code_grouped_greedy_batch_host_workspace_size(Dt, 48, 1)))
res["seeds_obj"], _ = tm(lambda: (np.full(48, 42, dtype=object) & 0xFFFFFFFF).astype(np.uint64)
                         .astype(np.uint32).view(np.int32))
res["list_args"], _ = tm(lambda: (list(T), list(P)))
res["thread_roundtrip"], _ = tm(lambda: S._batch_thread().submit(lambda: None).result())
res["current_stream"], _ = tm(lambda: torch.cuda.current_stream(dev).cuda_stream)


def _device_ctx():
    with torch.cuda.device(dev):
        pass


res["device_ctx"], _ = tm(_device_ctx)
print(" ".join(f"{k} {v:.3f}" for k, v in res.items()), "ms", flush=True)
