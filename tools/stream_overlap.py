"""Experiment: does splitting a multi-step grouped encode over two HIP streams
(group halves) hide the per-step tails?  Times encode_blocks on the C2-CLI
groups in one call vs two half calls on two streams (run on the GPU box)."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C
from compression_without_quantization_amd import _lib
from compression_without_quantization_amd.synthetic import make_latents
from oracle import oracle as O

D = 32 * 48 * 128
q_loc, q_scale, p_loc, p_scale = make_latents(D, bits_per_dim=float(os.environ.get("BPD", "1.1")))
tl, ts = O.standardise(q_loc, q_scale, p_loc, p_scale)
kl = O.kl_normal_normal(q_loc, q_scale, p_loc, p_scale)
starts = np.asarray(C.group_starts(kl, 14 * 30, 12), np.int64)
G = starts.size - 1
dev = torch.device("cuda")
d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
tl_d, ts_d = d(tl), d(ts)
z, o = torch.zeros(D, device=dev), torch.ones(D, device=dev)
h = G // 2


def one():
    return C.encode_blocks(tl_d, ts_d, z, o, 14, 30, 42, block_off=starts)


def parts(streams):
    k = len(streams)
    cut = [G * i // k for i in range(k + 1)]
    res = []
    for i, st in enumerate(streams):
        g0, g1 = cut[i], cut[i + 1]
        sl = slice(int(starts[g0]), int(starts[g1]))
        with torch.cuda.stream(st):
            res.append(C.encode_blocks(tl_d[sl], ts_d[sl], z[sl], o[sl], 14, 30, 42,
                                       block_off=starts[g0:g1 + 1] - starts[g0],
                                       block_id_base=g0))
    return res


S = [torch.cuda.Stream() for _ in range(4)]
i0, _ = one()
r = parts(S[:2])
torch.cuda.synchronize()
same = np.array_equal(np.concatenate([x[0].cpu().numpy() for x in r]), i0.cpu().numpy())
for name, f in (("one stream", one), ("two streams", lambda: parts(S[:2])),
                ("three streams", lambda: parts(S[:3])), ("four streams", lambda: parts(S))):
    f(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t) / 3 * 1e3:.2f} ms (G={G}, indices equal: {same})")
