"""Where the time of one reference-shaped code_grouped_greedy_sample call goes
(GPU box): the whole call for C3's two latent shapes (level 1: 196,608 dims,
level 2: 2,304 dims, 8 bits/group), then the call's body re-run with a lap
after each piece.  Mirrors coded_greedy_sampler.code_grouped_greedy_sample's
two-half path; the laps are host wall time (perf_counter), averaged.

  python tools/single_call_laps.py [calls]
CWQ_HOST_PARTITION=1 forces the library's host partition loop (A/B)."""
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
N = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
lib = _lib.load()


def latent(D, seed):
    q_loc, q_scale, p_loc, p_scale = make_latents(D, bits_per_dim=1.1, seed=seed)
    return (C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev)),
            C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev)))


def whole(t, p):
    for _ in range(20):
        S.code_grouped_greedy_sample(None, t, p, 1, 8, 42)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        S.code_grouped_greedy_sample(None, t, p, 1, 8, 42)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / N * 1e6


def laps(t, p):
    names = ["args", "ws alloc", "pinned out", "scratch", "begin", "tolist", "end", "str"]
    acc = np.zeros(len(names))
    n_steps, nb = 1, 8
    for it in range(N + 20):
        ts = [time.perf_counter()]
        q_loc, q_scale = S._dist_parts(t, dev, "Target")
        p_loc, p_scale = S._dist_parts(p, dev, "Proposal")
        D = p_loc.numel()
        stream = torch.cuda.current_stream(dev).cuda_stream
        n_nats = nb * n_steps * np.log(2) - 1
        args = (S._ptr(q_loc), S._ptr(q_scale), S._ptr(p_loc), S._ptr(p_scale), D, n_steps, nb,
                42, 1.0, S.group_size_threshold(12), float(n_nats))
        opts = _lib.options(None, None, None)
        ts.append(time.perf_counter())
        ws = torch.empty(int(lib.cwq_code_grouped_greedy_workspace_size(D, n_steps)),
                         dtype=torch.uint8, device=dev)
        ts.append(time.perf_counter())
        blk = torch.empty((D + 2) * 8 + max(D, 1) * 4, dtype=torch.uint8, pin_memory=True).numpy()
        starts_h = blk[:(D + 2) * 8].view(np.int64)
        sample_h = blk[(D + 2) * 8:].view(np.float32)[:D]
        ts.append(time.perf_counter())
        bits_h = S._scratch_bytes((D + 1) * nb)
        idx_h = S._pinned_scratch((D + 1) * 4)
        ts.append(time.perf_counter())
        G = _lib.check(lib.cwq_code_grouped_greedy_begin(
            *args, sample_h.ctypes.data, idx_h.data_ptr(), D + 1, starts_h.ctypes.data,
            starts_h.size, None, ws.data_ptr(), ws.numel(), opts, stream), "begin")
        ts.append(time.perf_counter())
        starts = starts_h[:G + 1].tolist()
        ts.append(time.perf_counter())
        _lib.check(lib.cwq_code_grouped_greedy_end(idx_h.data_ptr(), G, n_steps, nb,
                                                   bits_h.ctypes.data, bits_h.size, stream), "end")
        ts.append(time.perf_counter())
        bitcode = str(memoryview(bits_h)[:G * nb], 'ascii')
        ts.append(time.perf_counter())
        if it >= 20:
            acc += np.diff(ts)
        del starts, bitcode
    acc = acc / N * 1e6
    return ", ".join(f"{k} {v:.1f}" for k, v in zip(names, acc)) + f"; sum {acc.sum():.1f} us"


sizes = [int(x) for x in os.environ.get("LAPS_SIZES", "2304,196608").split(",")]
for D in sizes:
    seed = D
    t, p = latent(D, seed)
    print(f"D={D} (device partition from {os.environ.get('CWQ_DEV_PART_MIN_D', 'default')}) : whole call {whole(t, p):.1f} us; laps: {laps(t, p)}", flush=True)

if os.environ.get("LAPS_C3"):
    # C3's per-image loop as bench.py runs it: 24 images x (level 1, level 2),
    # distinct latents, the previous step's results held until replaced
    lat = [latent(D, 1000 * i + li) for i in range(24)
           for li, D in enumerate((32 * 48 * 128, 8 * 12 * 24))]
    res = None
    per = np.zeros(2)
    steps, warm = 20, 3
    for k in range(steps + warm):
        out = []
        t0 = time.perf_counter()
        for j, (t, p) in enumerate(lat):
            a = time.perf_counter()
            out.append(S.code_grouped_greedy_sample(None, t, p, 1, 8, 42))
            if k >= warm:
                per[j % 2] += time.perf_counter() - a
        t1 = time.perf_counter()
        res = out
        t2 = time.perf_counter()
        if k >= warm and k == steps + warm - 1:
            print(f"last step {1e3 * (t1 - t0):.2f} ms, replacing the results {1e3 * (t2 - t1):.2f} ms")
    print(f"C3 loop: level-1 call {per[0] / steps / 24 * 1e6:.1f} us, level-2 call "
          f"{per[1] / steps / 24 * 1e6:.1f} us, step {per.sum() / steps * 1e3:.2f} ms "
          f"({24 * steps / per.sum():.0f} images/s)", flush=True)
