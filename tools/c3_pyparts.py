"""Python-side cost pieces of code_grouped_greedy_sample_batch on C3 (GPU box)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
import compression_without_quantization_amd.coded_greedy_sampler as S  # noqa: E402
from compression_without_quantization_amd.synthetic import make_latents  # noqa: E402

dev = torch.device("cuda", 0)
lat = []
for i in range(24):
    for li, D in enumerate((32 * 48 * 128, 8 * 12 * 24)):
        q_loc, q_scale, p_loc, p_scale = make_latents(D, bits_per_dim=1.1, seed=1000 * i + li)
        lat.append((C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev)),
                    C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev))))


def tm(f, n=50):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        r = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3, r


dparts, parts = tm(lambda: [(S._dist_parts(t, dev, "T") + S._dist_parts(p, dev, "P")) for t, p in lat])
dcat, cat = tm(lambda: [torch.cat([pt[k] for pt in parts]) for k in range(4)])
D = int(sum(p[0].numel() for p in parts))
dpin, _ = tm(lambda: (torch.empty(95 << 20, dtype=torch.uint8, pin_memory=True),
                      torch.empty(D, dtype=torch.float32, pin_memory=True),
                      torch.empty(D + 96, dtype=torch.int64, pin_memory=True)))
buf = np.full(8_100_000, ord('1'), np.uint8)
off = np.linspace(0, 8_000_000, 49).astype(np.int64)
mv = memoryview(buf)
dstr, _ = tm(lambda: [str(mv[off[i]:off[i + 1]], 'ascii') for i in range(48)])
dstr2, _ = tm(lambda: [buf[off[i]:off[i + 1]].tobytes().decode('ascii') for i in range(48)])
print(f"dist_parts {dparts:.3f} ms, cat {dcat:.3f} ms, pinned allocs {dpin:.3f} ms, "
      f"str(memoryview) {dstr:.3f} ms, tobytes+decode {dstr2:.3f} ms")
dcall, _ = tm(lambda: S.code_grouped_greedy_sample_batch(None, [t for t, _ in lat], [p for _, p in lat],
                                                         1, 8, 1, max_group_size_bits=4), n=30)
print(f"whole call {dcall:.3f} ms")
