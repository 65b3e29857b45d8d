"""Where the time of one code_grouped_importance_sample_batch call on I2 goes
(GPU box): the whole call, then the wrapper's pieces (argument checks and
concatenation, the native call, the per-item Python results), averaged.

  python tools/imp_batch_laps.py [calls]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
import compression_without_quantization_amd.coded_importance_sampler as I  # noqa: E402
from compression_without_quantization_amd.binary_io import elias_delta_code_many  # noqa: E402
from compression_without_quantization_amd.synthetic import make_latents  # noqa: E402

I.VERBOSE = False
N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
T, P = [], []
for i in range(24):
    q_loc, q_scale, p_loc, p_scale = make_latents(8 * 12 * 24, seed=5000 + i)
    T.append(C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev)))
    P.append(C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev)))


def tm(f, n=N):
    for _ in range(10):
        r = f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        r = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3, r


call = lambda: I.code_grouped_importance_sample_batch(None, T, P, 42, 20, max_group_size_bits=2,
                                                      dim_kl_bit_limit=16)
ms, res = tm(call)
print(f"whole batch call {ms:.3f} ms ({24 / ms * 1e3:.0f} images/s)")
cat_ms, cat = tm(lambda: [torch.cat([getattr(d, k).reshape(-1) for d in ds])
                          for ds, k in ((T, "loc"), (T, "scale"), (P, "loc"), (P, "scale"))])
print(f"  four torch.cat of 24 tensors: {cat_ms:.3f} ms")
idx = [r[1] for r in I.code_grouped_importance_sample_batch(None, T, P, 42, 20,
                                                            max_group_size_bits=2,
                                                            dim_kl_bit_limit=16,
                                                            return_indices=True)]
el_ms, _ = tm(lambda: [elias_delta_code_many(x) for x in idx])
print(f"  24 elias_delta_code_many: {el_ms:.3f} ms")
q_ms, _ = tm(lambda: [I.quantize_quint16(r[3][1].astype(np.float32)) for r in res])
print(f"  24 quantize_quint16: {q_ms:.3f} ms")
tl_ms, _ = tm(lambda: [tuple((np.arange(578, dtype=np.int64) + 1).tolist()) for _ in range(24)])
print(f"  24 index tuples of 578: {tl_ms:.3f} ms")
