"""Wall time of decode_grouped_greedy_sample on one C2 image (GPU box): the
grouped decoder's host phases (bit parsing, offsets) and its device work."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
import compression_without_quantization_amd.coded_greedy_sampler as S  # noqa: E402
from compression_without_quantization_amd.binary_io import bitcode_to_indices  # noqa: E402
from compression_without_quantization_amd.synthetic import make_latents  # noqa: E402

dev = torch.device("cuda", 0)
D = 32 * 48 * 128
q_loc, q_scale, p_loc, p_scale = make_latents(D, bits_per_dim=1.1, seed=0)
t = C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev))
p = C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev))
sample, bitcode, starts = C.code_grouped_greedy_sample(None, t, p, 1, 8, 42, max_group_size_bits=4)


def tm(f, n=50):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        r = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3, r


d_all, dec = tm(lambda: C.decode_grouped_greedy_sample(None, bitcode, starts, p, 8, 1, 42))
assert np.array_equal(dec.view(np.uint32), np.asarray(sample).view(np.uint32))
d_bits, _ = tm(lambda: bitcode_to_indices(bitcode, 8, len(starts)))
d_arr, _ = tm(lambda: S._int64_array(starts))
print(f"groups {len(starts)}: decode_grouped_greedy_sample {d_all:.3f} ms "
      f"(bitcode_to_indices {d_bits:.3f} ms, starts list -> array {d_arr:.3f} ms)")
