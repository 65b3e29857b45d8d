"""cProfile of code_grouped_greedy_sample_batch on the C3 workload (GPU box):
where the Python side of a batched call spends its time around the native call."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
from compression_without_quantization_amd.synthetic import make_latents  # noqa: E402

dev = torch.device("cuda", 0)
lat = []
for i in range(24):
    for li, D in enumerate((32 * 48 * 128, 8 * 12 * 24)):
        q_loc, q_scale, p_loc, p_scale = make_latents(D, bits_per_dim=1.1, seed=1000 * i + li)
        lat.append((C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev)),
                    C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev))))
T, P = [t for t, _ in lat], [p for _, p in lat]


def step():
    return C.code_grouped_greedy_sample_batch(None, T, P, 1, 8, 42)


native_s = []
if os.environ.get("C3_SPLIT"):  # time the native call inside the wrapper
    from compression_without_quantization_amd import _lib
    lib = _lib.load()
    fn = lib.cwq_code_grouped_greedy_batch

    def timed_native(*a):
        t = time.perf_counter()
        r = fn(*a)
        native_s.append(time.perf_counter() - t)
        return r
    lib.cwq_code_grouped_greedy_batch = timed_native


for _ in range(3):
    step()
torch.cuda.synchronize()
n = int(os.environ.get("C3_CALLS", "20"))
t0 = time.perf_counter()
for _ in range(n):
    step()
print("ms per call", (time.perf_counter() - t0) / n * 1e3)
if native_s:
    print("native ms per call", sum(native_s[-n:]) / n * 1e3)
if os.environ.get("C3_NO_CPROFILE"):
    sys.exit(0)
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    step()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
