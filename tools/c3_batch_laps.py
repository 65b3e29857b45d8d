"""Timeline of one batched C3 call (bench.py --config c3's step: 24 images x
both levels in one code_grouped_greedy_sample_batch call) on the GPU box:
Python entry, the library's phase laps (a CWQ_PHASE_TIMES build,
tools/variants.sh phases, selected with CWQ_LIB_PATH) and Python exit, all on
CLOCK_MONOTONIC, averaged over the calls.

  CWQ_LIB_PATH=tools/vrun/libcwq_phases.so python tools/c3_batch_laps.py [calls] 2> laps.err"""
import os
import re
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
import compression_without_quantization_amd.coded_greedy_sampler as S  # noqa: E402
from compression_without_quantization_amd.synthetic import make_latents  # noqa: E402

S.VERBOSE = False
N = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
T, P = [], []
for i in range(24):
    for li, D in enumerate((32 * 48 * 128, 8 * 12 * 24)):
        q_loc, q_scale, p_loc, p_scale = make_latents(D, bits_per_dim=1.1, seed=1000 * i + li)
        T.append(C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev)))
        P.append(C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev)))


def call():
    return C.code_grouped_greedy_sample_batch(None, T, P, 1, 8, 42)


for _ in range(10):
    res = call()
torch.cuda.synchronize()
marks = []
for _ in range(N):
    t0 = time.clock_gettime(time.CLOCK_MONOTONIC) * 1e6
    sys.stderr.write(f"[py] start monotonic {t0:.1f}\n")
    res = call()
    t1 = time.clock_gettime(time.CLOCK_MONOTONIC) * 1e6
    sys.stderr.write(f"[py] end monotonic {t1:.1f}\n")
    marks.append(t1 - t0)
    del res
sys.stderr.flush()
print(f"C3 batched call: {np.mean(marks):.1f} us mean, {np.median(marks):.1f} median "
      f"({24e6 / np.median(marks):.0f} images/s)", flush=True)
