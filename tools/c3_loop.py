"""C3's batched call back to back (the bench's timed loop without its second,
timer-carrying pass), for a kernel-trace timeline of the steady state:
  rocprofv3 --kernel-trace -- python3 tools/c3_loop.py [CALLS]
then python tools/timeline.py DIR WINDOW_MS over the last calls."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
import compression_without_quantization_amd.coded_greedy_sampler as S  # noqa: E402
from compression_without_quantization_amd.synthetic import make_latents  # noqa: E402

S.VERBOSE = False
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
if os.environ.get("C3_SET_DEVICE"):
    torch.cuda.set_device(dev)
if os.environ.get("C3_IMPORT_BENCH"):
    import bench  # noqa: F401
T, P = [], []
for i in range(24):
    for li, D in enumerate((32 * 48 * 128, 8 * 12 * 24)):
        q_loc, q_scale, p_loc, p_scale = make_latents(D, bits_per_dim=1.1, seed=1000 * i + li)
        T.append(C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev)))
        P.append(C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev)))
for _ in range(int(os.environ.get("C3_WARMUP", "5"))):  # host clocks ramp over ~0.3 s
    res = C.code_grouped_greedy_sample_batch(None, T, P, 1, 8, 42)
torch.cuda.synchronize()
t0 = time.perf_counter()
per, marks = [], []
if os.environ.get("C3_DEFER"):  # pipelined two deep (defer=True), as bench.py's pipelined pass
    h = C.code_grouped_greedy_sample_batch(None, T, P, 1, 8, 42, defer=True)
    for _ in range(n - 1):
        h2 = C.code_grouped_greedy_sample_batch(None, T, P, 1, 8, 42, defer=True)
        res = h.result()
        h = h2
        per.append(time.perf_counter())
    res = h.result()
    per.append(time.perf_counter())
for _ in range(0 if os.environ.get("C3_DEFER") else n):
    m0 = time.monotonic()
    res = C.code_grouped_greedy_sample_batch(None, T, P, 1, 8, 42)
    per.append(time.perf_counter())
    marks.append((m0, time.monotonic()))
if os.environ.get("C3_TSTAMPS"):  # with a CWQ_PHASE_TIMES build: the Python side's
    for m0, m1 in marks[-4:]:     # entry / return on the native laps' clock
        print(f"[py] call entry {m0 * 1e6:.1f} return {m1 * 1e6:.1f} us (monotonic)",
              file=sys.stderr)
torch.cuda.synchronize()
el = time.perf_counter() - t0
if os.environ.get("CWQ_BENCH_STEP_TIMES"):
    print("step ms:", " ".join(f"{(b - a) * 1e3:.2f}" for a, b in zip([t0] + per, per)),
          flush=True)
print(f"{n} calls, {el / n * 1e3:.3f} ms per call, {24 * n / el:.0f} images/s", flush=True)
