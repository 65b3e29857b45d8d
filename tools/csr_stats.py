"""Counters of the general pruned kernel (k_encode_prune_csr) on the grouped
coder (run on the GPU box with a -DCWQ_PRUNE_STATS build through CWQ_LIB_PATH).
Usage: CWQ_LIB_PATH=tools/vrun/libcwq_stats.so python tools/csr_stats.py [config]"""
import ctypes, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from compression_without_quantization_amd import _lib
import compression_without_quantization_amd as C
import compression_without_quantization_amd.coded_greedy_sampler as S
from compression_without_quantization_amd.synthetic import make_latents
import bench

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2cli"
n_img, dims, bits, desc = bench.GROUPED[cfg][:4]
n_steps = bench.GROUPED[cfg][4] if len(bench.GROUPED[cfg]) > 4 else 1
bpd = bench.GROUPED[cfg][5] if len(bench.GROUPED[cfg]) > 5 else 1.1
S.VERBOSE = False
lib = _lib.load()
q = [torch.from_numpy(a).cuda() for a in make_latents(dims[0], bits_per_dim=bpd)]
tgt, prop = C.Normal(q[0], q[1]), C.Normal(q[2], q[3])
out = (ctypes.c_ulonglong * 72)()
lib.cwq_debug_prune_stats(out, 1)
torch.cuda.synchronize()
t0 = time.perf_counter()
C.code_grouped_greedy_sample(None, tgt, prop, n_steps, bits, 42)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
assert lib.cwq_debug_prune_stats(out, 1) == 1, "not a CWQ_PRUNE_STATS build"
a = np.array(out[:], dtype=np.float64)
print(f"{cfg}: {dt * 1e3:.1f} ms (stats build)")
print(f"tiles screened {a[40]:.0f} exact {a[41]:.0f}")
print(f"rows finished {a[42]:.0f} completed {a[44]:.0f} pushed {a[45]:.0f} "
      f"list-full {a[46]:.0f} re-evaluated {a[47]:.0f}")
print(f"dims screened {a[43]:.3e} = {a[43] / max(a[42], 1):.1f}/row; lane-iterations {a[48]:.3e}")
