"""Measure the screening Box-Muller approximations against the exact device
tables over all 2^23 inputs (run on the GPU box)."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from compression_without_quantization_amd import _lib

lib = _lib.load()
N = 1 << 23
t = [torch.empty(N, dtype=torch.float32, device="cuda") for _ in range(6)]
st = torch.cuda.current_stream().cuda_stream
assert lib.cwq_selftest_bm_tables(0, N, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), st) == 0
assert lib.cwq_selftest_screen_tables(0, N, t[3].data_ptr(), t[4].data_ptr(), t[5].data_ptr(), st) == 0
torch.cuda.synchronize()
a = [x.cpu().numpy().astype(np.float64) for x in t]
a[3] = a[3] * np.sqrt(2.0 * np.log(2.0))   # the screen table holds r~ / sqrt(2 ln 2)
er = np.abs(a[3] - a[0]); es = np.abs(a[4] - a[1]); ec = np.abs(a[5] - a[2])
print("Er max %.6g at m=%d (r=%.6g)" % (er.max(), er.argmax(), a[0][er.argmax()]))
print("Es max %.6g at m=%d" % (es.max(), es.argmax()))
print("Ec max %.6g at m=%d" % (ec.max(), ec.argmax()))
print("rmax exact %.9g screen %.9g" % (a[0].max(), a[3].max()))
for lo, hi in [(0, 1 << 20), (1 << 20, 1 << 22), (1 << 22, (1 << 23) - (1 << 16)), ((1 << 23) - (1 << 16), N)]:
    print("  Er in m[%d,%d): %.4g" % (lo, hi, er[lo:hi].max()))
