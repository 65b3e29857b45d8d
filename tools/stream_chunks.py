"""encode_blocks_host chunk size vs throughput on C4 (GPU box).

Host arrays of 10^6 blocks x d=32 (16 bits); prints blocks/s of one
device-resident encode_blocks call, of the unpipelined host path (copy in,
encode, copy out) and of encode_blocks_host at several chunk sizes.
Usage: python tools/stream_chunks.py [nb]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
from compression_without_quantization_amd.synthetic import make_blocks_range  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
d, bits = 32, 16
dev = torch.device("cuda", 0)
host = make_blocks_range(0, nb, d, bits)
arrs = [np.ascontiguousarray(host[k].reshape(-1)) for k in
        ("post_loc", "post_scale", "prior_loc", "prior_scale")]


def run(f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = f()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, r


x = [torch.from_numpy(a).to(dev) for a in arrs]
run(lambda: C.encode_blocks(*x, bits, 1, 42, block_dim=d))
t, (gi, gs) = run(lambda: C.encode_blocks(*x, bits, 1, 42, block_dim=d))
print(f"device-resident           {nb / t:12.4e} blocks/s  {t * 1e3:8.1f} ms", flush=True)
ref_i, ref_s = gi.cpu().numpy(), gs.cpu().numpy()
del x


def naive():
    th = [torch.from_numpy(a).to(dev) for a in arrs]
    i, s = C.encode_blocks(*th, bits, 1, 42, block_dim=d)
    return i.cpu().numpy(), s.cpu().numpy()


t, _ = run(naive)
print(f"host, unpipelined         {nb / t:12.4e} blocks/s  {t * 1e3:8.1f} ms", flush=True)
for cb in (65536, 131072, 262144, 500000, None):
    C.encode_blocks_host(*[a[:2 * 65536 * d] for a in arrs], bits, 1, 42, d, chunk_blocks=cb)
    t, (hi, hs) = run(lambda: C.encode_blocks_host(*arrs, bits, 1, 42, d, chunk_blocks=cb))
    ok = np.array_equal(hi, ref_i) and np.array_equal(hs.view(np.uint32), ref_s.view(np.uint32))
    print(f"streamed, chunk {str(cb):>9} {nb / t:12.4e} blocks/s  {t * 1e3:8.1f} ms  "
          f"{'bit-exact' if ok else 'MISMATCH'}", flush=True)
