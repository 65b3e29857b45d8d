"""Units-per-candidate histogram of the pruned encoder (run on the GPU box
with a -DCWQ_PRUNE_STATS build selected through CWQ_LIB_PATH).
Usage: CWQ_LIB_PATH=tools/vrun/libcwq_stats.so python tools/prune_stats.py [nb] [mode]
(PS_D / PS_BITS select the block shape; default the C4 shape d=32, 16 bits)"""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from compression_without_quantization_amd import _lib
import compression_without_quantization_amd as C
from compression_without_quantization_amd.synthetic import make_blocks

nb = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 20000
mode = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else 2
d = int(os.environ.get("PS_D", "32"))
bits = int(os.environ.get("PS_BITS", "16"))
lib = _lib.load()
h = make_blocks(nb, d, bits, seed=20261015)
t = {k: torch.from_numpy(v.reshape(-1)).cuda() for k, v in h.items()}
out = (ctypes.c_ulonglong * 72)()


def run(flags):
    lib.cwq_debug_prune_stats(out, 1 | flags)
    i, _ = C.encode_blocks(t["post_loc"], t["post_scale"], t["prior_loc"], t["prior_scale"], bits,
                           1, 42, block_dim=d, prune_mode=mode)
    torch.cuda.synchronize()
    assert lib.cwq_debug_prune_stats(out, 1) == 1, "not a CWQ_PRUNE_STATS build"
    return i.cpu().numpy(), np.array(out[:], dtype=np.float64)


i0, a = run(4)
if "--oracle-tau" in sys.argv:   # second launch seeded with each block's exact best value
    i1, a = run(2)
    lib.cwq_debug_prune_stats(out, 4)
    assert np.array_equal(i0, i1)
    print("oracle tau: each tile starts at its exact best value")
hist = a[:65]
ncand = hist.sum()
print(f"blocks {nb} mode {mode}: candidates finished {ncand:.0f} (expected {nb * 2**bits})")
print("units/candidate %.4f" % ((hist * np.arange(65)).sum() / ncand))
for k in range(1, 65):
    if hist[k]:
        print(f"  finished after {k:2d} units: {hist[k] / ncand:.5f}")
print(f"completed rows {a[65]:.0f} ({a[65] / nb:.2f}/block), survivors pushed {a[66]:.0f} "
      f"({a[66] / nb:.2f}/block), screened tiles {a[67]:.0f}")
print(f"survivors re-evaluated exactly {a[68]:.0f} ({a[68] / nb:.2f}/block), "
      f"in-loop exact evaluations (list full) {a[69]:.0f}")
if "--json" in sys.argv:   # record for bench.py's roofline.valu.evaluated
    import json
    path = sys.argv[sys.argv.index("--json") + 1]
    with open(path, "w") as f:
        json.dump({"config": os.environ.get("PS_CONFIG", "c4"), "blocks": nb, "block_dim": d,
                   "kl_bits": bits, "prune_mode": mode,
                   "units_per_candidate": float((hist * np.arange(65)).sum() / ncand),
                   "unit_dims": 4, "candidates": float(ncand),
                   "survivors_exact_per_block": float(a[68] / nb),
                   "method": "tools/prune_stats.py on a -DCWQ_PRUNE_STATS build of libcwq.so "
                             "(counters inside k_encode_prune; same inputs as bench.py --config "
                             "c4 but a block sample)"}, f, indent=1)
    print("wrote", path)
