"""Ad-hoc sweep (GPU box): random batches through the batched grouped
importance call against one single call per item (bit for bit: samples,
Elias-delta codes, group starts, outliers) and one small item per trial
against the CPU oracle's whole pipeline.  Random item counts (1-40), sizes
(0-6,000 dims), rates (0.2-3 bits/dim, so groups from a few candidates to
~10^5 and both encode kernels), group-size limits, seeds and outlier limits.
Prints one line per trial; exits 1 on a mismatch.

Usage: python tools/stress_imp_batch.py [trials] [first_seed] [max_seconds]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd as C  # noqa: E402
import compression_without_quantization_amd.coded_importance_sampler as I  # noqa: E402
from compression_without_quantization_amd.synthetic import make_latents  # noqa: E402
from oracle import oracle as O  # noqa: E402  (the checker only)

I.VERBOSE = False
trials = int(sys.argv[1]) if len(sys.argv) > 1 else 40
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
budget = float(sys.argv[3]) if len(sys.argv) > 3 else 100.0
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


t_end = time.time() + budget
bad = 0
for t in range(first, first + trials):
    if time.time() > t_end:
        break
    rng = np.random.default_rng(t)
    n_items = int(rng.integers(1, 41))
    gbits = int(rng.choice([2, 3, 4]))
    kl_lim = float(rng.choice([8.0, 12.0, 16.0]))
    nbits = int(rng.choice([12, 16, 20]))
    T, P, raw = [], [], []
    for i in range(n_items):
        D = int(rng.choice([0, 1, 3, int(rng.integers(2, 800)), int(rng.integers(800, 6000))]))
        bpd = float(rng.uniform(0.2, 3.0))
        ql, qs, pl, ps = make_latents(D, bits_per_dim=bpd, seed=int(rng.integers(1 << 30)))
        raw.append((ql, qs, pl, ps))
        T.append(C.Normal(torch.from_numpy(ql).to(dev), torch.from_numpy(qs).to(dev)))
        P.append(C.Normal(torch.from_numpy(pl).to(dev), torch.from_numpy(ps).to(dev)))
    seeds = [int(x) for x in rng.integers(-(1 << 31), 1 << 31, n_items)]
    res = I.code_grouped_importance_sample_batch(None, T, P, seeds, nbits, max_group_size_bits=gbits,
                                                 dim_kl_bit_limit=kl_lim)
    mism = 0
    for i in range(n_items):
        s = I.code_grouped_importance_sample(None, T[i], P[i], seeds[i], nbits,
                                             max_group_size_bits=gbits, dim_kl_bit_limit=kl_lim)
        b = res[i]
        ok = (np.array_equal(bits(b[0]), bits(s[0])) and b[1] == s[1] and
              np.array_equal(np.asarray(b[2]), np.asarray(s[2])) and
              np.array_equal(b[3][0], s[3][0]) and np.array_equal(b[3][1], s[3][1]))
        mism += 0 if ok else 1
    # one small item against the oracle's pipeline
    small = [i for i in range(n_items) if 0 < raw[i][0].size <= 1200]
    oracle_ok = None
    if small:
        i = small[0]
        wsm, wi, wst, (oi, oq) = O.code_grouped_importance_sample(*raw[i], seeds[i], nbits, gbits,
                                                                   kl_lim, 8)
        b = res[i]
        got = np.asarray(C.elias_delta_decode_many(b[1], len(b[2]) - 1)[0], np.int64)
        oracle_ok = (np.array_equal(got, np.asarray(wi, np.int64)) and
                     np.array_equal(bits(b[0]), bits(wsm)) and
                     np.array_equal(np.asarray(b[2]), np.asarray(wst, np.int64)) and
                     np.array_equal(b[3][0], oi) and np.array_equal(b[3][1], oq))
    groups = sum(len(r[2]) - 1 for r in res)
    print(f"trial {t}: {n_items} items, {sum(r[0].size for r in raw)} dims, {groups} groups, "
          f"bits/group {nbits}, size bits {gbits}, kl limit {kl_lim}: batch vs single "
          f"mismatched items {mism}, oracle item {oracle_ok}", flush=True)
    if mism or oracle_ok is False:
        bad += 1
print(f"{bad} bad trials")
sys.exit(1 if bad else 0)
