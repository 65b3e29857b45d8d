"""A numpy model of the device partition's chunked walk (csrc/cwq_partition.hip:
nxt pointers, per-chunk exits by pointer jumping, converged chunks, entries,
marks) checked against the host loop (cwq_group_starts) on the CPU.  It pins
the algorithm; tests/test_partition_gpu.py pins the kernels to the host loop."""
import numpy as np

import compression_without_quantization_amd.coded_greedy_sampler as S
from compression_without_quantization_amd import _lib

W, MAXJ, RUN = 1024, 512, 8


def host(kl, T, n_nats):
    lib = _lib.load()
    st = np.empty(kl.size + 2, np.int64)
    n = lib.cwq_group_starts(kl.ctypes.data, kl.size, T, float(n_nats), st.ctypes.data, st.size)
    return st[:n]


def thr_of(n_nats):
    t = np.float32(n_nats)
    while not (float(t) >= n_nats):
        t = np.nextafter(t, np.float32(np.inf))
    while float(np.nextafter(t, np.float32(-np.inf))) >= n_nats:
        t = np.nextafter(t, np.float32(-np.inf))
    return t


def model(kl, T, n_nats, item_off=None):
    """Per item its start list, or None where the device path falls back."""
    D = kl.size
    item_off = np.array([0, D]) if item_off is None else np.asarray(item_off)
    thr = thr_of(n_nats)
    nxt = np.zeros(D, np.int64)
    maxj = 0
    for i in range(D):
        iend = item_off[np.searchsorted(item_off, i, side="right")]
        j = i + 1
        if i < iend - 1:
            cur, size = kl[i], 1
            while j < iend - 1:
                s = np.float32(cur + kl[j])
                if size >= T or s >= thr:
                    break
                cur, size = s, size + 1
                if j - i >= MAXJ:
                    j += 1
                    break
                j += 1
        nxt[i] = j
        maxj = max(maxj, j - i)
    if maxj > MAXJ:
        return None
    nch = (D + W - 1) // W
    exg = {}
    conv = np.zeros(nch, bool)
    for c in range(nch):
        b = c * W
        lim = min(b + W, D)

        def ex(i):
            while i < lim:
                i = nxt[i]
            return i
        mc = b if c == 0 else max(nxt[max(0, b - MAXJ):b].max(), b)
        cands = range(b, min(mc, lim - 1) + 1)
        exits = [ex(i) for i in cands]
        for i, e in zip(cands, exits):
            exg[i] = e
        conv[c] = len(set(exits)) == 1
    marked = []
    for c in range(nch):
        b, lim = c * W, min(c * W + W, D)
        e = 0
        if c > 0:
            k, run = c - 1, 0
            while k > 0 and not conv[k] and run < RUN:
                k, run = k - 1, run + 1
            if k > 0 and not conv[k]:
                return None
            e = exg[k * W]
            for _ in range(k + 1, c):
                e = exg[e]
        while e < lim:
            marked.append(e)
            e = nxt[e]
    nodes = np.array(marked)
    out = []
    for k in range(item_off.size - 1):
        a, e = item_off[k], item_off[k + 1]
        if a == e:
            out.append(np.array([0, 0]))
            continue
        mine = nodes[(nodes >= a) & (nodes < e)] - a
        dup = int(T <= 0 or kl[a] >= thr or e - a == 1)
        # the kernel's st[0] = 0, st[dup + rank] = node (rank 0: the first dim), st[dup + cnt] = D
        out.append(np.concatenate([[0] * dup, mine, [e - a]]).astype(np.int64))
    return out


def test_model_matches_host_loop():
    rng = np.random.default_rng(3)
    T = S.group_size_threshold(12)
    n_nats = 8 * np.log(2) - 1
    covered = 0
    for trial in range(40):
        D = int(rng.integers(2, 6000))
        kl = rng.exponential(rng.uniform(0.2, 2.0), D).astype(np.float32)
        if trial % 5 == 0:
            kl[0] = np.float32(10.0)
        got = model(kl, T, n_nats)
        if got is None:
            continue
        covered += 1
        assert np.array_equal(got[0], host(kl, T, n_nats)), (trial, D)
    assert covered >= 30


def test_model_items_match_host_loop_per_item():
    rng = np.random.default_rng(4)
    T = S.group_size_threshold(12)
    n_nats = 8 * np.log(2) - 1
    sizes = [0, 1, 2, 700, 0, 3000, 1, 1500]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    kl = rng.exponential(0.8, int(off[-1])).astype(np.float32)
    got = model(kl, T, n_nats, off)
    assert got is not None
    for k in range(len(sizes)):
        want = host(kl[off[k]:off[k + 1]].copy(), T, n_nats) if sizes[k] else np.array([0, 0])
        assert np.array_equal(got[k], want), k


def _next_loop(kl, i, iend, T, thr):
    """nxt(i) as the reference loop restarts from a start at i (the shape of
    k_part_next before round 4's rewrite): size and sum carried, three tests."""
    j = i + 1
    if i < iend - 1:
        cur, size = kl[i], 1
        while j < iend - 1:
            s = np.float32(cur + kl[j])
            if size >= T or s >= thr:
                break
            cur, size = s, size + 1
            if j - i >= MAXJ:
                j += 1
                break
            j += 1
    return j


def _next_folded(kl, i, iend, T, thr):
    """k_part_next's scan (csrc/cwq_partition.hip): the three stops folded into
    one bound klim = min(iend - 1 - i, T, MAXJ + 1), one add and compare per dim."""
    k = 1
    if i < iend - 1:
        klim = min(iend - 1 - i, T, MAXJ + 1)
        cur = kl[i]
        while k < klim:
            s = np.float32(cur + kl[i + k])
            if s >= thr:
                break
            cur = s
            k += 1
    return i + k


def test_folded_scan_equals_loop():
    """The kernel's folded scan equals the loop's on every start: random and
    near-zero KL (long groups up to and past MAXJ), size thresholds 1..5 and
    large, NaN/inf entries, item ends at every distance."""
    rng = np.random.default_rng(11)
    n_nats = 8 * np.log(2) - 1
    thr = thr_of(n_nats)
    for trial in range(12):
        D = int(rng.integers(2, 1400))
        scale = [0.8, 0.02, 0.004, 1e-4][trial % 4]
        kl = rng.exponential(scale, D).astype(np.float32)
        if trial % 3 == 0:
            kl[rng.integers(0, D, 5)] = np.float32(np.nan)
            kl[rng.integers(0, D, 3)] = np.float32(np.inf)
        for T in (1, 2, 3, 5, 4095):
            for iend in (D, max(1, D // 2), min(D, 600)):
                for i in range(0, iend):
                    a = _next_loop(kl, i, iend, T, thr)
                    b = _next_folded(kl, i, iend, T, thr)
                    assert a == b, (trial, T, iend, i, a, b)
