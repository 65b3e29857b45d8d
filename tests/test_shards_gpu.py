"""GPU: the multi-GPU partitioning on the HIP path, the C3 workload, and the
bench's own N-rank launcher.

Sharding rests on one property of the reference: group g is coded with seed
``seed + g`` (coded_greedy_sampler.py:282), so a shard coded with
block_id_base = its first global block reproduces the single-call result.
These tests check that property bit for bit on the kernels (uniform and
ragged CSR blocks, the multi-step CSR path that forks onto the library's
streams, even and cost-balanced cuts), then run the C3 image set through the
grouped pipeline, and finally run ``bench.py --gpus 2`` as a fresh process.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import REPO

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cwq(cwqlib):
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import compression_without_quantization_amd as C
    return C


def _u32(a):
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


def _encode_sharded(cwq, arrays, cuts, bits, n_steps, seed, off=None, d=None):
    """Encode [cuts[r], cuts[r+1]) blocks per shard with block_id_base = cuts[r];
    return the concatenated (idx, sample) as host arrays."""
    tl, ts, pl, ps = arrays
    idx_parts, smp_parts = [], []
    for b0, b1 in zip(cuts[:-1], cuts[1:]):
        if off is None:
            sl = slice(b0 * d, b1 * d)
            i, s = cwq.encode_blocks(tl[sl], ts[sl], pl[sl], ps[sl], bits, n_steps, seed,
                                     block_dim=d, block_id_base=b0)
        else:
            sl = slice(int(off[b0]), int(off[b1]))
            i, s = cwq.encode_blocks(tl[sl], ts[sl], pl[sl], ps[sl], bits, n_steps, seed,
                                     block_off=off[b0:b1 + 1] - off[b0], block_id_base=b0)
        idx_parts.append(i.cpu().numpy().reshape(-1, n_steps))
        smp_parts.append(s.cpu().numpy())
    return np.concatenate(idx_parts), np.concatenate(smp_parts)


def _cuts(nb, world, cost=None):
    from compression_without_quantization_amd.parallel import shard_range
    spans = [shard_range(nb, world, r, cost) for r in range(world)]
    return [spans[0][0]] + [b for _, b in spans]


def test_uniform_shards_concatenate_to_single_call(cwq, oracle):
    """C4-shaped slice (d=32, 16 bits): one call == 2 even shards == 3
    cost-balanced shards, bit for bit; oracle on sampled blocks of each shard."""
    from compression_without_quantization_amd.synthetic import make_blocks_range
    nb, d, bits, seed = 6000, 32, 16, 42
    h = make_blocks_range(0, nb, d, bits)
    host = [h[k].reshape(-1) for k in ("post_loc", "post_scale", "prior_loc", "prior_scale")]
    dev = torch.device("cuda")
    arrays = [torch.from_numpy(a).to(dev) for a in host]
    i1, s1 = _encode_sharded(cwq, arrays, [0, nb], bits, 1, seed, d=d)
    for cuts in (_cuts(nb, 2), _cuts(nb, 3, cost=np.full(nb, d * 2.0 ** bits)), [0, 1, 4097, nb]):
        ik, sk = _encode_sharded(cwq, arrays, cuts, bits, 1, seed, d=d)
        assert np.array_equal(ik, i1), f"indices differ for cuts {cuts}"
        assert np.array_equal(_u32(sk), _u32(s1)), f"samples differ for cuts {cuts}"
    # oracle: first, last and a middle block of every 3-way shard
    for b in sorted({0, 1999, 2000, 2001, 3999, 4000, nb - 1}):
        sl = slice(b * d, (b + 1) * d)
        wi, ws = oracle.greedy_encode(host[0][sl], host[1][sl], host[2][sl], host[3][sl],
                                      np.array([0, d], np.int64), bits, 1, seed, 1.0, b)
        assert int(wi.reshape(-1)[0]) == int(i1[b, 0]), f"block {b}"
        assert np.array_equal(_u32(ws), _u32(s1[sl])), f"block {b}"


def test_ragged_csr_shards_multistep(cwq, oracle):
    """Ragged groups (sizes 1..4095, the C2/C3 group-size range), 14 bits x 3
    steps -- the general pruned kernel and the multi-stream step split -- one
    call vs 2 even and 3 cost-balanced shard_range cuts (cost d_g 2^b n_steps)."""
    rng = np.random.default_rng(2026)
    sizes = np.concatenate([rng.integers(1, 64, 40), rng.integers(64, 4096, 6), [1, 4095]])
    rng.shuffle(sizes)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D, nb = int(off[-1]), sizes.size
    bits, n_steps, seed = 14, 3, 7
    tl = rng.standard_normal(D).astype(np.float32) * 0.3
    ts = rng.uniform(0.5, 1.0, D).astype(np.float32)
    pl = np.zeros(D, np.float32)
    ps = np.ones(D, np.float32)
    dev = torch.device("cuda")
    arrays = [torch.from_numpy(a).to(dev) for a in (tl, ts, pl, ps)]
    i1, s1 = _encode_sharded(cwq, arrays, [0, nb], bits, n_steps, seed, off=off)
    cost = sizes.astype(np.float64) * 2.0 ** bits * n_steps
    for cuts in (_cuts(nb, 2), _cuts(nb, 3, cost=cost)):
        ik, sk = _encode_sharded(cwq, arrays, cuts, bits, n_steps, seed, off=off)
        assert np.array_equal(ik, i1), f"indices differ for cuts {cuts}"
        assert np.array_equal(_u32(sk), _u32(s1)), f"samples differ for cuts {cuts}"
    # oracle on a few groups (incl. the longest and a single-dim group)
    for g in sorted({0, int(np.argmax(sizes)), int(np.argmin(sizes)), nb - 1}):
        sl = slice(int(off[g]), int(off[g + 1]))
        wi, ws = oracle.greedy_encode(tl[sl], ts[sl], pl[sl], ps[sl],
                                      np.array([0, sizes[g]], np.int64), bits, n_steps, seed,
                                      1.0, g)
        assert np.array_equal(wi.reshape(-1), i1[g]), f"group {g}"
        assert np.array_equal(_u32(ws), _u32(s1[sl])), f"group {g}"


def test_q4_kernels_match_unaligned_fallback(cwq, oracle):
    """The float4 finalize/decode kernels (uniform d % 4 == 0) against the
    per-dim kernels they replace, reached through 4-byte-offset views (the
    launchers fall back when a base is not 16-byte aligned); d=12 (3 Philox
    blocks per row) and d=32, 1 and 3 steps."""
    rng = np.random.default_rng(5)
    dev = torch.device("cuda")
    for d, bits, n_steps in ((12, 10, 1), (32, 12, 3), (32, 16, 1)):
        nb = 300
        n = nb * d
        buf = [torch.from_numpy(np.concatenate([[0.0], a]).astype(np.float32)).to(dev)
               for a in (rng.standard_normal(n) * 0.5, rng.uniform(0.3, 0.9, n),
                         rng.standard_normal(n), rng.uniform(0.5, 2.0, n))]
        al = [b[1:].clone() for b in buf]          # aligned copies
        un = [b[1:] for b in buf]                  # offset views: 4 bytes past a 256-B base
        assert un[0].data_ptr() % 16 == 4
        ia, sa = cwq.encode_blocks(*al, bits, n_steps, 42, block_dim=d)
        out_u = torch.empty(n + 1, dtype=torch.float32, device=dev)[1:]
        iu, su = cwq.encode_blocks(*un, bits, n_steps, 42, block_dim=d, out_sample=out_u)
        assert torch.equal(ia, iu)
        assert torch.equal(sa.view(torch.int32), su.view(torch.int32))
        da = cwq.decode_blocks(ia, al[2], al[3], bits, n_steps, 42, block_dim=d)
        dec_u = torch.empty(n + 1, dtype=torch.float32, device=dev)[1:]
        du = cwq.decode_blocks(ia, un[2], un[3], bits, n_steps, 42, block_dim=d,
                               out_sample=dec_u)
        assert torch.equal(da.view(torch.int32), sa.view(torch.int32))
        assert torch.equal(du.view(torch.int32), sa.view(torch.int32))
        h = [a.cpu().numpy() for a in al]
        for b in (0, nb - 1):
            sl = slice(b * d, (b + 1) * d)
            wi, ws = oracle.greedy_encode(h[0][sl], h[1][sl], h[2][sl], h[3][sl],
                                          np.array([0, d], np.int64), bits, n_steps, 42, 1.0, b)
            assert np.array_equal(wi.reshape(-1), ia[b].cpu().numpy())
            assert np.array_equal(_u32(ws), _u32(sa[sl].cpu().numpy()))


def test_c3_image_set(cwq, oracle):
    """C3: 24 images x (196,608 level-1 + 2,304 level-2 latents) through
    code_grouped_greedy_sample at 8 bits/group (pln.py:350, :463-472; the two
    levels as independent latent sets -- no trained SynthesisTransform_2 links
    them offline).  Images 0 and 23 against the oracle in full; every image:
    bitcode length = groups x 8 and a bit-exact decode round trip."""
    from compression_without_quantization_amd.synthetic import make_latents
    cwq.coded_greedy_sampler.VERBOSE = False
    thr = cwq.group_size_threshold(12)
    for i in range(24):
        for li, D in enumerate((32 * 48 * 128, 8 * 12 * 24)):
            q_loc, q_scale, p_loc, p_scale = make_latents(D, seed=1000 * i + li)
            target, proposal = cwq.Normal(q_loc, q_scale), cwq.Normal(p_loc, p_scale)
            sample, bitcode, starts = cwq.code_grouped_greedy_sample(None, target, proposal, 1,
                                                                     8, 42)
            assert starts[0] == 0 and starts[-1] == D
            assert len(bitcode) == (len(starts) - 1) * 8, f"image {i} level {li}"
            dec = cwq.decode_grouped_greedy_sample(None, bitcode, starts, proposal, 8, 1, 42)
            assert np.array_equal(_u32(dec), _u32(sample)), f"image {i} level {li} decode"
            if i in (0, 23):
                ws, wi, wst = oracle.code_grouped_greedy_sample(q_loc, q_scale, p_loc, p_scale,
                                                                1, 8, 42, thr)
                assert starts == wst, f"image {i} level {li} groups"
                assert bitcode == cwq.indices_to_bitcode(wi, 8), f"image {i} level {li} code"
                assert np.array_equal(_u32(sample), _u32(ws)), f"image {i} level {li} sample"


def test_c3_batch_equals_per_image_calls(cwq):
    """code_grouped_greedy_sample_batch over C3's 48 latent sets (24 images x 2
    levels, one encode launch over every image's groups with per-group seeds)
    equals 48 code_grouped_greedy_sample calls: groups, bitcode, sample bits."""
    from compression_without_quantization_amd.synthetic import make_latents
    cwq.coded_greedy_sampler.VERBOSE = False
    tg, pr = [], []
    for i in range(24):
        for li, D in enumerate((32 * 48 * 128, 8 * 12 * 24)):
            q_loc, q_scale, p_loc, p_scale = make_latents(D, seed=1000 * i + li)
            tg.append(cwq.Normal(q_loc, q_scale))
            pr.append(cwq.Normal(p_loc, p_scale))
    got = cwq.code_grouped_greedy_sample_batch(None, tg, pr, 1, 8, 42)
    assert len(got) == 48
    for k in (0, 1, 2, 17, 46, 47):
        sample, bitcode, starts = cwq.code_grouped_greedy_sample(None, tg[k], pr[k], 1, 8, 42)
        bs, bb, bst = got[k]
        assert isinstance(bst, np.ndarray) and bst.tolist() == starts, k
        assert bb == bitcode, k
        assert np.array_equal(_u32(bs), _u32(sample)), k


@pytest.mark.parametrize("sizes,seeds,bits,n_steps", [
    ([3000, 1, 20000, 257, 4096], [42, -7, 2 ** 31 - 3, 0, -2 ** 31], 8, 1),
    ([5000, 300, 6000], [1, 2, 3], 14, 3),   # multi-step: the forked stream parts
    ([2, 1, 3], 9, 6, 2),                    # tiny items, one seed for all
    ([0, 5, 0, 0, 700], [3, 4, 5, 6, 7], 8, 1),  # empty items (one empty group each)
    # >= 65,536 dims: the pipelined path (several chunks, empty and 1-dim items
    # inside chunks, a chunk boundary next to an empty item)
    ([70000, 0, 1, 30000, 0, 50000, 2, 40000, 3, 0], list(range(10)), 8, 1),
    ([40000, 30000, 20000, 5, 25000], [11, -12, 13, 14, 15], 12, 3),  # chunked multi-step
])
def test_grouped_batch_equals_single_calls(cwq, sizes, seeds, bits, n_steps):
    """Per-item seeds (int32 wrap-around included), items of 1 dim, and
    multi-step batches whose launch forks onto the library streams: each item's
    result equals code_grouped_greedy_sample on that item alone."""
    cwq.coded_greedy_sampler.VERBOSE = False
    rng = np.random.default_rng(sum(sizes) + bits)
    tg, pr = [], []
    for D in sizes:
        pl = (0.1 * rng.standard_normal(D)).astype(np.float32)
        ps = rng.uniform(0.8, 1.2, D).astype(np.float32)
        ql = (pl + ps * rng.standard_normal(D) * 0.7).astype(np.float32)
        qs = (ps * rng.uniform(0.3, 1.0, D)).astype(np.float32)
        tg.append(cwq.Normal(torch.from_numpy(ql).cuda(), torch.from_numpy(qs).cuda()))
        pr.append(cwq.Normal(torch.from_numpy(pl).cuda(), torch.from_numpy(ps).cuda()))
    got = cwq.code_grouped_greedy_sample_batch(None, tg, pr, n_steps, bits, seeds)
    assert cwq.code_grouped_greedy_sample_batch(None, [], [], n_steps, bits, seeds) == []
    sl = seeds if isinstance(seeds, list) else [seeds] * len(sizes)
    for k in range(len(sizes)):
        sample, bitcode, starts = cwq.code_grouped_greedy_sample(None, tg[k], pr[k], n_steps,
                                                                 bits, sl[k])
        bs, bb, bst = got[k]
        assert isinstance(bst, np.ndarray) and bst.tolist() == starts, k
        assert bb == bitcode, k
        assert np.array_equal(_u32(bs), _u32(sample)), k


def test_grouped_batch_deferred_overlapping_calls(cwq):
    """defer=True: three batches queued before any is collected (different
    items, seeds and sizes; the large one takes the pipelined path), collected
    out of order and twice, each equal to the synchronous call; an invalid
    batch raises from result(), and again on a second result()."""
    cwq.coded_greedy_sampler.VERBOSE = False
    rng = np.random.default_rng(77)

    def batch(sizes):
        tg, pr = [], []
        for D in sizes:
            pl = (0.1 * rng.standard_normal(D)).astype(np.float32)
            ps = rng.uniform(0.8, 1.2, D).astype(np.float32)
            ql = (pl + ps * rng.standard_normal(D) * 0.7).astype(np.float32)
            qs = (ps * rng.uniform(0.3, 1.0, D)).astype(np.float32)
            tg.append(cwq.Normal(torch.from_numpy(ql).cuda(), torch.from_numpy(qs).cuda()))
            pr.append(cwq.Normal(torch.from_numpy(pl).cuda(), torch.from_numpy(ps).cuda()))
        return tg, pr

    jobs = [(batch([3000, 1, 500, 0, 70000, 9000]), [5, -7, 2 ** 31 - 1, 0, 11, 12]),
            (batch([4000, 4000]), 42),
            (batch([123]), 9)]
    handles = [cwq.code_grouped_greedy_sample_batch(None, tg, pr, 1, 8, sd, defer=True)
               for (tg, pr), sd in jobs]
    assert cwq.code_grouped_greedy_sample_batch(None, [], [], 1, 8, 0, defer=True).result() == []
    for k in (2, 0, 1, 0):  # out of order, and one handle twice
        got = handles[k].result()
        (tg, pr), sd = jobs[k]
        want = cwq.code_grouped_greedy_sample_batch(None, tg, pr, 1, 8, sd)
        assert len(got) == len(want)
        for (gs, gb, gst), (ws, wb, wst) in zip(got, want):
            assert gb == wb and gst.tolist() == wst.tolist()
            assert np.array_equal(_u32(gs), _u32(ws))
    (tg, pr), _ = jobs[1]
    bad = cwq.code_grouped_greedy_sample_batch(None, tg, pr, 1, 40, 0, defer=True)
    for _ in range(2):
        with pytest.raises(Exception):
            bad.result()

    # synchronous calls on this thread while deferred batches are in flight: a
    # single-item batch and code_grouped_greedy_sample run here, on this
    # thread's page-locked staging, while the queued calls use their own
    (tg0, pr0), sd0 = jobs[0]
    (tg1, pr1), sd1 = jobs[1]
    want0 = cwq.code_grouped_greedy_sample_batch(None, tg0, pr0, 1, 8, sd0)
    want1 = cwq.code_grouped_greedy_sample_batch(None, tg1, pr1, 1, 8, sd1)
    one_want = cwq.code_grouped_greedy_sample_batch(None, tg1[:1], pr1[:1], 1, 8, 3)
    single_want = cwq.code_grouped_greedy_sample(None, tg0[0], pr0[0], 1, 8, 4)
    for _ in range(3):
        h0 = cwq.code_grouped_greedy_sample_batch(None, tg0, pr0, 1, 8, sd0, defer=True)
        h1 = cwq.code_grouped_greedy_sample_batch(None, tg1, pr1, 1, 8, sd1, defer=True)
        one = cwq.code_grouped_greedy_sample_batch(None, tg1[:1], pr1[:1], 1, 8, 3)
        single = cwq.code_grouped_greedy_sample(None, tg0[0], pr0[0], 1, 8, 4)
        for got, want in ((h0.result(), want0), (h1.result(), want1), (one, one_want)):
            for (gs, gb, gst), (ws, wb, wst) in zip(got, want):
                assert gb == wb and gst.tolist() == wst.tolist()
                assert np.array_equal(_u32(gs), _u32(ws))
        assert single[1] == single_want[1] and list(single[2]) == list(single_want[2])
        assert np.array_equal(_u32(single[0]), _u32(single_want[0]))
    # a handle dropped without result(): its buffers return to the pools once
    # its call ends, and its error (if any) is reported as a warning
    import gc
    import warnings
    from compression_without_quantization_amd import coded_greedy_sampler as S
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        dropped = cwq.code_grouped_greedy_sample_batch(None, tg, pr, 1, 40, 0, defer=True)
        del dropped
        gc.collect()
        cwq.code_grouped_greedy_sample_batch(None, tg1, pr1, 1, 8, sd1, defer=True).result()
    assert any("result() was never requested" in str(x.message) for x in w)
    assert len(S._pinned_free) >= 1 and len(S._bits_free) >= 1


def test_grouped_batch_many_items(cwq):
    """More items than the device partition keeps in LDS (1,024): 1,300 items
    of 0..200 dims (empty and 1-dim ones among them, ~130k dims: the pipelined
    path), each equal to code_grouped_greedy_sample on that item alone."""
    cwq.coded_greedy_sampler.VERBOSE = False
    rng = np.random.default_rng(1300)
    sizes = rng.integers(0, 201, 1300)
    sizes[::97] = 0
    sizes[5::89] = 1
    seeds = [int(x) for x in rng.integers(-2 ** 31, 2 ** 31, sizes.size)]
    tg, pr = [], []
    for D in sizes:
        pl = (0.1 * rng.standard_normal(D)).astype(np.float32)
        ps = rng.uniform(0.8, 1.2, D).astype(np.float32)
        ql = (pl + ps * rng.standard_normal(D) * 0.7).astype(np.float32)
        qs = (ps * rng.uniform(0.3, 1.0, D)).astype(np.float32)
        tg.append(cwq.Normal(torch.from_numpy(ql).cuda(), torch.from_numpy(qs).cuda()))
        pr.append(cwq.Normal(torch.from_numpy(pl).cuda(), torch.from_numpy(ps).cuda()))
    got = cwq.code_grouped_greedy_sample_batch(None, tg, pr, 1, 8, seeds)
    assert len(got) == sizes.size
    for k in range(sizes.size):
        sample, bitcode, starts = cwq.code_grouped_greedy_sample(None, tg[k], pr[k], 1, 8,
                                                                 seeds[k])
        bs, bb, bst = got[k]
        assert bst.tolist() == starts, k
        assert bb == bitcode, k
        assert np.array_equal(_u32(bs), _u32(sample)), k


@pytest.mark.parametrize("D,bits,n_steps", [(0, 8, 1), (1, 8, 1), (3000, 8, 1), (20000, 10, 2),
                                             (9000, 14, 3)])
def test_grouped_two_halves_equal_one_shot(cwq, cwqlib, D, bits, n_steps):
    """code_grouped_greedy_sample takes cwq_code_grouped_greedy_begin / _end
    (the group-start list is built while the device codes) unless the caller
    asks the library to time the encode (eval_ms_out: the one-shot call); both
    give the same sample, bitcode and starts, also for D = 0 and 1 and
    multi-step groups on the forked streams.  _begin refuses eval_ms_out."""
    import ctypes
    cwq.coded_greedy_sampler.VERBOSE = False
    rng = np.random.default_rng(D + bits)
    pl = (0.1 * rng.standard_normal(D)).astype(np.float32)
    ps = rng.uniform(0.8, 1.2, D).astype(np.float32)
    ql = (pl + ps * rng.standard_normal(D) * 0.7).astype(np.float32)
    qs = (ps * rng.uniform(0.3, 1.0, D)).astype(np.float32)
    tg = cwq.Normal(torch.from_numpy(ql).cuda(), torch.from_numpy(qs).cuda())
    pr = cwq.Normal(torch.from_numpy(pl).cuda(), torch.from_numpy(ps).cuda())
    a = cwq.code_grouped_greedy_sample(None, tg, pr, n_steps, bits, 42)
    ms = ctypes.c_float(-1.0)
    b = cwq.code_grouped_greedy_sample(None, tg, pr, n_steps, bits, 42, eval_ms_out=ms)
    assert a[2] == b[2] and isinstance(a[2], list)
    assert a[1] == b[1]
    assert np.array_equal(_u32(a[0]), _u32(b[0]))
    assert len(a[1]) == (len(a[2]) - 1) * n_steps * bits
    if D > 0:
        assert ms.value >= 0.0
    # the C ABI: eval_ms_out is refused by _begin (it returns before the encode ends)
    from compression_without_quantization_amd import _lib
    ws = torch.empty(max(1, int(cwqlib.cwq_code_grouped_greedy_workspace_size(16, 1))),
                     dtype=torch.uint8, device="cuda")
    x = torch.ones(16, device="cuda")
    sample = np.empty(16, np.float32)
    idx = np.empty(17, np.int32)
    starts = np.empty(18, np.int64)
    rc = cwqlib.cwq_code_grouped_greedy_begin(
        x.data_ptr(), x.data_ptr(), x.data_ptr(), x.data_ptr(), 16, 1, 8, 42, 1.0, 4095, 4.5,
        sample.ctypes.data, idx.ctypes.data, 17, starts.ctypes.data, 18, None, ws.data_ptr(),
        ws.numel(), _lib.options(None, None, ctypes.c_float(0.0)),
        torch.cuda.current_stream().cuda_stream)
    assert rc < 0
    assert b"eval_ms_out" in cwqlib.cwq_last_error()


def _bench(args, timeout=300):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-u", os.path.join(REPO, "bench.py")] + args,
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_launches_two_ranks_itself(cwq):
    """`bench.py --gpus 2` with no launcher environment starts two rank
    processes (here sharing the one GPU over gloo), codes 8192 C4 blocks split
    between them (strong scaling) and checks every rank's sample against the
    oracle: one JSON line with n_gpus == 2 and no mismatch."""
    line = _bench(["--gpus", "2", "--blocks", "8192", "--steps", "1", "--warmup", "0",
                   "--no-e2e"])
    assert line["n_gpus"] == 2 and line["config"]["world_size_checked"] == 2
    assert line["scaling"] == "strong"
    assert line["config"]["blocks_total"] == 8192 and line["config"]["blocks_per_gpu"] == 4096
    _check_shards(line, 2, 8192)
    assert line["parity"]["index_mismatches"] == 0
    assert line["parity"]["sample_word_mismatches"] == 0
    assert line["parity"]["blocks_checked"] >= 2 * 16
    assert line["decode_roundtrip_bit_exact"] is True
    assert line["value"] > 0
    # rank -> device map in the line (both ranks on the box's one GPU: gloo)
    rd = line["config"]["rank_devices"]
    assert [m["rank"] for m in rd] == [0, 1] and line["config"]["backend"] == "gloo"
    # the N > 1 roofline is the job's: both shards' bytes over the slower kernel
    rf = line["roofline"]
    assert rf["scope"].startswith("all 2 GPUs")
    assert rf["algorithmic_bytes_per_launch"] == 8192 * (20 * 32 + 4)
    assert rf["rank0"]["algorithmic_bytes_per_launch"] == 4096 * (20 * 32 + 4)
    assert rf["kernel_ms"] == line["eval_kernel_ms_max_over_ranks"]


def _ragged_gather_worker(rank, world, port, q):
    """One rank of test_ragged_shards_gathered: codes its cost-balanced shard of
    ragged CSR groups on the GPU and all-gathers the indices (gloo, CPU)."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import compression_without_quantization_amd as C
    from compression_without_quantization_amd.parallel import gather_indices, shard_range
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tl, ts, pl, ps, off, bits, n_steps = _ragged_set()
    nb = off.size - 1
    cost = np.diff(off).astype(np.float64) * (1 << bits) * n_steps
    b0, b1 = shard_range(nb, world, rank, cost)
    a, b = int(off[b0]), int(off[b1])
    if b1 > b0:
        idx, _ = C.encode_blocks(tl[a:b], ts[a:b], pl[a:b], ps[a:b], bits, n_steps, 42,
                                 block_off=off[b0:b1 + 1] - a, block_id_base=b0)
        local = idx.cpu()
    else:
        local = torch.zeros((0, n_steps), dtype=torch.int32)
    full = gather_indices(local)
    if rank == 0:
        q.put((b1 - b0, full.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _ragged_set():
    rng = np.random.default_rng(5)
    sizes = np.concatenate([rng.integers(1, 40, 300), [2000, 1], rng.integers(1, 9, 200)])
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    D = int(off[-1])
    tl = rng.standard_normal(D).astype(np.float32)
    ts = rng.uniform(0.3, 0.9, D).astype(np.float32)
    pl = (0.1 * rng.standard_normal(D)).astype(np.float32)
    ps = rng.uniform(0.8, 1.2, D).astype(np.float32)
    return tl, ts, pl, ps, off, 10, 2


def test_ragged_shards_gathered(cwq):
    """Three ranks sharing the GPU (gloo) code cost-balanced, unequal shards of
    ragged groups (1 .. 2000 dims) with block_id_base = their first group, and
    parallel.gather_indices (which pads and trims internally) returns exactly
    the indices of one single-process encode of all groups."""
    import socket
    import torch.multiprocessing as mp
    tl, ts, pl, ps, off, bits, n_steps = _ragged_set()
    want, _ = cwq.encode_blocks(tl, ts, pl, ps, bits, n_steps, 42, block_off=off)
    want = want.cpu().numpy()
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ragged_gather_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    n0, got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert 0 < n0 < off.size - 1  # rank 0's shard is a strict part: shards are unequal
    assert np.array_equal(got, want)


def _check_shards(line, world, nb_total):
    sh = line["config"]["shards"]
    assert len(sh) == world
    assert sh[0][0] == 0 and sh[-1][1] == nb_total
    for (a0, a1), (b0, b1) in zip(sh[:-1], sh[1:]):
        assert a1 == b0 and a0 < a1  # contiguous, non-empty, in rank order


@pytest.mark.parametrize("config,blocks,check", [("c4", 8192, 4), ("c5", 64, 1)])
def test_bench_eight_ranks_rehearsal(cwq, config, blocks, check):
    """The scaling target's N = 8 on the box's one GPU: `bench.py --gpus 8`
    starts its eight ranks itself (gloo: they share the device), cuts the
    block set into 8 contiguous shards coded with block_id_base = their first
    block (coded_greedy_sampler.py:282, seed + g), all-reduces the timing and
    the oracle checks of every rank (first, last and evenly spaced blocks of
    its shard): one line, world size 8, no mismatch.  C4-shaped (16 bits) and
    C5-shaped (2^24 candidates per block, the multi-tile blocks) cases."""
    line = _bench(["--gpus", "8", "--config", config, "--blocks", str(blocks), "--steps", "1",
                   "--warmup", "0", "--no-e2e", "--check-blocks", str(check)], timeout=600)
    assert line["n_gpus"] == 8 and line["config"]["world_size_checked"] == 8
    assert line["scaling"] == "strong" and line["config"]["blocks_total"] == blocks
    _check_shards(line, 8, blocks)
    assert [m["rank"] for m in line["config"]["rank_devices"]] == list(range(8))
    assert line["parity"]["index_mismatches"] == 0
    assert line["parity"]["sample_word_mismatches"] == 0
    assert line["parity"]["blocks_checked"] >= 8 * 2
    assert line["decode_roundtrip_bit_exact"] is True
    assert line["roofline"]["scope"].startswith("all 8 GPUs")


def test_bench_weak_scaling_two_ranks(cwq):
    line = _bench(["--gpus", "2", "--blocks", "2048", "--steps", "1", "--warmup", "0",
                   "--no-e2e", "--scaling", "weak", "--config", "c4"])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["blocks_total"] == 4096 and line["config"]["blocks_per_gpu"] == 2048
    assert line["parity"]["index_mismatches"] == 0


@pytest.mark.parametrize("nb,d,chunk,n_steps,base", [
    (1000, 32, 256, 1, 0),      # 4 chunks, the last one partial
    (700, 8, 1000, 2, 5),       # one chunk larger than the job
    (513, 16, 64, 1, 77),       # many chunks: both slots reused repeatedly
    (3, 32, 1, 3, 0),           # one block per chunk
])
def test_encode_blocks_host_streamed_equals_one_call(cwq, nb, d, chunk, n_steps, base):
    """encode_blocks_host (copies straight from and to the caller's pageable
    arrays on a copy stream, coding on the compute stream, two device buffer
    slots; chunk c coded with block_id_base = base + c * chunk) equals one
    encode_blocks call over all blocks, bit for bit."""
    rng = np.random.default_rng(nb * d + chunk)
    tl = rng.standard_normal(nb * d).astype(np.float32)
    ts = rng.uniform(0.3, 0.9, nb * d).astype(np.float32)
    pl = (0.1 * rng.standard_normal(nb * d)).astype(np.float32)
    ps = rng.uniform(0.8, 1.2, nb * d).astype(np.float32)
    bits = 12
    gi, gs = cwq.encode_blocks(tl, ts, pl, ps, bits, n_steps, 42, block_dim=d,
                               block_id_base=base)
    hi, hs = cwq.encode_blocks_host(tl, ts, pl, ps, bits, n_steps, 42, d, block_id_base=base,
                                    chunk_blocks=chunk)
    assert hi.shape == (nb, n_steps) and hs.shape == (nb * d,)
    assert np.array_equal(hi, gi.cpu().numpy())
    assert np.array_equal(hs.view(np.uint32), gs.cpu().numpy().view(np.uint32))


def test_grouped_batch_errors_and_pageable_staging(cwq):
    """cwq_code_grouped_greedy_batch through ctypes: a short host workspace or
    bits buffer is refused (CWQ_ERR_WORKSPACE / CWQ_ERR_CAPACITY) and the call
    returns with no device work outstanding; with no host workspace (library
    pageable staging) the results equal the pinned path's."""
    import ctypes
    from compression_without_quantization_amd import _lib
    from compression_without_quantization_amd.coded_greedy_sampler import group_size_threshold
    lib = _lib.load()
    rng = np.random.default_rng(9)
    sizes = [50000, 3, 30000, 0, 20000]
    D, n = sum(sizes), len(sizes)
    cat = []
    pl = (0.1 * rng.standard_normal(D)).astype(np.float32)
    ps = rng.uniform(0.8, 1.2, D).astype(np.float32)
    ql = (pl + ps * rng.standard_normal(D) * 0.7).astype(np.float32)
    qs = (ps * rng.uniform(0.3, 1.0, D)).astype(np.float32)
    cat = [torch.from_numpy(x).cuda() for x in (ql, qs, pl, ps)]
    item_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    seeds = np.arange(n, dtype=np.int32)
    ws = torch.empty(lib.cwq_code_grouped_greedy_batch_workspace_size(D, n, 1), dtype=torch.uint8,
                     device="cuda")
    hneed = lib.cwq_code_grouped_greedy_batch_host_workspace_size(D, n, 1)
    hws = torch.empty(hneed, dtype=torch.uint8, pin_memory=True)

    def call(bits_cap, host_ws, host_bytes, opts=None):
        sample = np.empty(D, np.float32)
        bits = np.empty(max(bits_cap, 1), np.uint8)
        starts = np.empty(D + 2 * n, np.int64)
        bits_off = np.empty(n + 1, np.int64)
        n_starts = np.empty(n, np.int64)
        rc = lib.cwq_code_grouped_greedy_batch(
            n, item_off.ctypes.data, cat[0].data_ptr(), cat[1].data_ptr(), cat[2].data_ptr(),
            cat[3].data_ptr(), 1, 8, seeds.ctypes.data, 1.0, group_size_threshold(12),
            8 * np.log(2) - 1, sample.ctypes.data, bits.ctypes.data, bits_cap,
            bits_off.ctypes.data, starts.ctypes.data, starts.size, n_starts.ctypes.data,
            ws.data_ptr(), ws.numel(), host_ws, host_bytes, opts,
            torch.cuda.current_stream().cuda_stream)
        return rc, sample, bits[:bits_off[-1]].tobytes() if rc >= 0 else b"", starts, n_starts
    rc, s1, b1, st1, n1 = call((D + n) * 8, hws.data_ptr(), hneed)
    assert rc > 0
    rc2, s2, b2, st2, n2 = call((D + n) * 8, None, 0)  # pageable library staging
    assert rc2 == rc and b2 == b1 and np.array_equal(s2.view(np.uint32), s1.view(np.uint32))
    assert np.array_equal(n2, n1)
    rc3 = call((D + n) * 8, hws.data_ptr(), hneed - 1)[0]
    assert rc3 == -3 and b"host workspace" in lib.cwq_last_error()
    rc4 = call(100, hws.data_ptr(), hneed)[0]  # bits buffer far too small
    assert rc4 == -4 and b"bits_cap" in lib.cwq_last_error()
    # item_ready: every flag raised on success (results unchanged), not all on an error
    ready = np.zeros(n, np.int32)
    rc5, s5, b5, _, _ = call((D + n) * 8, hws.data_ptr(), hneed,
                             _lib.options(item_ready=ready.ctypes.data))
    assert rc5 == rc and b5 == b1 and np.array_equal(s5.view(np.uint32), s1.view(np.uint32))
    assert ready.tolist() == [1] * n
    ready[:] = 0
    assert call(100, hws.data_ptr(), hneed, _lib.options(item_ready=ready.ctypes.data))[0] == -4
    assert ready.sum() < n
    torch.cuda.synchronize()
    rc6, s6, b6, _, _ = call((D + n) * 8, hws.data_ptr(), hneed)  # the library still works
    assert rc6 == rc and b6 == b1


def test_grouped_batch_wrapper_raises_from_helper_thread(cwq):
    """code_grouped_greedy_sample_batch runs the native call on a helper thread
    for several items: a failing call still raises CwqError with the library's
    message (read on the thread that made the call), and the next call works."""
    from compression_without_quantization_amd import _lib
    rng = np.random.default_rng(3)
    items = []
    for D in (3000, 2000):
        pl = (0.1 * rng.standard_normal(D)).astype(np.float32)
        ps = rng.uniform(0.8, 1.2, D).astype(np.float32)
        ql = (pl + 0.5 * ps * rng.standard_normal(D)).astype(np.float32)
        qs = (ps * rng.uniform(0.3, 1.0, D)).astype(np.float32)
        items.append((cwq.Normal(torch.from_numpy(ql).cuda(), torch.from_numpy(qs).cuda()),
                      cwq.Normal(torch.from_numpy(pl).cuda(), torch.from_numpy(ps).cuda())))
    tg, pr = [t for t, _ in items], [p for _, p in items]
    with pytest.raises(_lib.CwqError, match="prune_mode"):
        cwq.code_grouped_greedy_sample_batch(None, tg, pr, 1, 8, 5, prune_mode=7)
    out = cwq.code_grouped_greedy_sample_batch(None, tg, pr, 1, 8, 5)
    for (t, p), (sample, bitcode, starts) in zip(items, out):
        s1, b1, st1 = cwq.code_grouped_greedy_sample(None, t, p, 1, 8, 5)
        assert bitcode == b1 and list(starts) == list(st1)
        assert np.array_equal(sample.view(np.uint32), np.asarray(s1).view(np.uint32))


def test_grouped_batch_wrapper_argument_forms(cwq):
    """The batch wrapper's fast argument path (float32 CUDA tensors, one
    torch.cat per column) and its general path give the same results: 1-D and
    multi-dim items of different shapes, numpy items, a mix; float64 inputs
    and size mismatches raise as the single call does."""
    rng = np.random.default_rng(17)
    shapes = [(1, 4, 6, 8), (1, 2, 3, 5), (700,)]
    arrs = []
    for shp in shapes:
        n = int(np.prod(shp))
        pl = (0.1 * rng.standard_normal(n)).astype(np.float32).reshape(shp)
        ps = rng.uniform(0.8, 1.2, n).astype(np.float32).reshape(shp)
        ql = (pl + 0.5 * ps * rng.standard_normal(shp)).astype(np.float32)
        qs = (ps * rng.uniform(0.3, 1.0, shp)).astype(np.float32)
        arrs.append((ql, qs, pl, ps))

    def run(conv):
        tg = [cwq.Normal(conv(a[0]), conv(a[1])) for a in arrs]
        pr = [cwq.Normal(conv(a[2]), conv(a[3])) for a in arrs]
        return cwq.code_grouped_greedy_sample_batch(None, tg, pr, 1, 8, 11)
    def same(r0, r1):
        for (s0, b0, st0), (s1, b1, st1) in zip(r0, r1):
            assert b0 == b1 and np.array_equal(st0, st1)
            assert np.array_equal(np.asarray(s0).view(np.uint32), np.asarray(s1).view(np.uint32))
    flat = run(lambda x: torch.from_numpy(x.reshape(-1).copy()).cuda())  # 1-D tensors
    same(flat, run(lambda x: torch.from_numpy(x).cuda()))  # multi-dim, shapes differ
    same(flat, run(lambda x: x))                           # numpy arrays
    # non-contiguous views code their logical (flattened) order
    tr = lambda x: torch.from_numpy(x).cuda().transpose(0, -1)  # noqa: E731
    same(run(lambda x: tr(x).reshape(-1).contiguous()), run(tr))
    tg = [cwq.Normal(torch.from_numpy(a[0]).cuda().double(), torch.from_numpy(a[1]).cuda())
          for a in arrs]
    pr = [cwq.Normal(torch.from_numpy(a[2]).cuda(), torch.from_numpy(a[3]).cuda()) for a in arrs]
    with pytest.raises(Exception, match="float32"):
        cwq.code_grouped_greedy_sample_batch(None, tg, pr, 1, 8, 11)
    tg = [cwq.Normal(torch.from_numpy(a[0]).cuda(), torch.from_numpy(a[1]).cuda()) for a in arrs]
    pr[1] = cwq.Normal(torch.from_numpy(arrs[1][2][..., :-1].copy()).cuda(),
                       torch.from_numpy(arrs[1][3][..., :-1].copy()).cuda())
    with pytest.raises(ValueError, match="same size"):
        cwq.code_grouped_greedy_sample_batch(None, tg, pr, 1, 8, 11)
