"""Benchmark: latent blocks encoded/s at KL=16 bits (BASELINE.json metric).

One "step" = one greedy-coding pass (code_greedy_sample semantics, 2^16
candidates per block, n_steps=1) over the job's synthetic blocks (config C4:
10^6 blocks x d=32), inputs resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c5|c1|...]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

With --gpus N > 1 and no launcher environment, bench.py starts the N rank
processes itself (one per GPU; the parent never touches the GPU).  Block
configs at N > 1 default to strong scaling: the config's block set (10^6 for
C4) is cut into N contiguous shards (parallel.shard_range), each coded with
block_id_base = its first global block, so every block's seed and result are
those of the single-GPU run (coded_greedy_sampler.py:282); --scaling weak
gives every rank the config's block count instead.  No collective touches the
data path: RCCL carries only the start/stop barriers and the max-reduce of
the step time (gloo when ranks share one device).

c4 (default) is BASELINE.json's metric; c5/c1 are the other block configs;
c2/c3 time the whole grouped greedy pipeline per image (code_grouped_greedy_sample)
and i1/i2 the grouped importance pipeline.

Rank 0 prints one JSON line.  `roofline` prices the dominant kernel (the
candidate-scoring eval kernel, timed with HIP events on its launch stream);
`cpu_baseline` times the CPU oracle (oracle/, a restatement of the reference's
semantics -- the TF1 reference cannot run here) on a bounded sample of the
same workload and checks the GPU's indices/samples on that sample bit-exactly
(at N > 1 every rank checks a sample of its shard instead).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import compression_without_quantization_amd as C  # noqa: E402
from compression_without_quantization_amd import _lib  # noqa: E402
from compression_without_quantization_amd.parallel import shard_range  # noqa: E402
from compression_without_quantization_amd.synthetic import DEFAULT_SEED, make_blocks_range  # noqa

GROUPED = {
    # name: (images, [latent dims per image], bits/step, description[, n_steps])
    "c2": (1, [32 * 48 * 128], 8,
           "C2: one 512x768 image, PLN level-1 latents (196,608 dims), 8 bits/group"),
    "c3": (24, [32 * 48 * 128, 8 * 12 * 24], 8,
           "C3: 24 images x (196,608 + 2,304) dims, both ladder levels, 8 bits/group"),
    "c2cli": (1, [32 * 48 * 128], 14,
              "C2 at the CLI's greedy defaults: 196,608 dims, n_steps=30 x 14 bits/step "
              "(miracle_arguments.py:159-165)", 30),
    "c2low": (1, [32 * 48 * 128], 14,
              "C2 at the CLI's greedy defaults, low-rate latents (0.06 bits/dim, the PLN "
              "bench's level 1): ~50 groups of up to 4095 dims, n_steps=30 x 14 bits/step",
              30, 0.06),
}
IMPORTANCE = {
    # name: (images, latent dims, n_bits_per_group, max_group_size_bits, dim_kl_bit_limit, desc)
    "i1": (1, 32 * 48 * 128, 20, 4, 16,
           "I1: one image's PLN level-1 latents (196,608 dims), grouped importance coder, "
           "20 bits/group, groups <= 16 dims (miracle_arguments.py:177-183)"),
    "i2": (24, 8 * 12 * 24, 20, 2, 16,
           "I2: 24 images' PLN level-2 latents (2,304 dims each), grouped importance coder, "
           "20 bits/group, groups <= 4 dims (miracle_arguments.py:168-174)"),
}
PLN = {
    # name: (images, H, W, level-1 coder, description)
    "pln": (1, 512, 768, "greedy",
            "PLN image codec: one 512x768 image, both levels (level 2 importance 20 bits/group, "
            "level 1 greedy 30 x 14 bits), group sizes arithmetic-coded, .miracle file "
            "(miracle.py compress/decompress defaults, miracle_arguments.py:146-189)"),
    "pln_is": (1, 512, 768, "importance",
               "PLN image codec, level 1 through the importance coder (--use_importance_sampling: "
               "20 bits/group, groups <= 16 dims), level 2 as pln; the path the reference's "
               "kodim05 timings most likely used (SURVEY.md 6)"),
}
CONFIGS = {
    # name: (blocks per GPU, block dim, kl bits, n_steps, description)
    "c4": (1_000_000, 32, 16, 1, "C4: 1e6 blocks x d=32, KL=16 bits (2^16 candidates/block)"),
    "c5": (1024, 16, 24, 1, "C5: 1024 blocks x d=16, KL=24 bits (2^24 candidates/block)"),
    "c1": (4096, 8, 4, 1, "C1 shape batched: d=8, KL=4 bits"),
}
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults per config (None): the block configs 3 steps after 1 warmup (C4: ~0.3 s a
    # step); the grouped, importance and PLN configs 20 after 3 (a step is 0.5-55 ms, and
    # their first steps grow torch's pinned-memory cache for the results they return)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--config", default="c4",
                    choices=sorted(CONFIGS) + sorted(GROUPED) + sorted(IMPORTANCE) + sorted(PLN))
    ap.add_argument("--blocks", type=int, default=0, help="override the config's block count (the whole job under strong scaling, "
                         "per rank under weak)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--per-image", action="store_true",
                    help="grouped configs: time one call per latent set only (no batched call)")
    ap.add_argument("--batch-only", action="store_true",
                    help="grouped configs of several latent sets: time the batched call only "
                         "(profiling runs: every scoring dispatch belongs to it)")
    ap.add_argument("--prune-mode", type=int, default=2, choices=(0, 1, 2),
                    help="0 unpruned, 1 exact pruning, 2 pruning + screening (default)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default=None,
                    help="block configs at N > 1: strong (default; the config's block set "
                         "split over the ranks) or weak (that many blocks per rank)")
    ap.add_argument("--check-blocks", type=int, default=16,
                    help="N > 1: blocks per rank checked against the CPU oracle")
    ap.add_argument("--rank-timeout", type=float,
                    default=float(os.environ.get("CWQ_BENCH_RANK_TIMEOUT", "480")),
                    help="N > 1: wall-clock seconds the ranks may take in all (the parent "
                         "stops ranks still running then and exits 124); also the process "
                         "group's timeout for its collectives")
    args = ap.parse_args()
    block = args.config in CONFIGS
    if args.steps is None:
        args.steps = 3 if block else 20
    if args.warmup is None:
        args.warmup = 1 if block else 3
    return args


def grouped_main(args):
    """C2/C3: the whole grouped pipeline per image (code_grouped_greedy_sample):
    standardise + KL on the GPU, host grouping, encode, bitcode.  Synthetic
    PLN-like latents (no Kodak images or checkpoints offline).  The line's
    roofline prices the candidate-scoring launches (HIP events recorded by the
    library around them, every call of the timed steps), cpu_baseline the
    oracle on image 0's latent sets (a prefix of its groups where the whole set
    would take too long)."""
    import compression_without_quantization_amd.coded_greedy_sampler as S
    from compression_without_quantization_amd.synthetic import make_latents
    S.VERBOSE = False
    n_img, dims, bits, desc = GROUPED[args.config][:4]
    n_steps = GROUPED[args.config][4] if len(GROUPED[args.config]) > 4 else 1
    bpd = GROUPED[args.config][5] if len(GROUPED[args.config]) > 5 else 1.1
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lat, lat_np = [], []
    for i in range(n_img):
        for li, D in enumerate(dims):
            q_loc, q_scale, p_loc, p_scale = make_latents(D, bits_per_dim=bpd, seed=1000 * i + li)
            if i == 0:
                lat_np.append((q_loc, q_scale, p_loc, p_scale))
            lat.append((C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev)),
                        C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev))))
    import ctypes
    evq = []  # the timed calls' scoring-launch milliseconds (cwq_options.eval_ms_out)
    evp = []  # single calls: (start, stop) events recorded around their scoring launches

    def ev():
        v = ctypes.c_float(0.0)
        evq.append(v)
        return v

    pool = []  # pre-made event pairs, taken in order by the timed single calls

    def make_pairs(n):
        pool.clear()
        for _ in range(n):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            b.record()  # materialise the hipEvent_t handles
            pool.append((a, b))
        pool.reverse()

    def ev_pair():
        a, b = pool.pop()
        evp.append((a, b))
        return a.cuda_event, b.cuda_event

    def step_single(timed_events=False):  # one code_grouped_greedy_sample call per latent set
        # (caller events, so the call takes its two-half path: eval_ms_out would
        # make it synchronous)
        out = []
        pairs = [ev_pair() if timed_events else None for _ in lat]
        for (target, proposal), pe in zip(lat, pairs):
            out.append(C.code_grouped_greedy_sample(None, target, proposal, n_steps, bits, 42,
                                                    eval_events=pe))
        return out

    def step_batch(timed_events=False):  # every latent set of the step in one batched call
        return C.code_grouped_greedy_sample_batch(None, [t for t, _ in lat], [p for _, p in lat],
                                                  n_steps, bits, 42,
                                                  eval_ms_out=ev() if timed_events else None)

    def timed(step):
        """(seconds for args.steps steps, results, scoring ms per step).  The
        steps are timed without the scoring timers; a second pass of the same
        steps records them (timing events between the chunks of a batched call
        cost C3 ~0.6 ms per step of host/device sync)."""
        res = None
        for _ in range(args.warmup):
            # hold each result as the timed loop does: a call then runs while the
            # previous call's results (page-locked host memory) are still alive,
            # so the pinned cache reaches its steady two blocks during warmup
            res = step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        per = []
        for _ in range(args.steps):
            res = step()
            per.append(time.perf_counter())
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if os.environ.get("CWQ_BENCH_STEP_TIMES"):  # diagnostics: each step's wall time
            print("step ms:", " ".join(f"{(b - a) * 1e3:.2f}" for a, b in zip([t0] + per, per)),
                  file=sys.stderr, flush=True)
        if step is step_single:
            make_pairs(args.steps * len(lat))
        evq.clear()
        evp.clear()
        for _ in range(args.steps):
            step(True)
        torch.cuda.synchronize()
        kms = (sum(v.value for v in evq) + sum(a.elapsed_time(b) for a, b in evp)) / \
            max(args.steps, 1)
        return el, res, kms

    batch = len(lat) > 1 and not args.per_image
    if batch and args.batch_only:
        el, res, kernel_ms = timed(step_batch)
        batched = {"latent_sets_per_call": len(lat), "equal_to_single_calls": None,
                   "single_call_images_per_s": None}
    else:
        el_single, res, kms_single = timed(step_single)
        el, kernel_ms = el_single, kms_single
        batched = None
    if batch and not args.batch_only:
        el, res_b, kernel_ms = timed(step_batch)
        same = all(list(a[2]) == list(b[2]) and a[1] == b[1] and
                   np.array_equal(np.asarray(a[0]).view(np.uint32), np.asarray(b[0]).view(np.uint32))
                   for a, b in zip(res, res_b))
        batched = {"latent_sets_per_call": len(lat), "equal_to_single_calls": bool(same),
                   "single_call_images_per_s": n_img * args.steps / el_single,
                   "single_call_scoring_kernel_ms": round(kms_single, 4)}
        if not same:
            raise SystemExit("bench.py: batched results differ from the single calls")
    if batch:
        # the same steps with the calls pipelined two deep (defer=True: step k + 1
        # is queued before step k's results are collected), so the host work
        # between calls overlaps the device work; reported beside value
        def step_deferred():
            return C.code_grouped_greedy_sample_batch(None, [t for t, _ in lat],
                                                      [p for _, p in lat], n_steps, bits, 42,
                                                      defer=True)

        def pipelined(k):
            h = step_deferred()
            out = None
            for _ in range(k - 1):
                h2 = step_deferred()
                out = h.result()
                h = h2
            return h.result() if k > 0 else out

        pipelined(max(args.warmup, 10))  # two calls in flight: more page-locked blocks to warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res_p = pipelined(args.steps)
        torch.cuda.synchronize()
        el_p = time.perf_counter() - t0
        same_p = all(list(a[2]) == list(b[2]) and a[1] == b[1] and
                     np.array_equal(np.asarray(a[0]).view(np.uint32),
                                    np.asarray(b[0]).view(np.uint32))
                     for a, b in zip(res, res_p))
        if not same_p:
            raise SystemExit("bench.py: pipelined batched results differ")
        batched["pipelined_images_per_s"] = n_img * args.steps / el_p
        batched["pipelined_ms_per_step"] = el_p / args.steps * 1e3
        batched["pipelined_note"] = ("defer=True, two calls in flight; the same results as the "
                                     "synchronous calls (checked); not value")
    groups = sum(len(r[2]) - 1 for r in res)
    bitlen = sum(len(r[1]) for r in res)
    D_step = sum(int(t.loc.numel()) for t, _ in lat)
    # SURVEY.md 8(d) per group: 16 d (four f32 inputs) + 4 n_steps (indices) + 4 d (sample)
    alg = 20 * D_step + 4 * groups * n_steps
    cand_dims = (1 << bits) * n_steps * D_step
    small = 64 <= (1 << bits) < 4096
    roofline = scoring_roofline(
        args.config, groups, alg, kernel_ms, cand_dims,
        ("k_small_prep1 + k_small_one + k_small_finalize (the small-candidate pipeline, "
         "DESIGN.md 5e; k_small_one dominant)" if small else
         "k_csr_prep + k_encode_prune_csr (+ finalize between steps)"),
        "HIP events recorded on the launch stream around the candidate-scoring launches: the "
        "caller's cwq_options events for single calls, cwq_options.eval_ms_out (per "
        "pipelined chunk) for the batched call; summed over the calls of a step, in a second "
        "pass of the timed steps (value and ms_per_step come from the pass without timers)")
    cpu = parity = None
    if not args.no_cpu:
        cpu, parity = grouped_cpu_baseline(args, lat_np, res[:len(dims)], bits, n_steps)
    line = {"metric": "images coded/s (grouped greedy pipeline)", "value": n_img * args.steps / el,
            "unit": "images/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic PLN-like latents",
            "config": {"workload": desc, "groups_per_step": groups, "bits_per_step": bitlen,
                       "groups_per_s": groups * args.steps / el,
                       "mode": ("code_grouped_greedy_sample_batch: every latent set of a step "
                                "in one call" if batched else
                                "one code_grouped_greedy_sample call per latent set"),
                       "batched": batched},
            "roofline": roofline, "cpu_baseline": cpu, "parity": parity}
    print(json.dumps(line), flush=True)


def grouped_cpu_baseline(args, lat_np, res0, bits, n_steps):
    """The CPU oracle on image 0 of a grouped config (its latent sets lat_np,
    the GPU's results res0 for them): the whole pipeline
    (oracle.code_grouped_greedy_sample) where image 0 fits ~cpu_seconds on
    every usable CPU, else the coder on a prefix of each set's groups (the
    GPU's partition) with the rate scaled by the prefix's share of the image's
    candidate-dims.  The sampled groups' indices and sample words are checked
    against the GPU's."""
    from oracle import oracle as O
    from compression_without_quantization_amd.binary_io import bitcode_to_indices
    from compression_without_quantization_amd.coded_greedy_sampler import group_size_threshold
    ncpu, quota = affinity_cores()
    nthr = min(ncpu, int(np.ceil(quota))) if quota else ncpu
    thr = group_size_threshold(12)
    sets = []
    for (ql, qs, pl, ps), (gs, gcode, gst) in zip(lat_np, res0):
        st = np.asarray(gst, dtype=np.int64)
        gidx = bitcode_to_indices(gcode, bits, (st.size - 1) * n_steps).reshape(-1, n_steps)
        sets.append((ql, qs, pl, ps, np.asarray(gs), gidx, st))
    work = [float(np.diff(st).sum()) * (1 << bits) * n_steps for *_, st in sets]

    def prefix(k_frac, threads):
        """Code the first k_frac of each set's groups; (seconds, cand-dims, mism)."""
        t_all = cd = 0.0
        mi = ms = 0
        for (ql, qs, pl, ps, gs, gidx, st) in sets:
            G = st.size - 1
            k = max(1, int(round(G * k_frac)))
            e = int(st[k])
            tl, ts = O.standardise(ql[:e], qs[:e], pl[:e], ps[:e])
            c0 = time.perf_counter()
            wi, wsm = O.greedy_encode(tl, ts, np.zeros(e, np.float32), np.ones(e, np.float32),
                                      st[:k + 1], bits, n_steps, 42, 1.0, 0, threads)
            t_all += time.perf_counter() - c0
            smp = O.destandardise(wsm, pl[:e], ps[:e])
            mi += int((wi != gidx[:k]).sum())
            ms += int((smp.view(np.uint32) != gs[:e].view(np.uint32)).sum())
            cd += float(e) * (1 << bits) * n_steps
        return t_all, cd, mi, ms
    # calibrate on ~1% of the groups, then size the sample to ~cpu_seconds
    dt, cd, _, _ = prefix(0.01, nthr)
    full_s = dt * sum(work) / max(cd, 1.0)
    if full_s <= args.cpu_seconds:
        # the whole image, repeated to ~3 s when it is short
        reps = int(max(1, min(100, 3.0 / max(full_s, 1e-6))))
        c0 = time.perf_counter()
        mi = ms = 0
        for (ql, qs, pl, ps, gs, gidx, st) in sets * reps:
            wsm, wi, wst = O.code_grouped_greedy_sample(ql, qs, pl, ps, n_steps, bits, 42, thr,
                                                        1.0, nthr)
            mi += int(len(wst) != st.size or (np.asarray(wst) != st).any())
            mi += int((np.asarray(wi).reshape(-1, n_steps) != gidx).sum()) \
                if len(wst) == st.size else 0
            ms += int((wsm.view(np.uint32) != gs.view(np.uint32)).sum())
        dt = (time.perf_counter() - c0) / reps
        mi, ms = mi // reps, ms // reps
        frac, kind = 1.0, (f"the whole pipeline (oracle.code_grouped_greedy_sample: standardise, "
                           f"KL, partition, coder, destandardise), {reps} run(s), per image")
    else:
        frac = min(1.0, args.cpu_seconds / full_s)
        dt, cd, mi, ms = prefix(frac, nthr)
        frac = cd / sum(work)
        kind = (f"the coder (oracle.greedy_encode) on the first {frac:.2%} of each latent "
                "set's candidate-dims (the GPU's partition); rate scaled by that share")
    # 1 core on a short prefix (~3 s)
    f1 = min(frac, 3.0 / max(full_s * nthr, 1e-9))
    dt1, cd1, _, _ = prefix(max(f1, 1e-4), 1)
    one_core = (cd1 / sum(work)) / dt1
    cpu = {"value": frac / dt, "unit": "images/s", "cores": nthr, "kind": "port",
           "sample": f"image 0 ({len(sets)} latent set(s), {sum(work):.3g} candidate-dims): "
                     f"{kind}, {dt:.3f} s, oracle/cwq_oracle.c OpenMP over groups",
           "affinity_cpus": ncpu, "cgroup_cpu_quota": quota, "one_core_value": one_core,
           "one_core_sample": f"{cd1 / sum(work):.3%} of image 0's candidate-dims, {dt1:.2f} s"}
    parity = {"groups_checked": int(round(sum(st.size - 1 for *_, st in sets) * frac)),
              "index_mismatches": mi, "sample_word_mismatches": ms,
              "oracle": "oracle/cwq_oracle.c (CPU restatement; TF reference unpinned)",
              "normaliser_sensitivity": normaliser_sensitivity("c2") if bits == 8 else None,
              # C3's level-1 sets are C2-shaped and its level-2 groups the same 8-bit coder
              "semantics_sensitivity": semantics_sensitivity(
                  {"c3": "c2"}.get(args.config, args.config))}
    return cpu, parity


def importance_main(args):
    """I1/I2: the grouped importance pipeline per image
    (code_grouped_importance_sample): standardise + KL on the GPU, host
    grouping and N_g plan, the tiled candidate kernel, Elias-delta bitcode and
    quint16 outliers.  Synthetic PLN-like latents.  The roofline prices the
    candidate-scoring launches (cwq_options.eval_ms_out: HIP events around
    them, summed over the step's calls); cpu_baseline / parity run the oracle's
    whole pipeline (oracle.code_grouped_importance_sample) on image 0."""
    import ctypes
    import compression_without_quantization_amd.coded_importance_sampler as I
    from compression_without_quantization_amd.synthetic import make_latents
    I.VERBOSE = False
    n_img, D, nbits, gbits, kl_lim, desc = IMPORTANCE[args.config]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lat, lat_np = [], []
    for i in range(n_img):
        q_loc, q_scale, p_loc, p_scale = make_latents(D, seed=5000 + i)
        if i == 0:
            lat_np.append((q_loc, q_scale, p_loc, p_scale))
        lat.append((C.Normal(torch.from_numpy(q_loc).to(dev), torch.from_numpy(q_scale).to(dev)),
                    C.Normal(torch.from_numpy(p_loc).to(dev), torch.from_numpy(p_scale).to(dev))))
    evq = []

    def step_single(timed=False):  # one code_grouped_importance_sample call per image
        out = []
        for t, p in lat:
            v = ctypes.c_float(0.0) if timed else None
            out.append(I.code_grouped_importance_sample(None, t, p, 42, nbits,
                                                        max_group_size_bits=gbits,
                                                        dim_kl_bit_limit=kl_lim, eval_ms_out=v))
            if v is not None:
                evq.append(v)
        return out

    def step_batch(timed=False):  # every image of the step in one batched call
        v = ctypes.c_float(0.0) if timed else None
        out = I.code_grouped_importance_sample_batch(None, [t for t, _ in lat],
                                                     [p for _, p in lat], 42, nbits,
                                                     max_group_size_bits=gbits,
                                                     dim_kl_bit_limit=kl_lim, eval_ms_out=v)
        if v is not None:
            evq.append(v)
        return out

    def timed(step):
        """(seconds for args.steps steps, results, scoring ms per step): the
        steps timed with the scoring timers on (each call synchronises anyway)."""
        res = None
        for _ in range(args.warmup):
            res = step()
        torch.cuda.synchronize()
        evq.clear()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            res = step(True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        return el, res, sum(v.value for v in evq) / max(args.steps, 1)

    batch = n_img > 1 and not args.per_image
    batched = None
    if batch and args.batch_only:
        el, res, kernel_ms = timed(step_batch)
        batched = {"images_per_call": n_img, "equal_to_single_calls": None,
                   "single_call_images_per_s": None}
    else:
        el, res, kernel_ms = timed(step_single)
        if batch:
            el_s, kms_s, res_s = el, kernel_ms, res
            el, res, kernel_ms = timed(step_batch)
            same = all(a[1] == b[1] and np.array_equal(np.asarray(a[2]), np.asarray(b[2])) and
                       np.array_equal(np.asarray(a[0]).view(np.uint32),
                                      np.asarray(b[0]).view(np.uint32)) and
                       np.array_equal(a[3][0], b[3][0]) and np.array_equal(a[3][1], b[3][1])
                       for a, b in zip(res_s, res))
            if not same:
                raise SystemExit("bench.py: batched importance results differ from the single calls")
            batched = {"images_per_call": n_img, "equal_to_single_calls": bool(same),
                       "single_call_images_per_s": n_img * args.steps / el_s,
                       "single_call_scoring_kernel_ms": round(kms_s, 4)}
    # work: sum over groups of N_g * d_g candidate-dims (the plan the coder used)
    cand_dims = 0
    for (t, p), r in zip(lat, res):
        starts = np.asarray(r[2], dtype=np.int64)
        cand_dims += _importance_work(t, p, starts, kl_lim, dev)
    groups = sum(len(r[2]) - 1 for r in res)
    bitlen = sum(len(r[1]) for r in res)
    # per group: 16 d (four f32 inputs) + 8 (int64 index) + 4 d (sample)
    alg = 20 * D * n_img + 8 * groups
    roofline = scoring_roofline(args.config, groups, alg, kernel_ms, cand_dims,
                                "k_imp_prep + k_imp_tiles + k_imp_eval + k_imp_rows "
                                "(DESIGN.md 8)", "cwq_options.eval_ms_out of each "
                                "code_grouped_importance_sample[_batch] call (HIP events around "
                                "its candidate-scoring launches), summed over the step's calls")
    cpu = parity = None
    if not args.no_cpu:
        cpu, parity = importance_cpu_baseline(args, lat_np[0], res[0], nbits, gbits, kl_lim)
    line = {"metric": "images coded/s (grouped importance pipeline)",
            "value": n_img * args.steps / el, "unit": "images/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic PLN-like latents",
            "config": {"workload": desc, "groups_per_step": groups, "bits_per_step": bitlen,
                       "groups_per_s": groups * args.steps / el,
                       "candidate_dims_per_step": cand_dims,
                       "candidate_dims_per_s": cand_dims * args.steps / el,
                       "mode": ("code_grouped_importance_sample_batch: every image of a step in "
                                "one call" if batched else
                                "one code_grouped_importance_sample call per image"),
                       "batched": batched},
            "roofline": roofline, "cpu_baseline": cpu, "parity": parity}
    print(json.dumps(line), flush=True)


def scoring_roofline(config, groups, alg, kernel_ms, cand_dims, kernel, timing):
    """The roofline block of a grouped line: the scoring launches' algorithmic
    bytes over their HIP-event time against HBM, and the VALU issue fraction
    and HBM traffic of the PMC evidence in profiles/traffic_CONFIG.json
    (tools/collect_profile.py; recomputable from the CSVs it lists) when it
    was taken on this workload (same group count)."""
    achieved = alg / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else None
    traffic = valu = agg = src = None
    tf = os.path.join(REPO, "profiles", f"traffic_{config}.json")
    if os.path.exists(tf):
        with open(tf) as f:
            tj = json.load(f)
        if tj.get("blocks") == groups:
            agg = tj.get("scoring") or {}
            traffic = agg.get("hbm_bytes_per_step", tj.get("hbm_bytes_per_launch"))
            valu = (tj.get("valu") or {}).get("valu_issue_frac")
            src = tj.get("sources")
    return {"bound": "valu", "achieved": None if achieved is None else round(achieved, 3),
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": None if achieved is None else achieved / HBM_PEAK_GBS, "traffic": traffic,
            "hbm_note": "achieved/peak/frac/traffic price the scoring launches' algorithmic "
                        "bytes (20 d + 4 n_steps per group) against HBM, as the north star "
                        "asks; the launches are bound by VALU issue (Philox + Box-Muller per "
                        "candidate), see `valu`",
            "kernel": kernel, "kernel_ms": round(kernel_ms, 4), "kernel_timing": timing,
            "algorithmic_bytes_per_launch": alg,
            "valu": {"unit": "candidate-dims/s",
                     "nominal_candidate_dims_per_s": (cand_dims / (kernel_ms * 1e-3)
                                                      if kernel_ms > 0 else None),
                     "valu_issue_frac": valu,
                     "valu_issue_frac_scoring_launches": (agg or {}).get("valu_issue_frac"),
                     "valu_issue_source": (f"profiles/traffic_{config}.json: 2 * SQ_INSTS_VALU / "
                                           "(1024 SIMDs x dispatch duration x 2.4 GHz), the "
                                           "dominant kernel; _scoring_launches: every scoring "
                                           "dispatch of the step; CSVs: " +
                                           ", ".join((src or {}).get("pmc_csvs", []))
                                           if valu is not None else None)}}


def importance_cpu_baseline(args, lat0, res0, nbits, gbits, kl_lim):
    """The oracle's grouped importance pipeline on image 0 (standardise, KL,
    outliers, partition, plan, coder, destandardise) where it fits
    ~cpu_seconds, else its coder on a prefix of the image's groups (the same
    plan) with the rate scaled by the prefix's share of the candidate-dims.
    The sampled groups' indices and sample words, the group starts and the
    outliers are checked against the GPU's."""
    from oracle import oracle as O
    ncpu, quota = affinity_cores()
    nthr = min(ncpu, int(np.ceil(quota))) if quota else ncpu
    ql, qs, pl, ps = lat0
    gs, gcode, gst, gout = res0
    D = ql.size
    tl, ts = O.standardise(ql, qs, pl, ps)
    kl_bits = O.kl_normal_normal(ql, qs, pl, ps) / np.float32(np.log(2))
    keep = kl_bits <= kl_lim
    tl = np.where(keep, tl, np.float32(0)).astype(np.float32)
    ts = np.where(keep, ts, np.float32(1)).astype(np.float32)
    zeros, ones = np.zeros(D, np.float32), np.ones(D, np.float32)
    kl_divs = O.kl_normal_normal(tl, ts, zeros, ones)
    st = np.asarray(O.importance_group_starts(kl_divs, nbits, gbits), np.int64)
    ns = np.asarray(O.importance_plan(kl_divs, st), np.int64)
    starts_equal = bool(np.array_equal(st, np.asarray(gst, np.int64)))
    G = st.size - 1
    gidx = np.asarray(C.elias_delta_decode_many(gcode, len(gst) - 1)[0]
                      if isinstance(gcode, str) else gcode, np.int64) - 1
    work = np.diff(st) * np.maximum(ns, 1)
    total = float(work.sum())

    def prefix(k, threads):
        e = int(st[k])
        c0 = time.perf_counter()
        wi, wsm = O.importance_encode(tl[:e], ts[:e], zeros[:e], ones[:e], st[:k + 1], ns[:k],
                                      42, 0, threads)
        dt = time.perf_counter() - c0
        smp = np.where(keep[:e], O.destandardise(wsm, pl[:e], ps[:e]), gs[:e])
        mi = int((wi != gidx[:k]).sum())
        ms = int((smp.astype(np.float32).view(np.uint32) != gs[:e].view(np.uint32)).sum())
        return dt, float(work[:k].sum()), mi, ms
    k0 = max(1, G // 100)
    dt, cd, _, _ = prefix(k0, nthr)
    full_s = dt * total / max(cd, 1.0)
    if full_s <= args.cpu_seconds:
        reps = int(max(1, min(100, 3.0 / max(full_s, 1e-6))))  # short images: ~3 s of runs
        c0 = time.perf_counter()
        for _ in range(reps):
            wsm, wi, wst, (oi, oq) = O.code_grouped_importance_sample(ql, qs, pl, ps, 42, nbits,
                                                                     gbits, kl_lim, nthr)
        dt = (time.perf_counter() - c0) / reps
        mi = int((np.asarray(wi, np.int64) - 1 != gidx).sum()) if len(wi) == gidx.size else G
        ms = int((wsm.view(np.uint32) != gs.view(np.uint32)).sum())
        out_equal = bool(np.array_equal(oi, gout[0]) and np.array_equal(oq, gout[1]))
        frac, kind, checked = 1.0, ("the whole pipeline (oracle.code_grouped_importance_sample: "
                                    "standardise, KL, outliers, partition, plan, coder, "
                                    f"destandardise), {reps} run(s), per image"), G
    else:
        frac_t = min(1.0, args.cpu_seconds / full_s)
        k = max(1, int(np.searchsorted(np.cumsum(work), frac_t * total)))
        dt, cd, mi, ms = prefix(k, nthr)
        frac = cd / total
        kind = (f"the coder (oracle.importance_encode) on the first {k} of the image's {G} "
                f"groups ({frac:.2%} of its candidate-dims, the same plan); rate scaled by that "
                "share")
        out_equal, checked = None, k
    k1 = max(1, min(G, int(np.searchsorted(np.cumsum(work), total * min(frac, 3.0 / max(
        full_s * nthr, 1e-9))))))
    dt1, cd1, _, _ = prefix(k1, 1)
    cpu = {"value": frac / dt, "unit": "images/s", "cores": nthr, "kind": "port",
           "sample": f"image 0 ({D} dims, {total:.3g} candidate-dims): {kind}, {dt:.3f} s, "
                     "oracle/cwq_oracle.c OpenMP over groups",
           "affinity_cpus": ncpu, "cgroup_cpu_quota": quota,
           "one_core_value": (cd1 / total) / dt1,
           "one_core_sample": f"{cd1 / total:.3%} of image 0's candidate-dims, {dt1:.2f} s"}
    parity = {"groups_checked": checked, "index_mismatches": mi, "sample_word_mismatches": ms,
              "group_starts_equal": starts_equal, "outliers_equal": out_equal,
              "oracle": "oracle/cwq_oracle.c + oracle/oracle.py (CPU restatement of "
                        "coded_importance_sampler.py:112-274; TF reference unpinned)"}
    return cpu, parity


def pln_main(args):
    """The PLN image codec end to end (pln.py:213-817): transforms (MIOpen),
    latent plumbing (HIP), both coders, the group-size arithmetic coder and
    the .miracle file, then the decoder.  Seeded random weights (no trained
    checkpoint offline) on a synthetic image."""
    import tempfile
    import compression_without_quantization_amd.coded_greedy_sampler as S
    import compression_without_quantization_amd.coded_importance_sampler as I
    from compression_without_quantization_amd import pln as P
    S.VERBOSE = I.VERBOSE = False
    n_img, H, W, level1, desc = PLN[args.config]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    model = P.ProbabilisticLadderNetwork().to(dev).eval()
    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:H, 0:W] / max(H, W)
    imgs = []
    for i in range(n_img):
        base = np.stack([np.sin((6 + i) * xx + c) * np.cos(4 * yy - c) for c in range(3)], -1)
        imgs.append(np.clip(0.5 + 0.35 * base + 0.05 * rng.standard_normal((H, W, 3)), 0, 1)
                    .astype(np.float32)[None])
    kw = dict(n_steps=30, n_bits_per_step=14, greedy_max_group_size_bits=12,
              use_importance_sampling=(level1 == "importance"),
              second_level_n_bits_per_group=20, second_level_max_group_size_bits=2,
              second_level_dim_kl_bit_limit=16, first_level_n_bits_per_group=20,
              first_level_max_group_size_bits=4, first_level_dim_kl_bit_limit=16)
    tmp = tempfile.mkdtemp()
    paths = [os.path.join(tmp, f"img{i}.miracle") for i in range(n_img)]

    # the last warmup compress (the first timed one when --warmup 0) captures
    # image 0's coder inputs, results and scoring-launch milliseconds: the
    # roofline prices those launches, the CPU oracle codes the same latents
    # (parity).  Capturing inside a compress that runs anyway keeps a `--steps 1
    # --warmup 0` PMC pass at exactly one compress per step; the last warmup's
    # launches are warm (the first call's scoring bracket includes one-off
    # module loads).
    cap = {}

    def compress(capture=False):
        c = cap if capture and not cap else None
        return [model.code_image_greedy(None, im, 42, comp_file_path=p,
                                        capture=(c if i == 0 else None), **kw)[1]
                for i, (im, p) in enumerate(zip(imgs, paths))]

    def decompress():
        return [model.decode_image_greedy(None, p, use_importance_sampling=kw[
            "use_importance_sampling"], second_level_max_group_size_bits=2,
            first_level_max_group_size_bits=4) for p in paths]
    for w in range(args.warmup):
        compress(capture=(w == args.warmup - 1))
        decompress()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        summ = compress(capture=(k == 0 and args.warmup == 0))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rec = decompress()
    torch.cuda.synchronize()
    eld = time.perf_counter() - t0
    l1, l2 = cap["level1"], cap["level2"]
    D1, D2 = l1["q_loc"].size, l2["q_loc"].size
    G1, G2 = len(l1["result"][2]) - 1, len(l2["result"][2]) - 1
    greedy1 = l1["kind"] == "greedy"
    alg = (20 * D1 + (4 * kw["n_steps"] if greedy1 else 8) * G1) + (20 * D2 + 8 * G2)
    kernel_ms = float(sum(cap["scoring_ms"]))
    roofline = scoring_roofline(
        args.config, (G1 + G2) * n_img, alg, kernel_ms, 0,
        ("level 1: " + ("k_csr_prep + k_encode_prune_csr (+ finalize), 30 x 14 bits"
                        if greedy1 else "k_imp_* (importance, 20 bits/group)") +
         "; level 2: k_imp_* (importance, 20 bits/group)"),
        "cwq_options.eval_ms_out of the two coders' calls (HIP events around their "
        "candidate-scoring launches) in one compress of image 0, summed")
    roofline["valu"]["nominal_candidate_dims_per_s"] = None
    roofline["scoring_ms_by_level"] = {"level2": cap["scoring_ms"][0],
                                       "level1": cap["scoring_ms"][1]}
    cpu = parity = None
    if not args.no_cpu:
        cpu, parity = pln_cpu_baseline(args, cap, kw)
    line = {"metric": "images compressed/s (PLN codec, miracle.py compress)",
            "value": n_img * args.steps / el, "unit": "images/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic image, seeded random PLN weights (no checkpoint offline)",
            "config": {"workload": desc, "groups_per_step": (G1 + G2) * n_img,
                       "decompress_images_per_s": n_img * args.steps / eld,
                       "bytes": summ[0]["actual_byte_size"], "bpp": summ[0]["bpp"],
                       "kl_bits_level1": summ[0]["first_level_theoretical"] * 8,
                       "kl_bits_level2": summ[0]["second_level_theoretical"] * 8,
                       "groups_level1": summ[0]["first_level_groups"],
                       "groups_level2": summ[0]["second_level_groups"],
                       "reconstruction_shape": list(rec[0].shape)},
            "roofline": roofline, "cpu_baseline": cpu, "parity": parity}
    print(json.dumps(line), flush=True)


def pln_cpu_baseline(args, cap, kw):
    """The CPU oracle coding image 0's two latent levels as the codec did
    (level 2 importance; level 1 greedy 30 x 14 bits or importance), on the
    coders' exact inputs captured from the GPU run: a per-level sample as in
    grouped_cpu_baseline / importance_cpu_baseline, the image rate combining
    the two levels' times.  The analysis / synthesis transforms (seeded random
    weights, MIOpen) and the arithmetic coder are outside the sample."""
    l1, l2 = cap["level1"], cap["level2"]
    half = argparse.Namespace(**{**vars(args), "cpu_seconds": args.cpu_seconds / 2})
    lat = lambda lv: (lv["q_loc"], lv["q_scale"], lv["p_loc"], lv["p_scale"])
    c2, p2 = importance_cpu_baseline(half, lat(l2), l2["result"],
                                     kw["second_level_n_bits_per_group"],
                                     kw["second_level_max_group_size_bits"],
                                     kw["second_level_dim_kl_bit_limit"])
    if l1["kind"] == "greedy":
        c1, p1 = grouped_cpu_baseline(half, [lat(l1)], [l1["result"]], kw["n_bits_per_step"],
                                      kw["n_steps"])
    else:
        c1, p1 = importance_cpu_baseline(half, lat(l1), l1["result"],
                                         kw["first_level_n_bits_per_group"],
                                         kw["first_level_max_group_size_bits"],
                                         kw["first_level_dim_kl_bit_limit"])
    comb = lambda a, b: 1.0 / (1.0 / a + 1.0 / b)
    cpu = {"value": comb(c1["value"], c2["value"]), "unit": "images/s", "cores": c1["cores"],
           "kind": "port",
           "sample": "image 0's latent coding on the CPU oracle (transforms and arithmetic "
                     "coder excluded): level 1 " + c1["sample"] + "; level 2 " + c2["sample"],
           "one_core_value": comb(c1["one_core_value"], c2["one_core_value"]),
           "levels": {"level1": c1, "level2": c2}}
    parity = {"level1": p1, "level2": p2,
              "index_mismatches": p1["index_mismatches"] + p2["index_mismatches"],
              "sample_word_mismatches": p1["sample_word_mismatches"] +
              p2["sample_word_mismatches"],
              "oracle": "oracle/cwq_oracle.c + oracle/oracle.py (CPU restatement; TF reference "
                        "unpinned); the coders' inputs are the GPU codec's (random-weight "
                        "transforms, TFC parity unpinned)"}
    return cpu, parity


def _importance_work(target, proposal, starts, kl_lim, dev):
    """sum_g N_g d_g for the plan code_grouped_importance_sample used."""
    import compression_without_quantization_amd.coded_importance_sampler as I
    lib = _lib.load()
    D = proposal.loc.numel()
    t_loc = torch.empty(D, dtype=torch.float32, device=dev)
    t_scale = torch.empty(D, dtype=torch.float32, device=dev)
    f = lambda x: x.contiguous().float()
    tl, ts, pl, ps = f(target.loc), f(target.scale), f(proposal.loc), f(proposal.scale)
    _lib.check(lib.cwq_standardise(tl.data_ptr(), ts.data_ptr(), pl.data_ptr(), ps.data_ptr(), D,
                                   t_loc.data_ptr(), t_scale.data_ptr(),
                                   torch.cuda.current_stream(dev).cuda_stream), "standardise")
    kl_bits = I._kl(dev, tl, ts, pl, ps).cpu().numpy() / np.float32(np.log(2))
    keep = torch.from_numpy(kl_bits <= kl_lim).to(dev)
    t_loc = torch.where(keep, t_loc, torch.zeros_like(t_loc))
    t_scale = torch.where(keep, t_scale, torch.ones_like(t_scale))
    z, o = torch.zeros_like(t_loc), torch.ones_like(t_loc)
    kl = I._kl(dev, t_loc, t_scale, z, o).cpu().numpy()
    n = I.num_samples_plan(kl, starts)
    sizes = np.diff(starts)
    return int((np.maximum(n, 1) * sizes).sum())


def _stop_processes(procs, grace=5.0):
    """SIGTERM the exact processes given, SIGKILL those still alive after
    `grace` seconds, and reap them all (nothing is left running)."""
    import signal
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t_end = time.monotonic() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.0, t_end - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def run_rank_processes(cmds, deadline_s, poll=0.05):
    """Start one process per (argv, env) of `cmds` (rank r = cmds[r]) and wait
    for them, with a wall-clock deadline.  The first rank to fail stops the
    others (exact PIDs) and its exit code is returned; past `deadline_s` the
    ranks still running are named on stderr, stopped, and 124 is returned (the
    code of `timeout`).  Returns 0 when every rank exits 0."""
    procs = [subprocess.Popen(argv, env=env) for argv, env in cmds]
    t_end = time.monotonic() + deadline_s
    rc = 0
    live = list(procs)
    try:
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    print(f"bench.py: rank {procs.index(p)} exited with {c}; stopping ranks "
                          f"{[procs.index(q) for q in live]}", file=sys.stderr, flush=True)
                    _stop_processes(live)
                    live = []
                    break
            if live and time.monotonic() > t_end:
                print(f"bench.py: ranks {[procs.index(q) for q in live]} still running after "
                      f"the {deadline_s:g} s deadline (--rank-timeout); stopping them",
                      file=sys.stderr, flush=True)
                _stop_processes(live)
                live = []
                rc = rc or 124
            time.sleep(poll)
    finally:
        _stop_processes([p for p in procs if p.poll() is None])
    return rc


def spawn_ranks(args):
    """`bench.py --gpus N` (N > 1) without a launcher: start N fresh rank
    processes (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their environment, one
    GPU each) and wait for them.  This parent never touches the GPU (it only
    imports torch), so no process that initialised HIP is replaced or forked.
    If a rank fails the others are stopped (exact PIDs) and its code returned;
    ranks still running at the --rank-timeout deadline are stopped and the
    parent exits 124."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmds = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        cmds.append(([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env))
    rc = run_rank_processes(cmds, args.rank_timeout)
    sys.exit(rc if rc >= 0 else 128 - rc)


def affinity_cores():
    """(CPUs in this process's affinity, the cgroup CPU quota or None)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return n, quota


def normaliser_sensitivity(section):
    """profiles/normaliser_sensitivity.json's record for one workload (the
    oracle re-encoded with log sigma from Eigen plog, +-1 ulp, random +-1 ulp:
    tools/normaliser_sensitivity.py) as the parity field's bound on how many
    indices hang on the undeclarable normaliser choice."""
    f = os.path.join(REPO, "profiles", "normaliser_sensitivity.json")
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        r = json.load(fh).get(section)
    if not r:
        return None
    var = ("plog", "plog_fma", "up", "down", "random")
    flips = {v: r[v]["index_flips"] for v in var if v in r}
    n = r["indices"]
    return {"normaliser_ulp_flip_rate": max(flips.values()) / n if flips else None,
            "indices_per_variant": n, "flips": flips,
            "flip_rate_95pct_upper": (3.0 / n if flips and max(flips.values()) == 0 else None),
            "best_second_gap_min": r.get("best_second_gap", {}).get("min"),
            "source": "profiles/normaliser_sensitivity.json (tools/normaliser_sensitivity.py, "
                      "CPU oracle; log sigma from Eigen plog / plog+FMA / logf +1 ulp / -1 ulp / "
                      "random +-1 ulp)"}


def semantics_sensitivity(section):
    """profiles/semantics_sensitivity.json's record for one workload: the
    oracle scoring every candidate also under TFP >= 0.8's log-prob form and
    five other Eigen sum orders (tools/semantics_sensitivity.py), i.e. how many
    indices hang on the per-candidate declared semantics."""
    f = os.path.join(REPO, "profiles", "semantics_sensitivity.json")
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        r = json.load(fh).get(section)
    if not r:
        return None
    flips = {v: x["index_flips"] for v, x in r["variants"].items()}
    n = r["indices"]
    return {"variants": len(flips), "indices_per_variant": n, "sample": r["sample"],
            "max_flips": max(flips.values()), "flips": flips,
            "flip_rate_95pct_upper": (3.0 / n if max(flips.values()) == 0 else None),
            "model_flip_rate_max": r.get("max_model_flip_rate_over_variants"),
            "best_second_gap_min": r["best_second_gap"]["min"],
            "source": "profiles/semantics_sensitivity.json (tools/semantics_sensitivity.py, CPU "
                      "oracle; TFP>=0.8 squared_difference log_prob x {Eigen AVX, SSE, AVX x2, "
                      "AVX-512, sequential, tree} row sums)"}


def rank_device_map(dist, rank, local_rank, dev):
    """[{rank, local_rank, host, device, pci_bus}] of every rank (all-gathered);
    with RCCL (one GPU per rank) two ranks on one GPU are refused."""
    import socket
    props = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "local_rank": local_rank, "host": socket.gethostname(),
          "device": dev.index, "pci_bus": getattr(props, "pci_bus_id", None),
          "visible": os.environ.get("HIP_VISIBLE_DEVICES",
                                    os.environ.get("CUDA_VISIBLE_DEVICES"))}
    if dist is None:
        return [me]
    allm = [None] * dist.get_world_size()
    dist.all_gather_object(allm, me)
    if dist.get_backend() == "nccl":
        seen = {}
        for m in allm:
            key = (m["host"], m["pci_bus"] if m["pci_bus"] is not None else
                   (m["visible"], m["device"]))
            if key in seen:
                raise SystemExit(f"bench.py: ranks {seen[key]} and {m['rank']} share GPU {key} "
                                 "under RCCL; one GPU per rank is required")
            seen[key] = m["rank"]
    return allm


def devices_distinct(rank_devices):
    """True when no two ranks share a GPU (same host and PCI bus, or, without a
    bus id, the same visible set and device index)."""
    keys = [(m["host"], m["pci_bus"] if m["pci_bus"] is not None else (m["visible"], m["device"]))
            for m in rank_devices]
    return len(set(keys)) == len(keys)


def oracle_check(O, host, d, bits, n_steps, seed, block_id_base, idx_h, samp_h, blocks, nthr):
    """Indices and sample words of `blocks` (local block numbers) against the
    CPU oracle: the checker, outside every timed region."""
    blocks = np.asarray(blocks, dtype=np.int64)
    mi = ms = 0
    for b in blocks:
        sl = slice(int(b) * d, (int(b) + 1) * d)
        wi, wsm = O.greedy_encode(host["post_loc"].reshape(-1)[sl],
                                  host["post_scale"].reshape(-1)[sl],
                                  host["prior_loc"].reshape(-1)[sl],
                                  host["prior_scale"].reshape(-1)[sl],
                                  np.array([0, d], np.int64), bits, n_steps, seed, 1.0,
                                  block_id_base + int(b), nthr)
        mi += int((wi.reshape(-1) != idx_h[b].reshape(-1)).sum())
        ms += int((wsm.view(np.uint32) != samp_h[sl].view(np.uint32)).sum())
    return mi, ms


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.config in GROUPED or args.config in IMPORTANCE or args.config in PLN:
        if world > 1:
            raise SystemExit(f"bench.py: --config {args.config} is a single-GPU workload")
        if args.config in GROUPED:
            return grouped_main(args)
        if args.config in IMPORTANCE:
            return importance_main(args)
        return pln_main(args)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local_rank % ndev)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # RCCL when every rank owns a GPU (the data path itself has no collective:
        # only the start/stop barriers and the max-reduce of the step time use
        # it); gloo when ranks share one device (a rehearsal on a 1-GPU box)
        import datetime
        pg_timeout = datetime.timedelta(seconds=max(30.0, min(args.rank_timeout, 300.0)))
        if ndev >= world:
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout)
        else:
            dist.init_process_group("gloo", timeout=pg_timeout)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, "
                             f"--gpus {args.gpus}")
    rank_devices = rank_device_map(dist, rank, local_rank, dev)
    if dist is not None and dist.get_backend() == "nccl" and not devices_distinct(rank_devices):
        raise SystemExit("bench.py: RCCL ranks must own distinct GPUs")  # (rank_device_map)

    nb_cfg, d, bits, n_steps, desc = CONFIGS[args.config]
    if args.blocks:
        nb_cfg = args.blocks
    scaling = args.scaling or ("strong" if world > 1 else "weak")
    if scaling == "strong":
        # the config's block set is the whole job, cut into contiguous shards
        # (parallel.shard_range); each shard keeps its global block ids
        nb_total = nb_cfg
        b0, b1 = shard_range(nb_total, world, rank)
    else:
        # nb_cfg blocks per rank: rank r owns global blocks [r nb, (r+1) nb)
        nb_total = nb_cfg * world
        b0, b1 = rank * nb_cfg, (rank + 1) * nb_cfg
    nb = b1 - b0
    block_id_base = b0
    shards = [[b0, b1]]
    if dist:  # every rank's block range, for the line (contiguous, disjoint: checked in tests)
        allr = [None] * world
        dist.all_gather_object(allr, [b0, b1])
        shards = allr
    seed = 42
    host = make_blocks_range(b0, b1, d, bits, seed=DEFAULT_SEED)
    t = {k: torch.from_numpy(v.reshape(-1)).to(dev) for k, v in host.items()}
    out_idx = torch.empty((nb, n_steps), dtype=torch.int32, device=dev)
    out_sample = torch.empty(nb * d, dtype=torch.float32, device=dev)
    ws = torch.empty(max(1, C.encode_workspace_bytes(nb, nb * d, block_dim=d)),
                     dtype=torch.uint8, device=dev)
    nst = max(args.steps, 1)
    events = []
    for _ in range(nst):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        b.record()  # materialise the hipEvent_t handles
        events.append((a, b))

    def step(ev=None):
        C.encode_blocks(t["post_loc"], t["post_scale"], t["prior_loc"], t["prior_scale"], bits,
                        n_steps, seed, block_dim=d, block_id_base=block_id_base,
                        out_idx=out_idx, out_sample=out_sample, workspace=ws,
                        prune_mode=args.prune_mode,
                        eval_events=None if ev is None else (ev[0].cuda_event, ev[1].cuda_event))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    eval_ms = float(np.mean([a.elapsed_time(b) for a, b in events[:args.steps]])) \
        if args.steps else float("nan")
    if dist:
        e = torch.tensor([elapsed, eval_ms], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed, eval_ms_max = float(e[0].item()), float(e[1].item())
    else:
        eval_ms_max = eval_ms

    # PCIe-inclusive single pass (host arrays in, indices + samples out): reported aside
    e2e = e2e_streamed = None
    if not args.no_e2e and rank == 0 and nb:
        torch.cuda.synchronize()
        te0 = time.perf_counter()
        th = {k: torch.from_numpy(v.reshape(-1)).to(dev) for k, v in host.items()}
        C.encode_blocks(th["post_loc"], th["post_scale"], th["prior_loc"], th["prior_scale"],
                        bits, n_steps, seed, block_dim=d, block_id_base=block_id_base,
                        out_idx=out_idx, out_sample=out_sample, workspace=ws,
                        prune_mode=args.prune_mode)
        idx_h = out_idx.cpu().numpy()
        samp_h = out_sample.cpu().numpy()
        te1 = time.perf_counter()
        e2e = nb / (te1 - te0)
        del th, idx_h, samp_h
        # the same pass through encode_blocks_host: chunks of blocks copied in on
        # a copy stream while the previous chunk codes, results copied out
        # behind the next chunk; one untimed call on the first blocks first
        # primes the caching allocator
        ha = [host[k].reshape(-1) for k in ("post_loc", "post_scale", "prior_loc",
                                            "prior_scale")]
        w = min(nb, 2 * 131072) * d
        C.encode_blocks_host(*[a[:w] for a in ha], bits, n_steps, seed, d,
                             block_id_base=block_id_base, device=dev,
                             prune_mode=args.prune_mode)
        torch.cuda.synchronize()
        te0 = time.perf_counter()
        C.encode_blocks_host(*ha, bits, n_steps, seed, d, block_id_base=block_id_base,
                             device=dev, prune_mode=args.prune_mode)
        te1 = time.perf_counter()
        e2e_streamed = nb / (te1 - te0)

    # decoder throughput on the same blocks (reported aside), with its own
    # HIP-event kernel time
    dec_out = torch.empty_like(out_sample)
    C.decode_blocks(out_idx, t["prior_loc"], t["prior_scale"], bits, n_steps, seed, block_dim=d,
                    block_id_base=block_id_base, out_sample=dec_out)
    torch.cuda.synchronize()
    da = torch.cuda.Event(enable_timing=True)
    db = torch.cuda.Event(enable_timing=True)
    n_dec = 5
    da.record()
    for _ in range(n_dec):
        C.decode_blocks(out_idx, t["prior_loc"], t["prior_scale"], bits, n_steps, seed,
                        block_dim=d, block_id_base=block_id_base, out_sample=dec_out)
    db.record()
    torch.cuda.synchronize()
    dec_ms = da.elapsed_time(db) / n_dec
    decode_bps = nb / (dec_ms * 1e-3) if nb else 0.0
    roundtrip_ok = bool(torch.equal(dec_out.view(torch.int32), out_sample.view(torch.int32)))
    if dist:
        ok_t = torch.tensor([0 if roundtrip_ok else 1], dtype=torch.int64,
                            device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(ok_t)
        roundtrip_ok = int(ok_t.item()) == 0

    value = nb_total * args.steps / elapsed
    bytes_per_launch = nb * (20 * d + 4 * n_steps)
    cand = nb * n_steps * (1 << bits)
    cand_dims = cand * d
    rank0_kernel = {"blocks": nb, "algorithmic_bytes_per_launch": bytes_per_launch,
                    "kernel_ms": round(eval_ms, 3)}
    if dist:
        # the job's roofline: every rank's launch bytes and candidate-dims
        # summed, over the slowest rank's kernel time (each rank's GPU runs its
        # shard concurrently)
        tot = torch.tensor([bytes_per_launch, cand, cand_dims], dtype=torch.float64,
                           device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tot)
        bytes_per_launch, cand, cand_dims = (int(v) for v in tot.tolist())
        eval_ms = eval_ms_max
    achieved = bytes_per_launch / (eval_ms * 1e-3) / 1e9
    traffic = None
    valu = None
    units = None
    tsrc = {}
    tf = os.path.join(REPO, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tf):
        with open(tf) as f:
            tj = json.load(f)
        if tj.get("blocks") == nb:
            traffic = tj.get("hbm_bytes_per_launch")
            valu = tj.get("valu")
            tsrc = tj.get("sources") or {}
    pf = os.path.join(REPO, "profiles", f"prune_stats_{args.config}.json")
    if os.path.exists(pf):
        with open(pf) as f:
            units = json.load(f)
    fast = args.prune_mode and d % 8 == 0 and 8 <= d <= 64
    evaluated = None
    if units and fast and args.prune_mode == units.get("prune_mode"):
        # each evaluated 4-dim unit costs the same; candidates stop after
        # units_per_candidate of the d/4 units on average
        evaluated = {"units_per_candidate": units["units_per_candidate"],
                     "units_per_candidate_nominal": d // 4,
                     "candidate_dims_per_s": cand / (eval_ms * 1e-3)
                     * units["units_per_candidate"] * 4,
                     "source": f"profiles/prune_stats_{args.config}.json "
                               "(tools/prune_stats.py on a -DCWQ_PRUNE_STATS build)"}
    roofline = {"bound": "valu",
                "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "hbm_note": "achieved/peak/frac/traffic are the HBM figures the north star "
                            "asks for; the kernel is bound by VALU issue (Philox + "
                            "Box-Muller per candidate), see `valu` and DESIGN.md 4",
                # third argument: tiles run block-interleaved when a block spans
                # several tiles (fewer than 16,384 blocks, csrc choose_tiling)
                "kernel": (f"k_encode_prune<{d},true,{'true' if 0 < nb < 16384 else 'false'}>"
                           if fast else "k_encode_eval"),
                "kernel_ms": round(eval_ms, 3),
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "scope": ("one GPU" if world == 1 else
                          f"all {world} GPUs: algorithmic bytes and candidate-dims summed "
                          "over the ranks' launches, kernel_ms the slowest rank's (HIP "
                          "events on each rank's launch stream, max-reduced); achieved and "
                          "nominal rates are whole-job, peak is one GPU's"),
                "rank0": rank0_kernel if world > 1 else None,
                "valu": {"unit": "candidate-dims/s",
                         "nominal_candidate_dims_per_s": cand_dims / (eval_ms * 1e-3),
                         "evaluated": evaluated,
                         "valu_issue_frac": (valu or {}).get("valu_issue_frac"),
                         "valu_issue_source": (f"profiles/traffic_{args.config}.json: 2 * "
                                               "SQ_INSTS_VALU / (1024 SIMDs x dispatch duration "
                                               "x 2.4 GHz) of the same kernel; CSVs: " +
                                               ", ".join(tsrc.get("pmc_csvs", []))
                                               if valu else None)}}

    cpu = None
    parity = None
    if not args.no_cpu and nb:
        from oracle import oracle as O
        ncpu, quota = affinity_cores()
        idx_h = out_idx.cpu().numpy()
        samp_h = out_sample.cpu().numpy()
        # every CPU the process may use: the affinity set, capped by the
        # cgroup's CPU quota (the GPU box grants a 16-CPU share of a larger
        # host; threads beyond the quota only time-slice -- measured 2x slower)
        usable = min(ncpu, int(np.ceil(quota))) if quota else ncpu
        if rank == 0 and world == 1:
            nthr = usable
            # calibrate on a small sample, then size the sample to ~cpu_seconds

            def run(n):
                off = np.arange(n + 1, dtype=np.int64) * d
                sl = slice(0, n * d)
                c0 = time.perf_counter()
                wi, wsm = O.greedy_encode(host["post_loc"].reshape(-1)[sl],
                                          host["post_scale"].reshape(-1)[sl],
                                          host["prior_loc"].reshape(-1)[sl],
                                          host["prior_scale"].reshape(-1)[sl], off, bits,
                                          n_steps, seed, 1.0, block_id_base, nthr)
                return time.perf_counter() - c0, wi, wsm
            n = min(nb, 2 * nthr)
            dt, wi, wsm = run(n)
            if dt < args.cpu_seconds / 4 and n < nb:
                rate = n / max(dt, 1e-3)
                n = int(min(nb, max(n, rate * args.cpu_seconds)))
                if n < min(nb, 10_000) and min(nb, 10_000) / rate <= 30.0:
                    n = min(nb, 10_000)  # the first 10^4 blocks where that fits 30 s
                n = max(min(nb, nthr), (n // nthr) * nthr)
                dt, wi, wsm = run(n)
            mism_idx = int((wi != idx_h[:n]).sum())
            mism_smp = int((wsm.view(np.uint32) != samp_h[:n * d].view(np.uint32)).sum())
            # 1-core figure on a short sample
            n1 = max(1, min(n, int(max(1.0, n / dt / nthr * 3.0))))
            off1 = np.arange(n1 + 1, dtype=np.int64) * d
            c0 = time.perf_counter()
            O.greedy_encode(host["post_loc"].reshape(-1)[:n1 * d],
                            host["post_scale"].reshape(-1)[:n1 * d],
                            host["prior_loc"].reshape(-1)[:n1 * d],
                            host["prior_scale"].reshape(-1)[:n1 * d],
                            off1, bits, n_steps, seed, 1.0, block_id_base, 1)
            dt1 = time.perf_counter() - c0
            model = ""
            try:
                with open("/proc/cpuinfo") as f:
                    model = next((ln.split(":", 1)[1].strip() for ln in f
                                  if ln.startswith("model name")), "")
            except OSError:
                pass
            cpu = {"value": n / dt, "unit": "blocks/s", "cores": nthr, "kind": "port",
                   "sample": f"first {n} blocks of the same {args.config} workload "
                             f"({n * (1 << bits) * d * n_steps:.3g} candidate-dims, {dt:.1f} s), "
                             "oracle/cwq_oracle.c OpenMP over blocks, one thread per usable "
                             "CPU (affinity capped by the cgroup quota)",
                   "affinity_cpus": ncpu, "cgroup_cpu_quota": quota,
                   "one_core_value": n1 / dt1, "one_core_sample": f"first {n1} blocks, {dt1:.1f} s",
                   "cpu_model": model}
            checked = n
        else:
            # N > 1: every rank checks a sample of its own shard (first, last
            # and evenly spaced blocks) against the oracle; counts summed
            nthr = max(1, usable // world)
            pick = np.unique(np.concatenate([[0, nb - 1],
                                             np.linspace(0, nb - 1, args.check_blocks)
                                             .astype(np.int64)]))
            mism_idx, mism_smp = oracle_check(O, host, d, bits, n_steps, seed, block_id_base,
                                              idx_h.reshape(nb, n_steps), samp_h, pick, nthr)
            checked = int(pick.size)
        if dist:
            m = torch.tensor([checked, mism_idx, mism_smp], dtype=torch.int64,
                             device=dev if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(m)
            checked, mism_idx, mism_smp = (int(v) for v in m.tolist())
        parity = {"blocks_checked": checked, "index_mismatches": mism_idx,
                  "sample_word_mismatches": mism_smp,
                  "oracle": "oracle/cwq_oracle.c (CPU restatement; TF reference unpinned)",
                  "normaliser_sensitivity": (normaliser_sensitivity("c4")
                                             if (d, bits, n_steps) == (32, 16, 1) else None),
                  "semantics_sensitivity": semantics_sensitivity(
                      {(32, 16, 1): "c4", (16, 24, 1): "c5"}.get((d, bits, n_steps), ""))}

    if rank == 0:
        line = {
            "metric": "latent blocks encoded/s at KL=16 bits" if bits == 16 else
                      f"latent blocks encoded/s at KL={bits} bits",
            "value": value, "unit": "blocks/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / max(args.steps, 1) * 1e3,
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic diagonal-Gaussian blocks (PCG64(SeedSequence([20261015, chunk])) "
                    "per 65,536-block chunk of the global block set)",
            "config": {"workload": desc, "blocks_total": nb_total, "blocks_per_gpu": nb,
                       "block_dim": d, "kl_bits": bits, "n_steps": n_steps, "seed": seed,
                       "parallelism": f"block-sharded x{world} ({scaling} scaling), "
                                      "no collective on the data path",
                       "world_size_checked": (dist.get_world_size() if dist else 1),
                       "shards": shards,
                       "backend": (dist.get_backend() if dist else None),
                       "rank_devices": rank_devices,
                       "rank_devices_distinct": devices_distinct(rank_devices)},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity": parity,
            "pcie_inclusive_blocks_per_s": e2e,
            "pcie_inclusive_streamed_blocks_per_s": e2e_streamed,
            "decode_blocks_per_s": decode_bps,
            "decode_kernel_ms": round(dec_ms, 4),
            "decode_hbm_gbs": nb * (12 * d + 4 * n_steps) / (dec_ms * 1e-3) / 1e9 if nb else None,
            "decode_roundtrip_bit_exact": roundtrip_ok,
            "eval_kernel_ms_max_over_ranks": round(eval_ms_max, 3),
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
