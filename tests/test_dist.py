"""CPU: multi-rank block sharding over gloo (world_size 2, 3 and 8), as bench.py
--gpus N uses it (no collective on the data path; optional all-gather of
indices).  Each rank codes its shard with the CPU oracle (the checker, allowed
in tests) using block_id_base = its first global block; the gathered indices
must equal one single-process encode of all blocks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from compression_without_quantization_amd.parallel import gather_indices, shard_range


def test_shard_range_covers():
    for nb in (0, 1, 7, 1000, 10 ** 6):
        for w in (1, 2, 3, 8):
            spans = [shard_range(nb, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == nb
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))


def test_shard_range_cost_balanced():
    rng = np.random.default_rng(0)
    cost = rng.integers(1, 4096, 5000).astype(np.float64) * 256
    w = 8
    spans = [shard_range(cost.size, w, r, cost) for r in range(w)]
    loads = [cost[a:b].sum() for a, b in spans]
    assert spans[0][0] == 0 and spans[-1][1] == cost.size
    assert max(loads) / (cost.sum() / w) < 1.01


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nb, cost, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from oracle import oracle as O
    from compression_without_quantization_amd.synthetic import make_blocks_range
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d, bits = 8, 6
    b0, b1 = shard_range(nb, world, rank, cost)
    h = make_blocks_range(b0, b1, d, bits)
    idx, _ = O.greedy_encode(h["post_loc"], h["post_scale"], h["prior_loc"], h["prior_scale"],
                             np.arange(b1 - b0 + 1, dtype=np.int64) * d, bits, 1, 42, 1.0, b0, 1)
    # ranks may own different block counts (cost-balanced cuts): gather_indices
    # pads and trims internally; [nb, n_steps] rows, an empty shard included
    local = torch.from_numpy(idx.astype(np.int32))
    full = gather_indices(local)
    if rank == 0:
        out.put(full.reshape(-1).numpy().tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,balanced", [(2, False), (3, True), (3, "empty"), (8, True)])
def test_gloo_ranks_gather_oracle_coded_shards(world, balanced):
    from oracle import oracle as O
    from compression_without_quantization_amd.synthetic import make_blocks_range
    O.build()
    nb, d, bits = 40, 8, 6
    cost = None
    if balanced == "empty":  # all the cost in the first block: ranks 1.. own nothing
        cost = [1e9] + [0.0] * (nb - 1)
    elif balanced:
        cost = np.random.default_rng(3).integers(1, 50, nb).astype(np.float64).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nb, cost, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    h = make_blocks_range(0, nb, d, bits)
    want, _ = O.greedy_encode(h["post_loc"], h["post_scale"], h["prior_loc"], h["prior_scale"],
                              np.arange(nb + 1, dtype=np.int64) * d, bits, 1, 42)
    assert got == want.reshape(-1).tolist()


def test_make_blocks_range_is_shard_independent():
    from compression_without_quantization_amd.synthetic import make_blocks_range
    full = make_blocks_range(0, 70000, 4, 8, chunk=1 << 15)
    for b0, b1 in ((0, 1), (32767, 32769), (40000, 70000), (65535, 65536)):
        part = make_blocks_range(b0, b1, 4, 8, chunk=1 << 15)
        for k in full:
            assert np.array_equal(part[k], full[k][b0:b1])


def test_rank_device_map_refuses_shared_gpu_under_rccl(monkeypatch):
    """bench.py's rank -> device check: with the nccl (RCCL) backend two ranks
    on one GPU are refused; distinct GPUs (or gloo, the shared-GPU rehearsal)
    pass and the map is returned for the bench line."""
    import sys
    from conftest import REPO
    sys.path.insert(0, REPO)
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    import bench

    class P:
        pci_bus_id = None

    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda dev: P())

    class FakeDist:
        def __init__(self, backend, devices):
            self.backend, self.devices = backend, devices

        def get_world_size(self):
            return len(self.devices)

        def get_backend(self):
            return self.backend

        def all_gather_object(self, out, me):
            for r, dv in enumerate(self.devices):
                out[r] = dict(me, rank=r, local_rank=r, device=dv)

    dev = torch.device("cuda", 0)
    m = bench.rank_device_map(FakeDist("nccl", [0, 1, 2, 3]), 0, 0, dev)
    assert [x["device"] for x in m] == [0, 1, 2, 3]
    assert len(bench.rank_device_map(FakeDist("gloo", [0, 0]), 0, 0, dev)) == 2
    with pytest.raises(SystemExit, match="share GPU"):
        bench.rank_device_map(FakeDist("nccl", [0, 1, 1]), 0, 0, dev)


def test_rank_deadline_stops_stuck_and_failed_ranks():
    """bench.py --gpus N's own launcher cannot hang the SCALE run: a rank that
    exits non-zero stops the others at once (its code is returned), and ranks
    still running at the deadline are stopped and 124 returned, within the
    deadline plus the stop grace, with no child left running."""
    import subprocess
    import sys
    import time
    from conftest import REPO
    sys.path.insert(0, REPO)
    import bench
    env = dict(os.environ)
    sleeper = [sys.executable, "-c", "import time; time.sleep(600)"]
    failer = [sys.executable, "-c", "import time, sys; time.sleep(0.5); sys.exit(3)"]
    ok = [sys.executable, "-c", "pass"]
    # one rank fails, one would sleep for ten minutes
    t0 = time.monotonic()
    procs = []
    real_popen = subprocess.Popen

    def track(*a, **k):
        p = real_popen(*a, **k)
        procs.append(p)
        return p
    try:
        subprocess.Popen = track
        rc = bench.run_rank_processes([(failer, env), (sleeper, env)], deadline_s=60)
        assert rc == 3
        assert time.monotonic() - t0 < 30
        assert all(p.poll() is not None for p in procs)
        # both sleep past the deadline: stopped, 124
        procs.clear()
        t0 = time.monotonic()
        rc = bench.run_rank_processes([(sleeper, env), (ok, env), (sleeper, env)], deadline_s=2)
        assert rc == 124
        assert time.monotonic() - t0 < 2 + 5 + 5
        assert all(p.poll() is not None for p in procs)
        # a rank that ignores SIGTERM is killed after the grace period
        stubborn = [sys.executable, "-c", "import signal, time; "
                    "signal.signal(signal.SIGTERM, signal.SIG_IGN); time.sleep(600)"]
        procs.clear()
        t0 = time.monotonic()
        rc = bench.run_rank_processes([(stubborn, env)], deadline_s=1)
        assert rc == 124 and time.monotonic() - t0 < 1 + 5 + 5
        assert all(p.poll() is not None for p in procs)
        assert bench.run_rank_processes([(ok, env), (ok, env)], deadline_s=60) == 0
    finally:
        subprocess.Popen = real_popen
        for p in procs:
            if p.poll() is None:
                p.kill()


def test_devices_distinct():
    import sys
    from conftest import REPO
    sys.path.insert(0, REPO)
    import bench
    m = [{"host": "h", "pci_bus": b, "visible": None, "device": i} for i, b in enumerate([3, 4])]
    assert bench.devices_distinct(m)
    assert not bench.devices_distinct(m + [dict(m[0], device=5)])
    m2 = [{"host": "h", "pci_bus": None, "visible": "0,1", "device": i} for i in (0, 1, 1)]
    assert not bench.devices_distinct(m2) and bench.devices_distinct(m2[:2])
