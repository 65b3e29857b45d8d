"""CPU: multi-rank block sharding over gloo (world_size 2), as bench.py --gpus N
uses it (no collective on the data path; optional all-gather of indices)."""
import os
import socket

import numpy as np
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


def _worker(rank, world, port, nb, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b0, b1 = shard_range(nb, world, rank)
    # stand-in for per-rank coded indices: a deterministic function of the
    # global block id (what block_id_base guarantees for the real coder)
    local = torch.arange(b0, b1, dtype=torch.int32) * 7 + 3
    full = gather_indices(local, b1 - b0)
    if rank == 0:
        out.put(full.numpy().tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_gather():
    world, nb = 2, 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nb, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == [b * 7 + 3 for b in range(nb)]
