"""Multi-GPU block sharding.

Blocks are independent and their seeds depend only on the global block index
(coded_greedy_sampler.py:282 ``seed + i``), so each rank codes a contiguous
block range with ``block_id_base`` = its first block: no collective is needed
on the data path.  ``gather_indices`` is the optional all-gather for a caller
that wants every rank to hold the whole index array.
"""
import numpy as np
import torch


def shard_range(nb, world_size, rank, cost=None):
    """Contiguous [b0, b1) block range of ``rank``.

    Without ``cost`` blocks are split evenly; with a per-block ``cost`` (e.g.
    d_g * 2^b * n_steps for ragged groups) the cut points equalise the
    prefix sums of cost.
    """
    if world_size < 1 or not (0 <= rank < world_size):
        raise ValueError("bad world_size / rank")
    if cost is None:
        b0 = (nb * rank) // world_size
        b1 = (nb * (rank + 1)) // world_size
        return b0, b1
    c = np.asarray(cost, dtype=np.float64).reshape(-1)
    if c.size != nb:
        raise ValueError("cost must have one entry per block")
    pref = np.concatenate([[0.0], np.cumsum(c)])
    tot = pref[-1]
    cuts = [0] + [int(np.searchsorted(pref, tot * r / world_size, side="left"))
                  for r in range(1, world_size)] + [nb]
    cuts = np.maximum.accumulate(np.clip(cuts, 0, nb))
    return int(cuts[rank]), int(cuts[rank + 1])


def gather_indices(local_idx, nb_per_rank, group=None):
    """All-gather each rank's int32 index block (ranks own equal block counts).

    Works with any torch.distributed backend (RCCL on GPU, gloo on CPU).
    """
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [torch.empty_like(local_idx) for _ in range(world)]
    dist.all_gather(parts, local_idx.contiguous(), group=group)
    return torch.cat(parts, dim=0)
