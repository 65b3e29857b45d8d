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


def gather_indices(local_idx, nb_per_rank=None, group=None):
    """All-gather every rank's index block along dim 0, in rank order.

    Ranks may own different block counts (``shard_range`` cuts are uneven, and
    cost-balanced cuts for ragged groups more so): the row counts are
    all-gathered first, each rank's block is padded to the largest, gathered,
    and the padding dropped.  ``nb_per_rank`` is accepted for compatibility and
    ignored.  Works with any torch.distributed backend (RCCL on GPU, gloo on
    CPU); the tensors stay on local_idx's device.  This is the optional
    collective of SURVEY.md 8(e): the coding itself needs none.
    """
    import torch.distributed as dist
    world = dist.get_world_size(group)
    x = local_idx.contiguous()
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    sizes = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(v.item()) for v in sizes]
    m = max(sizes) if sizes else 0
    if m == 0:
        return x[:0]
    if x.shape[0] < m:
        pad = torch.zeros((m - x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        x = torch.cat([x, pad], dim=0)
    parts = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(parts, x, group=group)
    return torch.cat([p[:k] for p, k in zip(parts, sizes)], dim=0)
