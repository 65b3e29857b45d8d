"""Host-resident blocks through the encoder with the PCIe copies hidden.

``encode_blocks`` codes blocks that are already in HBM.  A caller holding the
distributions in host memory (numpy, as ``code/pln.py`` does after its TF
session) would otherwise pay the host->device copy of 16 d bytes per block and
the device->host copy of the results in series with the coding: ~7% on C4.
``encode_blocks_host`` streams the blocks in chunks instead, two device buffer
slots alternating:

* chunk c's inputs are copied to HBM (on a copy stream) while the compute
  stream still codes chunk c - 1;
* chunk c - 1's indices and sample come back into the caller's result arrays
  once it is coded, while chunk c is already queued behind it.

The copies go straight from and to the caller's pageable arrays: the HIP
runtime stages them through its own pinned buffers faster than a Python-side
copy into pinned memory (measured: that variant was CPU-bound at ~1.5 GB/s).
The host thread blocks only while a copy runs or while it waits for chunk
c - 1; the GPU always has the next chunk queued.  Chunk c is coded with
``block_id_base = base + c * chunk``, so the result is bit-identical to one
``encode_blocks`` call over all blocks (the seed of block g depends only on its
global index, coded_greedy_sampler.py:282).
"""
import numpy as np
import torch

from .coded_greedy_sampler import encode_blocks, encode_workspace_bytes


def encode_blocks_host(t_loc, t_scale, p_loc, p_scale, n_bits_per_step, n_steps, seed,
                       block_dim, rho=1., block_id_base=0, chunk_blocks=None, device=None,
                       prune_mode=None):
    """Uniform blocks (``block_dim`` dims each) from host float32 arrays.

    Returns (idx np.int32 [nb, n_steps], sample np.float32 [D]) equal to
    ``encode_blocks`` on the same inputs.  ``chunk_blocks`` blocks move and
    code per step of the pipeline; by default an eighth of the job (at least
    131,072 blocks): each launch ends with a tail in which the chip drains, so
    fewer, larger chunks code faster, while the first chunk's inputs and the
    last chunk's results are the copies left exposed (C4 on one MI355X,
    tools/stream_chunks.py: 65,536-block chunks 2.99e6 blocks/s, 131,072
    3.05e6, 262,144 3.04e6, 500,000 2.99e6; unpipelined 2.89e6,
    device-resident 3.09e6).  A job of one chunk takes the plain copy-in /
    encode / copy-out sequence.
    """
    arrs = [np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1))
            for a in (t_loc, t_scale, p_loc, p_scale)]
    D = arrs[0].size
    if any(a.size != D for a in arrs[1:]):
        raise ValueError("t_loc, t_scale, p_loc, p_scale must have the same size")
    d = int(block_dim)
    if d <= 0 or D % d:
        raise ValueError(f"D={D} is not a multiple of block_dim={block_dim}")
    nb = D // d
    n_steps = int(n_steps)
    idx_out = np.empty((nb, n_steps), dtype=np.int32)
    sample_out = np.empty(D, dtype=np.float32)
    if nb == 0:
        return idx_out, sample_out
    dev = torch.device(device) if device is not None else torch.device("cuda",
                                                                       torch.cuda.current_device())
    if chunk_blocks is None:
        chunk_blocks = max(131072, -(-nb // 8))
    cb = max(1, min(int(chunk_blocks), nb))
    n_chunks = (nb + cb - 1) // cb
    if n_chunks == 1:
        # nothing to overlap: one copy in, one encode, one copy out on the
        # caller's stream (the pipeline's extra stream, events and slots only
        # cost here: C5's 1,024 blocks ran 23.9k blocks/s through them against
        # 28.1k for the plain sequence, round 4)
        with torch.cuda.device(dev):
            x = [torch.from_numpy(a).to(dev) for a in arrs]
            idx, smp = encode_blocks(x[0], x[1], x[2], x[3], n_bits_per_step, n_steps, seed,
                                     rho=rho, block_dim=d, block_id_base=int(block_id_base),
                                     prune_mode=prune_mode)
            idx_out[:] = idx.cpu().numpy().reshape(nb, n_steps)
            sample_out[:] = smp.cpu().numpy().reshape(-1)
        return idx_out, sample_out
    nslot = min(2, n_chunks)
    host_in = [torch.from_numpy(a) for a in arrs]
    host_idx, host_smp = torch.from_numpy(idx_out), torch.from_numpy(sample_out)
    with torch.cuda.device(dev):
        compute = torch.cuda.current_stream(dev)
        copy = torch.cuda.Stream(dev)
        dev_in = [torch.empty((4, cb * d), dtype=torch.float32, device=dev)
                  for _ in range(nslot)]
        dev_idx = [torch.empty((cb, n_steps), dtype=torch.int32, device=dev)
                   for _ in range(nslot)]
        dev_smp = [torch.empty(cb * d, dtype=torch.float32, device=dev) for _ in range(nslot)]
        ws = [torch.empty(max(encode_workspace_bytes(cb, cb * d, block_dim=d), 1),
                          dtype=torch.uint8, device=dev) for _ in range(nslot)]
        in_done = [torch.cuda.Event() for _ in range(nslot)]  # the slot's inputs are in HBM
        coded = [torch.cuda.Event() for _ in range(nslot)]    # the slot's chunk is coded

        def fetch(c):  # chunk c's results into the caller's arrays (blocks until coded)
            s = c % nslot
            b0, b1 = c * cb, min(nb, (c + 1) * cb)
            n = b1 - b0
            with torch.cuda.stream(copy):
                copy.wait_event(coded[s])
                host_idx[b0:b1].copy_(dev_idx[s][:n])
                host_smp[b0 * d:b1 * d].copy_(dev_smp[s][:n * d])

        for c in range(n_chunks):
            s = c % nslot
            b0, b1 = c * cb, min(nb, (c + 1) * cb)
            n = b1 - b0
            with torch.cuda.stream(copy):
                # after chunk c - 2's encode (which read dev_in[s]) and its fetch
                copy.wait_event(coded[s])
                for k in range(4):
                    dev_in[s][k, :n * d].copy_(host_in[k][b0 * d:b1 * d], non_blocking=True)
                in_done[s].record(copy)
            with torch.cuda.stream(compute):
                compute.wait_event(in_done[s])
                x = dev_in[s]
                encode_blocks(x[0, :n * d], x[1, :n * d], x[2, :n * d], x[3, :n * d],
                              n_bits_per_step, n_steps, seed, rho=rho, block_dim=d,
                              block_id_base=int(block_id_base) + b0,
                              out_idx=dev_idx[s][:n], out_sample=dev_smp[s][:n * d],
                              workspace=ws[s], prune_mode=prune_mode)
                coded[s].record(compute)
            if c >= 1:
                fetch(c - 1)
        fetch(n_chunks - 1)
        compute.wait_stream(copy)
    return idx_out, sample_out
