"""Synthetic diagonal-Gaussian latent blocks.

No Kodak images or trained PLN checkpoints exist offline, so benchmarks and
parity tests use blocks of the configured shape:

  prior      p_loc ~ N(0,1), p_scale ~ U[0.5, 2]
  target     t_scale ~ U[0.3, 0.9], t_loc = alpha * m, m ~ N(0,1), with alpha
             solved per block so that the block KL
             sum_j 0.5 (t_loc^2 + t_scale^2 - 1 - 2 ln t_scale) equals K nats
             (K = kl_bits*ln2 - 1, the reference's n_nats_per_group,
             coded_greedy_sampler.py:226; C1 uses K = 4 ln2 exactly);
             blocks whose scale part alone exceeds K get their log-scale
             deviations shrunk until it takes K/2.
  posterior  post_loc = p_loc + p_scale * t_loc, post_scale = p_scale * t_scale

Generator: numpy PCG64(20261015) unless a seed is given.
"""
import numpy as np

DEFAULT_SEED = 20261015


def target_nats(kl_bits, exact=False):
    return kl_bits * np.log(2) if exact else kl_bits * np.log(2) - 1


def make_blocks(nb, d, kl_bits, seed=DEFAULT_SEED, exact_kl=False, chunk=1 << 16):
    """Returns dict of float32 arrays [nb, d]: prior_loc, prior_scale, post_loc, post_scale."""
    rng = np.random.Generator(np.random.PCG64(seed))
    K = target_nats(kl_bits, exact_kl)
    out = {k: np.empty((nb, d), dtype=np.float32)
           for k in ("prior_loc", "prior_scale", "post_loc", "post_scale")}
    for b0 in range(0, nb, chunk):
        n = min(chunk, nb - b0)
        p_loc = rng.standard_normal((n, d))
        p_scale = rng.uniform(0.5, 2.0, (n, d))
        t_scale = rng.uniform(0.3, 0.9, (n, d))
        m = rng.standard_normal((n, d))
        rhs = 2 * K - np.sum(t_scale ** 2 - 1 - 2 * np.log(t_scale), axis=1)
        bad = rhs <= 0
        if bad.any():
            # the scale part alone exceeds K (large d, small K): shrink the
            # log-scale deviations of those blocks so it uses K/2 nats
            ls = np.log(t_scale[bad])
            lo = np.zeros(ls.shape[0])
            hi = np.ones(ls.shape[0])
            for _ in range(60):
                lam = 0.5 * (lo + hi)
                f = np.sum(np.exp(2 * lam[:, None] * ls) - 1 - 2 * lam[:, None] * ls, axis=1)
                over = f > K
                hi = np.where(over, lam, hi)
                lo = np.where(over, lo, lam)
            t_scale[bad] = np.exp(lo[:, None] * ls)
            rhs = 2 * K - np.sum(t_scale ** 2 - 1 - 2 * np.log(t_scale), axis=1)
        alpha = np.sqrt(rhs / np.sum(m ** 2, axis=1))
        t_loc = alpha[:, None] * m
        out["prior_loc"][b0:b0 + n] = p_loc
        out["prior_scale"][b0:b0 + n] = p_scale
        out["post_loc"][b0:b0 + n] = p_loc + p_scale * t_loc
        out["post_scale"][b0:b0 + n] = p_scale * t_scale
    return out


def make_blocks_range(b0, b1, d, kl_bits, seed=DEFAULT_SEED, chunk=1 << 16):
    """Blocks [b0, b1) of a global synthetic set of the make_blocks kind whose
    chunk c (blocks [c*chunk, (c+1)*chunk)) comes from its own generator
    PCG64(SeedSequence([seed, c])): any rank can build its shard without
    generating the blocks before it, and every sharding of the same global
    set sees the same data (bench.py strong/weak scaling)."""
    out = {k: np.empty((max(b1 - b0, 0), d), dtype=np.float32)
           for k in ("prior_loc", "prior_scale", "post_loc", "post_scale")}
    for c in range(b0 // chunk, (b1 + chunk - 1) // chunk if b1 > b0 else 0):
        part = make_blocks(chunk, d, kl_bits, seed=np.random.SeedSequence([seed, c]))
        lo, hi = max(b0, c * chunk), min(b1, (c + 1) * chunk)
        for k in out:
            out[k][lo - b0:hi - b0] = part[k][lo - c * chunk:hi - c * chunk]
    return out


def make_latents(D, bits_per_dim=1.1, off_fraction=0.5, seed=DEFAULT_SEED):
    """Flat PLN-like latents for the grouped path (configs C2/C3).

    A fraction of dims carries ~no information (posterior == prior up to
    noise, as inactive latent channels do); the rest have per-dim KL drawn
    from a Gamma distribution so the mean KL is ``bits_per_dim`` bits.
    Returns float32 arrays (q_loc, q_scale, p_loc, p_scale) of length D.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    p_loc = rng.standard_normal(D)
    p_scale = rng.uniform(0.5, 2.0, D)
    active = rng.uniform(size=D) >= off_fraction
    mean_nats = bits_per_dim * np.log(2) / max(1e-9, 1 - off_fraction)
    kl = np.where(active, rng.gamma(1.5, mean_nats / 1.5, D), rng.uniform(0, 1e-3, D))
    # split each dim's KL between a scale and a mean part
    t_scale = np.exp(-rng.uniform(0, 1, D) * np.sqrt(kl))  # <= 1
    kl_scale = 0.5 * (t_scale ** 2 - 1 - 2 * np.log(t_scale))
    t_loc2 = np.maximum(2 * (kl - kl_scale), 0.0)
    t_loc = np.sqrt(t_loc2) * np.where(rng.uniform(size=D) < 0.5, -1, 1)
    q_loc = p_loc + p_scale * t_loc
    q_scale = p_scale * t_scale
    f = lambda a: a.astype(np.float32)
    return f(q_loc), f(q_scale), f(p_loc), f(p_scale)
