"""code/misc.py:3-17 -- the candidate RNG, on the GPU."""
import numpy as np
import torch

from . import _lib
from .coded_greedy_sampler import _device_of, _f32, _like_input, _ptr


def stateless_normal_sample(loc, scale, num_samples, seed):
    """misc.py:3-17: loc + scale * tf.random.stateless_normal([N] + shape, seed=[seed, 42]).

    ``loc``/``scale`` are float32 of any shape; returns [num_samples, *shape].
    """
    lib = _lib.load()
    dev = _device_of(loc, scale)
    shape = tuple(loc.shape) if isinstance(loc, torch.Tensor) else tuple(np.shape(loc))
    l = _f32(loc, dev, "loc")
    s = _f32(scale, dev, "scale")
    if l.numel() != s.numel():
        raise ValueError("loc and scale must have the same size")
    d = l.numel()
    out = torch.empty((int(num_samples),) + shape, dtype=torch.float32, device=dev)
    seed32 = int(np.int32(np.uint32(int(seed) & 0xFFFFFFFF)))
    rc = lib.cwq_stateless_normal_sample(_ptr(l), _ptr(s), d, int(num_samples), seed32,
                                         _ptr(out), torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(rc, "cwq_stateless_normal_sample")
    return _like_input(out, loc)
