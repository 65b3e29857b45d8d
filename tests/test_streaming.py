"""Host-side argument handling of encode_blocks_host (no GPU needed); the
streamed results themselves are checked on the GPU in test_shards_gpu.py."""
import numpy as np
import pytest

import compression_without_quantization_amd as C


def test_streamed_rejects_mismatched_sizes():
    a = np.zeros(64, np.float32)
    with pytest.raises(ValueError, match="same size"):
        C.encode_blocks_host(a, a, a, np.zeros(63, np.float32), 8, 1, 42, 8)


def test_streamed_rejects_partial_blocks():
    a = np.zeros(60, np.float32)
    with pytest.raises(ValueError, match="multiple of block_dim"):
        C.encode_blocks_host(a, a, a, a, 8, 1, 42, 8)
    with pytest.raises(ValueError, match="multiple of block_dim"):
        C.encode_blocks_host(a, a, a, a, 8, 1, 42, 0)


def test_streamed_empty_job_returns_empty_arrays():
    a = np.zeros(0, np.float32)
    idx, sample = C.encode_blocks_host(a, a, a, a, 8, 3, 42, 16)
    assert idx.shape == (0, 3) and idx.dtype == np.int32
    assert sample.shape == (0,) and sample.dtype == np.float32
