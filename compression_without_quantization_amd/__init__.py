"""MI355X-native greedy coded sampler (compression without quantization).

Public surface mirrors the reference's code/coded_greedy_sampler.py,
code/misc.py and code/binary_io.py (bit-string helpers); every sample is
computed by the gfx950 kernels in libcwq.so (see include/cwq.h).
"""
from .binary_io import (bitcode_to_indices, elias_delta_code, elias_delta_decode,
                        elias_delta_code_many, elias_delta_decode_many,
                        from_bit_string, indices_to_bitcode, read_bin_code, to_bit_string,
                        write_bin_code)
from .coding import ArithmeticCoder
from .coded_greedy_sampler import (Normal, code_greedy_sample, code_grouped_greedy_sample,
                                   code_grouped_greedy_sample_batch,
                                   decode, decode_blocks, decode_greedy_sample,
                                   decode_grouped_greedy_sample, encode, encode_blocks,
                                   encode_workspace_bytes, group_size_threshold, group_starts)
from .coded_importance_sampler import (code_grouped_importance_sample,
                                       code_grouped_importance_sample_batch,
                                       code_importance_sample,
                                       decode_grouped_importance_sample,
                                       decode_importance_sample, importance_decode_blocks,
                                       importance_encode_blocks)
from .misc import stateless_normal_sample
from .pln import ProbabilisticLadderNetwork, build_empirical_dists
from .parallel import gather_indices, shard_range
from .streaming import encode_blocks_host

__all__ = [
    "Normal", "code_greedy_sample", "decode_greedy_sample", "code_grouped_greedy_sample",
    "decode_grouped_greedy_sample", "encode", "decode", "encode_blocks", "decode_blocks",
    "encode_workspace_bytes", "group_starts", "group_size_threshold",
    "stateless_normal_sample", "to_bit_string", "from_bit_string", "indices_to_bitcode",
    "bitcode_to_indices", "shard_range", "gather_indices", "elias_delta_code",
    "elias_delta_decode", "elias_delta_code_many", "elias_delta_decode_many",
    "code_importance_sample", "decode_importance_sample",
    "code_grouped_importance_sample", "decode_grouped_importance_sample",
    "code_grouped_importance_sample_batch",
    "importance_encode_blocks", "importance_decode_blocks", "ArithmeticCoder",
    "write_bin_code", "read_bin_code", "ProbabilisticLadderNetwork", "build_empirical_dists",
    "encode_blocks_host", "code_grouped_greedy_sample_batch",
]
