"""First-call latency of the PLN codec (MIOpen algorithm selection) vs later calls."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import compression_without_quantization_amd.coded_greedy_sampler as S
import compression_without_quantization_amd.coded_importance_sampler as I
from compression_without_quantization_amd import pln as P
S.VERBOSE = I.VERBOSE = False
m = P.ProbabilisticLadderNetwork().cuda().eval()
rng = np.random.default_rng(0)
img = rng.uniform(0, 1, (1, 512, 768, 3)).astype(np.float32)
for i in range(3):
    torch.cuda.synchronize(); t = time.perf_counter()
    m.code_image_greedy(None, img, 42, comp_file_path="/tmp/x.miracle", second_level_max_group_size_bits=2,
                        second_level_dim_kl_bit_limit=16, first_level_dim_kl_bit_limit=16)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    m.decode_image_greedy(None, "/tmp/x.miracle", use_importance_sampling=False,
                          second_level_max_group_size_bits=2)
    torch.cuda.synchronize(); t2 = time.perf_counter()
    print(f"call {i}: compress {1e3 * (t1 - t):.1f} ms, decompress {1e3 * (t2 - t1):.1f} ms", flush=True)
