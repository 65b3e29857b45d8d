import os, sys, time
sys.argv = ["bench.py", "--config", "c3", "--no-cpu", "--no-e2e", "--batch-only"]
sys.path.insert(0, os.getcwd())
import bench
import compression_without_quantization_amd as C
import torch
args = bench.parse()
# run grouped_main but intercept timed() by monkeypatching time.perf_counter? simpler: call it
bench.grouped_main(args)
