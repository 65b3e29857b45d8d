"""Build libcwq.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libcwq.so")
SOURCES = ["cwq_kernels.hip", "cwq_importance.hip", "cwq_pln.hip", "cwq_partition.hip", "cwq_capi.hip",
           "cwq_ac.cpp"]
HEADERS = ["cwq_math.h", "cwq_kernels.h", "cwq_device.h", "cwq_debug.h"]

# -ffp-contract=off: every FMA in the arithmetic is explicit (bit-exactness).
# Division and sqrt stay IEEE correctly rounded (hipcc's default
# -fhip-fp32-correctly-rounded-divide-sqrt); no fast-math.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
         "-fPIC", "-shared", "-Wall", "-Wno-unused-function"]
# the batch call's result copies go to the SDMA engines through the HSA runtime
LIBS = ["-L/opt/rocm/lib", "-lhsa-runtime64"]


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "cwq.h"))
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force=False, verbose=True):
    if not force and not _stale():
        return OUT
    cmd = ["hipcc"] + FLAGS + ["-o", OUT] + [os.path.join(CSRC, s) for s in SOURCES] + LIBS
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
