"""CPU: libcwq.so loads, exports every symbol include/cwq.h declares, and its
host-side validation / host functions behave (no GPU compute is called)."""
import os
import re

import numpy as np

from conftest import REPO
from compression_without_quantization_amd import _lib


def _header_symbols():
    with open(os.path.join(REPO, "include", "cwq.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cwq_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_header_symbol(cwqlib):
    syms = _header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(cwqlib, s), s
    assert sorted(_lib.SIGNATURES) == syms


def test_version_and_error(cwqlib):
    assert cwqlib.cwq_version() >= 1
    # the message is thread-local and kept until the next call: an empty
    # (n = 0) call succeeds without touching the device and clears it
    assert cwqlib.cwq_pln_posterior(None, None, None, None, 0, 1e-12, None, None, None) == 0
    assert cwqlib.cwq_last_error() == b""


def test_invalid_args_rejected_before_launch(cwqlib):
    # argument validation happens on the host before any HIP call
    rc = cwqlib.cwq_greedy_encode_uniform(None, None, None, None, 1, 4, 31, 1, 42, 1.0, 0,
                                          None, None, None, 0, None, None)
    assert rc == -1 and b"n_bits_per_step" in cwqlib.cwq_last_error()
    rc = cwqlib.cwq_greedy_encode_uniform(None, None, None, None, 1, 4, 8, 0, 42, 1.0, 0,
                                          None, None, None, 0, None, None)
    assert rc == -1 and b"n_steps" in cwqlib.cwq_last_error()
    need = cwqlib.cwq_greedy_encode_uniform_workspace_size(10, 4)
    assert need >= 10 * 8 + 3 * 40 * 4
    rc = cwqlib.cwq_greedy_encode_uniform(1, 1, 1, 1, 10, 4, 8, 1, 42, 1.0, 0, 1, 1, 1,
                                          need - 1, None, None)
    assert rc == -3


def test_workspace_sizes_and_options_rejected(cwqlib):
    """CSR encodes need the general pruned kernel's arrays: the CSR size always
    holds them, so a CSR call given only the uniform-kernel size is refused
    with CWQ_ERR_WORKSPACE (no silent unpruned run); bad options are refused
    before any launch."""
    from compression_without_quantization_amd import _lib
    nb, d = 10, 32
    uni = cwqlib.cwq_greedy_encode_uniform_workspace_size(nb, d)
    csr = cwqlib.cwq_greedy_encode_workspace_size(nb, nb * d, d)
    assert csr >= uni + 16 * nb * d + 180 * nb
    # uniform d outside the fast kernel: the general layout either way
    assert cwqlib.cwq_greedy_encode_uniform_workspace_size(nb, 9) == \
        cwqlib.cwq_greedy_encode_workspace_size(nb, nb * 9, 9)
    # blocks longer than 1024 dims add the visit-order records (32 B/dim)
    long_ = cwqlib.cwq_greedy_encode_workspace_size(nb, nb * 2000, 2000)
    assert long_ >= cwqlib.cwq_greedy_encode_workspace_size(nb, nb * 2000, 1024) + 32 * nb * 2000
    assert cwqlib.cwq_greedy_encode_uniform_workspace_size(nb, 2000) == long_
    rc = cwqlib.cwq_greedy_encode(1, 1, 1, 1, 1, nb, nb * d, d, 8, 1, 42, 1.0, 0, 1, 1, 1,
                                  uni, None, None)
    assert rc == -3 and b"workspace" in cwqlib.cwq_last_error()
    for bad in (_lib.options(prune_mode=3), _lib.options(prune_mode=-1),
                _lib.options(eval_events=(1, None))):
        rc = cwqlib.cwq_greedy_encode_uniform(1, 1, 1, 1, nb, d, 8, 1, 42, 1.0, 0, 1, 1, 1,
                                              uni, bad, None)
        assert rc == -1 and b"cwq_options" in cwqlib.cwq_last_error()
    o = _lib.options(prune_mode=1)
    o.contents.reserved = 5
    assert cwqlib.cwq_greedy_encode_uniform(1, 1, 1, 1, nb, d, 8, 1, 42, 1.0, 0, 1, 1, 1, uni,
                                            o, None) == -1


def test_group_starts_host(cwqlib):
    kl = np.array([0.5, 0.5, 5.0, 0.1, 0.1], np.float32)
    starts = np.zeros(16, np.int64)
    n = cwqlib.cwq_group_starts(kl.ctypes.data, kl.size, 4095, 2 * np.log(2) - 1,
                                starts.ctypes.data, 16)
    # n_nats = 0.386: dim0 alone (0.5 >= n_nats at idx 0 -> duplicate 0) ...
    assert list(starts[:n]) == [0, 0, 1, 2, 3, 4, 5]


def test_missing_library_fails_loudly(tmp_path):
    """No CPU fallback: with the library absent the product path raises on
    first use instead of routing anywhere else."""
    import subprocess
    import sys
    code = ("import numpy as np, compression_without_quantization_amd as C\n"
            "try:\n"
            "    C.encode_blocks(np.zeros(4, np.float32), np.ones(4, np.float32),\n"
            "                    np.zeros(4, np.float32), np.ones(4, np.float32), 4, 1, 0)\n"
            "except (ImportError, OSError) as e:\n"
            "    print('raised', type(e).__name__)\n")
    env = dict(os.environ, CWQ_LIB_PATH=str(tmp_path / "absent" / "libcwq.so"))
    out = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env,
                         capture_output=True, text=True, timeout=120)
    assert "raised" in out.stdout, (out.stdout, out.stderr)


def test_abi_version_checked(cwqlib, tmp_path):
    """The header's CWQ_ABI_VERSION, the bindings' and the library's agree, and
    a library reporting another version is refused at load time even when
    selected through CWQ_LIB_PATH (its argument lists would differ)."""
    import subprocess
    import sys
    with open(os.path.join(REPO, "include", "cwq.h")) as f:
        m = re.search(r"#define CWQ_ABI_VERSION \(\((\d+) << 16\) \| (\d+)\)", f.read())
    assert m, "CWQ_ABI_VERSION missing from include/cwq.h"
    hdr = (int(m.group(1)) << 16) | int(m.group(2))
    assert hdr == _lib.ABI_VERSION == cwqlib.cwq_version()
    src = tmp_path / "old.c"
    src.write_text("int cwq_version(void) { return 1; }\n")
    so = tmp_path / "libold.so"
    subprocess.check_call(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)])
    code = ("from compression_without_quantization_amd import _lib\n"
            "try:\n    _lib.load()\nexcept ImportError as e:\n    print('refused', e)\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True,
                       env=dict(os.environ, CWQ_LIB_PATH=str(so)), timeout=120)
    assert "refused" in r.stdout and "ABI version 0.1" in r.stdout, r.stdout + r.stderr
