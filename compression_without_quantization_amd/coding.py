"""Arithmetic coder -- code/coding.pyx:27-310 (the reference's Cython
ArithmeticCoder) on the C++ implementation in libcwq.so (csrc/cwq_ac.cpp).

Used by the reference's image codec for group-size side information
(pln.py:517-529 encode, pln.py:708-709 decode): symbol 0 is EOF, callers
append it to the message and strip it after decoding.
"""
import numpy as np

from . import _lib


class ArithmeticCoder(object):
    """ArithmeticCoder(P, precision=32) with encode / decode / decode_fast.

    The reference builds an interval AVL tree for decode_fast and prints its
    depth (coding.pyx:50-51); here decode_fast is a binary search over the
    same scaled CDF (identical symbols, no tree, no print).
    """

    def __init__(self, P, precision=32):
        self._P = np.ascontiguousarray(np.asarray(P, dtype=np.int64).reshape(-1))
        self._precision = int(precision)
        self.C = np.concatenate([[0], np.cumsum(self._P)[:-1]]).astype(np.int64)
        self.D = np.cumsum(self._P).astype(np.int64)
        self.R = int(self.D[-1]) if self.D.size else 0

    def encode(self, message):
        """coding.pyx:59-125 -> list of '0'/'1' characters."""
        lib = _lib.load()
        msg = np.ascontiguousarray(np.asarray(message, dtype=np.int64).reshape(-1))
        P = self._P
        mp = msg.ctypes.data if msg.size else None
        # one pass into a buffer of a generous size (group sizes code at a few
        # bits a symbol); a message that needs more is sized by a counting pass
        cap = 32 * msg.size + 1024
        buf = np.empty(cap, dtype=np.uint8)
        n = lib.cwq_ac_encode(P.ctypes.data, P.size, self._precision, mp, msg.size,
                              buf.ctypes.data, cap)
        if n == -4:  # CWQ_ERR_CAPACITY
            n = _lib.check(lib.cwq_ac_encode(P.ctypes.data, P.size, self._precision, mp,
                                             msg.size, None, 0), "cwq_ac_encode")
            buf = np.empty(max(n, 1), dtype=np.uint8)
            n = lib.cwq_ac_encode(P.ctypes.data, P.size, self._precision, mp, msg.size,
                                  buf.ctypes.data, n)
        _lib.check(n, "cwq_ac_encode")
        return list(buf[:n].tobytes().decode("ascii"))

    def decode_fast(self, code, verbose=False):
        """coding.pyx:220-310 -> list of symbols up to and including EOF (0)."""
        lib = _lib.load()
        if isinstance(code, (list, tuple)):
            code = ''.join(code)
        bits = np.frombuffer(code.encode("ascii") if isinstance(code, str) else bytes(code),
                             dtype=np.uint8)
        cap = max(64, 2 * bits.size + 64)
        while True:
            out = np.empty(cap, dtype=np.int64)
            n = lib.cwq_ac_decode(self._P.ctypes.data, self._P.size, self._precision,
                                  bits.ctypes.data if bits.size else None, bits.size,
                                  out.ctypes.data, cap)
            if n == -4 and cap < (1 << 34):  # CWQ_ERR_CAPACITY: very skewed counts
                cap *= 8
                continue
            _lib.check(n, "cwq_ac_decode")
            if verbose:
                print("decoded {} symbols".format(n))
            return [int(v) for v in out[:n]]

    decode = decode_fast  # coding.pyx:129-216 yields the same symbols
