"""Index <-> bit-string helpers (code/binary_io.py:41-67).

``to_bit_string`` / ``from_bit_string`` keep the reference's semantics exactly
(LSB first; overflow raises the reference's exception).  The vectorised
helpers turn whole index arrays into the concatenated bitcode the grouped
coder emits (coded_greedy_sampler.py:81-87, :288) and back.
"""
import numpy as np


def to_bit_string(num, num_bits):
    """binary_io.py:41-53 -- ``num`` as ``num_bits`` '0'/'1' chars, LSB first."""
    if num >= 2 ** num_bits:
        raise Exception("The number {} (>= {}) is bigger than what we can encode!".format(
            num, 2 ** num_bits))
    bitcode = []
    for _ in range(num_bits):
        bitcode.append(str(num % 2))
        num //= 2
    return ''.join(bitcode)


def from_bit_string(bitcode):
    """binary_io.py:55-67 -- LSB-first '0'/'1' string (str or bytes) -> int."""
    num = 0
    if isinstance(bitcode, bytes):
        bitcode = bitcode.decode("utf-8")
    for i in range(len(bitcode)):
        if bitcode[i] == "1":
            num += 2 ** i
    return num


def indices_to_bitcode(indices, num_bits):
    """Concatenate ``to_bit_string(i, num_bits)`` over a flat index array.

    Row-major order of ``indices`` is the reference's order (steps within a
    group, then groups, coded_greedy_sampler.py:81-87 and :288).
    """
    idx = np.ascontiguousarray(np.asarray(indices).reshape(-1)).astype(np.int64)
    if num_bits == 0:
        if idx.size and (idx != 0).any():
            bad = int(idx[idx != 0][0])
            to_bit_string(bad, 0)  # raises the reference's exception
        return ''
    if idx.size and (idx.min() < 0 or idx.max() >= (1 << num_bits)):
        bad = int(idx[(idx < 0) | (idx >= (1 << num_bits))][0])
        to_bit_string(bad, num_bits)  # raises the reference's exception
    shifts = np.arange(num_bits, dtype=np.int64)
    bits = ((idx[:, None] >> shifts[None, :]) & 1).astype(np.uint8) + ord('0')
    return bits.tobytes().decode('ascii')


def bitcode_to_indices(bitcode, num_bits, count, dtype=np.int64):
    """Inverse of indices_to_bitcode for ``count`` indices (as ``dtype``).

    Missing trailing characters read as '0' (``from_bit_string`` of a short
    substring, as tf.strings.substr yields at the end of the string).  Widths
    up to 30 bits (CWQ_MAX_BITS_PER_STEP) are parsed by one native pass
    (cwq_bitcode_to_indices).
    """
    raw_b = bitcode if isinstance(bitcode, bytes) else bitcode.encode('ascii')
    count, num_bits = int(count), int(num_bits)
    if 0 <= num_bits <= 30 and count >= 0:
        from . import _lib
        out = np.empty(count, dtype=np.int32)
        _lib.check(_lib.load().cwq_bitcode_to_indices(raw_b, len(raw_b), num_bits, count,
                                                      out.ctypes.data), "bitcode parse")
        return out if dtype == np.int32 else out.astype(dtype)
    raw = np.frombuffer(raw_b, dtype=np.uint8)
    need = count * num_bits
    bits = np.zeros(need, dtype=np.int64)
    m = min(need, raw.size)
    bits[:m] = (raw[:m] == ord('1'))
    if num_bits == 0:
        return np.zeros(count, dtype=np.int64)
    bits = bits.reshape(count, num_bits)
    weights = (np.int64(1) << np.arange(num_bits, dtype=np.int64))
    return (bits * weights[None, :]).sum(axis=1).astype(dtype)


def elias_delta_code(x):
    """binary_io.py:7-21 -- Elias-delta code of x >= 1 as a '0'/'1' string.

    n = floor(log2 x) and l = floor(log2(n + 1)) are evaluated exactly as the
    reference does (np.log ratio in float64); for x < 2^31 that equals the
    bit length (pinned by tests/test_importance.py).
    """
    x = int(x)
    lg2 = np.log(2)
    n = int(np.floor(np.log(x) / lg2).astype(np.int32))
    l = int(np.floor(np.log(n + 1) / lg2).astype(np.int32))
    length_length_code = ''.join(["0"] * l)
    length_code = to_bit_string(n + 1, l + 1)[::-1]
    num_code = to_bit_string(x, n + 1)[::-1][1:]
    return length_length_code + length_code + num_code


def elias_delta_decode(x):
    """binary_io.py:23-39 -- decode one Elias-delta code at the start of x
    (bytes or str).  Returns (num, code_length)."""
    if isinstance(x, str):
        x = x.encode("ascii")
    l = 0
    while x[l] == 48:  # '0'
        l += 1
    x = x[l:]
    n_plus_one = from_bit_string(x[:l + 1][::-1])
    x = x[l + 1:]
    num = from_bit_string(x[:n_plus_one - 1][::-1] + b"1")
    return num, 2 * l + n_plus_one


def elias_delta_code_many(values):
    """''.join(elias_delta_code(v) for v in values), in one native call
    (cwq_elias_delta_encode).  Values >= 2^30, where the reference's float64
    formulas are not proven equal to the bit lengths, take the Python path."""
    from . import _lib
    x = np.ascontiguousarray(np.asarray(values, dtype=np.int64).reshape(-1))
    if x.size == 0:
        return ''
    if x.min() < 1 or x.max() >= (1 << 30):
        return ''.join(elias_delta_code(int(v)) for v in x)
    lib = _lib.load()
    # one pass into a buffer of the longest codes (x < 2^30: at most 38 chars)
    buf = np.empty(38 * x.size, dtype=np.uint8)
    n = _lib.check(lib.cwq_elias_delta_encode(x.ctypes.data, x.size, buf.ctypes.data, buf.size),
                   "elias encode")
    return str(memoryview(buf)[:n], 'ascii')


def elias_delta_decode_many(bitcode, count):
    """Parse ``count`` concatenated Elias-delta codes from the start of
    ``bitcode`` (str or bytes).  Returns (values int64 [count], chars consumed).
    Raises ValueError when the code runs out (cwq_elias_delta_decode)."""
    from . import _lib
    raw = bitcode.encode('ascii') if isinstance(bitcode, str) else bytes(bitcode)
    out = np.empty(max(int(count), 0), dtype=np.int64)
    if count <= 0:
        return out, 0
    lib = _lib.load()
    r = lib.cwq_elias_delta_decode(raw, len(raw), int(count), out.ctypes.data)
    if r < 0:
        raise ValueError("bitcode exhausted or corrupt: " +
                         lib.cwq_last_error().decode("utf-8", "replace"))
    return out, int(r)


# ---------------------------------------------------------------------------
# .miracle container (binary_io.py:69-197)
# ---------------------------------------------------------------------------
def _pack_bits(bits):
    """'0'/'1' string -> bytes, MSB first, zero padded to a byte (:76-78)."""
    if len(bits) % 8:
        bits = bits + "0" * (8 - len(bits) % 8)
    if not bits:
        return b""
    a = np.frombuffer(bits.encode("ascii"), dtype=np.uint8) - ord("0")
    return np.packbits(a).tobytes()


def write_bin_code(code, path, extras=None, extra_var_bits=None, var_length_extras=None,
                   var_length_bits=None):
    """binary_io.py:69-133: 4-byte big-endian extras, 16-bit-length variable
    bit strings, 16-bit-length + 8-bit-width integer lists, then the message
    bits, each section packed MSB-first with zero padding."""
    if var_length_extras is not None:
        if var_length_bits is None or len(var_length_extras) != len(var_length_bits):
            raise Exception("Each var length extra needs to have a bitlength associated!")
    out = bytearray()
    if extras is not None:
        for extra in extras:
            extra = int(extra)
            eb = []
            for _ in range(4):
                eb.append(extra % 256)
                extra = extra // 256
            out += bytes(eb[::-1])
    if extra_var_bits is not None:
        for bits in extra_var_bits:
            bits = ''.join(bits)
            out += bytes([len(bits) // 256, len(bits) % 256])
            out += _pack_bits(bits)
    if var_length_extras is not None:
        for extra, extra_bit_size in zip(var_length_extras, var_length_bits):
            extra = list(extra)
            out += bytes([len(extra) // 256, len(extra) % 256])
            out += bytes([extra_bit_size])
            out += _pack_bits(''.join(to_bit_string(int(item), extra_bit_size)
                                      for item in extra))
    out += _pack_bits(''.join(code))
    with open(path, "wb") as f:
        f.write(bytes(out))


class _ByteCursor:
    """Sequential reader over a .miracle file's bytes (every section of the
    container starts on a byte boundary, binary_io.py:69-133)."""

    def __init__(self, data):
        self.data = data
        self.pos = 0

    def take(self, n):
        if n < 0 or self.pos + n > len(self.data):
            raise ValueError(f"truncated .miracle file: {n} bytes wanted at byte {self.pos} "
                             f"of {len(self.data)}")
        out = self.data[self.pos:self.pos + n]
        self.pos += n
        return out

    def uint(self, n):
        """n-byte big-endian unsigned integer."""
        return int.from_bytes(self.take(n), "big")

    def bits(self, nbits):
        """The next ceil(nbits / 8) bytes as nbits MSB-first '0'/'1' flags (uint8)."""
        raw = np.frombuffer(self.take(-(-nbits // 8)), dtype=np.uint8)
        return np.unpackbits(raw)[:nbits]


def _chars(flags):
    return (flags + ord("0")).astype(np.uint8).tobytes().decode("ascii")


def read_bin_code(path, num_extras=0, num_extra_var_bits=0, num_var_length_extras=0,
                  extras_bytes=4, extra_bytes=2):
    """binary_io.py:135-197 -> (remaining message bits incl. padding, extras,
    extra_var_bits, var_length_extras).

    Parsed section by section from the file's bytes: ``extras_bytes``-byte
    big-endian extras; for each variable bit string an ``extra_bytes``-byte bit
    length and its bits, padded to a byte; for each integer list an
    ``extra_bytes``-byte length, a one-byte width w and its w-bit LSB-first
    values, padded to a byte; the rest of the file is the message."""
    with open(path, "rb") as f:
        cur = _ByteCursor(f.read())
    extras = [cur.uint(extras_bytes) for _ in range(num_extras)]
    extra_var_bits = []
    for _ in range(num_extra_var_bits):
        extra_var_bits.append(_chars(cur.bits(cur.uint(extra_bytes))))
    var_length_extras = []
    for _ in range(num_var_length_extras):
        n, w = cur.uint(extra_bytes), cur.uint(1)
        if w == 0:  # the reference's slicing loop has step 0 here (ValueError)
            raise ValueError("integer list of bit width 0")
        flags = cur.bits(n * w).astype(np.int64).reshape(n, w)
        weights = np.int64(1) << np.arange(w, dtype=np.int64)  # LSB first (from_bit_string)
        var_length_extras.append([int(v) for v in (flags * weights).sum(axis=1)])
    rest = cur.bits(8 * (len(cur.data) - cur.pos))
    return _chars(rest), extras, extra_var_bits, var_length_extras
