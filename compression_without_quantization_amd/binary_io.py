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


def bitcode_to_indices(bitcode, num_bits, count):
    """Inverse of indices_to_bitcode for ``count`` indices.

    Missing trailing characters read as '0' (``from_bit_string`` of a short
    substring, as tf.strings.substr yields at the end of the string).
    """
    if isinstance(bitcode, bytes):
        raw = np.frombuffer(bitcode, dtype=np.uint8)
    else:
        raw = np.frombuffer(bitcode.encode('ascii'), dtype=np.uint8)
    need = count * num_bits
    bits = np.zeros(need, dtype=np.int64)
    m = min(need, raw.size)
    bits[:m] = (raw[:m] == ord('1'))
    if num_bits == 0:
        return np.zeros(count, dtype=np.int64)
    bits = bits.reshape(count, num_bits)
    weights = (np.int64(1) << np.arange(num_bits, dtype=np.int64))
    return (bits * weights[None, :]).sum(axis=1)


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
