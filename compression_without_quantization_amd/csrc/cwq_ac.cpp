// cwq_ac.cpp -- integer arithmetic coder, the native-code equivalent of the
// reference's only compiled component, code/coding.pyx:27-310 (SURVEY.md
// 8(f) row 3).  Host code: the coder is a serial integer renormalisation
// loop with nothing to parallelise, so it stays on the CPU.
//
// Semantics follow coding.pyx exactly:
//   * C[i] = sum_{k<i} P[k], D[i] = C[i] + P[i], R = D[K-1] (:35-55);
//   * interval update high = low + (width*D[s]) // R, low = low + (width*C[s]) // R
//     with the old `low` in both (:85-89);
//   * renormalisation on `high < half` / `low > half` (strict, as written,
//     :92-109), middle rescaling on `low > quarter && high < 3 quarter`
//     (:112-115), pending bits `s`, final emission (:118-123);
//   * decoding (:129-216) stops at symbol 0 (EOF) and returns it too.
// decode_fast's AVL search (:220-310, data_structures.py:188-215) is a binary
// search here: the symbol containing z is the last j with
// (width*C[j]) // R <= z - low, which is what the linear decoder (:162-181)
// finds as well.  Products are formed in 128-bit integers, so no count
// total can overflow (the reference's int64 arithmetic would for R > 2^31).
// The bit-string codecs of binary_io.py (Elias-delta, the greedy coder's
// fixed-width index parse) sit here too: host-side, serial byte work.
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <immintrin.h>

#include <vector>

#include "../../include/cwq.h"
#include "cwq_kernels.h"

namespace {

typedef __int128 i128;

struct Model {
  std::vector<int64_t> C, D;
  int64_t R = 0;
};

bool build_model(const int64_t* counts, int64_t K, Model* m) {
  if (K <= 0 || !counts) return false;
  m->C.resize((size_t)K);
  m->D.resize((size_t)K);
  int64_t c = 0;
  for (int64_t i = 0; i < K; ++i) {
    if (counts[i] < 0) return false;
    m->C[(size_t)i] = c;
    c += counts[i];
    m->D[(size_t)i] = c;
  }
  m->R = c;
  return c > 0;
}

inline int64_t scale(int64_t width, int64_t x, int64_t R) {
  return (int64_t)(((i128)width * (i128)x) / (i128)R);  // non-negative: floor == trunc
}

}  // namespace

extern "C" {

int64_t cwq_ac_encode(const int64_t* counts, int64_t K, int precision, const int64_t* message,
                      int64_t n, char* out_bits, int64_t cap) {
  Model m;
  if (precision < 3 || precision > 62 || n < 0 || (n > 0 && !message) || !build_model(counts, K, &m))
    return cwq::set_error(CWQ_ERR_INVALID, "cwq_ac_encode: bad counts/precision/message");
  const int64_t whole = (int64_t)1 << precision;
  const int64_t half = (int64_t)1 << (precision - 1);
  const int64_t quarter = (int64_t)1 << (precision - 2);
  int64_t low = 0, high = whole;
  int64_t s = 0;
  int64_t nbits = 0;
  auto emit = [&](char b) -> bool {
    if (out_bits) {
      if (nbits >= cap) return false;
      out_bits[nbits] = b;
    }
    ++nbits;
    return true;
  };
  for (int64_t k = 0; k < n; ++k) {
    const int64_t sym = message[k];
    if (sym < 0 || sym >= K)
      return cwq::set_error(CWQ_ERR_INVALID, "cwq_ac_encode: symbol outside [0, K)");
    // a zero-count symbol has an empty interval: the reference's loop would
    // spin forever at low == high == half (coding.pyx:92-115); reject it
    if (m.C[(size_t)sym] == m.D[(size_t)sym])
      return cwq::set_error(CWQ_ERR_INVALID, "cwq_ac_encode: symbol has a zero count");
    const int64_t width = high - low;
    high = low + scale(width, m.D[(size_t)sym], m.R);
    low = low + scale(width, m.C[(size_t)sym], m.R);
    while (high < half || low > half) {
      if (high < half) {
        if (!emit('0')) return cwq::set_error(CWQ_ERR_CAPACITY, "cwq_ac_encode: cap");
        for (; s > 0; --s)
          if (!emit('1')) return cwq::set_error(CWQ_ERR_CAPACITY, "cwq_ac_encode: cap");
        low *= 2;
        high *= 2;
      } else {
        if (!emit('1')) return cwq::set_error(CWQ_ERR_CAPACITY, "cwq_ac_encode: cap");
        for (; s > 0; --s)
          if (!emit('0')) return cwq::set_error(CWQ_ERR_CAPACITY, "cwq_ac_encode: cap");
        low = (low - half) * 2;
        high = (high - half) * 2;
      }
    }
    while (low > quarter && high < 3 * quarter) {
      s += 1;
      low = (low - quarter) * 2;
      high = (high - quarter) * 2;
    }
  }
  s += 1;
  const char first = (low <= quarter) ? '0' : '1';
  const char rest = (low <= quarter) ? '1' : '0';
  if (!emit(first)) return cwq::set_error(CWQ_ERR_CAPACITY, "cwq_ac_encode: cap");
  for (; s > 0; --s)
    if (!emit(rest)) return cwq::set_error(CWQ_ERR_CAPACITY, "cwq_ac_encode: cap");
  cwq::set_error(CWQ_OK, "");
  return nbits;
}

int64_t cwq_ac_decode(const int64_t* counts, int64_t K, int precision, const char* bits,
                      int64_t nbits, int64_t* out_msg, int64_t cap) {
  Model m;
  if (precision < 3 || precision > 62 || nbits < 0 || (nbits > 0 && !bits) || !out_msg ||
      !build_model(counts, K, &m))
    return cwq::set_error(CWQ_ERR_INVALID, "cwq_ac_decode: bad counts/precision/bits");
  const int64_t whole = (int64_t)1 << precision;
  const int64_t half = (int64_t)1 << (precision - 1);
  const int64_t quarter = (int64_t)1 << (precision - 2);
  int64_t low = 0, high = whole;
  int64_t z = 0;
  int64_t i = 0;
  while (i < precision && i < nbits) {
    if (bits[i] == '1') z += (int64_t)1 << (precision - i - 1);
    ++i;
  }
  int64_t nout = 0;
  for (;;) {
    const int64_t width = high - low;
    const int64_t target = z - low;
    // last j with scale(width, C[j]) <= target
    int64_t lo = 0, hi = K;  // invariant: answer in [lo, hi)
    if (target < 0) return cwq::set_error(CWQ_ERR_INVALID, "cwq_ac_decode: corrupt code");
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (scale(width, m.C[(size_t)mid], m.R) <= target) lo = mid; else hi = mid;
    }
    const int64_t j = lo;
    const int64_t high_ = low + scale(width, m.D[(size_t)j], m.R);
    const int64_t low_ = low + scale(width, m.C[(size_t)j], m.R);
    if (!(low_ <= z && z < high_))  // corrupt code (the reference loops forever)
      return cwq::set_error(CWQ_ERR_INVALID, "cwq_ac_decode: corrupt code");
    if (nout >= cap) return cwq::set_error(CWQ_ERR_CAPACITY, "cwq_ac_decode: cap");
    out_msg[nout++] = j;
    high = high_;
    low = low_;
    if (j == 0) {  // EOF symbol
      cwq::set_error(CWQ_OK, "");
      return nout;
    }
    while (high < half || low > half) {
      if (high < half) {
        low *= 2;
        high *= 2;
        z *= 2;
      } else {
        low = (low - half) * 2;
        high = (high - half) * 2;
        z = (z - half) * 2;
      }
      if (i < nbits && bits[i] == '1') z += 1;
      ++i;
    }
    while (low > quarter && high < 3 * quarter) {
      low = (low - quarter) * 2;
      high = (high - quarter) * 2;
      z = (z - quarter) * 2;
      if (i < nbits && bits[i] == '1') z += 1;
      ++i;
    }
  }
}

// Elias-delta strings for the importance sampler's indices (binary_io.py:7-39),
// vectorised: the reference's float64 formulas n = floor(log2 x),
// l = floor(log2(n + 1)) equal the bit lengths for 1 <= x < 2^30
// (tests/test_importance.py); larger x is rejected so the caller can fall back.
// The code of v is l '0's, n + 1 in l + 1 bits and v's low n bits, all MSB
// first: the len = 2l + 1 + n bit binary of W = ((n + 1) << n) | (v mod 2^n)
// (its top bit is n + 1's, so the l leading zeros are the padding).
namespace {
int elias_len(int64_t v, uint64_t* w) {
  const int nb = 63 - __builtin_clzll((unsigned long long)v);        // n = floor(log2 v)
  const int l = 63 - __builtin_clzll((unsigned long long)(nb + 1));  // floor(log2(n + 1))
  *w = ((uint64_t)(nb + 1) << nb) | ((uint64_t)v & ((1ull << nb) - 1));
  return 2 * l + 1 + nb;
}
void elias_chars(uint64_t w, int len, char* o) {
  for (int k = len - 1; k >= 0; --k) *o++ = (char)('0' + ((w >> k) & 1));
}
// BMI2: the code left-aligned in 64 bits, then 8 chars per pdep (bit k -> the
// low bit of byte k), a byte swap (the first char is the byte's top bit) and
// an OR with '0' x 8; writes whole 8-byte words, so it needs 8 * ceil(len / 8)
// bytes of room (<= 40).  14k I2 indices: ~3x faster than a char at a time.
__attribute__((target("bmi2"))) void elias_chars_pdep(uint64_t w, int len, char* o) {
  constexpr uint64_t kLow = 0x0101010101010101ull, kZero = 0x3030303030303030ull;
  const uint64_t a = w << (64 - len);
  for (int k = 0; k < len; k += 8) {
    const uint64_t c = __builtin_bswap64(_pdep_u64((a >> (56 - k)) & 0xffu, kLow)) | kZero;
    memcpy(o + k, &c, 8);
  }
}
}  // namespace

int64_t cwq_elias_delta_encode(const int64_t* x, int64_t n, char* out, int64_t cap) {
  if (n < 0 || (n > 0 && !x)) return cwq::set_error(CWQ_ERR_INVALID, "cwq_elias_delta_encode: bad arguments");
  static const bool bmi2 = __builtin_cpu_supports("bmi2");
  int64_t pos = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t v = x[i];
    if (v < 1 || v >= ((int64_t)1 << 30))
      return cwq::set_error(CWQ_ERR_INVALID, "cwq_elias_delta_encode: value outside [1, 2^30)");
    uint64_t w;
    const int len = elias_len(v, &w);
    if (out) {
      if (pos + len > cap) return cwq::set_error(CWQ_ERR_CAPACITY, "cwq_elias_delta_encode: cap");
      if (bmi2 && pos + 40 <= cap)
        elias_chars_pdep(w, len, out + pos);
      else
        elias_chars(w, len, out + pos);
    }
    pos += len;
  }
  cwq::set_error(CWQ_OK, "");
  return pos;
}

int64_t cwq_elias_delta_decode(const char* bits, int64_t nbits, int64_t count, int64_t* out) {
  if (nbits < 0 || count < 0 || (nbits > 0 && !bits) || (count > 0 && !out))
    return cwq::set_error(CWQ_ERR_INVALID, "cwq_elias_delta_decode: bad arguments");
  int64_t pos = 0;
  for (int64_t i = 0; i < count; ++i) {
    int l = 0;
    while (pos + l < nbits && bits[pos + l] == '0') ++l;
    if (l > 30 || pos + 2 * l + 1 > nbits)
      return cwq::set_error(CWQ_ERR_INVALID, "cwq_elias_delta_decode: code exhausted or corrupt");
    pos += l;
    int64_t np1 = 0;
    for (int k = 0; k <= l; ++k) np1 = (np1 << 1) | (bits[pos + k] == '1');
    pos += l + 1;
    if (np1 < 1 || np1 > 31 || pos + (np1 - 1) > nbits)
      return cwq::set_error(CWQ_ERR_INVALID, "cwq_elias_delta_decode: code exhausted or corrupt");
    int64_t v = 1;
    for (int64_t k = 0; k < np1 - 1; ++k) v = (v << 1) | (bits[pos + k] == '1');
    pos += np1 - 1;
    out[i] = v;
  }
  cwq::set_error(CWQ_OK, "");
  return pos;
}

int64_t cwq_bitcode_to_indices(const char* bits, int64_t nbits, int num_bits, int64_t count,
                               int32_t* out) {
  if (nbits < 0 || count < 0 || num_bits < 0 || num_bits > CWQ_MAX_BITS_PER_STEP ||
      (nbits > 0 && !bits) || (count > 0 && !out) || count > (INT64_MAX >> 5))
    return cwq::set_error(CWQ_ERR_INVALID, "cwq_bitcode_to_indices: bad arguments");
  const int64_t need = count * num_bits;
  const int64_t m = nbits < need ? nbits : need;  // chars past the string read as '0'
  // the chars as a packed LSB-first bit stream (8 spare zero bytes for the
  // 64-bit field reads below), 8 chars per step: a byte of x ^ "11111111" is
  // zero iff its char is '1'; folding each byte's complement onto its bit 0
  // and gathering those bits with one multiply gives the 8 flags in order
  thread_local std::vector<uint8_t> packed;
  packed.assign((size_t)((need + 7) >> 3) + 8, 0);
  int64_t k = 0;
  for (; k + 8 <= m; k += 8) {
    uint64_t x;
    memcpy(&x, bits + k, 8);
    uint64_t y = ~(x ^ 0x3131313131313131ull);
    y &= y >> 4;
    y &= y >> 2;
    y &= y >> 1;
    packed[(size_t)(k >> 3)] = (uint8_t)(((y & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56);
  }
  for (; k < m; ++k)
    if (bits[k] == '1') packed[(size_t)(k >> 3)] |= (uint8_t)(1u << (k & 7));
  const uint64_t mask = (1ull << num_bits) - 1;
  for (int64_t i = 0; i < count; ++i) {
    const int64_t off = i * num_bits;
    uint64_t w;
    memcpy(&w, packed.data() + (off >> 3), 8);
    out[i] = (int32_t)((w >> (off & 7)) & mask);
  }
  cwq::set_error(CWQ_OK, "");
  return count;
}

}  // extern "C"
