// cwq_math.h -- bit-level arithmetic of the greedy coded sampler, shared by the
// gfx950 kernels (device) and the host-side exhaustive self-check.
//
// Everything here reproduces the arithmetic that the reference reaches through
// TensorFlow / TFP / glibc:
//   * Philox4x32-10 + TF GenerateKey          (misc.py:10-11 -> tf.random.stateless_normal)
//   * TF Uint32ToFloat + BoxMullerFloat        (A.3, A.4)
//   * glibc 2.35 x86_64 logf / sincosf, FMA ifunc variant (the libm TF's CPU
//     kernel calls for `std::log(float)` / `sincosf`).  The algorithms are the
//     glibc ones (sysdeps/ieee754/flt-32/e_logf.c, s_sincosf.c); the constant
//     tables below were checked byte-for-byte against the host
//     /lib/x86_64-linux-gnu/libm.so.6 (.rodata of __logf_data and
//     __sincosf_table), and the Box-Muller domains (2^23 inputs each) are
//     verified exhaustively against that libm by tests/test_math_exhaustive.py
//     (host) and tests/test_gpu.py (device, via cwq_selftest_bm_tables).
//   * TFP (<=0.7) Normal.log_prob and the Eigen inner-dim sum order (A.5, A.6).
//
// Compile with -ffp-contract=off: every fused multiply-add below is explicit.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define CWQ_HD __host__ __device__ __forceinline__
#else
#define CWQ_HD static inline
#endif

namespace cwq {

// ---------------------------------------------------------------------------
// bit casts
// ---------------------------------------------------------------------------
CWQ_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
CWQ_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }

// ---------------------------------------------------------------------------
// A.1 Philox4x32-10
// ---------------------------------------------------------------------------
constexpr uint32_t kPhiloxM0 = 0xD2511F53u;
constexpr uint32_t kPhiloxM1 = 0xCD9E8D57u;
constexpr uint32_t kPhiloxW0 = 0x9E3779B9u;
constexpr uint32_t kPhiloxW1 = 0xBB67AE85u;

struct U4 { uint32_t x, y, z, w; };

CWQ_HD void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                         uint32_t k0, uint32_t k1) {
  uint64_t p0 = (uint64_t)kPhiloxM0 * c0;
  uint64_t p1 = (uint64_t)kPhiloxM1 * c2;
  uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
  uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
  c1 = (uint32_t)p1;
  c3 = (uint32_t)p0;
  c0 = n0;
  c2 = n2;
}

// Ten rounds; the key bump after the last round is dead code (the compiler
// drops it).  When the key is uniform the bumped keys live in SGPRs.
CWQ_HD U4 philox10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                   uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += kPhiloxW0;
    k1 += kPhiloxW1;
  }
  return U4{c0, c1, c2, c3};
}

// A.2 TF GenerateKey for seed = [s0, s1] (int32, sign-extended to 64 bits).
struct PhiloxStream {
  uint32_t k0, k1;  // key
  uint32_t c2, c3;  // counter words 2,3 (words 0,1 start at 0)
};

CWQ_HD PhiloxStream generate_key(int32_t s0, int32_t s1) {
  uint64_t a = (uint64_t)(int64_t)s0, b = (uint64_t)(int64_t)s1;
  U4 m = philox10((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32),
                  0x3ec8f720u, 0x02461e29u);
  return PhiloxStream{m.x, m.y, m.z, m.w};
}

// int32 `1000 * seed + i` with wrap-around (coded_greedy_sampler.py:55).
CWQ_HD int32_t step_seed(int32_t seed, int32_t i) {
  return (int32_t)((uint32_t)1000u * (uint32_t)seed + (uint32_t)i);
}

// Philox output block `grp` of a stream: counter = (0,0,c2,c3) + grp.
// Counter words 0/1 start at zero, so the 128-bit skip never carries.
CWQ_HD U4 philox_block(const PhiloxStream& s, uint64_t grp) {
  return philox10((uint32_t)grp, (uint32_t)(grp >> 32), s.c2, s.c3, s.k0, s.k1);
}

// ---------------------------------------------------------------------------
// TF Uint32ToFloat: 23 random mantissa bits -> [0,1).
// ---------------------------------------------------------------------------
CWQ_HD float uint32_to_float(uint32_t x) {
  return u2f((127u << 23) | (x & 0x7fffffu)) - 1.0f;
}

// ---------------------------------------------------------------------------
// glibc 2.35 logf (FMA variant).  __logf_data, LOGF_TABLE_BITS = 4.
// Table layout: {invc, logc} x 16 (doubles).
// ---------------------------------------------------------------------------
#define CWQ_LOGF_TAB_INIT                                                              \
  {                                                                                    \
    0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2, 0x1.571ed4aaf883dp+0,                 \
        -0x1.2bef0a7c06ddbp-2, 0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2,             \
        0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3, 0x1.30d190c8864a5p+0,             \
        -0x1.6574f0ac07758p-3, 0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3,               \
        0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4, 0x1.12358f08ae5bap+0,             \
        -0x1.1973c5a611cccp-4, 0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5, 0x1p+0,    \
        0x0p+0, 0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5, 0x1.ca4b31f026aap-1,       \
        0x1.c5e53aa362eb4p-4, 0x1.b2036576afce6p-1, 0x1.526e57720db08p-3,              \
        0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3, 0x1.886e6037841edp-1,               \
        0x1.1058bc8a07ee1p-2, 0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2               \
  }
constexpr double kLogfLn2 = 0x1.62e42fefa39efp-1;
constexpr double kLogfA0 = -0x1.00ea348b88334p-2;
constexpr double kLogfA1 = 0x1.5575b0be00b6ap-2;
constexpr double kLogfA2 = -0x1.ffffef20a4123p-2;

// Core of glibc logf for a positive, normal, finite x (the Box-Muller domain
// u1 in [1e-7, 1) and every positive normal scale).  `tab` = CWQ_LOGF_TAB_INIT
// (lives in LDS on the device).
CWQ_HD float logf_core(float x, const double* tab) {
  uint32_t ix = f2u(x);
  uint32_t tmp = ix - 0x3f330000u;
  uint32_t i = (tmp >> 19) & 15u;
  int32_t k = (int32_t)tmp >> 23;
  uint32_t iz = ix - (tmp & 0xff800000u);
  double invc = tab[2 * i], logc = tab[2 * i + 1];
  double z = (double)u2f(iz);
  double r = __builtin_fma(z, invc, -1.0);
  double y0 = __builtin_fma((double)k, kLogfLn2, logc);
  double r2 = r * r;
  double y = __builtin_fma(kLogfA1, r, kLogfA2);
  y = __builtin_fma(kLogfA0, r2, y);
  y = __builtin_fma(y, r2, y0 + r);
  return (float)y;
}

// Full glibc logf (special cases + subnormal normalisation).  Used for the
// per-dimension normaliser log(scale) and for the KL, where inputs are
// arbitrary floats.
CWQ_HD float logf_full(float x, const double* tab) {
  uint32_t ix = f2u(x);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    if (ix * 2 == 0) return -__builtin_inff();  // log(+-0) = -inf
    if (ix == 0x7f800000u) return x;            // log(inf) = inf
    if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __builtin_nanf("");
    // subnormal: normalise
    ix = f2u(x * 0x1p23f);
    ix -= 23u << 23;
    uint32_t tmp = ix - 0x3f330000u;
    uint32_t i = (tmp >> 19) & 15u;
    int32_t k = (int32_t)tmp >> 23;
    uint32_t iz = ix - (tmp & 0xff800000u);
    double invc = tab[2 * i], logc = tab[2 * i + 1];
    double z = (double)u2f(iz);
    double r = __builtin_fma(z, invc, -1.0);
    double y0 = __builtin_fma((double)k, kLogfLn2, logc);
    double r2 = r * r;
    double y = __builtin_fma(kLogfA1, r, kLogfA2);
    y = __builtin_fma(kLogfA0, r2, y);
    y = __builtin_fma(y, r2, y0 + r);
    return (float)y;
  }
  return logf_core(x, tab);
}

// ---------------------------------------------------------------------------
// glibc 2.35 sincosf (FMA variant), restricted to y in [0, 120): the
// reduce_fast path.  For y < pi/4 the reduction has n == 0 and is the
// identity, so it coincides with glibc's unreduced polynomial branch; for
// y < 2^-12 glibc returns (y, 1.0f) directly, which the polynomial also
// rounds to -- both facts are checked exhaustively over the Box-Muller angle
// domain.  __sincosf_table[0]; table[1] only negates the cosine
// coefficients, which (round-to-nearest being symmetric) negates the cosine
// polynomial's result exactly.
// ---------------------------------------------------------------------------
constexpr double kSinHpiInv = 0x1.45f306dc9c883p+23;  // 2/pi * 2^24
constexpr double kSinHpi = 0x1.921fb54442d18p+0;
constexpr double kSinC0 = 0x1p0;
constexpr double kSinC1 = -0x1.ffffffd0c621cp-2;
constexpr double kSinS1 = -0x1.555545995a603p-3;
constexpr double kSinC2 = 0x1.55553e1068f19p-5;
constexpr double kSinS2 = 0x1.1107605230bc4p-7;
constexpr double kSinC3 = -0x1.6c087e89a359dp-10;
constexpr double kSinS3 = -0x1.994eb3774cf24p-13;
constexpr double kSinC4 = 0x1.99343027bf8c3p-16;

CWQ_HD void sincosf_pos(float y, float& so, float& co) {
  double x = (double)y;
  double r = x * kSinHpiInv;
  int32_t n = ((int32_t)r + 0x800000) >> 24;
  x = __builtin_fma(-(double)n, kSinHpi, x);
  // sincosf_poly(x * sign[n&3], x*x, table[(n>>1)&1], n)
  double x2 = x * x;
  double x4 = x2 * x2;
  double x3 = x2 * x;
  double c2 = __builtin_fma(x2, kSinC4, kSinC3);
  double s1 = __builtin_fma(x2, kSinS3, kSinS2);
  double c1 = __builtin_fma(x2, kSinC1, kSinC0);
  double x5 = x3 * x2;
  double x6 = x4 * x2;
  double s = __builtin_fma(x3, kSinS1, x);
  double c = __builtin_fma(x4, kSinC2, c1);
  float sp = (float)__builtin_fma(x5, s1, s);   // odd poly of +x
  float cp = (float)__builtin_fma(x6, c2, c);   // even poly, table[0]
  // sign[] = {1,-1,-1,1}: negate the odd poly for n&3 in {1,2};
  // table[1] (n&2) negates the even poly.
  uint32_t nq = (uint32_t)n & 3u;
  uint32_t sflip = ((nq == 1u) | (nq == 2u)) ? 0x80000000u : 0u;
  uint32_t cflip = (nq & 2u) ? 0x80000000u : 0u;
  float sv = u2f(f2u(sp) ^ sflip);
  float cv = u2f(f2u(cp) ^ cflip);
  if (nq & 1u) {  // quadrant swap
    so = cv;
    co = sv;
  } else {
    so = sv;
    co = cv;
  }
}

// ---------------------------------------------------------------------------
// A.4 Box-Muller pieces.  Each depends on 23 bits of one Philox word.
// ---------------------------------------------------------------------------
// u2 = sqrt(-2 log(max(u1, 1e-7)))
CWQ_HD float bm_radius(uint32_t x0, const double* logtab) {
  float u1 = uint32_to_float(x0);
  u1 = u1 < 1.0e-7f ? 1.0e-7f : u1;
  return __builtin_sqrtf(-2.0f * logf_core(u1, logtab));
}

// v1 = (float)(2*pi (double) * Uint32ToFloat(x1)).  Uint32ToFloat(x1) =
// m * 2^-23 exactly, so the double product equals RN64(2pi*m) * 2^-23.
CWQ_HD float bm_angle(uint32_t x1) {
  return (float)(6.283185307179586 * (double)uint32_to_float(x1));
}

CWQ_HD void box_muller(uint32_t x0, uint32_t x1, const double* logtab, float& f0, float& f1) {
  float u2 = bm_radius(x0, logtab);
  float s, c;
  sincosf_pos(bm_angle(x1), s, c);
  f0 = s * u2;
  f1 = c * u2;
}

// Four normals of Philox block `grp` (NormalDistribution<PhiloxRandom,float>).
struct F4 { float a, b, c, d; };
CWQ_HD F4 normal4(const PhiloxStream& s, uint64_t grp, const double* logtab) {
  U4 x = philox_block(s, grp);
  F4 z;
  box_muller(x.x, x.y, logtab, z.a, z.b);
  box_muller(x.z, x.w, logtab, z.c, z.d);
  return z;
}

// ---------------------------------------------------------------------------
// A.5 TFP Normal.log_prob with a precomputed normaliser c = 0.9189385f + log(s)
// ---------------------------------------------------------------------------
constexpr float kHalfLog2Pi = 0x1.d67f1cp-1f;  // float32(0.5*math.log(2*math.pi))

CWQ_HD float log_prob(float x, float loc, float scale, float c) {
  float z = (x - loc) / scale;
  float u = -0.5f * (z * z);
  return u - c;
}

// Orderable argmax key: max key <=> max value, lowest index on ties.
// NaN and values <= -FLT_MAX never beat the reducer's initial accumulator
// (index 0, value lowest()), so they are clamped to lowest(); -0 == +0.
CWQ_HD uint64_t argmax_key(float v, uint32_t idx) {
  const float lowest = -0x1.fffffep+127f;
  v = (v > lowest) ? v : lowest;
  v = v + 0.0f;  // -0 -> +0
  uint32_t b = f2u(v);
  uint32_t o = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  return ((uint64_t)o << 32) | (uint64_t)(0xFFFFFFFFu - idx);
}
// ord(lowest()): keys at this level carry no information about the index.
constexpr uint32_t kArgmaxClampOrd = 0x00800000u;
CWQ_HD uint32_t argmax_key_index(uint64_t key) {
  return 0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull);
}

}  // namespace cwq
