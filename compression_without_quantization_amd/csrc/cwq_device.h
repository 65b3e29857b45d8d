// cwq_device.h -- device helpers shared by the gfx950 kernels (greedy and
// importance coders): LDS log table, wave reductions, block spans, the
// device-tuned Philox / Box-Muller / division, and the Eigen-order row
// evaluator.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cwq_math.h"

namespace cwq {

static __constant__ double kLogTabConst[32] = CWQ_LOGF_TAB_INIT;

__device__ __forceinline__ void fill_logtab(double* lds) {
  if (threadIdx.x < 32) lds[threadIdx.x] = kLogTabConst[threadIdx.x];
  __syncthreads();
}

__device__ __forceinline__ uint32_t wave_id() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

__device__ __forceinline__ double wave_sum_f64(double v) {  // full exec mask
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ double wave_max_f64(double v) {  // full exec mask
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    uint64_t o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

// ---------------------------------------------------------------------------
// Device-tuned arithmetic.  Same results as the portable restatement in
// cwq_math.h (the Box-Muller pieces are verified exhaustively on the GPU by
// tests/test_gpu.py via cwq_selftest_bm_tables), fewer instructions:
//   * Philox: the two 3-input XORs of a round are one v_bitop3_b32 each.
//   * sqrt for the Box-Muller radius: the argument -2 logf(u1) lies in
//     [2.4e-7, 32.3] (normal, finite), so the correctly rounded sqrt is
//     v_sqrt_f32 plus the two one-ulp corrections, without the denormal
//     scaling and special-case fixups of the general sequence.
//   * angle: Uint32ToFloat(x1) = m * 2^-23 exactly, so
//     RN64(2pi * U) = RN64((2pi * 2^-23) * m) and m converts exactly.
// ---------------------------------------------------------------------------
__device__ __forceinline__ U4 philox10_dev(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                           uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)kPhiloxM0 * c0;
    const uint64_t p1 = (uint64_t)kPhiloxM1 * c2;
    const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
    const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += kPhiloxW0;
    k1 += kPhiloxW1;
  }
  return U4{c0, c1, c2, c3};
}

// Philox-10 of the counter (c0, 0, c2, c3) with c2, c3 and the key
// wave-uniform (a stream's blocks below 2^32).  Rounds 0-2 then carry
// wave-uniform terms: round 0's n0 and round 1's products of it, round 1's c3.
// Their XORs with the round keys are folded per stream into four scalars
// (philox_lo_key), so each of those rounds needs one two-operand v_xor_b32
// with a scalar instead of a three-input v_bitop3_b32 with two scalars (the
// constant bus takes one: a v_mov per round) or a uniform value held in a VGPR.
// Same results as philox10_dev(c0, 0, c2, c3, k0, k1) (tests/test_gpu.py).
struct PhiloxLo {
  uint32_t A, B, C, D;
};
__device__ __forceinline__ PhiloxLo philox_lo_key(const PhiloxStream& s) {
  const uint64_t p1 = (uint64_t)kPhiloxM1 * s.c2;
  const uint32_t n0 = (uint32_t)(p1 >> 32) ^ s.k0;       // round 0's n0
  const uint64_t q0 = (uint64_t)kPhiloxM0 * n0;           // round 1's first product
  PhiloxLo o;
  o.A = s.c3 ^ s.k1;                                      // round 0: n2 = hi(M0 c0) ^ A
  o.B = (uint32_t)p1 ^ (s.k0 + kPhiloxW0);                // round 1: n0 = hi(M1 n2) ^ B
  o.C = (uint32_t)(q0 >> 32) ^ (s.k1 + kPhiloxW1);        // round 1: n2 = lo(M0 c0) ^ C
  o.D = (uint32_t)q0 ^ (s.k1 + 2u * kPhiloxW1);           // round 2: n2 = hi(M0 c0') ^ D
  // opaque scalars: the compiler must not re-associate the XORs into
  // three-input bitop3 forms with two scalar operands
  asm volatile("" : "+s"(o.A), "+s"(o.B), "+s"(o.C), "+s"(o.D));
  return o;
}
// k0, k1: the stream's key (callers may pass it through an opaque move)
__device__ __forceinline__ U4 philox10_lo(uint32_t c0, const PhiloxLo& K, uint32_t k0,
                                          uint32_t k1) {
  const uint64_t p0 = (uint64_t)kPhiloxM0 * c0;                 // round 0
  const uint32_t r0n2 = (uint32_t)(p0 >> 32) ^ K.A;
  const uint64_t q1 = (uint64_t)kPhiloxM1 * r0n2;               // round 1
  uint32_t x0 = (uint32_t)(q1 >> 32) ^ K.B;
  uint32_t x1 = (uint32_t)q1;
  uint32_t x2 = (uint32_t)p0 ^ K.C;
  const uint64_t s0 = (uint64_t)kPhiloxM0 * x0;                 // round 2
  const uint64_t s1 = (uint64_t)kPhiloxM1 * x2;
  x0 = __builtin_amdgcn_bitop3_b32((uint32_t)(s1 >> 32), x1, k0 + 2u * kPhiloxW0, 0x96);
  x2 = (uint32_t)(s0 >> 32) ^ K.D;
  x1 = (uint32_t)s1;
  uint32_t x3 = (uint32_t)s0;
  k0 += 3u * kPhiloxW0;
  k1 += 3u * kPhiloxW1;
#pragma unroll
  for (int r = 3; r < 10; ++r) {
    const uint64_t a0 = (uint64_t)kPhiloxM0 * x0;
    const uint64_t a1 = (uint64_t)kPhiloxM1 * x2;
    const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(a1 >> 32), x1, k0, 0x96);
    const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(a0 >> 32), x3, k1, 0x96);
    x1 = (uint32_t)a1;
    x3 = (uint32_t)a0;
    x0 = n0;
    x2 = n2;
    k0 += kPhiloxW0;
    k1 += kPhiloxW1;
  }
  return U4{x0, x1, x2, x3};
}

__device__ __forceinline__ U4 philox_block_dev(const PhiloxStream& s, uint64_t grp) {
  return philox10_dev((uint32_t)grp, (uint32_t)(grp >> 32), s.c2, s.c3, s.k0, s.k1);
}

__device__ __forceinline__ float sqrt_cr_bm(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sd = u2f(f2u(s) - 1u);
  const float su = u2f(f2u(s) + 1u);
  const float rd = __builtin_fmaf(-sd, s, x);
  const float ru = __builtin_fmaf(-su, s, x);
  const float t = (rd <= 0.0f) ? sd : s;
  return (ru > 0.0f) ? su : t;
}

__device__ __forceinline__ float bm_radius_dev(uint32_t x0, const double* logtab) {
  float u1 = uint32_to_float(x0);
  u1 = fmaxf(u1, 1.0e-7f);  // == (u1 < 1e-7f ? 1e-7f : u1): u1 is never NaN
  return sqrt_cr_bm(-2.0f * logf_core(u1, logtab));
}

__device__ __forceinline__ float bm_angle_dev(uint32_t x1) {
  return (float)((double)(x1 & 0x7fffffu) * 0x1.921fb54442d18p-21);
}

__device__ __forceinline__ void box_muller_dev(uint32_t x0, uint32_t x1, const double* logtab,
                                               float& f0, float& f1) {
  const float u2 = bm_radius_dev(x0, logtab);
  float s, c;
  sincosf_pos(bm_angle_dev(x1), s, c);
  f0 = s * u2;
  f1 = c * u2;
}

// Screening Box-Muller (approximate).  The hardware transcendentals
// v_log_f32 / v_sqrt_f32 / v_sin_f32 / v_cos_f32 (sin and cos take the angle in
// revolutions, so U = Uint32ToFloat(x1) needs no scaling or range reduction).
// Used ONLY by the screening passes, which turn the values into rigorous
// bounds: the largest deviation from the exact pair over every possible input
// (2^23 each) is a measured constant, kScreenEr / kScreenEs, re-checked
// exhaustively on the GPU by tests/test_gpu.py.
//
// The radius is carried without its constant factor: q~ = sqrt(-log2 u1) =
// r~ / sqrt(2 ln 2), and box_muller_screen returns z~ / sqrt(2 ln 2); callers
// fold kSqrt2Ln2 into their per-dim constants (one multiply less per pair).
constexpr double kSqrt2Ln2 = 1.1774100225154747;  // sqrt(2 ln 2)
__device__ __forceinline__ float bm_qradius_screen(uint32_t x0) {
  const float u1 = fmaxf(uint32_to_float(x0), 1.0e-7f);
  return __builtin_amdgcn_sqrtf(-__builtin_amdgcn_logf(u1));
}
__device__ __forceinline__ void bm_sincos_screen(uint32_t x1, float& s, float& c) {
  // 1 + U (exact, in [1, 2)): sin/cos in revolutions are 1-periodic, so the
  // "- 1.0f" of Uint32ToFloat is not needed here (the error table covers it)
  const float V = u2f((x1 & 0x7fffffu) | 0x3f800000u);
  s = __builtin_amdgcn_sinf(V);
  c = __builtin_amdgcn_cosf(V);
}
__device__ __forceinline__ void box_muller_screen(uint32_t x0, uint32_t x1, float& f0, float& f1) {
  const float q = bm_qradius_screen(x0);
  float s, c;
  bm_sincos_screen(x1, s, c);
  f0 = s * q;
  f1 = c * q;
}

// Error constants of the screening Box-Muller, shared by both screening passes.
// measured maxima over all 2^23 inputs (tools/screen_err.py, re-checked by
// tests/test_gpu.py): |sqrt(2 ln 2) q~ - r| <= 5.82e-7, |sin~ - sin|, |cos~ - cos| <= 2.99e-7
constexpr double kScreenEr = 1.0e-6;
constexpr double kScreenEs = 6.0e-7;
constexpr double kScreenRmax = 5.68;  // r <= sqrt(-2 ln 1e-7) = 5.6777
// |sqrt(2 ln 2) RN(s~ q~) - RN(s r)| <= (1 + Es) Er + Rmax Es + 2^-23 (Rmax + Er)
constexpr double kScreenEz =
    (1.0 + kScreenEs) * kScreenEr + kScreenRmax * kScreenEs + 0x1p-23 * (kScreenRmax + kScreenEr);
constexpr double kScreenZm = 5.7;     // bound on |z| and |z~|

__device__ __forceinline__ F4 normal4_screen(const PhiloxStream& s, uint64_t grp) {
  const U4 x = philox_block_dev(s, grp);
  F4 z;
  box_muller_screen(x.x, x.y, z.a, z.b);
  box_muller_screen(x.z, x.w, z.c, z.d);
  return z;
}

// normal4_screen of a block below 2^32, K = philox_lo_key(s)
__device__ __forceinline__ F4 normal4_screen_lo(const PhiloxStream& s, const PhiloxLo& K,
                                                uint32_t grp) {
  const U4 x = philox10_lo(grp, K, s.k0, s.k1);
  F4 z;
  box_muller_screen(x.x, x.y, z.a, z.b);
  box_muller_screen(x.z, x.w, z.c, z.d);
  return z;
}

__device__ __forceinline__ F4 normal4_dev(const PhiloxStream& s, uint64_t grp,
                                          const double* logtab) {
  const U4 x = philox_block_dev(s, grp);
  F4 z;
  box_muller_dev(x.x, x.y, logtab, z.a, z.b);
  box_muller_dev(x.z, x.w, logtab, z.c, z.d);
  return z;
}

// Correctly rounded a / b for 2^-60 <= |a| <= 2^60 (or a == 0) and
// 2^-60 <= b <= 2^60, given y = RN(1/b).  q0 = RN(a y) is within 2 ulps;
// one residual step brings q1 within 1 ulp; with q1 within 1 ulp and y within
// half an ulp of 1/b, the residual b*q1 - a is exact and the final fused step
// rounds to RN(a/b) (Markstein's theorem).  The ranges keep
// every intermediate normal.  Callers route other operands to IEEE division.
__device__ __forceinline__ float div_rn_markstein(float a, float b, float y) {
  const float q0 = a * y;
  const float r0 = __builtin_fmaf(-b, q0, a);
  const float q1 = __builtin_fmaf(r0, y, q0);
  const float r1 = __builtin_fmaf(-b, q1, a);
  return __builtin_fmaf(r1, y, q1);
}
// 2^-60 <= |a| < 2^60 (biased exponent 67..186) or a == +-0, branch-free.
// True when all four numerators lie in [2^-60, 2^60].  Exact zeros fail
// too (they are rare, and the caller's IEEE fallback handles them), which lets
// the test be two 3-input min/max ops and two compares.  A NaN numerator may
// pass: both division paths then yield NaN, which the score clamps anyway.
__device__ __forceinline__ bool markstein_ok4(float a, float b, float c, float d) {
  const float ma = __builtin_fabsf(a), mb = __builtin_fabsf(b);
  const float mc = __builtin_fabsf(c), md = __builtin_fabsf(d);
  const float hi = __builtin_fmaxf(__builtin_fmaxf(ma, mb), __builtin_fmaxf(mc, md));
  const float lo = __builtin_fminf(__builtin_fminf(ma, mb), __builtin_fminf(mc, md));
  return (hi <= 0x1p60f) & (lo >= 0x1p-60f);
}
__device__ __forceinline__ bool markstein_ok_den(float b) {
  return b >= 0x1p-60f && b <= 0x1p60f;
}

struct BlockSpan {
  int64_t off;
  int64_t d;
};

__device__ __forceinline__ BlockSpan block_span(const int64_t* __restrict__ block_off,
                                                int64_t ud, int64_t g) {
  if (block_off == nullptr) return BlockSpan{g * ud, ud};
  int64_t a = block_off[g];
  int64_t b = block_off[g + 1];
  return BlockSpan{a, b - a};
}

__device__ __forceinline__ int32_t block_seed(int32_t seed, int64_t block_id) {
  return (int32_t)((uint32_t)seed + (uint32_t)block_id);
}

// The encoders' block seeds: block g of a launch is coded with seed
// `seed + base + g` (coded_greedy_sampler.py:282), or with per_block[g] when
// the launch codes several independent jobs at once (a batch of images, each
// numbering its groups from 0 with its own seed).
struct SeedSpec {
  int32_t seed;
  int64_t base;
  const int32_t* per_block;  // device [nb] or nullptr
  __device__ __forceinline__ int32_t of(int64_t g) const {
    return per_block ? per_block[g] : block_seed(seed, base + g);
  }
};

__device__ __forceinline__ uint32_t ord_f32(float v) {
  const uint32_t b = f2u(v);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(uint32_t o) {
  return u2f((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
#ifndef CWQ_WAVE_MAX_ASM
#define CWQ_WAVE_MAX_ASM 1  // 1: one v_max_f32_dpp per step (inline asm)
#endif
// Wave-wide max with GFX9 DPP (quad perms, row mirrors, row_bcast:15/31):
// six v_max_f32_dpp and one readlane.  Requires a full exec mask.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_max_step(float v) {
  const int ninf = (int)0xff800000u;  // -inf: identity for the rows DPP leaves unwritten
  const int o = __builtin_amdgcn_update_dpp(ninf, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf,
                                            false);
  return fmaxf(v, __builtin_bit_cast(float, o));
}
#if CWQ_WAVE_MAX_ASM
// The same six steps as one v_max_f32_dpp each: v = max(v[dpp], v), and lanes a
// step's row mask leaves unwritten keep v.  Through the builtins each step is a
// v_mov_b32_dpp from a -inf "old" value plus two v_max_f32 (fmaxf's IEEE
// canonicalisation of the moved value): 25 VALU instructions against 6 (the
// tau sharing of the pruned loops, every 16 units).  Each step starts with the
// two wait states a DPP read of a VGPR written by the previous VALU needs, and
// the last ends with them before the readlane.  tau is never a signalling NaN,
// for which the two forms would differ.
#define CWQ_DPP_MAX_STEP(v, ctl, rmask) \
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 " ctl " row_mask:" rmask " bank_mask:0xf" \
               : "+v"(v))
__device__ __forceinline__ float wave_max_f32(float v) {
  CWQ_DPP_MAX_STEP(v, "quad_perm:[1,0,3,2]", "0xf");
  CWQ_DPP_MAX_STEP(v, "quad_perm:[2,3,0,1]", "0xf");
  CWQ_DPP_MAX_STEP(v, "row_half_mirror", "0xf");
  CWQ_DPP_MAX_STEP(v, "row_mirror", "0xf");
  CWQ_DPP_MAX_STEP(v, "row_bcast:15", "0xa");
  CWQ_DPP_MAX_STEP(v, "row_bcast:31", "0xc");
  asm volatile("s_nop 1" : "+v"(v));
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
#else
__device__ __forceinline__ float wave_max_f32(float v) {
  v = dpp_max_step<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
  v = dpp_max_step<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
  v = dpp_max_step<0x141, 0xf>(v);  // row_half_mirror
  v = dpp_max_step<0x140, 0xf>(v);  // row_mirror: every lane holds its row's max
  v = dpp_max_step<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  v = dpp_max_step<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3: lane 63 holds the max
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
#endif
// Sum over each 16-lane DPP row, the same value in all 16 lanes: butterflies
// (quad xor 1, quad xor 2, half-row mirror, row mirror) pair lanes
// symmetrically and float addition commutes, so every lane forms the
// identical ((x0+x1)+(x2+x3)) + ... tree.  Requires a full exec mask.
template <int CTRL>
__device__ __forceinline__ float dpp_add_step(float v) {
  const int o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false);
  return v + __builtin_bit_cast(float, o);
}
__device__ __forceinline__ float row16_sum_f32(float v) {
  v = dpp_add_step<0xb1>(v);   // quad_perm [1,0,3,2]
  v = dpp_add_step<0x4e>(v);   // quad_perm [2,3,0,1]
  v = dpp_add_step<0x141>(v);  // row_half_mirror: quad 0 <-> quad 1 of each half row
  v = dpp_add_step<0x140>(v);  // row_mirror: half 0 <-> half 1
  return v;
}
// smallest float >= b (+inf for non-finite b: such a bound never drops anything)
__device__ __forceinline__ float round_up_f32(double b) {
  if (!(b == b) || b > 3.0e38 || b < -3.0e38) return __builtin_inff();
  float f = (float)b;
  if ((double)f < b) {
    const uint32_t u = f2u(f);
    f = (f >= 0.0f) ? u2f(f == 0.0f ? 1u : u + 1u) : u2f(u - 1u);
  }
  return f;
}
__device__ __forceinline__ float round_dn_f32(double b) { return -round_up_f32(-b); }

template <int DC, class ElemF>
__device__ __forceinline__ float eval_row_f(const PhiloxStream& st, uint64_t kbase, int64_t d_rt,
                                            int align_rt, const double* logtab, ElemF&& val) {
  const int64_t d = DC > 0 ? (int64_t)DC : d_rt;
  const int align = (DC > 0 && (DC % 4) == 0) ? 0 : align_rt;
  const int64_t vec = d & ~(int64_t)7;
  float p[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  F4 z = {0.f, 0.f, 0.f, 0.f};

  auto elem = [&](int64_t e) -> float {
    const int w = (align + (int)(e & 3)) & 3;  // wave-uniform
    if (w == 0 || e == 0) z = normal4_dev(st, (kbase + (uint64_t)e) >> 2, logtab);
    const float zz = w == 0 ? z.a : (w == 1 ? z.b : (w == 2 ? z.c : z.d));
    return val(e, zz);
  };

  for (int64_t j = 0; j < vec; j += 8) {
#pragma unroll
    for (int l = 0; l < 8; ++l) p[l] = p[l] + elem(j + l);
  }
  float t = 0.0f;
  for (int64_t j = vec; j < d; ++j) t = t + elem(j);
  const float q0 = p[0] + p[4], q1 = p[1] + p[5], q2 = p[2] + p[6], q3 = p[3] + p[7];
  return t + ((q0 + q2) + (q1 + q3));
}

static inline unsigned grid_for(int64_t work, int64_t per_block, unsigned cap) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

}  // namespace cwq
