// cwq_importance.hip -- gfx950 kernels of the coded importance sampler
// (code/coded_importance_sampler.py:29-110), SURVEY.md 8(f) row 2.
//
// Same candidate stream as the greedy coder (stateless Philox, seed
// [seed + g, 42] -- the group seed itself, not 1000*seed + i), but:
//   * each group draws its own count N_g = ceil(exp(sum KL)) (host plan),
//   * a candidate's score is sum_j (log q(x_j) - log p(x_j)) in Eigen order,
//   * the emitted index is the argmax (coded as Elias-delta of index + 1 by
//     the host, binary_io.py:7-39).
// Groups have very different N_g, so work is cut into fixed-size tiles of one
// group's candidates; a device prefix over tiles-per-group lets a persistent
// grid find each tile's group by binary search (no host round trip); groups
// of at most kImpSmallN candidates take one wave each instead (k_imp_small).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cwq_device.h"
#include "cwq_kernels.h"

namespace cwq {

constexpr int64_t kImpCandPerTile = 16384;
constexpr int kImpScreenMaxD = 256;   // screening pass: per-dim constants live in LDS
constexpr int64_t kImpPruneMinD = 5;  // rows of >= 5 dims take the pruned screening loop
#ifndef CWQ_IMP_SURVIVOR_CAP
#define CWQ_IMP_SURVIVOR_CAP 1024
#endif

__global__ void __launch_bounds__(256) k_imp_prep(const float* __restrict__ t_scale,
                                                  const float* __restrict__ p_scale, int64_t n,
                                                  float* __restrict__ lnt,
                                                  float* __restrict__ lnp) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    lnt[i] = kHalfLog2Pi + logf_full(t_scale[i], kLogTabConst);
    lnp[i] = kHalfLog2Pi + logf_full(p_scale[i], kLogTabConst);
  }
}

// Tile size: the launch's candidates cut into about kImpTargetTiles tiles (a
// few per CU, so one image's ~600 groups do not leave most of a fixed grid
// idle), a power of two in [kImpMinCandPerTile, kImpCandPerTile].
#ifndef CWQ_IMP_TARGET_TILES
#define CWQ_IMP_TARGET_TILES 2048
#endif
#ifndef CWQ_IMP_MIN_CPT
#define CWQ_IMP_MIN_CPT 1024
#endif
constexpr int64_t kImpMinCandPerTile = CWQ_IMP_MIN_CPT;
constexpr int64_t kImpEvalGrid = 256 * 16;  // persistent k_imp_eval workgroups

// The tile-size rule (k_imp_tiles on the device; the launcher on the host
// when it knows the launch's candidate count T = sum max(N_g, 1)).
__host__ __device__ inline int64_t imp_cand_per_tile(int64_t T) {
  int64_t cpt = kImpMinCandPerTile;
  while (cpt < kImpCandPerTile && cpt * CWQ_IMP_TARGET_TILES < T) cpt <<= 1;
  return cpt;
}

// Groups of at most this many candidates are coded by k_imp_small (one wave
// per group, every row exact) and get no k_imp_eval tile: most groups of a
// batch of small latents draw a few dozen candidates (I2: 81% of 13,852
// groups have N <= 128, 1.6% of the candidates), and a tile's fixed cost (its
// group search, the screening constants, four barriers, the hand-out
// counter) exceeded their rows' work.  A/B (tools/variants.sh is0..is1024,
// one box, two rounds): I2's scoring 0.299 -> 0.207 ms, pln_is 0.36 -> 0.18 ms,
// I1 unchanged (8.39 / 8.41 ms); 128 and 256 tie, 1024 is slower on I1.
// 0 disables.
#ifndef CWQ_IMP_SMALL_N
#define CWQ_IMP_SMALL_N 128
#endif
constexpr int64_t kImpSmallN = CWQ_IMP_SMALL_N;

// Exclusive prefix over the 1024 threads of the workgroup (inclusive wave scans
// by shuffles, then the 16 wave totals).  Returns the prefix and
// sets *total.
__device__ __forceinline__ int64_t block_exclusive_scan_1024(int64_t v, int64_t* wsum,
                                                            int64_t* total) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  int64_t inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t o = __shfl_up(inc, off, 64);
    if ((int)lane >= off) inc += o;
  }
  if (lane == 63u) wsum[wv] = inc;
  __syncthreads();
  int64_t base = 0, all = 0;
  for (uint32_t w = 0; w < 16u; ++w) {
    const int64_t t = wsum[w];
    base += w < wv ? t : 0;
    all += t;
  }
  __syncthreads();
  *total = all;
  return base + inc - v;
}

// Chooses the launch's candidates per tile (*cpt_out), then
// tprefix[g] = sum_{h<g} tiles(N_h), tiles(N) = 0 for max(N, 1) <= kImpSmallN
// (k_imp_small's groups), else ceil(N / cpt); tprefix[nb] = total tiles.
// Also resets the per-group shared screening threshold gtau[g], the argmax
// keys and the dynamic hand-out counter.  One workgroup of 1024 threads.
__global__ void __launch_bounds__(1024) k_imp_tiles(const int64_t* __restrict__ n_samples,
                                                    int64_t nb, int64_t* __restrict__ cpt_out,
                                                    int64_t* __restrict__ tprefix,
                                                    uint32_t* __restrict__ gtau,
                                                    unsigned long long* __restrict__ next_tile,
                                                    unsigned long long* __restrict__ keys) {
  __shared__ int64_t wsum[16];
  if (threadIdx.x == 0) *next_tile = 0ull;
  // thread t takes groups t, t + 1024, ... (coalesced loads and stores); the
  // prefix is one block scan per 1,024 groups with a running carry.  (I2's
  // 13,852 groups: ~27 us either way -- neither the strided accesses nor the
  // 64-bit divisions of the previous per-thread-run form were the cost)
  const int64_t rounds = (nb + 1023) / 1024;
  constexpr int kRegs = 16;  // nb <= 16,384: every count held in registers
  const bool in_regs = rounds <= kRegs;
  auto count_at = [&](int64_t g) -> int64_t {
    const int64_t n = n_samples[g];
    return n > 1 ? n : 1;
  };
  int64_t nv[kRegs];
  int64_t cand = 0;
  if (in_regs) {
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const int64_t g = (int64_t)r * 1024 + threadIdx.x;
      nv[r] = g < nb ? count_at(g) : 0;
    }
#pragma unroll
    for (int r = 0; r < kRegs; ++r) cand += nv[r];
  } else {
    for (int64_t g = threadIdx.x; g < nb; g += 1024) cand += count_at(g);
  }
  for (int64_t g = threadIdx.x; g < nb; g += 1024) {
    gtau[g] = ord_f32(-__builtin_inff());
    keys[g] = 0ull;  // every group's argmax key (no separate memset launch)
  }
  int64_t T = 0;
  (void)block_exclusive_scan_1024(cand, wsum, &T);
  const int64_t cpt = imp_cand_per_tile(T);
  // a group k_imp_small codes takes no tile; cpt is a power of two
  const int lg = __builtin_ctzll((unsigned long long)cpt);
  auto ntiles = [&](int64_t n) -> int64_t { return n <= kImpSmallN ? 0 : (n + cpt - 1) >> lg; };
  int64_t carry = 0;
  for (int64_t r = 0; r < rounds; ++r) {
    const int64_t g = r * 1024 + threadIdx.x;
    int64_t n = 0;
    if (in_regs) {
#pragma unroll
      for (int i = 0; i < kRegs; ++i) n = r == i ? nv[i] : n;
    } else if (g < nb) {
      n = count_at(g);
    }
    const int64_t v = g < nb ? ntiles(n) : 0;
    int64_t tot = 0;
    const int64_t ex = block_exclusive_scan_1024(v, wsum, &tot);
    if (g < nb) tprefix[g] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    tprefix[nb] = carry;
    *cpt_out = cpt;
  }
}

// Screening row value: sum_j (A_j z_j + B_j) z_j + C_j over the candidate's
// dims, z from the hardware-transcendental Box-Muller ("screening
// the importance sampler").  `align` = (kbase mod 4) must be wave-uniform.
// HI0: every block index of the row is below 2^32 (lok = philox_lo_key(st))
template <bool HI0>
__device__ __forceinline__ float screen_row_imp(const PhiloxStream& st, const PhiloxLo& lok,
                                                uint64_t kbase, int64_t d, int align,
                                                const float4* __restrict__ coef) {
  float s = 0.0f;
  F4 z = {0.f, 0.f, 0.f, 0.f};
  for (int64_t e = 0; e < d; ++e) {
    const int w = (align + (int)(e & 3)) & 3;  // wave-uniform
    if (w == 0 || e == 0) {
      const uint64_t grp = (kbase + (uint64_t)e) >> 2;
      z = HI0 ? normal4_screen_lo(st, lok, (uint32_t)grp) : normal4_screen(st, grp);
    }
    const float zz = w == 0 ? z.a : (w == 1 ? z.b : (w == 2 ? z.c : z.d));
    const float4 c = coef[e];
    s = s + __builtin_fmaf(__builtin_fmaf(c.x, zz, c.y), zz, c.z);
  }
  return s;
}

// Per-dim screening constants and error bound (host-free, in double).  The
// exact term is t = RN(lt - lq), lt = RN(RN(-0.5 RN(yt^2)) - ct),
// yt = RN(RN(x - tl) / ts), lq likewise with (pl, ps, cp), x = RN(pl + RN(ps z)).
// In real arithmetic t(z) = A z^2 + B z + C with a = ps/ts, b = (pl - tl)/ts,
// A = (1 - a^2)/2, B = -a b, C = cp - ct - b^2/2.  Returns false if the dim
// must not be screened.
struct ImpScreenDim {
  float A, B, C, err, mag, umax;
};
__device__ __forceinline__ bool imp_screen_dim(float tl, float ts, float pl, float ps, float ct,
                                               float cp, ImpScreenDim& o) {
  if (!(ts >= 0x1p-60f && ts <= 0x1p60f && ps >= 0x1p-60f && ps <= 0x1p60f)) return false;
  if (!(tl - tl == 0.0f && pl - pl == 0.0f && ct - ct == 0.0f && cp - cp == 0.0f)) return false;
  const double u = 0x1p-24, r = 1.0001, Zm = kScreenZm, Ez = kScreenEz;
  const double dtl = tl, dts = ts, dpl = pl, dps = ps, dct = ct, dcp = cp;
  // rounding of the exact chain, bounded with |z| <= Zm
  const double m1 = __builtin_fabs(dps) * Zm;
  const double mx = __builtin_fabs(dpl) + m1;
  const double ex = u * (m1 + mx) * r;
  const double mdt = mx + __builtin_fabs(dtl), mdq = mx + __builtin_fabs(dpl);
  const double Myt = mdt / dts * (1.0 + 4.0 * u), Myq = mdq / dps * (1.0 + 4.0 * u);
  const double eyt = ((ex + u * mdt) / dts + u * Myt) * r;
  const double eyq = ((ex + u * mdq) / dps + u * Myq) * r;
  const double lt_mag = 0.5 * Myt * Myt + __builtin_fabs(dct);
  const double lq_mag = 0.5 * Myq * Myq + __builtin_fabs(dcp);
  const double rho = (0.5 * (2.0 * Myt * eyt + eyt * eyt + u * Myt * Myt) + u * lt_mag +
                      0.5 * (2.0 * Myq * eyq + eyq * eyq + u * Myq * Myq) + u * lq_mag +
                      u * (lt_mag + lq_mag)) * r;
  // the real quadratic in z and its float coefficients in z' = z / sqrt(2 ln 2)
  // (the screening Box-Muller's output): A' = 2 ln2 A, B' = sqrt(2 ln 2) B
  const double a = dps / dts, b = (dpl - dtl) / dts;
  const double A = 0.5 * (1.0 - a * a), B = -a * b, C = dcp - dct - 0.5 * b * b;
  const double A1 = A * (kSqrt2Ln2 * kSqrt2Ln2), B1 = B * kSqrt2Ln2;
  const double Zq = Zm / kSqrt2Ln2 * (1.0 + 4.0 * u);  // bound on |z'|
  o.A = (float)A1;
  o.B = (float)B1;
  o.C = (float)C;
  const double dA = __builtin_fabs((double)o.A - A1) + 0x1p-50 * (1.0 + a * a) * 1.4;
  const double dB = __builtin_fabs((double)o.B - B1) + 0x1p-50 * __builtin_fabs(a * b) * 1.2;
  const double dC = __builtin_fabs((double)o.C - C) +
                    0x1p-50 * (__builtin_fabs(dcp) + __builtin_fabs(dct) + b * b);
  const double fA = __builtin_fabs((double)o.A), fB = __builtin_fabs((double)o.B);
  const double fC = __builtin_fabs((double)o.C);
  const double h1 = fA * Zq + fB;  // |A' z' + B'|
  const double horner = dA * Zq * Zq + dB * Zq + dC + Zq * u * h1 * r + u * (h1 * Zq * r + fC);
  // z~ vs z: |t(z) - t(z~)| <= max|t'| Ez + |A| Ez^2
  const double slope = 2.0 * __builtin_fabs(A) * Zm + __builtin_fabs(B);
  const double e = (rho + slope * Ez + __builtin_fabs(A) * Ez * Ez + horner) * (1.0 + 0x1p-20) +
                   0x1p-140;
  o.err = round_up_f32(e);
  o.mag = round_up_f32(lt_mag + lq_mag + e);  // bounds |t| and |t~|
  // largest exact term over |z| <= Zm (pruning): the real quadratic's maximum
  // on the interval (vertex or an end) plus the chain error
  double qmax = A * Zm * Zm + __builtin_fabs(B) * Zm + C;
  if (A < 0.0) {
    double zv = -B / (2.0 * A);
    zv = zv < -Zm ? -Zm : (zv > Zm ? Zm : zv);
    qmax = A * zv * zv + B * zv + C;
  }
  qmax += 0x1p-40 * (__builtin_fabs(A) * Zm * Zm + __builtin_fabs(B) * Zm + __builtin_fabs(C));
  o.umax = round_up_f32(qmax + e);
  return o.err - o.err == 0.0f && o.mag - o.mag == 0.0f && o.A - o.A == 0.0f &&
         o.B - o.B == 0.0f && o.C - o.C == 0.0f && o.umax - o.umax == 0.0f;
}

#ifndef CWQ_IMP_DYNAMIC_MIN_GROUPS
#define CWQ_IMP_DYNAMIC_MIN_GROUPS 4096  // dynamic tile hand-out from this many groups
#endif
// ... or, when the host knows the launch's tile count, from this many tiles:
// below it the one-address hand-out counter (an atomic per tile from every
// workgroup) cost more than the balance it buys (I2's batch, ~4.4k tiles:
// 0.206 -> 0.185 ms static; pln_is 0.18 -> 0.13 ms; I1's 99.9k tiles need it:
// 8.40 -> 9.83 ms static)
#ifndef CWQ_IMP_DYNAMIC_MIN_TILES
#define CWQ_IMP_DYNAMIC_MIN_TILES 8192
#endif
#ifndef CWQ_IMP_MIN_WAVES
#define CWQ_IMP_MIN_WAVES 1  // waves/SIMD the register allocator must allow (tools/variants.sh)
#endif
// PER_BLOCK: group seeds from seeds.per_block (a batch of items); else
// seed + base + g.  CPT_MAX: the launch's tile size is kImpCandPerTile (the
// host knows its candidate count; k_imp_tiles picks the same size).  Both as
// template flags: the pointer and the tile size held in SGPRs through the
// loops cost I1 6% (more scalar spills in the screening loop).
template <bool PER_BLOCK, bool CPT_MAX>
__global__ void __launch_bounds__(256, CWQ_IMP_MIN_WAVES) k_imp_eval(
    const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ p_loc, const float* __restrict__ p_scale,
    const float* __restrict__ lnt, const float* __restrict__ lnp,
    const int64_t* __restrict__ block_off, const int64_t* __restrict__ n_samples, int64_t nb,
    const int64_t* __restrict__ tprefix, const int64_t* __restrict__ cpt_p, SeedSpec seeds,
    int allow_screen, uint32_t* __restrict__ gtau, unsigned long long* __restrict__ keys,
    unsigned long long* __restrict__ next_tile) {
  const int64_t total = tprefix[nb];
  // the grid is fixed (the tile count is only known on the device): workgroups
  // without a tile of the static assignment leave at once
  if (!next_tile && (int64_t)blockIdx.x >= total) return;
  const int64_t cpt = CPT_MAX ? kImpCandPerTile : *cpt_p;
  __shared__ int64_t s_tile;
  __shared__ double logtab[32];
  __shared__ float4 coef[kImpScreenMaxD];   // A, B, C per dim (screening)
  __shared__ float derr[kImpScreenMaxD];    // per-dim error bound
  __shared__ float dmag[kImpScreenMaxD];    // per-dim magnitude bound
  __shared__ float dumax[kImpScreenMaxD];   // per-dim largest exact term
  __shared__ float dsuf[kImpScreenMaxD + 1];  // pruning: sum of dumax[j..d)
  __shared__ float etot_sh;
  __shared__ uint32_t tau_ord;
  __shared__ uint32_t sq_cnt;
  __shared__ uint32_t sq_n[CWQ_IMP_SURVIVOR_CAP];
  __shared__ float sq_up[CWQ_IMP_SURVIVOR_CAP];
  __shared__ unsigned long long wkey[4];
  fill_logtab(logtab);
  const uint32_t wv = wave_id();
  const uint32_t lane = threadIdx.x & 63u;

  // Many groups: tiles differ in size by orders of magnitude (N_g from 1 to
  // ~4e5), so they are handed out one at a time through a global counter
  // (I1: -7%).  Few groups (fewer tiles than workgroups): the fixed
  // assignment, which saves the counter's round trip per tile (I2: -5%).
  int64_t tile = blockIdx.x;
  if (next_tile) {
    if (threadIdx.x == 0) s_tile = (int64_t)atomicAdd(next_tile, 1ull);
    __syncthreads();
    tile = s_tile;
    __syncthreads();
  }
#ifndef CWQ_IMP_PERMUTE
#define CWQ_IMP_PERMUTE 1
#endif
#ifndef CWQ_IMP_GTAU_MASK
#define CWQ_IMP_GTAU_MASK 63u  // 0: share tau with other tiles only at tile ends
#endif
  // dynamic hand-out order t -> tile (t * P) mod total, P = 2^31 - 1 prime
  // (a permutation while total < P): a group's tiles go out spread over the
  // launch, so most start after an earlier one has published its tau in
  // gtau[g] instead of all starting from -inf side by side (I1: -6%)
  const uint64_t pm = (CWQ_IMP_PERMUTE && next_tile && total > 1 && total < 0x7FFFFFFFll)
                          ? 0x7FFFFFFFull % (uint64_t)total : 1ull;
  for (; tile < total;) {
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int64_t tq = (int64_t)(((uint64_t)tile * pm) % (uint64_t)total);
    // group of this tile: last g with tprefix[g] <= tq
    int64_t lo = 0, hi = nb;  // tprefix[lo] <= tq < tprefix[hi]
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (tprefix[mid] <= tq) lo = mid; else hi = mid;
    }
    const int64_t g = lo;
    const int64_t off = block_off[g];
    const int64_t d = block_off[g + 1] - off;
    const int64_t N = n_samples[g] > 1 ? n_samples[g] : 1;
    const int64_t n0 = (tq - tprefix[g]) * cpt;
    const int64_t n1 = (n0 + cpt < N) ? n0 + cpt : N;
    const PhiloxStream st = generate_key(
        PER_BLOCK ? seeds.per_block[g] : block_seed(seeds.seed, seeds.base + g), 42);
    const int align = (int)(((uint64_t)(n0 + wv) * (uint64_t)d) & 3u);
    const float* tl = t_loc + off;
    const float* ts = t_scale + off;
    const float* pl = p_loc + off;
    const float* ps = p_scale + off;
    const float* ct = lnt + off;
    const float* cp = lnp + off;
    auto exact_row = [&](int64_t n) __attribute__((always_inline)) -> float {
      return eval_row_f<0>(st, (uint64_t)n * (uint64_t)d, d, (int)(((uint64_t)n * d) & 3u), logtab,
                           [&](int64_t e, float zz) -> float {
                             float x = ps[e] * zz;  // misc.py:14
                             x = pl[e] + x;         // misc.py:15
                             const float lt = log_prob(x, tl[e], ts[e], ct[e]);
                             const float lq = log_prob(x, pl[e], ps[e], cp[e]);
                             return lt - lq;        // :60
                           });
    };

    // screening gate and constants
    int ok = (allow_screen && d >= 1 && d <= kImpScreenMaxD) ? 1 : 0;
    if (ok && tid < d) {
      ImpScreenDim o;
      ok = imp_screen_dim(tl[tid], ts[tid], pl[tid], ps[tid], ct[tid], cp[tid], o) ? 1 : 0;
      coef[tid] = float4{o.A, o.B, o.C, 0.0f};
      derr[tid] = o.err;
      dmag[tid] = o.mag;
      dumax[tid] = o.umax;
    }
    const bool screen = __syncthreads_and(ok) != 0;
    if (screen && tid == 0) {
      double es = 0.0, ms = 0.0;
      for (int64_t j = 0; j < d; ++j) {
        es += (double)derr[j];
        ms += (double)dmag[j];
      }
      // |screened sum - exact Eigen-order sum| <= sum err_j + 2 gamma_d sum mag_j
      const double gam = 1.01 * (double)d * 0x1p-24;
      const double et = (es + 2.0 * gam * ms) * (1.0 + 0x1p-20) + 0x1p-126;
      etot_sh = et < 1.0e3 ? round_up_f32(et) : __builtin_inff();
      double suf = 0.0;
      dsuf[d] = 0.0f;
      for (int64_t j = d - 1; j >= 0; --j) {
        suf += (double)dumax[j];
        dsuf[j] = round_up_f32(suf * (1.0 + 0x1p-20) + 0x1p-126);  // covers the test's adds
      }
      // start from what earlier tiles of the group found (agent-scope load;
      // the loop reads gtau again every 64 units: per-iteration global
      // atomics on it cost more than they prune)
      tau_ord = __hip_atomic_load(&gtau[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sq_cnt = 0u;
    }
    __syncthreads();
    const float E = etot_sh;

    uint64_t bestk = 0;
    if (screen && E - E == 0.0f) {
      float tau = unord_f32(tau_ord);
      // may be the best: list it
      auto keep = [&](int64_t n, float sh, float slack) __attribute__((always_inline)) {
        const float up = sh + slack;
        tau = fmaxf(tau, sh - slack);
        const uint32_t slot = atomicAdd(&sq_cnt, 1u);
        if (slot < CWQ_IMP_SURVIVOR_CAP) {
          sq_n[slot] = (uint32_t)(n - n0);
          sq_up[slot] = up;
        } else {  // list full: evaluate exactly now
          const uint64_t k = argmax_key(exact_row(n), (uint32_t)n);
          bestk = k > bestk ? k : bestk;
        }
      };
      // every Philox block index (n d + j) / 4 of the group below 2^32:
      // counter word 1 is 0 (normal4_screen_lo: one multiply less per block)
      const bool lo32 = (uint64_t)N * (uint64_t)d <= (1ull << 34);
      auto scan = [&](auto HI0T) __attribute__((always_inline)) {
        constexpr bool HI0 = decltype(HI0T)::value;
        [[maybe_unused]] const PhiloxLo lok = HI0 ? philox_lo_key(st) : PhiloxLo{};
        if (d >= kImpPruneMinD) {
          // pruned screening: one Philox block of the lane's row per iteration;
          // a row stops once s + E + sum of the unvisited dims' maxima < tau.
          // Lanes refill from the wave's contiguous candidate range.
          const int64_t per_wave = (n1 - n0 + 3) / 4;
          const int64_t w0 = n0 + (int64_t)wv * per_wave;
          const int64_t w1 = (w0 + per_wave < n1) ? w0 + per_wave : n1;
          int64_t wnext = w0 + 64;
          int64_t n = w0 + lane;
          bool active = n < w1;
          int j = 0;
          float s = 0.0f;
          uint32_t iter = 0;
          while (__ballot(active) != 0ull) {
            const uint64_t k = (uint64_t)n * (uint64_t)d + (uint64_t)j;
            const F4 z = HI0 ? normal4_screen_lo(st, lok, (uint32_t)(k >> 2))
                             : normal4_screen(st, k >> 2);
            const int wa = (int)(k & 3u);
            const int cnt = (4 - wa) < (int)(d - j) ? (4 - wa) : (int)(d - j);
  #pragma unroll
            for (int t = 0; t < 4; ++t) {
              if (t < cnt) {
                const int w = wa + t;
                const float zz = w == 0 ? z.a : (w == 1 ? z.b : (w == 2 ? z.c : z.d));
                const float4 c = coef[j + t];
                s = s + __builtin_fmaf(__builtin_fmaf(c.x, zz, c.y), zz, c.z);
              }
            }
            j += cnt;
            const bool complete = (j == (int)d);
            const float slack = E + __builtin_fabsf(s) * 0x1p-22f;
            const float upper = (s + slack) + dsuf[j];
            const bool prune = !complete && (upper < tau);
            if (complete && active && upper >= tau) keep(n, s, slack);
            const bool done = complete || prune || !active;
            const uint64_t m = __ballot(done);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (done) {
              n = wnext + rank;
              j = 0;
              s = 0.0f;
            }
            wnext += (int64_t)__builtin_popcountll(m);
            active = n < w1;
            if (((++iter) & 15u) == 0u) {  // share tau with the workgroup
              const float tm = wave_max_f32(tau);
              if (lane == 0) atomicMax(&tau_ord, ord_f32(tm));
              uint32_t o = __atomic_load_n(&tau_ord, __ATOMIC_RELAXED);
  #if CWQ_IMP_GTAU_MASK
              // and every 64 units with the group's other tiles (publishing only
              // an improvement; I1 -2.5% on top of the permuted hand-out)
              if ((iter & CWQ_IMP_GTAU_MASK) == 0u) {
                const uint32_t o2 = __hip_atomic_load(&gtau[g], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
                if (lane == 0 && ord_f32(tm) > o2) atomicMax(&gtau[g], ord_f32(tm));
                o = o > o2 ? o : o2;
              }
  #endif
              tau = fmaxf(tau, unord_f32(o));
            }
          }
        } else {
          // short rows, no pruning: every row screened, listed if it may be
          // the best.  tau is shared in the wave after each of the first four
          // rounds and every fourth after (a lane-private tau lists ~ln(rows)
          // rows per lane, which overflowed the list into in-line exact rows),
          // and with the workgroup and the group's other tiles every 16.
          const int64_t iters = (n1 - n0 + 255) >> 8;  // wave-uniform trip count
          for (int64_t it = 0; it < iters; ++it) {
            const int64_t n = n0 + (it << 8) + 4 * (int64_t)lane + wv;
            if (n < n1) {
              const float sh =
                  screen_row_imp<HI0>(st, lok, (uint64_t)n * (uint64_t)d, d, align, coef);
              const float slack = E + __builtin_fabsf(sh) * 0x1p-22f;
              if (sh + slack >= tau) keep(n, sh, slack);
            }
            if (it < 4 || (it & 3) == 3) tau = wave_max_f32(tau);
            if ((it & 15) == 15) {
              if (lane == 0) atomicMax(&tau_ord, ord_f32(tau));
              uint32_t o = __atomic_load_n(&tau_ord, __ATOMIC_RELAXED);
              const uint32_t o2 = __hip_atomic_load(&gtau[g], __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
              if (lane == 0 && ord_f32(tau) > o2) atomicMax(&gtau[g], ord_f32(tau));
              o = o > o2 ? o : o2;
              tau = fmaxf(tau, unord_f32(o));
            }
          }
        }
      };
      if (lo32)
        scan(std::integral_constant<bool, true>{});
      else
        scan(std::integral_constant<bool, false>{});
      {
        const float tm = wave_max_f32(tau);
        if (lane == 0) atomicMax(&tau_ord, ord_f32(tm));
      }
      __syncthreads();
      // this tile's threshold, raised by what other tiles of the group published
      if (tid == 0) {
        const uint32_t mine = tau_ord;
        const uint32_t prev = atomicMax(&gtau[g], mine);
        tau_ord = prev > mine ? prev : mine;
      }
      __syncthreads();
      const float tau_final = unord_f32(tau_ord);
      const uint32_t ns = sq_cnt < CWQ_IMP_SURVIVOR_CAP ? sq_cnt : CWQ_IMP_SURVIVOR_CAP;
      for (uint32_t i = tid; i < ns; i += blockDim.x) {
        if (sq_up[i] >= tau_final) {
          const int64_t n = n0 + (int64_t)sq_n[i];
          const uint64_t k = argmax_key(exact_row(n), (uint32_t)n);
          bestk = k > bestk ? k : bestk;
        }
      }
    } else {
      for (int64_t n = n0 + 4 * (int64_t)lane + wv; n < n1; n += 256) {
        const float v = eval_row_f<0>(st, (uint64_t)n * (uint64_t)d, d, align, logtab,
                                      [&](int64_t e, float zz) -> float {
                                        float x = ps[e] * zz;  // misc.py:14
                                        x = pl[e] + x;         // misc.py:15
                                        const float lt = log_prob(x, tl[e], ts[e], ct[e]);
                                        const float lq = log_prob(x, pl[e], ps[e], cp[e]);
                                        return lt - lq;        // :60
                                      });
        const uint64_t k = argmax_key(v, (uint32_t)n);
        bestk = k > bestk ? k : bestk;
      }
    }
    bestk = wave_max_u64(bestk);
    if (lane == 0) wkey[wv] = bestk;
    __syncthreads();
    if (tid == 0) {
      uint64_t m = wkey[0];
      for (int i = 1; i < 4; ++i) m = wkey[i] > m ? wkey[i] : m;
      if (m) atomicMax(&keys[g], (unsigned long long)m);
    }
    __syncthreads();
    if (next_tile) {
      if (threadIdx.x == 0) s_tile = (int64_t)atomicAdd(next_tile, 1ull);
      __syncthreads();
      tile = s_tile;
      __syncthreads();
    } else {
      tile += gridDim.x;
    }
  }
}

// The groups of at most kImpSmallN candidates (no k_imp_eval tile): one wave
// per group, every row exact (the same rows, sums and argmax keys as
// k_imp_eval's exact evaluation, so the emitted index is the same), the
// wave's best key stored to keys[g] (zeroed by the launcher; no other kernel
// writes a small group's key).
__global__ void __launch_bounds__(256) k_imp_small(
    const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ p_loc, const float* __restrict__ p_scale,
    const float* __restrict__ lnt, const float* __restrict__ lnp,
    const int64_t* __restrict__ block_off, const int64_t* __restrict__ n_samples, int64_t nb,
    SeedSpec seeds, unsigned long long* __restrict__ keys) {
  __shared__ double logtab[32];
  fill_logtab(logtab);
  const uint32_t wv = wave_id();
  const uint32_t lane = threadIdx.x & 63u;
  for (int64_t g = (int64_t)blockIdx.x * 4 + wv; g < nb; g += (int64_t)gridDim.x * 4) {
    const int64_t N = n_samples[g] > 1 ? n_samples[g] : 1;
    if (N > kImpSmallN) continue;  // wave-uniform
    const int64_t off = block_off[g];
    const int64_t d = block_off[g + 1] - off;
    const PhiloxStream st = generate_key(seeds.of(g), 42);
    const float* tl = t_loc + off;
    const float* ts = t_scale + off;
    const float* pl = p_loc + off;
    const float* ps = p_scale + off;
    const float* ct = lnt + off;
    const float* cp = lnp + off;
    uint64_t bestk = 0;
    for (int64_t n = lane; n < N; n += 64) {
      const float v = eval_row_f<0>(st, (uint64_t)n * (uint64_t)d, d, (int)(((uint64_t)n * d) & 3u),
                                    logtab, [&](int64_t e, float zz) -> float {
                                      float x = ps[e] * zz;  // misc.py:14
                                      x = pl[e] + x;         // misc.py:15
                                      const float lt = log_prob(x, tl[e], ts[e], ct[e]);
                                      const float lq = log_prob(x, pl[e], ps[e], cp[e]);
                                      return lt - lq;        // :60
                                    });
      const uint64_t k = argmax_key(v, (uint32_t)n);
      bestk = k > bestk ? k : bestk;
    }
    bestk = wave_max_u64(bestk);
    if (lane == 0 && bestk) keys[g] = (unsigned long long)bestk;
  }
}

// Row `index` of group g's candidate stream: p_loc + p_scale * z (misc.py:14-15).
// With keys != nullptr the index comes from the argmax key (encoder), else
// from index_in (decoder, coded_importance_sampler.py:82-109).  out_sample
// (if given) gets the row; dst_out (if given) the row destandardised,
// dst_scale * row + dst_loc, exactly as k_destandardise computes it (the
// grouped calls' :265 rescale without a launch of its own).
__global__ void __launch_bounds__(256) k_imp_rows(
    const unsigned long long* __restrict__ keys, const int64_t* __restrict__ index_in,
    const float* __restrict__ p_loc, const float* __restrict__ p_scale,
    const int64_t* __restrict__ block_off, int64_t nb, SeedSpec seeds,
    int64_t* __restrict__ index_out, float* __restrict__ out_sample,
    const float* __restrict__ dst_loc, const float* __restrict__ dst_scale,
    float* __restrict__ dst_out) {
  __shared__ double logtab[32];
  fill_logtab(logtab);
  const uint32_t wv = wave_id();
  const uint32_t lane = threadIdx.x & 63u;
  for (int64_t g = (int64_t)blockIdx.x * 4 + wv; g < nb; g += (int64_t)gridDim.x * 4) {
    const int64_t off = block_off[g];
    const int64_t d = block_off[g + 1] - off;
    int64_t idx;
    if (keys) {
      const uint64_t key = keys[g];
      idx = (key >> 32) > kArgmaxClampOrd ? (int64_t)argmax_key_index(key) : 0;
      if (lane == 0) index_out[g] = idx;
    } else {
      idx = index_in[g];
    }
    const PhiloxStream st = generate_key(seeds.of(g), 42);
    for (int64_t j = lane; j < d; j += 64) {
      float v = __builtin_nanf("");
      if (idx >= 0) {
        const uint64_t k = (uint64_t)idx * (uint64_t)d + (uint64_t)j;
        const F4 z = normal4_dev(st, k >> 2, logtab);
        const uint32_t w = (uint32_t)(k & 3u);
        const float zz = w == 0 ? z.a : (w == 1 ? z.b : (w == 2 ? z.c : z.d));
        v = p_scale[off + j] * zz;
        v = p_loc[off + j] + v;
      }
      if (out_sample) out_sample[off + j] = v;
      if (dst_out) {
        const float m = dst_scale[off + j] * v;
        dst_out[off + j] = m + dst_loc[off + j];
      }
    }
  }
}

// :142-145, :148: per-dim KL in bits against dim_kl_bit_limit (float32, as
// numpy compares the float32 array); outlier dims get the standard target
// N(0, 1) (t_loc = 0, t_scale = 1).  keep[j] = 1 for coded dims.
__global__ void __launch_bounds__(256) k_imp_outliers(const float* __restrict__ kl, int64_t n,
                                                      float limit, float* __restrict__ t_loc,
                                                      float* __restrict__ t_scale,
                                                      uint8_t* __restrict__ keep) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float bits = kl[i] / 0.6931472f;  // kl / np.float32(np.log(2))
    const bool k = bits <= limit;           // NaN: an outlier, as in numpy
    if (!k) {
      t_loc[i] = 0.0f;
      t_scale[i] = 1.0f;
    }
    keep[i] = k ? 1 : 0;
  }
}

hipError_t launch_imp_outliers(const float* kl, int64_t n, float limit, float* t_loc,
                               float* t_scale, uint8_t* keep, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int64_t g = (n + 255) / 256;
  g = g < 8192 ? g : 8192;
  hipLaunchKernelGGL(k_imp_outliers, dim3((unsigned)g), dim3(256), 0, stream, kl, n, limit,
                     t_loc, t_scale, keep);
  return hipGetLastError();
}

size_t importance_workspace_size(int64_t nb, int64_t total_dims) {
  auto up = [](size_t v) { return (v + 255) / 256 * 256; };
  return up((size_t)nb * 8) + up((size_t)(nb + 1) * 8) + 2 * up((size_t)total_dims * 4) +
         up((size_t)nb * 4) + 256;
}

// block_seeds: device [nb] per-group seeds (a batch of items, each numbering
// its groups from 0 with its own seed), or nullptr: seed + block_id_base + g.
// total_cands: sum over groups of max(n_samples[g], 1) when the host knows it
// (-1: unknown; it only selects a kernel instantiation, never the results)
hipError_t launch_importance_encode(const float* t_loc, const float* t_scale, const float* p_loc,
                                    const float* p_scale, const int64_t* block_off,
                                    const int64_t* n_samples, int64_t nb, int64_t total_dims,
                                    int32_t seed, int64_t block_id_base,
                                    const int32_t* block_seeds, int allow_screen,
                                    int64_t* out_index, float* out_sample, void* workspace,
                                    hipStream_t stream, int64_t total_cands,
                                    int64_t total_tiles, const float* dst_loc,
                                    const float* dst_scale, float* dst_out) {
  if (nb <= 0) return hipSuccess;
  auto up = [](size_t v) { return (v + 255) / 256 * 256; };
  char* w = (char*)workspace;
  unsigned long long* keys = (unsigned long long*)w;
  int64_t* tprefix = (int64_t*)(w + up((size_t)nb * 8));
  float* lnt = (float*)(w + up((size_t)nb * 8) + up((size_t)(nb + 1) * 8));
  float* lnp = lnt + up((size_t)total_dims * 4) / 4;
  uint32_t* gtau = (uint32_t*)((char*)lnp + up((size_t)total_dims * 4));
  unsigned long long* next_tile = (unsigned long long*)((char*)gtau + up((size_t)nb * 4));
  int64_t* cpt = (int64_t*)(next_tile + 1);
  const SeedSpec ss{seed, block_id_base, block_seeds};
  if (total_dims > 0)
    hipLaunchKernelGGL(k_imp_prep, dim3(grid_for(total_dims, 256, 65536)), dim3(256), 0, stream,
                       t_scale, p_scale, total_dims, lnt, lnp);
  hipLaunchKernelGGL(k_imp_tiles, dim3(1), dim3(1024), 0, stream, n_samples, nb, cpt, tprefix,
                     gtau, next_tile, keys);
  const bool cmax = total_cands >= 0 && imp_cand_per_tile(total_cands) == kImpCandPerTile;
  auto eval = block_seeds ? (cmax ? k_imp_eval<true, true> : k_imp_eval<true, false>)
                          : (cmax ? k_imp_eval<false, true> : k_imp_eval<false, false>);
  hipLaunchKernelGGL(eval, dim3((unsigned)kImpEvalGrid), dim3(256), 0, stream, t_loc, t_scale,
                     p_loc, p_scale, lnt, lnp, block_off, n_samples, nb, (const int64_t*)tprefix,
                     (const int64_t*)cpt, ss, allow_screen, gtau, keys,
                     (total_tiles >= 0 ? total_tiles >= CWQ_IMP_DYNAMIC_MIN_TILES
                                       : nb >= CWQ_IMP_DYNAMIC_MIN_GROUPS)
                         ? next_tile
                         : nullptr);
  if (kImpSmallN > 0)
    hipLaunchKernelGGL(k_imp_small, dim3(grid_for(nb, 4, 65536)), dim3(256), 0, stream, t_loc,
                       t_scale, p_loc, p_scale, lnt, lnp, block_off, n_samples, nb, ss, keys);
  hipLaunchKernelGGL(k_imp_rows, dim3(grid_for(nb, 4, 65536)), dim3(256), 0, stream,
                     (const unsigned long long*)keys, (const int64_t*)nullptr, p_loc, p_scale,
                     block_off, nb, ss, out_index, out_sample, dst_loc, dst_scale, dst_out);
  return hipGetLastError();
}

int64_t importance_tile_count(const int64_t* n_samples_host, int64_t nb, int64_t total_cands) {
  const int64_t cpt = imp_cand_per_tile(total_cands);  // k_imp_tiles' rule
  int64_t tiles = 0;
  for (int64_t g = 0; g < nb; ++g) {
    const int64_t n = n_samples_host[g] > 1 ? n_samples_host[g] : 1;
    tiles += n <= kImpSmallN ? 0 : (n + cpt - 1) / cpt;
  }
  return tiles;
}

hipError_t launch_importance_decode(const int64_t* index, const float* p_loc,
                                    const float* p_scale, const int64_t* block_off, int64_t nb,
                                    int32_t seed, int64_t block_id_base, float* out_sample,
                                    hipStream_t stream) {
  if (nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_imp_rows, dim3(grid_for(nb, 4, 65536)), dim3(256), 0, stream,
                     (const unsigned long long*)nullptr, index, p_loc, p_scale, block_off, nb,
                     SeedSpec{seed, block_id_base, nullptr}, (int64_t*)nullptr, out_sample,
                     (const float*)nullptr, (const float*)nullptr, (float*)nullptr);
  return hipGetLastError();
}

}  // namespace cwq
