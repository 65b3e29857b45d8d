// cwq_kernels.hip -- gfx950 kernels of the greedy coded sampler.
//
// Hot path: for every block (the reference's "group")
// and every step, 2^b candidates are drawn from the proposal shard with the
// stateless Philox stream, scored by the target log-density and reduced to
// the argmax; the decoder regenerates only the selected row.
//
// Mapping:
//   * one "tile" = (block g, candidate range [n0, n1)), one 256-thread
//     workgroup per tile; a block whose 2^b candidates would leave the chip
//     idle is split over several tiles and merged with one 64-bit atomicMax
//     per workgroup on an orderable (value, ~index) key.
//   * inside a workgroup, wave v owns the candidates n == n0 + v (mod 4), so
//     the Philox word alignment (n*d) mod 4 is uniform within a wave and the
//     "start a new Philox block" branch is a scalar branch even for odd d.
//   * candidates are never materialised: each lane regenerates its row's
//     normals in registers (Philox -> Box-Muller -> shard -> log-prob) and
//     accumulates them in the Eigen AVX summation order.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <stdint.h>

#include "cwq_device.h"
#include "cwq_kernels.h"

namespace cwq {

// ---------------------------------------------------------------------------
// Per-dimension constants of a step (coded_greedy_sampler.py:42-48).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_prep_dims(
    const float* __restrict__ t_scale, const float* __restrict__ p_loc,
    const float* __restrict__ p_scale, int64_t n, float nst, float sdiv, float rho,
    float* __restrict__ loc_s, float* __restrict__ scale_s, float* __restrict__ lognorm,
    float* __restrict__ out_sample, unsigned long long* __restrict__ keys, int64_t nb) {
  // step 0's argmax keys start at 0 (one launch less than a memset)
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < nb;
       g += (int64_t)gridDim.x * blockDim.x)
    keys[g] = 0ull;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    loc_s[i] = p_loc[i] / nst;                // p_loc / n_steps
    float rs = rho * p_scale[i];              // rho * p_scale
    scale_s[i] = rs / sdiv;                   //   / sqrt(n_steps)
    lognorm[i] = kHalfLog2Pi + logf_full(t_scale[i], kLogTabConst);
    out_sample[i] = 0.0f;                     // best_sample = tf.zeros (:68)
  }
}

// ---------------------------------------------------------------------------
// One candidate row: sum_j log N(best_j + loc_s_j + scale_s_j z_j; mu_j, s_j)
// in the Eigen 3.3 AVX inner-dim reduction order.
//   kbase = n*d (flat index of the row's first normal), align = kbase & 3
//   (wave-uniform).  DC > 0: compile-time dimension (DC % 4 == 0 -> align 0).
// ---------------------------------------------------------------------------
// Greedy candidate row (coded_greedy_sampler.py:57-59).
template <int DC, bool STEP0>
__device__ __forceinline__ float eval_row(const PhiloxStream& st, uint64_t kbase, int64_t d_rt,
                                          int align_rt, const float* __restrict__ loc_s,
                                          const float* __restrict__ scale_s,
                                          const float* __restrict__ mu,
                                          const float* __restrict__ sg,
                                          const float* __restrict__ lognorm,
                                          const float* __restrict__ best,
                                          const double* logtab) {
  return eval_row_f<DC>(st, kbase, d_rt, align_rt, logtab, [&](int64_t e, float zz) -> float {
    float s = scale_s[e] * zz;  // misc.py:14
    s = loc_s[e] + s;           // misc.py:15
    const float tv = STEP0 ? s : best[e] + s;  // :57 (best == +0 at step 0)
    return log_prob(tv, mu[e], sg[e], lognorm[e]);
  });
}

// ---------------------------------------------------------------------------
// Encoder, one step: every tile scores its candidate range and folds its best
// (value, index) into keys[g] with one atomicMax.
// ---------------------------------------------------------------------------
template <int DC, bool STEP0>
__global__ void __launch_bounds__(256) k_encode_eval(
    const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ loc_s, const float* __restrict__ scale_s,
    const float* __restrict__ lognorm, const float* __restrict__ best,
    const int64_t* __restrict__ block_off, int64_t ud, int64_t ntiles, int64_t tiles_per_block,
    int64_t cand_per_tile, int64_t n_cand, SeedSpec sd, int32_t step,
    unsigned long long* __restrict__ keys) {
  __shared__ double logtab[32];
  __shared__ unsigned long long wkey[4];
  fill_logtab(logtab);
  const uint32_t wv = wave_id();
  const uint32_t lane = threadIdx.x & 63u;

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t g = tile / tiles_per_block;
    const int64_t tt = tile - g * tiles_per_block;
    const BlockSpan sp = block_span(block_off, ud, g);
    const int64_t n0 = tt * cand_per_tile;
    const int64_t n1 = (n0 + cand_per_tile < n_cand) ? n0 + cand_per_tile : n_cand;
    const PhiloxStream st =
        generate_key(step_seed(sd.of(g), step), 42);
    const int align = (int)(((uint64_t)(n0 + wv) * (uint64_t)sp.d) & 3u);

    uint64_t bestk = 0;
    for (int64_t n = n0 + 4 * (int64_t)lane + wv; n < n1; n += 256) {
      const float v = eval_row<DC, STEP0>(st, (uint64_t)n * (uint64_t)sp.d, sp.d, align,
                                          loc_s + sp.off, scale_s + sp.off, t_loc + sp.off,
                                          t_scale + sp.off, lognorm + sp.off,
                                          STEP0 ? nullptr : best + sp.off, logtab);
      const uint64_t k = argmax_key(v, (uint32_t)n);
      bestk = k > bestk ? k : bestk;
    }
    bestk = wave_max_u64(bestk);
    if (lane == 0) wkey[wv] = bestk;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t m = wkey[0];
      for (int i = 1; i < 4; ++i) m = wkey[i] > m ? wkey[i] : m;
      if (m) atomicMax(&keys[g], (unsigned long long)m);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Pruned encoder for uniform blocks, D % 8 == 0, D <= 64 (the C1/C4/C5 shapes).
//
// Same result as k_encode_eval, less work: a candidate whose log-density can
// no longer reach a value already achieved in this tile is dropped before its
// remaining dims are generated.
//
// Order: each block's D/4 Philox groups are visited in decreasing order of
// their expected log-density deficit under the proposal shard (the dims that
// discriminate most first), one group (4 dims, one Philox block) per step.
//
// Drop rule ("pruning bound"): after the first k visited groups,
// with float running sum s of their log-densities, candidate n is dropped iff
//     s + 2^-14 |s| + B_k  <  tau
// where B_k >= sum_{unvisited j} f(M_j) + 2^-14 K_k (+ float evaluation
// margin), M_j = -c_j is the largest value the float log-density of dim j can
// take, f(x) = x + g|x| with g >= gamma_{D-1} + gamma_{D}, and K_k sums
// |M_j| + M_j over the visited dims.  The left side bounds from above the
// float Eigen-order value of every completion of the row; tau is a lower
// bound of the exact value of a candidate already completed in this tile.  So
// a dropped candidate is strictly worse than an existing one: neither the
// argmax nor a tie.
//
// Completion: after all groups, s brackets the exact value within
// [s - 2^-14|s| - L, s + 2^-14|s| + B_D].  Candidates whose upper end reaches
// tau go to an LDS survivor list; at the end of the tile the survivors whose
// upper end reaches the final tau are re-evaluated exactly (natural order,
// Eigen summation, eval_row) and only those produce argmax keys.
//
// Lanes keep one candidate each and refill from a per-wave counter with
// ballot/mbcnt when theirs completes or is dropped, so waves stay full even
// though candidates stop after different numbers of groups.
// ---------------------------------------------------------------------------
constexpr float kPruneC1 = 0x1p-14f;
#ifndef CWQ_PRUNE_MIN_WAVES
#define CWQ_PRUNE_MIN_WAVES 6  // waves/SIMD the register allocator must allow (tools/variants.sh)
#endif
#ifndef CWQ_XCD_BALANCE
#define CWQ_XCD_BALANCE 1  // INTER tiles: each XCD runs every block (see k_encode_prune)
#endif
#ifndef CWQ_TAU_SHARE_MASK
#define CWQ_TAU_SHARE_MASK 15u  // share tau across the workgroup every 16 units
#endif
#ifndef CWQ_SURVIVOR_CAP
#define CWQ_SURVIVOR_CAP 1024
#endif

// best + (loc_s + scale_s z) - mu  (misc.py:14-15, coded_greedy_sampler.py:57, TFP _z numerator)
template <bool STEP0>
__device__ __forceinline__ float cand_diff(float z, float ls, float ss, float mu, float bb) {
  float s = ss * z;  // misc.py:14
  s = ls + s;        // misc.py:15
  const float tv = STEP0 ? s : bb + s;
  return tv - mu;
}
__device__ __forceinline__ float lp_from_z(float z, float cc) {
  const float u = -0.5f * (z * z);
  return u - cc;
}

// Screening pass ("screening bound").  On tiles whose constants
// pass the range gate below, the drop decisions are taken on cheap
// approximations instead of exact values: z~ from the hardware
// transcendentals (|z~ - z| <= kScreenEz for every Philox output), and per dim
//     a_j = RN(sA_j z~ + sB_j),  sA_j ~ ss_j K_j,  sB_j ~ (best + loc_s - mu)_j K_j,
// K_j = sqrt(phi (1 - 2^-24) / 2) / sigma_j, with the guarantee
//     0.5 y_j^2 (1 - 2^-24)  >=  a_j^2 - C_j
// for the exact standardised value y_j (C_j a tiny per-dim constant).  With s
// the float sum of -a_j^2 over the visited dims, every completion of the row
// has an exact Eigen-order value
//     E  <=  (1 - 2^-14) s + Bs_k,    Bs_k ~ sum_j M_j + sum_{visited} C_j,
// and a completed row has E >= (1 + 2^-13) s + As - Pq sqrt(-s), which
// feeds tau.  Survivors are re-evaluated exactly as in the exact pass, so the
// screening arithmetic never reaches the output.
constexpr float kScreenC1 = 1.0f - 0x1p-14f;
constexpr float kScreenC2 = 1.0f + 0x1p-13f;
constexpr double kScreenEps = 0x1p-15;  // split of the additive error: (x-A)^2 >= (1-e)x^2 - (1/e-1)A^2
constexpr double kScreenPhi = (1.0 - kScreenEps) * (1.0 - 0x1p-21);
constexpr double kScreenKappa = 0.7070958018530696;  // sqrt(phi (1 - 2^-24) / 2), rounded down


#ifdef CWQ_TILE_TIMES
// timing builds only (tools/tile_times.py): per tile of k_encode_prune its
// start / end wall clock (s_memrealtime, 100 MHz) and the workgroup that ran it
constexpr int kTileTimes = 1 << 18;
__device__ unsigned long long g_tile_t0[kTileTimes], g_tile_t1[kTileTimes];
__device__ unsigned int g_tile_wg[kTileTimes];
#endif
#ifdef CWQ_PRUNE_STATS
// tuning builds only (tools/prune_stats.py): [0..64] candidates finished after
// k units, [65] completed rows, [66] survivors pushed, [67] screened tiles;
// general kernel (tools/csr_stats.py): [40]/[41] screened/exact tiles, [42] rows
// finished, [43] dims screened, [44] rows completed, [45] survivors pushed,
// [46] list-full exact rows, [47] survivors re-evaluated, [48] lane-iterations
__device__ unsigned long long g_prune_stats[72];
// "oracle tau" experiment: each tile's best key is saved; with g_seed_tau set
// the next launch starts every tile at the exact best value of the last one
constexpr int kDbgBlocks = 1 << 20;
__device__ unsigned long long g_dbg_best[kDbgBlocks];
__device__ int g_seed_tau;
#endif

template <int D, bool STEP0, bool INTER>
__global__ void __launch_bounds__(256, CWQ_PRUNE_MIN_WAVES) k_encode_prune(
    const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ loc_s, const float* __restrict__ scale_s,
    const float* __restrict__ lognorm, const float* __restrict__ best, int64_t ntiles,
    int64_t tiles_per_block, int64_t cand_per_tile, int64_t n_cand, SeedSpec sd, int32_t step,
    int allow_screen, unsigned long long* __restrict__ keys, int64_t tail_from, int tail_div,
    uint32_t* __restrict__ tq) {
  static_assert(D % 8 == 0 && D >= 8 && D <= 64, "pruned path: D % 8 == 0, D <= 64");
  constexpr int G = D / 4;
  constexpr int NF = STEP0 ? 6 : 7;  // loc_s, scale_s, mu, sigma, c, 1/sigma[, best]
  constexpr int NS = 2;              // screening: sA, sB
  __shared__ double logtab[32];
  __shared__ float4 cst[G * NF];     // constants of the k-th visited group
  __shared__ float4 scst[G * NS];    // screening constants of the k-th visited group
  __shared__ int2 meta[G];           // {Philox group of visit k, bits of B_{k+1}}
  __shared__ float dscore[D];
  __shared__ float dA[D];            // screening: A_j (additive error, a units)
  __shared__ float dC[D];            // screening: C_j
  __shared__ float gscore[G];
  __shared__ int gpos[G];
  __shared__ float lowc;             // L: lower-end constant of a completed row
  __shared__ float scr_a, scr_pq;    // screening: As, Pq
  __shared__ uint32_t tau_ord;
  __shared__ uint32_t sq_cnt;
  __shared__ uint32_t sq_n[CWQ_SURVIVOR_CAP];
  __shared__ float sq_ub[CWQ_SURVIVOR_CAP];
  __shared__ unsigned long long wkey[4];
  __shared__ uint32_t s_next;
#ifdef CWQ_PRUNE_STATS
  // per-workgroup counters (LDS atomics), added to g_prune_stats once per tile:
  // one global atomic per finished candidate made C5-sized runs take minutes
  __shared__ uint32_t s_ps[72];
  for (int i = threadIdx.x; i < 72; i += blockDim.x) s_ps[i] = 0u;
#endif
  fill_logtab(logtab);
  const uint32_t wv = wave_id();
  const uint32_t lane = threadIdx.x & 63u;

  // INTER (several tiles per block, high rates): tiles run block-interleaved
  // (tile t is tile t / nb of block t % nb), so a block's later tiles start
  // after its first ones have finished and begin from the exact best value
  // they left in keys[g] instead of from -inf
  constexpr bool inter = INTER;
  const int64_t nbt = INTER ? ntiles / tiles_per_block : 0;
  // tile queue (tq != nullptr): a workgroup's first tile is its id, later ones
  // come from one atomic counter, so workgroups stay resident until the queue
  // is empty.  With one tile per workgroup the resident count fell from 1,514
  // to 1,414 of 1,536 slots over a C5 launch as finished workgroups were
  // replaced (tools/tile_times.py); the queue keeps every slot busy to the end.
  auto next_tile = [&](int64_t cur) -> int64_t {
    if (tq == nullptr) return cur + gridDim.x;
    __syncthreads();
    if (threadIdx.x == 0) s_next = gridDim.x + atomicAdd(tq, 1u);
    __syncthreads();
    return (int64_t)s_next;
  };
  for (int64_t tile = blockIdx.x; tile < ntiles; tile = next_tile(tile)) {
    // thread index re-derived per tile behind an opaque move: the per-thread
    // addresses below are then recomputed (cheap) instead of hoisted out of the
    // tile loop and spilled under the 6-waves/SIMD register budget
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
#ifdef CWQ_TILE_TIMES
    if (tid == 0 && tile < kTileTimes) {
      g_tile_t0[tile] = __builtin_amdgcn_s_memrealtime();
      // HW_REG_XCC_ID (hwreg 20), bits [3:0]: the XCD this workgroup runs on
      const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));
      g_tile_wg[tile] = (xcc << 24) | (blockIdx.x & 0xffffffu);
    }
#endif
    // XCD balance (INTER): workgroups go to the 8 XCDs round-robin by id, so
    // with the block-interleaved order XCD x would run only the blocks == x
    // (mod 8), and with few blocks per XCD their uneven pruning left XCDs idle
    // at the end (tools/tile_times.py: 84% of the slots busy on 128 blocks).
    // XCD x instead runs the x-th eighth of the interleaved order: every block,
    // a contiguous range of its tiles.
    // Only the full-size tiles are spread so: the short tail tiles (below) come
    // last in their natural order, so every XCD gets its share of them too.
    int64_t tord = tile;
    const int64_t treg = inter ? nbt * tail_from : 0;  // full-size tiles
    if (inter && CWQ_XCD_BALANCE && tq == nullptr && tile < treg && (treg & 7) == 0 &&
        (gridDim.x & 7u) == 0)
      tord = (tile & 7) * (treg >> 3) + (tile >> 3);
    const int64_t g = inter ? tord % nbt : tile / tiles_per_block;
    const int64_t tt = inter ? tord / nbt : tile - g * tiles_per_block;
    const int64_t off = g * D;
    // a block's tiles from tail_from on are tail_div times smaller: the last
    // rounds of the launch drain in short tiles (INTER; tail_div 1: no tail)
    int64_t n0, csz;
    if (tt < tail_from) {
      n0 = tt * cand_per_tile;
      csz = cand_per_tile;
    } else {
      csz = cand_per_tile / tail_div;
      n0 = tail_from * cand_per_tile + (tt - tail_from) * csz;
    }
    const int64_t n1 = (n0 + csz < n_cand) ? n0 + csz : n_cand;
    if (n0 >= n1) continue;  // (uniform) a tail piece past the block's candidates
    const PhiloxStream st =
        generate_key(step_seed(sd.of(g), step), 42);

    // (a) expected deficit of dim j under the proposal shard:
    //     E[0.5((T - mu)/sigma)^2], T ~ N(best + loc_s, scale_s^2)
    if (tid < D) {
      const int j = tid;
      const float ls = loc_s[off + j], ss = scale_s[off + j], mu = t_loc[off + j];
      const float rs = 1.0f / t_scale[off + j];
      const float m = (STEP0 ? ls : best[off + j] + ls) - mu;
      float e = 0.5f * (ss * ss + m * m) * (rs * rs);
      dscore[j] = (e == e) ? e : -1.0f;
    }
    __syncthreads();
    // (b) group scores, (c) visit order: rank by decreasing score, ties by index
    if (tid < G) {
      const int q = tid;
      gscore[q] = ((dscore[4 * q] + dscore[4 * q + 1]) + dscore[4 * q + 2]) + dscore[4 * q + 3];
    }
    __syncthreads();
    if (tid < G) {
      const int q = tid;
      const float sq = gscore[q];
      int r = 0;
      for (int q2 = 0; q2 < G; ++q2) {
        const float s2 = gscore[q2];
        r += (s2 > sq || (s2 == sq && q2 < q)) ? 1 : 0;
      }
      gpos[q] = r;
      meta[r].x = q;
    }
    __syncthreads();
    // (d) constants in visit order (reloaded: nothing is held across the syncs)
    int den_ok = 1, scr_ok = 1;
    if (tid < D) {
      const int j = tid, k = gpos[j >> 2], w = j & 3;
      float fj[7];
      const float sgj = t_scale[off + j];
      fj[0] = loc_s[off + j];
      fj[1] = scale_s[off + j];
      fj[2] = t_loc[off + j];
      fj[3] = sgj;
      fj[4] = lognorm[off + j];
      fj[5] = 1.0f / sgj;
      fj[6] = STEP0 ? 0.0f : best[off + j];
      float* c = reinterpret_cast<float*>(cst);
#pragma unroll
      for (int f = 0; f < NF; ++f) c[(k * NF + f) * 4 + w] = fj[f];
      den_ok = markstein_ok_den(sgj) ? 1 : 0;
      // screening constants (see kScreen* above and DESIGN.md)
      const double ssa = __builtin_fabs((double)fj[1]), lsa = __builtin_fabs((double)fj[0]);
      const double mua = __builtin_fabs((double)fj[2]);
      const double bba = STEP0 ? 0.0 : __builtin_fabs((double)fj[6]);
      const double zs = kScreenZm * ssa;
      const double mag = bba + lsa + zs + mua;
      // rounding of the exact chain RN(RN(RN(bb +) RN(ls + RN(ss z))) - mu)
      const double rho = 0x1p-24 * 1.0001 * (zs + (lsa + zs) + (STEP0 ? 0.0 : bba + lsa + zs) + mag);
      const double offd = (STEP0 ? 0.0 : (double)fj[6]) + (double)fj[0] - (double)fj[2];
      const double sig = (double)sgj;
      const double kq = kScreenKappa / sig;
      const float sa = (float)((double)fj[1] * kq * kSqrt2Ln2);  // z~ arrives / sqrt(2 ln 2)
      const float sb = (float)(offd * kq);
      float* sc = reinterpret_cast<float*>(scst);
      sc[(k * NS + 0) * 4 + w] = sa;
      sc[(k * NS + 1) * 4 + w] = sb;
      const double a0 = (kq * (rho + ssa * kScreenEz) +
                         kq * 0x1p-24 * 1.0001 * (zs + __builtin_fabs(offd))) * (1.0 + 0x1p-20) +
                        0x1p-140;
      const float cdim = round_up_f32((1.0 / kScreenEps - 1.0) * a0 * a0 / kScreenPhi * (1.0 + 0x1p-20));
      dA[j] = round_up_f32(a0 * 1.0001);
      dC[j] = cdim;
      const float cj = fj[4];
      scr_ok = (den_ok && mag <= 0x1p100 && mag / sig <= 0x1p50 && cdim <= 0x1p60f &&
                sa - sa == 0.0f && sb - sb == 0.0f && cj - cj == 0.0f)
                   ? 1
                   : 0;
    }
    const bool fastdiv = __syncthreads_and(den_ok) != 0;
    const bool scr_all = __syncthreads_and(scr_ok) != 0;
    // (e) drop bounds: thread k computes B_k for the first k visited groups
    //     (exact or screening form); thread G + 1 the screening constants
    const bool screen = allow_screen && scr_all;
    if (tid <= G + 1) {
      const int kb = tid;
      const float* c = reinterpret_cast<const float*>(cst);
      double rf = 0.0, kk = 0.0, asum = 0.0, msum = 0.0, kall = 0.0, cvis = 0.0, a2 = 0.0,
             amax = 0.0;
#pragma unroll 1
      for (int p = 0; p < D; ++p) {  // p = 4 * (visit position) + w
        const double mj = -(double)c[((p >> 2) * NF + 4) * 4 + (p & 3)];  // M_j = -c_j
        const double aj = __builtin_fabs(mj);
        asum += aj;
        msum += mj;
        kall += aj + mj;
        if (p >= 4 * kb) {
          rf += mj + 0x1p-17 * aj;
        } else {
          kk += aj + mj;
          if (screen) cvis += (double)dC[(meta[p >> 2].x << 2) + (p & 3)];
        }
        if (screen && kb == G + 1) {
          const double av = (double)dA[p];
          a2 += av * av;
          amax = av > amax ? av : amax;
        }
      }
      const double marg = 0x1p-20 * (__builtin_fabs(rf) + asum) + 0x1p-126;
      const double sl = 0x1p-14 * (__builtin_fabs(msum) + asum + kall) + 0x1p-126;
      if (kb <= G) {
        const float bk = screen ? round_up_f32(msum + cvis * (1.0 + 0x1p-20) + sl)
                                : round_up_f32(rf + 0x1p-14 * kk + marg);
        if (kb >= 1) meta[kb - 1].y = (int)f2u(bk);
        if (kb == G) lowc = round_up_f32(0x1p-14 * kk + marg);
      } else if (screen) {
        scr_a = round_dn_f32(msum - sl - 1.01 * a2 * (1.0 + 0x1p-11));
        scr_pq = round_up_f32(2.01 * amax * __builtin_sqrt((double)D) * (1.0 + 0x1p-11));
      }
      if (kb == 0) {
        uint32_t t0 = ord_f32(-__builtin_inff());
        if (inter) {  // an actual row's exact value: no larger than the block's best
          const unsigned long long kv =
              __hip_atomic_load(&keys[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((uint32_t)(kv >> 32) > kArgmaxClampOrd) t0 = (uint32_t)(kv >> 32);
        }
        tau_ord = t0;
#ifdef CWQ_PRUNE_STATS
        if (g_seed_tau && g < kDbgBlocks && (g_dbg_best[g] >> 32) > kArgmaxClampOrd)
          tau_ord = (uint32_t)(g_dbg_best[g] >> 32);
#endif
        sq_cnt = 0u;
      }
    }
    __syncthreads();
    const float lc = lowc;
#ifdef CWQ_PRUNE_STATS
    const float tau_seed = unord_f32(tau_ord);
#endif
    const float sA = scr_a, sPq = scr_pq;

    // this wave's contiguous share of the tile's candidates
    const int64_t per_wave = (n1 - n0 + 3) / 4;
    const int64_t w0 = n0 + (int64_t)wv * per_wave;
    // candidate indices stay below 2^32 in this kernel (launch_prune_t):
    // 32-bit counters (a 64-bit add and compare cost two VALU slots each)
    const uint32_t w1 = (uint32_t)((w0 + per_wave < n1) ? w0 + per_wave : n1);
    uint32_t wnext = (uint32_t)w0 + 64u;
    uint32_t n = (uint32_t)w0 + lane;
    int k = 0;
    float s = 0.0f;
#ifndef CWQ_TAU_FROM_KEYS
#define CWQ_TAU_FROM_KEYS 1  // INTER: start the lanes' tau at keys[g]'s value, not at the first share
#endif
    float tau = (INTER && CWQ_TAU_FROM_KEYS) ? unord_f32(tau_ord) : -__builtin_inff();
#ifdef CWQ_PRUNE_STATS
    tau = tau_seed;
#endif
    uint64_t bestk = 0;
    uint32_t iter = 0;

    const PhiloxLo lok = philox_lo_key(st);  // block indices < 2^32 (launch_prune_t)
    auto pass = [&](auto screen_tag) {
      constexpr bool SCREEN = decltype(screen_tag)::value;
      for (;;) {
        // a lane is active while its row index is in the wave's range (a
        // compare each iteration, not a flag carried in a VGPR)
        const bool active = n < w1;
        if (__ballot(active) == 0ull) break;
        const int2 mt = meta[k];
        const uint32_t grp = (uint32_t)n * (uint32_t)G + (uint32_t)mt.x;
        const U4 x = philox10_lo(grp, lok, st.k0, st.k1);
        float z0, z1, z2, z3;
        float upper;
        if constexpr (SCREEN) {
          box_muller_screen(x.x, x.y, z0, z1);
          box_muller_screen(x.z, x.w, z2, z3);
          const float4* cq = scst + k * NS;
          const float4 sa = cq[0], sb = cq[1];
          const float a0 = __builtin_fmaf(sa.x, z0, sb.x);
          const float a1 = __builtin_fmaf(sa.y, z1, sb.y);
          const float a2 = __builtin_fmaf(sa.z, z2, sb.z);
          const float a3 = __builtin_fmaf(sa.w, z3, sb.w);
          s = __builtin_fmaf(-a0, a0, s);
          s = __builtin_fmaf(-a1, a1, s);
          s = __builtin_fmaf(-a2, a2, s);
          s = __builtin_fmaf(-a3, a3, s);
          upper = __builtin_fmaf(s, kScreenC1, u2f((uint32_t)mt.y));
        } else {
          box_muller_dev(x.x, x.y, logtab, z0, z1);
          box_muller_dev(x.z, x.w, logtab, z2, z3);
          const float4* cq = cst + k * NF;
          const float4 ls = cq[0], ss = cq[1], mu = cq[2], sg = cq[3], cc = cq[4], ry = cq[5];
          const float4 bb = STEP0 ? float4{0.f, 0.f, 0.f, 0.f} : cq[6];
          const float d0 = cand_diff<STEP0>(z0, ls.x, ss.x, mu.x, bb.x);
          const float d1 = cand_diff<STEP0>(z1, ls.y, ss.y, mu.y, bb.y);
          const float d2 = cand_diff<STEP0>(z2, ls.z, ss.z, mu.z, bb.z);
          const float d3 = cand_diff<STEP0>(z3, ls.w, ss.w, mu.w, bb.w);
          // fast correctly rounded quotients; lanes whose operands leave the
          // Markstein ranges (never, for sane inputs) redo them with IEEE division
          // inside a wave-uniform branch, so the common path issues no fallback.
          float y0 = div_rn_markstein(d0, sg.x, ry.x);
          float y1 = div_rn_markstein(d1, sg.y, ry.y);
          float y2 = div_rn_markstein(d2, sg.z, ry.z);
          float y3 = div_rn_markstein(d3, sg.w, ry.w);
          const bool ok = fastdiv & markstein_ok4(d0, d1, d2, d3);
          if (__builtin_expect(__ballot(!ok) != 0ull, 0)) {
            if (!ok) {
              y0 = d0 / sg.x;
              y1 = d1 / sg.y;
              y2 = d2 / sg.z;
              y3 = d3 / sg.w;
            }
          }
          s = s + lp_from_z(y0, cc.x);
          s = s + lp_from_z(y1, cc.y);
          s = s + lp_from_z(y2, cc.z);
          s = s + lp_from_z(y3, cc.w);
          upper = (s + __builtin_fabsf(s) * kPruneC1) + u2f((uint32_t)mt.y);
        }
        k += 1;
        const bool complete = (k == G);
        const bool below = upper < tau;
#ifdef CWQ_PRUNE_STATS
        const bool prune = !complete && below;
#endif
        const bool done = complete || below || !active;
        // the finished lanes' mask from the compares' own masks (SALU): a
        // ballot of the combined flag costs a v_cndmask + v_cmp to rebuild it
        const uint64_t m = __ballot(complete) | __ballot(below) |
                           (__builtin_amdgcn_read_exec() & ~__ballot(active));
        if (complete && active && upper >= tau) {  // may be the best: keep it
          float lower;
          if constexpr (SCREEN)
            lower = __builtin_fmaf(s, kScreenC2, sA) - sPq * __builtin_amdgcn_sqrtf(-s);  // ~1 ulp: inside Pq's 0.4% slack
          else
            lower = (s - __builtin_fabsf(s) * kPruneC1) - lc;
          tau = fmaxf(tau, lower);
          const uint32_t slot = atomicAdd(&sq_cnt, 1u);
          if (slot < CWQ_SURVIVOR_CAP) {
            sq_n[slot] = (uint32_t)n;
            sq_ub[slot] = upper;
          } else {  // list full (near-ties everywhere): evaluate exactly now
#ifdef CWQ_PRUNE_STATS
            atomicAdd(&g_prune_stats[69], 1ull);
#endif
            const float v = eval_row<D, STEP0>(st, (uint64_t)n * D, D, 0, loc_s + off,
                                               scale_s + off, t_loc + off, t_scale + off,
                                               lognorm + off, STEP0 ? nullptr : best + off, logtab);
            const uint64_t kv = argmax_key(v, (uint32_t)n);
            bestk = kv > bestk ? kv : bestk;
          }
        }
#ifdef CWQ_PRUNE_STATS
        if (active && (complete || prune)) atomicAdd(&s_ps[k], 1u);
        if (active && complete) atomicAdd(&s_ps[65], 1u);
        if (active && complete && upper >= tau) atomicAdd(&s_ps[66], 1u);
#endif
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (done) {
          n = wnext + rank;
          k = 0;
          s = 0.0f;
        }
        wnext += (uint32_t)__builtin_popcountll(m);
        if (((++iter) & CWQ_TAU_SHARE_MASK) == 0u) {  // share tau across the workgroup's waves
          const float tm = wave_max_f32(tau);
          if (lane == 0) atomicMax(&tau_ord, ord_f32(tm));
          tau = fmaxf(tau, unord_f32(__atomic_load_n(&tau_ord, __ATOMIC_RELAXED)));
        }
      }
    };
#ifdef CWQ_PRUNE_STATS
    if (screen && tid == 0) atomicAdd(&g_prune_stats[67], 1ull);
#endif
    if (screen)
      pass(std::true_type{});
    else
      pass(std::false_type{});

    // exact evaluation of the survivors that can still reach the final tau
    {
      const float tm = wave_max_f32(tau);
      if (lane == 0) atomicMax(&tau_ord, ord_f32(tm));
    }
    __syncthreads();
    const float tau_final = unord_f32(tau_ord);
    const uint32_t nsurv = sq_cnt < CWQ_SURVIVOR_CAP ? sq_cnt : CWQ_SURVIVOR_CAP;
    for (uint32_t i = tid; i < nsurv; i += blockDim.x) {
      if (sq_ub[i] >= tau_final) {
#ifdef CWQ_PRUNE_STATS
        atomicAdd(&g_prune_stats[68], 1ull);
#endif
        const uint32_t nn = sq_n[i];
        const float v = eval_row<D, STEP0>(st, (uint64_t)nn * D, D, 0, loc_s + off,
                                           scale_s + off, t_loc + off, t_scale + off,
                                           lognorm + off, STEP0 ? nullptr : best + off, logtab);
        const uint64_t kv = argmax_key(v, nn);
        bestk = kv > bestk ? kv : bestk;
      }
    }

    bestk = wave_max_u64(bestk);
    if (lane == 0) wkey[wv] = bestk;
    __syncthreads();
    if (tid == 0) {
      uint64_t mk = wkey[0];
      for (int i = 1; i < 4; ++i) mk = wkey[i] > mk ? wkey[i] : mk;
      if (mk) atomicMax(&keys[g], (unsigned long long)mk);
#ifdef CWQ_PRUNE_STATS
      if (!g_seed_tau && g < kDbgBlocks) g_dbg_best[g] = mk;
#endif
#ifdef CWQ_TILE_TIMES
      if (tile < kTileTimes) g_tile_t1[tile] = __builtin_amdgcn_s_memrealtime();
#endif
    }
#ifdef CWQ_PRUNE_STATS
    if (tid < 72) {
      if (s_ps[tid]) atomicAdd(&g_prune_stats[tid], (unsigned long long)s_ps[tid]);
      s_ps[tid] = 0u;
    }
#endif
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// General pruned encoder: any block dimension, CSR or uniform (the greedy
// coder's ragged groups, coded_greedy_sampler.py:207-284).  Same screening
// bound as k_encode_prune (DESIGN.md "screening bound"), with three changes:
//   * dims are visited in natural order (a candidate row starts at any word of
//     a Philox block: each lane walks its row one Philox block at a time);
//   * the per-dim constants live in global memory, computed once per step by
//     k_csr_prep (one workgroup per block), with the float-summation factors
//     of the bound scaled for the block's d (gamma_d = 1.01 (d+1) 2^-24);
//   * tiles of one block share their threshold through gtau[g].
// Blocks whose constants fail the gate are scored exactly.
// ---------------------------------------------------------------------------
struct CsrDim {
  float sa, sb;     // a = RN(sa z' + sb), z' = screening z / sqrt(2 ln 2)
  float A, C;       // additive error (a units) and C_j of the bound
  double M;         // M_j = -c_j
  bool ok;
};

template <bool STEP0>
__device__ __forceinline__ CsrDim csr_dim(float ls, float ss, float mu, float sg, float c,
                                          float bb) {
  CsrDim o;
  const double ssa = __builtin_fabs((double)ss), lsa = __builtin_fabs((double)ls);
  const double mua = __builtin_fabs((double)mu);
  const double bba = STEP0 ? 0.0 : __builtin_fabs((double)bb);
  const double zs = kScreenZm * ssa;
  const double mag = bba + lsa + zs + mua;
  const double rho = 0x1p-24 * 1.0001 * (zs + (lsa + zs) + (STEP0 ? 0.0 : bba + lsa + zs) + mag);
  const double offd = (STEP0 ? 0.0 : (double)bb) + (double)ls - (double)mu;
  const double sig = (double)sg;
  const double kq = kScreenKappa / sig;
  o.sa = (float)((double)ss * kq * kSqrt2Ln2);
  o.sb = (float)(offd * kq);
  const double a0 = (kq * (rho + ssa * kScreenEz) +
                     kq * 0x1p-24 * 1.0001 * (zs + __builtin_fabs(offd))) * (1.0 + 0x1p-20) +
                    0x1p-140;
  o.A = round_up_f32(a0 * 1.0001);
  o.C = round_up_f32((1.0 / kScreenEps - 1.0) * a0 * a0 / kScreenPhi * (1.0 + 0x1p-20));
  o.M = -(double)c;
  o.ok = markstein_ok_den(sg) && mag <= 0x1p100 && mag / sig <= 0x1p50 && o.C <= 0x1p60f &&
         o.sa - o.sa == 0.0f && o.sb - o.sb == 0.0f && c - c == 0.0f;
  return o;
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// Visit order.  A row starting at flat normal k0 = n*d has alignment class
// c = k0 & 3; its Philox blocks ("units") u = 0..U_c-1, U_c = (d + c + 3) / 4,
// hold dims 4u - c + t (t = word 0..3, kept if 0 <= dim < d).  Per block and
// class, k_csr_prep sorts the units by expected a^2 (most informative first,
// so rows cross tau early) and stores for visit position k the unit ord[k] and
// the drop bound bpre[k] (units visited before position k).  Region of block g:
// off + 12 g, class c at c * csr_cls_stride(d), csr_cls_stride(d) =
// (d + 6) / 4 + 1 >= U_c + 1; 4 strides <= d + 10 entries.
__host__ __device__ __forceinline__ int64_t csr_cls_stride(int64_t d) { return (d + 6) / 4 + 1; }
constexpr int64_t kCsrSortUnits = 2048;  // sorted if U_3 <= this (d <= 8189); else natural order

// Per block: the per-dim constants and sums, then for each alignment class
// its sorted visit order and drop bounds.  Each dim's constants are computed
// once (double arithmetic) into sab (sA, sB) and cdim (C_j) in global memory,
// where the class passes read them back; the prep workgroup keeps a small LDS
// footprint, so it can start on a CU that the other streams' scoring kernels
// occupy.  With few blocks the four classes go to four workgroups
// (blockIdx.y), each computing the block's constants and sums (identical
// values, so their stores to sab / cdim agree), so the sorts run side by
// side; the blockIdx.y == 0 workgroup also writes sab's zero pads and the
// block's gate constants.  Sums and the drop-bound prefix sums are wave
// reductions / scans (a few barriers per block); classes of <= 256 units are
// ordered by a rank sort (one barrier), longer ones by a bitonic sort.
// Blocks longer than lds_dims (whose constants the scoring kernel reads from
// global memory, not LDS) also get abp: for visit position k of class c the
// (sa, sb) of unit ord[k]'s four words in one 32-byte record, so the scoring
// lanes of a slot read consecutive records instead of gathering.
template <bool STEP0>
__global__ void __launch_bounds__(256) k_csr_prep(
    const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ loc_s, const float* __restrict__ scale_s,
    const float* __restrict__ lognorm, const float* __restrict__ best,
    const int64_t* __restrict__ block_off, int64_t ud, int64_t nb, float2* __restrict__ sab,
    float* __restrict__ cdim, float* __restrict__ bpre, uint32_t* __restrict__ ordu,
    float4* __restrict__ grp, uint32_t* __restrict__ gtau, float4* __restrict__ abp,
    int64_t lds_dims, int64_t coop_min_d) {
  __shared__ double red[5][4];
  __shared__ double wscan[4];
  __shared__ double ucs[256];  // classes of <= 256 units: unit u's C sum
  __shared__ unsigned long long skey[kCsrSortUnits];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  // gridDim.y == 4: one class per workgroup (few blocks: the four sorts run
  // side by side); gridDim.y == 1: one workgroup walks all four classes (many
  // blocks: the per-dim constants are computed once per block, not per class)
  const bool lead = blockIdx.y == 0;  // writes the block's class-independent outputs
  for (int64_t g = blockIdx.x; g < nb; g += gridDim.x) {
    const BlockSpan sp = block_span(block_off, ud, g);
    const int64_t off = sp.off, d = sp.d;
    double sm = 0.0, sa = 0.0, sk = 0.0, s2 = 0.0, mx = 0.0;
    int ok = 1;
    float2* sabg = sab + off + 8 * g + 4;  // 4 zero pads either side (partial units)
    float* cg = cdim + off;
    if (lead && tid < 8) {  // 8 trailing zeros: the last 4 are the next block's
      if (tid < 4) sabg[tid - 4] = float2{0.f, 0.f};  // leading pads (or the slack
      sabg[d + tid] = float2{0.f, 0.f};               // past the last block)
    }
    for (int64_t j = tid; j < d; j += 256) {
      const CsrDim o =
          csr_dim<STEP0>(loc_s[off + j], scale_s[off + j], t_loc[off + j], t_scale[off + j],
                         lognorm[off + j], STEP0 ? 0.0f : best[off + j]);
      sabg[j] = float2{o.sa, o.sb};
      cg[j] = o.C;
      sm += o.M;
      sa += __builtin_fabs(o.M);
      sk += __builtin_fabs(o.M) + o.M;
      s2 += (double)o.A * (double)o.A;
      mx = (double)o.A > mx ? (double)o.A : mx;
      ok &= o.ok ? 1 : 0;
    }
    sm = wave_sum_f64(sm);
    sa = wave_sum_f64(sa);
    sk = wave_sum_f64(sk);
    s2 = wave_sum_f64(s2);
    mx = wave_max_f64(mx);
    if (lane == 0) {
      red[0][wv] = sm;
      red[1][wv] = sa;
      red[2][wv] = sk;
      red[3][wv] = s2;
      red[4][wv] = mx;
    }
    // the sab / cdim stores are read back below by other threads: wait for
    // them to complete (they write through to L2) and read them with
    // agent-scope loads, which bypass the CU's L1 (a line another block's
    // workgroup on this CU filled earlier may hold this block's previous-step
    // values at its edges)
    __threadfence_block();
    const bool all_ok = __syncthreads_and(ok) != 0;
    const double SM = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    const double SA = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    const double SK = ((red[2][0] + red[2][1]) + red[2][2]) + red[2][3];
    const double S2 = ((red[3][0] + red[3][1]) + red[3][2]) + red[3][3];
    double MX = red[4][0];
    for (int w = 1; w < 4; ++w) MX = red[4][w] > MX ? red[4][w] : MX;
    // Float summation error of depth h: gamma_h = 1.01 (h + 1) 2^-24 bounds
    // |fl(sum) - sum| / sum|x| for any summation tree in which every term
    // passes through at most h roundings.  Two sums of d terms enter the
    // bound: the screening sum s (sequential over the row: h = d; cooperative
    // rows: 4 in-lane + 4 butterfly + one per 16-unit chunk, <= 16 + d/64) and
    // the exact Eigen-order row value (8 strided accumulators, predux, tail:
    // <= d/8 + 8).  gamma is taken at the larger depth.  The additive margin
    // 2^-20 covers the float rounding of B_k and of the tests' fma (u |B_k|)
    // and the double roundings of the sums here; u |s| is covered by the
    // 2^-22 / 2^-14 terms of c1 / c2.
    const bool coop_blk = d >= coop_min_d;
    const double h_s = coop_blk ? 16.0 + (double)d / 64.0 : (double)d;
    const double h_e = (double)d / 8.0 + 8.0;
    const double gam = 1.01 * ((h_s > h_e ? h_s : h_e) + 1.0) * 0x1p-24;
    const double sl = (3.0 * gam + 0x1p-20) * (__builtin_fabs(SM) + SA + SK) + 0x1p-126;
    const int64_t reg = off + 12 * g, cs = csr_cls_stride(d);
    const bool recs = abp != nullptr && d > lds_dims;
    auto sab_at = [&](int64_t j) {
      const unsigned long long v = __hip_atomic_load(
          reinterpret_cast<unsigned long long*>(sabg + j), __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_AGENT);
      return float2{u2f((uint32_t)v), u2f((uint32_t)(v >> 32))};
    };
    for (int c = (int)blockIdx.y; c < 4; c += (int)gridDim.y) {
      // word t of unit u of class c is dim 4u - c + t (absent outside [0, d));
      // unit u: its sum of C_j and its expected sum of a_j^2 - C_j
      auto unit = [&](int64_t u, double& csum, double& gain) {
        csum = 0.0;
        gain = 0.0;
        for (int t = 0; t < 4; ++t) {
          const int64_t j = 4 * u - c + t;
          if (j >= 0 && j < d) {
            const float2 ab = sab_at(j);
            const float xc = u2f(__hip_atomic_load(reinterpret_cast<uint32_t*>(cg + j),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            csum += (double)xc;
            gain += (double)ab.x * (double)ab.x * (0.5 / 0.6931471805599453) +
                    (double)ab.y * (double)ab.y - (double)xc;
          }
        }
      };
      auto key_of = [&](int64_t u) {
        double cu, gu;
        unit(u, cu, gu);
        const float gf = (float)(gu > 0.0 ? gu : 0.0);
        return ((unsigned long long)ord_f32(gf) << 32) | (0xffffffffull - (uint64_t)u);
      };
      const int64_t U = (d + c + 3) / 4;
      const bool sorted = all_ok && U <= kCsrSortUnits;
      const bool small = U <= 256;  // one unit per thread: its C sum kept in LDS
      if (sorted && small) {  // rank sort of (gain desc, u asc) keys: keys are distinct
        unsigned long long key = 0ull;
        if (tid < U) {
          double cu, gu;
          unit(tid, cu, gu);
          ucs[tid] = cu;
          const float gf = (float)(gu > 0.0 ? gu : 0.0);
          key = ((unsigned long long)ord_f32(gf) << 32) | (0xffffffffull - (uint64_t)tid);
          skey[tid] = key;
        }
        __syncthreads();
        int r = 0;
        if (tid < U)
          for (int i = 0; i < (int)U; ++i) r += skey[i] > key ? 1 : 0;
        __syncthreads();
        if (tid < U) skey[r] = key;
        __syncthreads();
      } else if (sorted) {  // bitonic sort of (gain desc, u asc) keys
        int64_t P = 1;
        while (P < U) P <<= 1;
        for (int64_t u = tid; u < P; u += 256) skey[u] = u < U ? key_of(u) : 0ull;
        __syncthreads();
        for (int64_t k = 2; k <= P; k <<= 1) {
          for (int64_t jj = k >> 1; jj > 0; jj >>= 1) {
            for (int64_t i = tid; i < P; i += 256) {
              const int64_t l = i ^ jj;
              if (l > i) {
                const unsigned long long x = skey[i], y = skey[l];
                const bool desc = (i & k) == 0;  // overall descending
                if (desc ? (x < y) : (x > y)) {
                  skey[i] = y;
                  skey[l] = x;
                }
              }
            }
            __syncthreads();
          }
        }
      }
      // drop bounds along the visit order, positions k = 0..U
      double carry = 0.0;
      for (int64_t base = 0; base <= U; base += 256) {
        const int64_t k = base + tid;
        int64_t u = k;
        if (sorted && k < U) u = (int64_t)(0xffffffffull - (skey[k] & 0xffffffffull));
        double cu = 0.0, gu;
        if (all_ok && k < U) {
          if (sorted && small)
            cu = ucs[u];
          else
            unit(u, cu, gu);
        }
        if (recs && k <= U) {  // the unit's four (sa, sb), zero for absent words
          float e[8];          // (position U: the zero record of the pad unit)
          for (int t = 0; t < 4; ++t) {
            const int64_t j = 4 * u - c + t;
            float2 ab = float2{0.f, 0.f};
            if (k < U && j >= 0 && j < d) ab = sab_at(j);
            e[2 * t] = ab.x;
            e[2 * t + 1] = ab.y;
          }
          float4* rr = abp + 2 * (csr_rec_base(off) + c * cs + k);
          rr[0] = float4{e[0], e[1], e[2], e[3]};
          rr[1] = float4{e[4], e[5], e[6], e[7]};
        }
        double v = cu;  // inclusive scan: in the wave, then across the four waves
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const double t = __shfl_up(v, (unsigned)o, 64);
          if (lane >= o) v += t;
        }
        if (lane == 63) wscan[wv] = v;
        __syncthreads();
        double pre = 0.0;
        for (int w = 0; w < wv; ++w) pre += wscan[w];
        const double total = ((wscan[0] + wscan[1]) + wscan[2]) + wscan[3];
        const double excl = carry + (pre + v) - cu;
        if (k <= U) {
          bpre[reg + c * cs + k] = round_up_f32(SM + excl * (1.0 + 0x1p-20) + sl);
          // position U: the pad unit U, whose words all fall on zero constants
          // (sab's and the scoring kernel's LDS pads), so a unit read past a
          // row's end scores exactly 0 without a mask
          ordu[reg + c * cs + k] = (uint32_t)(k < U ? u : U);
        }
        carry += total;
        __syncthreads();
      }
    }
    if (lead && tid == 0) {
      const float c1 = round_dn_f32(1.0 - 3.0 * gam - 0x1p-22);
      const float c2 = round_up_f32(1.0 + 3.0 * gam + 0x1p-14);
      const float as = round_dn_f32(SM - sl - 1.01 * S2 * (1.0 + 0x1p-11));
      const float pq = round_up_f32(2.01 * MX * __builtin_sqrt((double)(d > 0 ? d : 1)) *
                                    (1.0 + 0x1p-11));
      const bool fin = as - as == 0.0f && pq - pq == 0.0f;
      grp[g] = (all_ok && fin && d > 0) ? float4{c1, c2, as, pq} : float4{0.f, 0.f, 0.f, 0.f};
      gtau[g * CWQ_CSR_GTAU_STRIDE] = ord_f32(-__builtin_inff());
    }
    __syncthreads();
  }
}

// One candidate row evaluated exactly by a whole wave (the survivors of the
// general pruned kernel; d is large there, so one lane per row would leave the
// other 63 idle for a full row).  Lanes compute the terms of up to 63 Philox
// blocks per 248-dim chunk into LDS; lanes 0-7 then fold them into the eight
// Eigen accumulators and lane 8 into the tail, in exactly eval_row_f's order.
// Every lane returns the row value.
constexpr int kRowChunk = 248;  // multiple of 8; spans <= 63 Philox blocks

template <bool STEP0>
__device__ __forceinline__ float exact_row_wave(
    const PhiloxStream& st, uint64_t kbase, int64_t d, const float* __restrict__ loc_s,
    const float* __restrict__ scale_s, const float* __restrict__ mu,
    const float* __restrict__ sg, const float* __restrict__ lognorm,
    const float* __restrict__ best, const double* logtab, float* buf, uint32_t lane) {
  const int64_t vec = d & ~(int64_t)7;
  float acc = 0.0f;  // lane l < 8: p[l]; lane 8: the tail sum
  for (int64_t j0 = 0; j0 < d; j0 += kRowChunk) {
    const int64_t cnt = (d - j0) < kRowChunk ? d - j0 : kRowChunk;
    const uint64_t k0 = kbase + (uint64_t)j0;
    const uint64_t blk = (k0 >> 2) + lane;
    const int64_t ef = (int64_t)(blk << 2) - (int64_t)k0;  // chunk index of the block's word 0
    if (ef < cnt) {
      const F4 z = normal4_dev(st, blk, logtab);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int64_t e = ef + t;
        if (e >= 0 && e < cnt) {
          const int64_t j = j0 + e;
          const float zz = t == 0 ? z.a : (t == 1 ? z.b : (t == 2 ? z.c : z.d));
          float v = scale_s[j] * zz;  // misc.py:14
          v = loc_s[j] + v;           // misc.py:15
          const float tv = STEP0 ? v : best[j] + v;
          buf[e] = log_prob(tv, mu[j], sg[j], lognorm[j]);
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane < 8) {
      for (int64_t e = lane; e < cnt && j0 + e < vec; e += 8) acc = acc + buf[e];
    } else if (lane == 8) {
      for (int64_t e = (vec > j0 ? vec - j0 : 0); e < cnt; ++e) acc = acc + buf[e];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  float p[8];
#pragma unroll
  for (int l = 0; l < 8; ++l) p[l] = __shfl(acc, l, 64);
  const float t = __shfl(acc, 8, 64);
  const float q0 = p[0] + p[4], q1 = p[1] + p[5], q2 = p[2] + p[6], q3 = p[3] + p[7];
  return t + ((q0 + q2) + (q1 + q3));
}

#ifndef CWQ_CSR_GTAU_SHARE
#define CWQ_CSR_GTAU_SHARE 1  // 1: also share tau with the block's other tiles in the loop
#endif
#ifndef CWQ_CSR_GTAU_MASK
#define CWQ_CSR_GTAU_MASK 63u  // ... every CWQ_CSR_GTAU_MASK + 1 iterations
#endif
#ifndef CWQ_CSR_SURVIVOR_CAP
#define CWQ_CSR_SURVIVOR_CAP 512
#endif
#ifndef CWQ_CSR_COOP_ROWS_PER_LANE
#define CWQ_CSR_COOP_ROWS_PER_LANE 8  // cooperative rows below this many rows per lane ...
#endif
#ifndef CWQ_CSR_TILE
#define CWQ_CSR_TILE 1024             // smallest tile (candidates), per-lane rows
#endif
#ifndef CWQ_CSR_TILES
#define CWQ_CSR_TILES 8192            // tiles a launch aims for
#endif
#ifndef CWQ_CSR_COOP_TILE
#define CWQ_CSR_COOP_TILE 128         // smallest tile (candidates) in cooperative launches
#endif
#ifndef CWQ_CSR_COOP_TILES
#define CWQ_CSR_COOP_TILES 6144       // tiles a cooperative launch aims for (4 x 1536 slots)
#endif
#ifndef CWQ_CSR_COOP_CLASS_WAVES
#define CWQ_CSR_COOP_CLASS_WAVES 1    // 1: cooperative rows n = wave (mod 4) per wave
#endif
#ifndef CWQ_CSR_COOP_MIN_D
#define CWQ_CSR_COOP_MIN_D 256        // ... for blocks of at least this many dims
#endif
#ifndef CWQ_CSR_COOP_MIN_WAVES
#define CWQ_CSR_COOP_MIN_WAVES 4      // waves/SIMD the cooperative kernel's registers allow
#endif
#ifndef CWQ_CSR_RUN_MIN_WAVES
#define CWQ_CSR_RUN_MIN_WAVES 6       // waves/SIMD the per-lane kernel's registers allow
#endif
#ifndef CWQ_RUN_UPL
#define CWQ_RUN_UPL 2                 // units per lane per iteration of a per-lane row
#endif
#ifndef CWQ_COOP_UPL
#define CWQ_COOP_UPL 4                // units per lane per iteration of a cooperative row
#endif
#ifndef CWQ_COOP_CLASS_TILES
#define CWQ_COOP_CLASS_TILES 1        // 1: cooperative tiles hold one alignment class (rows n = R mod 4)
#endif
#ifndef CWQ_COOP_LOAD_ORDER
#define CWQ_COOP_LOAD_ORDER 0         // 1: a cooperative iteration's loads issued in unit order
#endif

// element idx of base through an unsigned 32-bit byte offset (base + voffset)
template <class T>
__device__ __forceinline__ T ld_u32off(const T* base, uint32_t idx) {
  return *(const T*)((const char*)base + (uint64_t)(idx * (uint32_t)sizeof(T)));
}

static_assert(CWQ_CSR_COOP_MIN_D <= CWQ_CSR_LDS_DIMS, "short rows of a cooperative launch use LDS");

// COOP: the kernel of cooperative launches (few long rows; blocks of at least
// coop_min_d dims walked by 16-lane slots, shorter ones per lane from LDS);
// otherwise one row per lane for every block.
template <bool STEP0, bool COOP>
__global__ void __launch_bounds__(256, COOP ? CWQ_CSR_COOP_MIN_WAVES : CWQ_CSR_RUN_MIN_WAVES) k_encode_prune_csr(
    const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ loc_s, const float* __restrict__ scale_s,
    const float* __restrict__ lognorm, const float* __restrict__ best,
    const int64_t* __restrict__ block_off, int64_t ud, int64_t ntiles, int64_t tiles_per_block,
    int64_t cand_per_tile, int64_t n_cand, SeedSpec sd, int32_t step,
    const float2* __restrict__ sab, const float* __restrict__ bpre,
    const uint32_t* __restrict__ ordu, const float4* __restrict__ grp,
    uint32_t* __restrict__ gtau, unsigned long long* __restrict__ keys, int64_t coop_min_d,
    const float4* __restrict__ abp) {
  __shared__ double logtab[32];
  __shared__ uint32_t tau_ord;
  __shared__ uint32_t sq_cnt;
  __shared__ uint32_t sq_n[CWQ_CSR_SURVIVOR_CAP];
  __shared__ float sq_ub[CWQ_CSR_SURVIVOR_CAP];
  __shared__ unsigned long long wkey[4];
  // One LDS region, two uses that never overlap in time: a short block's
  // natural-order constants, drop bounds and visit order (l_ab, l_bp, l_ord),
  // and the survivors' exact-row buffers (rowbuf, after the loops).
  constexpr int kNatF4 = (CWQ_CSR_LDS_DIMS + 12) * 2 / 4;   // l_ab in float4s
  constexpr int kIdxF4 = (CWQ_CSR_LDS_DIMS + 12) / 4;       // l_bp, l_ord
  static_assert((CWQ_CSR_LDS_DIMS + 12) % 4 == 0, "LDS sub-arrays in whole float4s");
  constexpr int kUnionF4 = kNatF4 + 2 * kIdxF4;
  static_assert(kUnionF4 * 4 >= 4 * kRowChunk, "rowbuf fits the region");
  __shared__ float4 l_u[kUnionF4];
  float2* const l_ab = reinterpret_cast<float2*>(l_u);
  float* const l_bp = reinterpret_cast<float*>(l_u + kNatF4);
  uint32_t* const l_ord = reinterpret_cast<uint32_t*>(l_u + kNatF4 + kIdxF4);
  float(*const rowbuf)[kRowChunk] = reinterpret_cast<float(*)[kRowChunk]>(l_u);
  fill_logtab(logtab);
  const uint32_t wv = wave_id();
  const uint32_t lane = threadIdx.x & 63u;

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    // tile-major order: a block's later tiles start after its first ones have
    // published their threshold in gtau (the loop shares tau inside the
    // workgroup only: per-iteration global atomics cost more than they prune)
    const int64_t nbk = ntiles / tiles_per_block;
    const int64_t tt = tile / nbk;
    const int64_t g = tile - tt * nbk;
    const BlockSpan sp = block_span(block_off, ud, g);
    const int64_t off = sp.off, d = sp.d;
    // the tile's rows: n0 + rstep m, m < nrt
    int64_t n0, nrt;
    uint32_t rlog = 0;  // log2 rstep
#if CWQ_COOP_CLASS_TILES && CWQ_CSR_COOP_CLASS_WAVES
    if (COOP && d >= coop_min_d && (tiles_per_block & 3) == 0) {
      // one alignment class per workgroup: tile tt takes the rows n = R (mod 4)
      // of chunk J (4 tiles' worth of candidates), R = tt mod 4, J = tt / 4, so
      // its four waves read one class's visit-order records, not four
      const int64_t J = tt >> 2, C4 = 4 * cand_per_tile;
      const int64_t lim = (J + 1) * C4 < n_cand ? (J + 1) * C4 : n_cand;
      n0 = J * C4 + (tt & 3);
      nrt = lim > n0 ? (lim - n0 + 3) / 4 : 0;
      rlog = 2;
    } else
#endif
    {
      n0 = tt * cand_per_tile;
      nrt = ((n0 + cand_per_tile < n_cand) ? n0 + cand_per_tile : n_cand) - n0;
    }
    if (nrt <= 0) continue;  // empty tile
    const int64_t n1 = n0 + nrt;  // contiguous tiles (rlog == 0): the rows' end
    const PhiloxStream st =
        generate_key(step_seed(sd.of(g), step), 42);
    const float4 gc = grp[g];
    const bool in_lds = d <= CWQ_CSR_LDS_DIMS;
    const int64_t reg = off + 12 * g, cs = csr_cls_stride(d);
    if (gc.x != 0.0f && in_lds) {
      // 4 zero pads before, 8 after (the pad unit U's words reach d + 7 + 4)
      for (int64_t j = tid; j < d + 12; j += blockDim.x)
        l_ab[j] = j < d + 8 ? sab[off + 8 * g + j] : float2{0.f, 0.f};
      for (int64_t j = tid; j < 4 * cs; j += blockDim.x) {
        l_bp[j] = bpre[reg + j];
        l_ord[j] = ordu[reg + j];
      }
    }
    if (tid == 0) {
      tau_ord = __hip_atomic_load(&gtau[g * CWQ_CSR_GTAU_STRIDE], __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);  // earlier tiles of the block
      sq_cnt = 0u;
    }
    __syncthreads();
    uint64_t bestk = 0;
#ifdef CWQ_PRUNE_STATS
    if (tid == 0) atomicAdd(&g_prune_stats[gc.x != 0.0f ? 40 : 41], 1ull);
#endif
    bool exact_tile = gc.x == 0.0f;
    if (!exact_tile) {
      const int64_t per_wave = (n1 - n0 + 3) / 4;
      const int64_t w0 = n0 + (int64_t)wv * per_wave;
      const int64_t w1 = (w0 + per_wave < n1) ? w0 + per_wave : n1;
      // lane state: row n0 + r (class c, first Philox block rb, U units), visit
      // position k.  ab is the padded constant array: entry 4 + j for dim j,
      // zeros for the out-of-row words of a row's first and last unit.
      const uint32_t r0 = (uint32_t)(w0 - n0), r1 = (uint32_t)(w1 - n0);
      const int d32 = (int)d;
      // ab: natural-order (sa, sb) (LDS or global); rec (REC true): the
      // visit-order records of k_csr_prep's abp, read at the lane's position
      // Past-the-end positions read the pad unit's zero constants (LDS, sab or
      // records: k_csr_prep), so their units add exactly 0 without a mask.
      // HI0: every Philox block index of the launch is below 2^32 (counter
      // word 1 is 0, which makes round 2's first product lane-invariant).
      auto run = [&](const float2* ab, const float* bp, const uint32_t* od, const float4* rec,
                     auto REC, auto HI0T) __attribute__((always_inline)) {
        constexpr bool HI0 = decltype(HI0T)::value;
        [[maybe_unused]] const PhiloxLo lok = HI0 ? philox_lo_key(st) : PhiloxLo{};
        uint32_t wnext = r0 + 64u;
        uint32_t r = r0 + lane;
        bool active = r < r1;
        float s = 0.0f;
        float tau = unord_f32(tau_ord);
        uint32_t iter = 0;
        uint64_t rb;
        int c, U, cb;
        auto start_row = [&]() __attribute__((always_inline)) {
          const uint64_t k0 = (uint64_t)(n0 + (int64_t)r) * (uint64_t)d;
          rb = k0 >> 2;
          c = (int)(k0 & 3u);
          U = (d32 + c + 3) >> 2;
          cb = c * (int)cs;
        };
        start_row();
        int k = 0;
        // RUPL units per iteration (positions k .. k + RUPL - 1; a unit past
        // the row end adds exactly 0: its a is forced to 0).  The units of the
        // next positions are loaded one iteration ahead (the Philox counter
        // needs them first thing: a load at the top of the iteration would
        // expose its latency every time); a new row reloads.  Loads index
        // their uniform base with an unsigned 32-bit byte offset.
        constexpr int RUPL = COOP ? 1 : CWQ_RUN_UPL;  // the cooperative kernel: short rows only
        uint32_t u_nx[RUPL];
        auto load_units = [&](int p0) __attribute__((always_inline)) {
#pragma unroll
          for (int i = 0; i < RUPL; ++i) {
            const int pp = p0 + i;
            u_nx[i] = ld_u32off(od, (uint32_t)(cb + (pp < U ? pp : U)));
          }
        };
        load_units(0);
        while (__ballot(active) != 0ull) {
          uint32_t u[RUPL];
#pragma unroll
          for (int i = 0; i < RUPL; ++i) u[i] = u_nx[i];
          load_units(k + RUPL);
          // this iteration's constants and the next drop bound are loaded
          // here, ahead of the opaque key move below, so their latency
          // overlaps the Philox rounds (the compiler otherwise issues them
          // after the transcendentals and waits on them at once)
          float2 e[RUPL][4];
#pragma unroll
          for (int i = 0; i < RUPL; ++i) {
            const int pp = k + i;
            if constexpr (decltype(REC)::value) {
              const uint32_t pc = (uint32_t)(cb + (pp < U ? pp : U));
              const float4 ra = ld_u32off(rec, 2u * pc), rb2 = ld_u32off(rec, 2u * pc + 1u);
              e[i][0] = float2{ra.x, ra.y};
              e[i][1] = float2{ra.z, ra.w};
              e[i][2] = float2{rb2.x, rb2.y};
              e[i][3] = float2{rb2.z, rb2.w};
            } else {
              const uint32_t jp = (uint32_t)(4 * (int)u[i] - c + 4);
              e[i][0] = ld_u32off(ab, jp);  // padded index of word 0
              e[i][1] = ld_u32off(ab, jp + 1u);
              e[i][2] = ld_u32off(ab, jp + 2u);
              e[i][3] = ld_u32off(ab, jp + 3u);
            }
          }
          const int kn = (k + RUPL < U) ? k + RUPL : U;
          const float bnext = ld_u32off(bp, (uint32_t)(cb + kn));
          // round keys recomputed in SALU each iteration (opaque key): keeping
          // all 20 live costs SGPRs the loop then spills into VGPR lanes
          uint32_t kk0 = st.k0, kk1 = st.k1;
          asm volatile("" : "+s"(kk0), "+s"(kk1));
#pragma unroll
          for (int i = 0; i < RUPL; ++i) {
            const uint64_t blk = rb + u[i];
            const U4 x = HI0 ? philox10_lo((uint32_t)blk, lok, kk0, kk1)
                             : philox10_dev((uint32_t)blk, (uint32_t)(blk >> 32), st.c2, st.c3,
                                            kk0, kk1);
            F4 z;
            box_muller_screen(x.x, x.y, z.a, z.b);
            box_muller_screen(x.z, x.w, z.c, z.d);
            const float a0 = __builtin_fmaf(e[i][0].x, z.a, e[i][0].y);
            const float a1 = __builtin_fmaf(e[i][1].x, z.b, e[i][1].y);
            const float a2 = __builtin_fmaf(e[i][2].x, z.c, e[i][2].y);
            const float a3 = __builtin_fmaf(e[i][3].x, z.d, e[i][3].y);
            s = __builtin_fmaf(-a0, a0, s);
            s = __builtin_fmaf(-a1, a1, s);
            s = __builtin_fmaf(-a2, a2, s);
            s = __builtin_fmaf(-a3, a3, s);
#ifdef CWQ_PRUNE_STATS
            if (active && (i == 0 || k + i < U)) atomicAdd(&g_prune_stats[43], 1ull);
#endif
          }
          k = kn;
          const bool complete = k == U;
          const float upper = __builtin_fmaf(s, gc.x, bnext);
          const bool prune = !complete && (upper < tau);
          if (complete && active && upper >= tau) {  // may be the best: keep it
            const float lower =
                __builtin_fmaf(s, gc.y, gc.z) - gc.w * __builtin_amdgcn_sqrtf(-s);
            tau = fmaxf(tau, lower);
            const uint32_t slot = atomicAdd(&sq_cnt, 1u);
            if (slot < CWQ_CSR_SURVIVOR_CAP) {  // else: overflow, the tile is redone
              sq_n[slot] = r;
              sq_ub[slot] = upper;
            }
          }
          const bool done = complete || prune || !active;
#ifdef CWQ_PRUNE_STATS
          if (active && (complete || prune)) atomicAdd(&g_prune_stats[42], 1ull);
          if (active && complete) atomicAdd(&g_prune_stats[44], 1ull);
          if (active && complete && upper >= tau) atomicAdd(&g_prune_stats[45], 1ull);
          atomicAdd(&g_prune_stats[48], 1ull);
#endif
          const uint64_t m = __ballot(done);
          const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
              (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (done) {
            r = wnext + rank;
            start_row();
            k = 0;
            s = 0.0f;
            load_units(0);
          }
          wnext += (uint32_t)__builtin_popcountll(m);
          active = r < r1;
          if (((++iter) & CWQ_TAU_SHARE_MASK) == 0u) {  // share with the workgroup
            const float tm = wave_max_f32(tau);
            if (lane == 0) atomicMax(&tau_ord, ord_f32(tm));
            uint32_t o = __atomic_load_n(&tau_ord, __ATOMIC_RELAXED);
#if CWQ_CSR_GTAU_SHARE
            if ((iter & CWQ_CSR_GTAU_MASK) == 0u) {
              // publish only an improvement (atomics are rare once tau settles),
              // read the block's threshold every time
              uint32_t* gt = &gtau[g * CWQ_CSR_GTAU_STRIDE];
              const uint32_t o2 = __hip_atomic_load(gt, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
              if (lane == 0 && ord_f32(tm) > o2) atomicMax(gt, ord_f32(tm));
              o = o > o2 ? o : o2;
            }
#endif
            tau = fmaxf(tau, unord_f32(o));
          }
        }
        const float tm = wave_max_f32(tau);
        if (lane == 0) atomicMax(&tau_ord, ord_f32(tm));
      };
      // Cooperative rows (long rows, few rows per lane): each 16-lane DPP row
      // ("slot") walks one candidate row, lane t taking visit position k + t,
      // 16 units per iteration.  The partial sums are added over the slot with
      // a symmetric butterfly (row16_sum_f32), so s, the drop test and the
      // refill are uniform within the slot; the drop test runs every 16 units.
      // The bound's float-summation factor is taken at this tree's depth
      // (k_csr_prep: 4 in-lane + 4 butterfly + one per chunk).
      auto run_coop = [&](const float2* ab, const float* bp, const uint32_t* od,
                          const float4* rec, auto REC, auto HI0T) __attribute__((always_inline)) {
        constexpr bool HI0 = decltype(HI0T)::value;
        [[maybe_unused]] const PhiloxLo lok = HI0 ? philox_lo_key(st) : PhiloxLo{};
        const uint32_t t = lane & 15u, slot = lane >> 4;
        const uint64_t below = (1ull << (slot * 16u)) - 1ull;  // lanes of lower slots
#if CWQ_CSR_COOP_CLASS_WAVES
        // wave wv walks rows wv, wv + 4, wv + 8, ... of the tile: one alignment
        // class per wave, so its slots share one class's visit order
        const uint32_t nrows = (uint32_t)nrt;
        const uint32_t q0 = 0u, q1 = nrows > wv ? (nrows - wv + 3u) / 4u : 0u;
        auto row_of = [&](uint32_t q) { return (wv + 4u * q) << rlog; };
#else
        const uint32_t q0 = r0, q1 = r1;
        auto row_of = [&](uint32_t q) { return q; };
#endif
        uint32_t wnext = q0 + 4u;
        uint32_t q = q0 + slot;
        bool active = q < q1;
        uint32_t r = row_of(q);
        float s = 0.0f;
        float tau = unord_f32(tau_ord);
        uint32_t iter = 0;
        uint64_t rb;
        int c, U, cb;
        auto start_row = [&]() __attribute__((always_inline)) {
          const uint64_t k0 = (uint64_t)(n0 + (int64_t)r) * (uint64_t)d;
          rb = k0 >> 2;
          c = (int)(k0 & 3u);
          U = (d32 + c + 3) >> 2;
          cb = c * (int)cs;
        };
        start_row();
        int k = 0;
        // lane t takes visit positions k + t + 16 i, i < UPL: a slot advances
        // CH = 16 UPL units per iteration.  The units of the next positions
        // are loaded one iteration ahead, as in run.
        constexpr int UPL = CWQ_COOP_UPL, CH = 16 * UPL;
        // Loads index their (uniform) base with an unsigned 32-bit byte offset,
        // so they address as base + voffset: no 64-bit address arithmetic in
        // the loop.  Offsets stay far below 2^32 (a block's region holds
        // d + 10 entries of at most 32 bytes).
        uint32_t u_nx[UPL];
        auto load_units = [&](int p0) __attribute__((always_inline)) {
#pragma unroll
          for (int i = 0; i < UPL; ++i) {
            const int pp = p0 + 16 * i;
            u_nx[i] = ld_u32off(od, (uint32_t)cb + (uint32_t)(pp < U ? pp : U));
          }
        };
        load_units((int)t);
        while (__ballot(active) != 0ull) {
          const int p = k + (int)t;
          float part = 0.0f;
          uint32_t u[UPL];
#pragma unroll
          for (int i = 0; i < UPL; ++i) u[i] = u_nx[i];
          load_units(p + CH);
          // constants and the slot's next drop bound ahead of the Philox
          // rounds, as in run (positions past U clamp to U, the pad unit)
          const int kn = (k + CH < U) ? k + CH : U;
          const float bnext = ld_u32off(bp, (uint32_t)(cb + kn));
          float2 e[UPL][4];
#pragma unroll
          for (int i = 0; i < UPL; ++i) {
            const int pp = p + 16 * i;
            if constexpr (decltype(REC)::value) {
              const uint32_t pc = (uint32_t)(cb + (pp < U ? pp : U));
              const float4 ra = ld_u32off(rec, 2u * pc), rb2 = ld_u32off(rec, 2u * pc + 1u);
              e[i][0] = float2{ra.x, ra.y};
              e[i][1] = float2{ra.z, ra.w};
              e[i][2] = float2{rb2.x, rb2.y};
              e[i][3] = float2{rb2.z, rb2.w};
            } else {
              const uint32_t jp = (uint32_t)(4 * (int)u[i] - c + 4);
              e[i][0] = ld_u32off(ab, jp);
              e[i][1] = ld_u32off(ab, jp + 1u);
              e[i][2] = ld_u32off(ab, jp + 2u);
              e[i][3] = ld_u32off(ab, jp + 3u);
            }
#if CWQ_COOP_LOAD_ORDER
            // issue unit i's loads before unit i + 1's: the first unit's
            // constants then arrive first (loads complete in order), so its
            // wait does not also cover the later units' loads
            asm volatile("" ::: "memory");
#endif
          }
          if (active && p < U) {
            uint32_t kk0 = st.k0, kk1 = st.k1;
            asm volatile("" : "+s"(kk0), "+s"(kk1));
            // the UPL units are independent chains (ILP); a unit past the row
            // end reads the pad unit's zero constants and adds exactly 0
#pragma unroll
            for (int i = 0; i < UPL; ++i) {
              const uint64_t blk = rb + u[i];
              const U4 x = HI0 ? philox10_lo((uint32_t)blk, lok, kk0, kk1)
                               : philox10_dev((uint32_t)blk, (uint32_t)(blk >> 32), st.c2,
                                              st.c3, kk0, kk1);
              F4 z;
              box_muller_screen(x.x, x.y, z.a, z.b);
              box_muller_screen(x.z, x.w, z.c, z.d);
              const float a0 = __builtin_fmaf(e[i][0].x, z.a, e[i][0].y);
              const float a1 = __builtin_fmaf(e[i][1].x, z.b, e[i][1].y);
              const float a2 = __builtin_fmaf(e[i][2].x, z.c, e[i][2].y);
              const float a3 = __builtin_fmaf(e[i][3].x, z.d, e[i][3].y);
              float pu = -(a0 * a0);
              pu = __builtin_fmaf(-a1, a1, pu);
              pu = __builtin_fmaf(-a2, a2, pu);
              pu = __builtin_fmaf(-a3, a3, pu);
              if (i == 0)
                part = pu;
              else
                part = part + pu;
            }
          }
#ifdef CWQ_PRUNE_STATS
#pragma unroll
          for (int i = 0; i < UPL; ++i)
            if (active && p + 16 * i < U) atomicAdd(&g_prune_stats[43], 1ull);
#endif
          s = s + row16_sum_f32(part);
          k = kn;
          const bool complete = k == U;
          const float upper = __builtin_fmaf(s, gc.x, bnext);
          const bool prune = !complete && (upper < tau);
          if (complete && active && upper >= tau) {  // may be the best: keep it
            const float lower =
                __builtin_fmaf(s, gc.y, gc.z) - gc.w * __builtin_amdgcn_sqrtf(-s);
            tau = fmaxf(tau, lower);
            if (t == 0u) {
              const uint32_t sl = atomicAdd(&sq_cnt, 1u);
              if (sl < CWQ_CSR_SURVIVOR_CAP) {  // else: overflow, the tile is redone
                sq_n[sl] = r;
                sq_ub[sl] = upper;
              }
            }
          }
          const bool done = complete || prune || !active;
#ifdef CWQ_PRUNE_STATS
          if (t == 0u && active && (complete || prune)) atomicAdd(&g_prune_stats[42], 1ull);
          if (t == 0u && active && complete) atomicAdd(&g_prune_stats[44], 1ull);
          if (t == 0u && active && complete && upper >= tau) atomicAdd(&g_prune_stats[45], 1ull);
          atomicAdd(&g_prune_stats[48], 1ull);
#endif
          const uint64_t m = __ballot(done);  // 16 bits per finished slot
          if (done) {
            q = wnext + (uint32_t)(__builtin_popcountll(m & below) >> 4);
            r = row_of(q);
            start_row();
            k = 0;
            s = 0.0f;
            load_units((int)t);
          }
          wnext += (uint32_t)(__builtin_popcountll(m) >> 4);
          active = q < q1;
          if (((++iter) & CWQ_TAU_SHARE_MASK) == 0u) {  // share with the workgroup
            const float tm = wave_max_f32(tau);
            if (lane == 0) atomicMax(&tau_ord, ord_f32(tm));
            tau = fmaxf(tau, unord_f32(__atomic_load_n(&tau_ord, __ATOMIC_RELAXED)));
          }
        }
        const float tm = wave_max_f32(tau);
        if (lane == 0) atomicMax(&tau_ord, ord_f32(tm));
      };
      const bool coop = d >= coop_min_d;
      // the block's largest Philox block index, ((n_cand - 1) d + d - 1) / 4
      const bool lo32 = (uint64_t)n_cand * (uint64_t)d <= (1ull << 34);
      // survivor list overflow (near-ties everywhere, or a weak early tau):
      // redo the pass starting from the final tau, then score exactly
      for (int pass = 0;; ++pass) {
        using NoRec = std::integral_constant<int, 0>;
        using Rec = std::integral_constant<int, 1>;
        using Lo32 = std::integral_constant<bool, true>;   // block indices < 2^32
        using Hi32 = std::integral_constant<bool, false>;
        // each launch mode instantiates only its own loops (register
        // allocation is per kernel: the largest loop sets every loop's budget)
        auto any_run = [&](auto HI0T) __attribute__((always_inline)) {
          if constexpr (COOP) {
            if (coop) {
              if (in_lds)
                run_coop(l_ab, l_bp, l_ord, nullptr, NoRec{}, HI0T);
              else if (abp)
                run_coop(nullptr, bpre + reg, ordu + reg, abp + 2 * csr_rec_base(off), Rec{}, HI0T);
              else
                run_coop(sab + off + 8 * g, bpre + reg, ordu + reg, nullptr, NoRec{}, HI0T);
            } else {  // d < coop_min_d <= CWQ_CSR_LDS_DIMS: the constants are in LDS
              run(l_ab, l_bp, l_ord, nullptr, NoRec{}, HI0T);
            }
          } else if (in_lds)
            run(l_ab, l_bp, l_ord, nullptr, NoRec{}, HI0T);
          else if (abp)
            run(nullptr, bpre + reg, ordu + reg, abp + 2 * csr_rec_base(off), Rec{}, HI0T);
          else
            run(sab + off + 8 * g, bpre + reg, ordu + reg, nullptr, NoRec{}, HI0T);
        };
        if (lo32)
          any_run(Lo32{});
        else
          any_run(Hi32{});
        __syncthreads();
        if (tid == 0) {
          const uint32_t mine = tau_ord;
          const uint32_t prev = atomicMax(&gtau[g * CWQ_CSR_GTAU_STRIDE], mine);
          tau_ord = prev > mine ? prev : mine;
        }
        __syncthreads();
        if (sq_cnt <= CWQ_CSR_SURVIVOR_CAP) break;
#ifdef CWQ_PRUNE_STATS
        if (tid == 0) atomicAdd(&g_prune_stats[46], 1ull);
#endif
        if (pass == 1) {
          exact_tile = true;
          break;
        }
        __syncthreads();
        if (tid == 0) sq_cnt = 0u;
        __syncthreads();
      }
    }
    if (!exact_tile) {
      const float tau_final = unord_f32(tau_ord);
      const uint32_t nsurv = sq_cnt < CWQ_CSR_SURVIVOR_CAP ? sq_cnt : CWQ_CSR_SURVIVOR_CAP;
      for (uint32_t i = wv; i < nsurv; i += 4) {  // one survivor per wave
        if (sq_ub[i] >= tau_final) {
          const int64_t nn = n0 + (int64_t)sq_n[i];
#ifdef CWQ_PRUNE_STATS
          if (lane == 0) atomicAdd(&g_prune_stats[47], 1ull);
#endif
          const float v = exact_row_wave<STEP0>(
              st, (uint64_t)nn * (uint64_t)d, d, loc_s + off, scale_s + off, t_loc + off,
              t_scale + off, lognorm + off, STEP0 ? nullptr : best + off, logtab, rowbuf[wv],
              lane);
          const uint64_t kv = argmax_key(v, (uint32_t)nn);
          bestk = kv > bestk ? kv : bestk;
        }
      }
    } else {
      const int align = (int)(((uint64_t)(n0 + ((int64_t)wv << rlog)) * (uint64_t)d) & 3u);
      for (int64_t m = 4 * (int64_t)lane + wv; m < nrt; m += 256) {
        const int64_t n = n0 + (m << rlog);
        const float v = eval_row<0, STEP0>(st, (uint64_t)n * (uint64_t)d, d, align, loc_s + off,
                                           scale_s + off, t_loc + off, t_scale + off,
                                           lognorm + off, STEP0 ? nullptr : best + off, logtab);
        const uint64_t kv = argmax_key(v, (uint32_t)n);
        bestk = kv > bestk ? kv : bestk;
      }
    }
    bestk = wave_max_u64(bestk);
    if (lane == 0) wkey[wv] = bestk;
    __syncthreads();
    if (tid == 0) {
      uint64_t mk = wkey[0];
      for (int i = 1; i < 4; ++i) mk = wkey[i] > mk ? wkey[i] : mk;
      if (mk) atomicMax(&keys[g], (unsigned long long)mk);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Screened encoder for few candidates (64 <= 2^b < 4096, CSR or uniform d the
// fast kernel does not take): C2/C3's 8-bit groups of ~5 dims.  Every
// candidate is screened -- k_csr_prep's bound with the row summed
// sequentially in natural order, no pruning -- and only survivors are scored
// exactly, densely, in a separate pass:
//   k_small_prep      per block (a lane each for short blocks): per-dim (sA, sB)
//                     into sab, the block's (c1, c2, As, Pq) into grp (c1 == 0:
//                     the block is scored exactly), its full-row bound B and
//                     stream key into bpre[off + 12 g ...]; gtau = -inf; the
//                     survivor count = 0.
//   k_small_screen    a wave per tile, each lane 4 consecutive rows at a time
//                     (d whole Philox blocks): screened value s of each row; tau = the wave's
//                     best lower bound fma(s, c2, As) - Pq sqrt(-s); rows whose
//                     upper bound fma(s, c1, B) reaches tau take one of the
//                     block's CWQ_SLIST_PER_BLOCK slots; tau is published to
//                     gtau[g].  Full slots mark the block exact.
//   k_small_survivors listed rows still reaching gtau[g], scored exactly one
//                     per lane; then every candidate of the blocks marked exact.
// The exact pass costs about 3x a screened row (f64 Box-Muller against the
// hardware transcendentals); survivors are ~1 per block, so the step costs
// about a third of scoring every candidate exactly.
// ---------------------------------------------------------------------------
#ifndef CWQ_SMALL_SCREEN_WAVES
#define CWQ_SMALL_SCREEN_WAVES 8  // waves/SIMD k_small_screen's registers must allow
#endif
#ifndef CWQ_SMALL_MIN_CAND
#define CWQ_SMALL_MIN_CAND 64  // fewer candidates: the exact kernel (screening would not pay)
#endif

// A wave prepares 64 consecutive blocks: lane i block i when it has at most
// kSmallLaneD dims (C2's groups: ~5), sequentially; longer blocks afterwards
// with the whole wave, lanes over dims.  The block's stream key for this step
// (a Philox-10 call) is stored too, so the screening rows do not repeat it.
constexpr int64_t kSmallLaneD = 32;
// Per-block header of the small path, 12 words at bpre + 12 g (bpre holds
// total_dims + 12 nb words; a forked part's bpre moves by 12 g0): [0] the
// full-row bound B, [1..4] the step's stream key, [5..8] grp's (c1, c2, As, Pq),
// [9..10] the block's dim offset, [11] its dims.  The slot count is at
// scnt[12 g].
constexpr int64_t kSmallHdr = 12;
struct SmallHdr {
  float bf;
  PhiloxStream st;
  float4 gc;
  int64_t off;
  int d;
};
__device__ __forceinline__ SmallHdr small_hdr(const float4 h0, const float4 h1, const float4 h2) {
  SmallHdr h;
  h.bf = h0.x;
  h.st = PhiloxStream{f2u(h0.y), f2u(h0.z), f2u(h0.w), f2u(h1.x)};
  h.gc = float4{h1.y, h1.z, h1.w, h2.x};
  h.off = (int64_t)(((uint64_t)f2u(h2.z) << 32) | (uint64_t)f2u(h2.y));
  h.d = (int)f2u(h2.w);
  return h;
}

template <bool STEP0>
__global__ void __launch_bounds__(256) k_small_prep(
    const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ loc_s, const float* __restrict__ scale_s,
    const float* __restrict__ lognorm, const float* __restrict__ best,
    const int64_t* __restrict__ block_off, int64_t ud, int64_t nb, SeedSpec sd, int32_t step,
    float2* __restrict__ sab, float* __restrict__ bpre, float4* __restrict__ grp,
    uint32_t* __restrict__ gtau, uint32_t* __restrict__ scnt) {
  const uint32_t lane = threadIdx.x & 63u;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  struct Sums {
    double sm = 0.0, sa = 0.0, sk = 0.0, s2 = 0.0, cs = 0.0, mx = 0.0;
    int ok = 1;
  };
  auto dim = [&](Sums& u, int64_t off, int64_t g, int64_t j) {
    const CsrDim o = csr_dim<STEP0>(loc_s[off + j], scale_s[off + j], t_loc[off + j],
                                    t_scale[off + j], lognorm[off + j],
                                    STEP0 ? 0.0f : best[off + j]);
    sab[off + 8 * g + 4 + j] = float2{o.sa, o.sb};  // k_csr_prep's padded layout
    u.sm += o.M;
    u.sa += __builtin_fabs(o.M);
    u.sk += __builtin_fabs(o.M) + o.M;
    u.s2 += (double)o.A * (double)o.A;
    u.cs += (double)o.C;
    u.mx = (double)o.A > u.mx ? (double)o.A : u.mx;
    u.ok &= o.ok ? 1 : 0;
  };
  // as k_csr_prep: gamma at the larger depth of the two float sums, the
  // screening sum (sequential over the row here: h = d) and the exact
  // Eigen-order row value (h <= d/8 + 8)
  auto finish = [&](const Sums& u, int64_t off, int64_t g, int64_t d) {
    const double h_s = (double)d, h_e = (double)d / 8.0 + 8.0;
    const double gam = 1.01 * ((h_s > h_e ? h_s : h_e) + 1.0) * 0x1p-24;
    const double sl = (3.0 * gam + 0x1p-20) * (__builtin_fabs(u.sm) + u.sa + u.sk) + 0x1p-126;
    const float bf = round_up_f32(u.sm + u.cs * (1.0 + 0x1p-20) + sl);
    const float c1 = round_dn_f32(1.0 - 3.0 * gam - 0x1p-22);
    const float c2 = round_up_f32(1.0 + 3.0 * gam + 0x1p-14);
    const float as = round_dn_f32(u.sm - sl - 1.01 * u.s2 * (1.0 + 0x1p-11));
    const float pq = round_up_f32(2.01 * u.mx * __builtin_sqrt((double)(d > 0 ? d : 1)) *
                                  (1.0 + 0x1p-11));
    const bool fin = as - as == 0.0f && pq - pq == 0.0f && bf - bf == 0.0f;
    const float4 gc = (u.ok && fin && d > 0) ? float4{c1, c2, as, pq} : float4{0.f, 0.f, 0.f, 0.f};
    grp[g] = gc;
    // the block's header (kSmallHdr), indexed by g alone: the screen reads it
    // with one load level and prefetches the next tile's
    const PhiloxStream st = generate_key(step_seed(sd.of(g), step), 42);
    float4* hg = reinterpret_cast<float4*>(bpre + kSmallHdr * g);
    hg[0] = float4{bf, u2f(st.k0), u2f(st.k1), u2f(st.c2)};
    hg[1] = float4{u2f(st.c3), gc.x, gc.y, gc.z};
    hg[2] = float4{gc.w, u2f((uint32_t)off), u2f((uint32_t)((uint64_t)off >> 32)), u2f((uint32_t)d)};
    scnt[kSmallHdr * g] = 0u;
    gtau[g * CWQ_CSR_GTAU_STRIDE] = ord_f32(-__builtin_inff());
  };
  for (int64_t gb = ((int64_t)blockIdx.x * 4 + wave_id()) * 64; gb < nb; gb += nwaves * 64) {
    const int64_t g = gb + lane;
    bool longb = false;
    if (g < nb) {
      const BlockSpan sp = block_span(block_off, ud, g);
      if (sp.d <= kSmallLaneD) {
        Sums u;
        for (int64_t j = 0; j < sp.d; ++j) dim(u, sp.off, g, j);
        finish(u, sp.off, g, sp.d);
      } else {
        longb = true;
      }
    }
    for (uint64_t m = __ballot(longb); m != 0ull; m &= m - 1ull) {  // the long blocks, a wave each
      const int64_t gl = gb + (int64_t)__builtin_ctzll(m);
      const BlockSpan sp = block_span(block_off, ud, gl);
      Sums u;
      for (int64_t j = lane; j < sp.d; j += 64) dim(u, sp.off, gl, j);
      const bool all_ok = __ballot(u.ok == 0) == 0ull;
      u.sm = wave_sum_f64(u.sm);
      u.sa = wave_sum_f64(u.sa);
      u.sk = wave_sum_f64(u.sk);
      u.s2 = wave_sum_f64(u.s2);
      u.cs = wave_sum_f64(u.cs);
      u.mx = wave_max_f64(u.mx);
      u.ok = all_ok ? 1 : 0;
      if (lane == 0) finish(u, sp.off, gl, sp.d);
    }
  }
}

template <bool STEP0>
__global__ void __launch_bounds__(256, CWQ_SMALL_SCREEN_WAVES) k_small_screen(
    const int64_t* __restrict__ block_off, int64_t ud, int64_t ntiles, int64_t tiles_per_block,
    int64_t cand_per_tile, int64_t n_cand, SeedSpec sd, int32_t step,
    const float2* __restrict__ sab, const float* __restrict__ bpre, float4* __restrict__ grp,
    uint32_t* __restrict__ gtau, uint32_t* __restrict__ scnt, uint2* __restrict__ slist) {
  const uint32_t lane0 = threadIdx.x & 63u;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  // a wave takes a whole tile (the block's header, key and threshold once per
  // tile), 256 rows per round.  The header (k_small_prep) is one load level.
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wave_id(); tile < ntiles; tile += nwaves) {
    // the lane index behind an opaque move: the many span variants' lane-derived
    // values are then computed per tile instead of hoisted out of the tile loop
    // (and spilled)
    uint32_t lane = lane0;
    asm volatile("" : "+v"(lane));
    const int64_t g = tiles_per_block == 1 ? tile : tile / tiles_per_block;
    const int64_t tt = tile - g * tiles_per_block;
    const float4* hp = reinterpret_cast<const float4*>(bpre + kSmallHdr * g);
    const SmallHdr h = small_hdr(hp[0], hp[1], hp[2]);
    const float4 gc = h.gc;
    if (gc.x == 0.0f) continue;  // scored exactly by k_small_survivors
    const int64_t off = h.off;
    const int d = h.d;
    const int64_t n0 = tt * cand_per_tile;
    const int64_t n1 = (n0 + cand_per_tile < n_cand) ? n0 + cand_per_tile : n_cand;
    const float bf = h.bf;
    const PhiloxStream st = h.st;
    const float2* ab = sab + off + 8 * g + 4;
    // A block that is one tile (C2/C3's 256 candidates) belongs to this wave
    // alone: its threshold starts at k_small_prep's -inf and its slot count
    // lives in a scalar, both stored once at the end -- no global atomics.
    const bool own = tiles_per_block == 1;
    float tau = own ? -__builtin_inff()
                    : unord_f32(__hip_atomic_load(&gtau[g * CWQ_CSR_GTAU_STRIDE],
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    uint32_t used = 0;  // own block: slots taken so far (wave-uniform)
    // lane span m: rows n0 + 4 (lane + 64 m) + q, q = 0..3.  n0 is a multiple
    // of 4 (tiles are multiples of 256 candidates), so a span's 4d words are
    // exactly Philox blocks [n d / 4, n d / 4 + d): every block is computed
    // once (a row alone would start and end inside blocks its neighbours also
    // compute), and the dim index of each word is the same in every lane, so
    // the per-dim constants are wave-uniform loads.
    const PhiloxLo K = philox_lo_key(st);
    // tau, survivor slots of one span's four rows (rs: their screened values)
    auto span_tail = [&](int64_t ns, const float (&rs)[4]) __attribute__((always_inline)) {
      // tau from the lane's best valid row: the lower bound is monotone in
      // the screened value, and any row's lower bound is a valid threshold,
      // so one wave max per span replaces one per row
      float smax = -__builtin_inff();
      bool any = false;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        if (ns + qq < n1) {
          smax = fmaxf(smax, rs[qq]);
          any = true;
        }
      const float lower = any ? __builtin_fmaf(smax, gc.y, gc.z) -
                                    gc.w * __builtin_amdgcn_sqrtf(-smax)
                              : -__builtin_inff();
      tau = fmaxf(tau, wave_max_f32(lower));
      uint64_t m[4];
      uint32_t cnt = 0;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        m[qq] = __ballot(ns + qq < n1 && __builtin_fmaf(rs[qq], gc.x, bf) >= tau);
        cnt += (uint32_t)__builtin_popcountll(m[qq]);
      }
      if (cnt) {
        // the block's slots: this wave's scalar count, or a global counter
        // shared with the block's other tiles
        uint32_t base = used;
        if (own) {
          used += cnt;
        } else {
          if (lane == 0) base = atomicAdd(&scnt[kSmallHdr * g], cnt);
          base = (uint32_t)__shfl((int)base, 0, 64);
        }
        uint32_t pre = base;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const uint64_t mq = m[qq];
          if ((mq >> lane) & 1ull) {
            const uint32_t slot = pre + __builtin_amdgcn_mbcnt_hi(
                                            (uint32_t)(mq >> 32),
                                            __builtin_amdgcn_mbcnt_lo((uint32_t)mq, 0u));
            if (slot < CWQ_SLIST_PER_BLOCK)
              slist[CWQ_SLIST_PER_BLOCK * g + slot] =
                  uint2{(uint32_t)(ns + qq), f2u(__builtin_fmaf(rs[qq], gc.x, bf))};
          }
          pre += (uint32_t)__builtin_popcountll(mq);
        }
        if (base + cnt > CWQ_SLIST_PER_BLOCK && lane == 0)  // slots full: score the block exactly
          __hip_atomic_store(reinterpret_cast<uint32_t*>(&grp[g].x), 0u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    };
    // lane span m: rows n0 + 4 (lane + 64 m) + q, q = 0..3.  n0 is a multiple
    // of 4 (tiles are multiples of 256 candidates), so a span's 4d words are
    // exactly Philox blocks [n d / 4, n d / 4 + d): every block is computed
    // once (a row alone would start and end inside blocks its neighbours also
    // compute), and the dim index of each word is the same in every lane, so
    // the per-dim constants are wave-uniform loads.
    auto spans = [&](auto lo_tag) __attribute__((always_inline)) {
      constexpr bool LO = decltype(lo_tag)::value;  // every Philox block index < 2^32
      for (int64_t m0 = 0; n0 + 256 * m0 < n1; ++m0) {
        const int64_t ns = n0 + 4 * ((int64_t)lane + 64 * m0);
        const uint64_t b0 = (uint64_t)ns * (uint64_t)d / 4u;
        float rs[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // the span's four row sums
        float cur = 0.0f;  // natural order, sequential sum (h = d), as k_small_prep's bound
        int j = 0, q = 0;
        for (int b = 0; b < d; ++b) {
          const uint64_t blk = b0 + (uint64_t)b;
          const U4 x = LO ? philox10_lo((uint32_t)blk, K, st.k0, st.k1)
                          : philox10_dev((uint32_t)blk, (uint32_t)(blk >> 32), st.c2, st.c3,
                                         st.k0, st.k1);
          float z[4];
          box_muller_screen(x.x, x.y, z[0], z[1]);
          box_muller_screen(x.z, x.w, z[2], z[3]);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const float2 e = ab[j];
            const float a = __builtin_fmaf(e.x, z[t], e.y);
            cur = __builtin_fmaf(-a, a, cur);
            if (++j == d) {  // wave-uniform: a row of the span is complete
              if (q == 0) rs[0] = cur;
              else if (q == 1) rs[1] = cur;
              else if (q == 2) rs[2] = cur;
              else rs[3] = cur;
              cur = 0.0f;
              j = 0;
              ++q;
            }
          }
        }
        span_tail(ns, rs);
      }
    };
    const bool lo = (uint64_t)(n1 + 4) * (uint64_t)d / 4u + (uint64_t)d <= 0xffffffffull;
    if (lo) {
      spans(std::true_type{});
    } else {
      spans(std::false_type{});
    }
    if (lane == 0) {
      if (own) {
        scnt[kSmallHdr * g] = used;
        gtau[g * CWQ_CSR_GTAU_STRIDE] = ord_f32(tau);
      } else {
        atomicMax(&gtau[g * CWQ_CSR_GTAU_STRIDE], ord_f32(tau));
      }
    }
  }
}

template <bool STEP0>
__global__ void __launch_bounds__(256) k_small_survivors(
    const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ loc_s, const float* __restrict__ scale_s,
    const float* __restrict__ lognorm, const float* __restrict__ best,
    const int64_t* __restrict__ block_off, int64_t ud, int64_t nb, int64_t n_cand, SeedSpec sd,
    int32_t step, const float4* __restrict__ grp, const uint32_t* __restrict__ gtau,
    const uint32_t* __restrict__ scnt, const uint2* __restrict__ slist,
    const float* __restrict__ bpre, unsigned long long* __restrict__ keys) {
  __shared__ double logtab[32];
  // per wave: the listed rows still reaching their block's final threshold,
  // queued until 64 of them can be scored at once, one per lane (a lane per
  // slot left ~6% of the lanes busy: ~1 survivor per block, 8 slots)
  constexpr int kQueue = 64 + 64 * CWQ_SLIST_PER_BLOCK;
  __shared__ int64_t q_g[4][kQueue];
  __shared__ uint32_t q_n[4][kQueue];
  fill_logtab(logtab);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = wave_id();
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  auto score = [&](int64_t g, uint32_t n) {
    const BlockSpan sp = block_span(block_off, ud, g);
    const float* bg = bpre + kSmallHdr * g;  // k_small_prep's header: the step's stream key
    const PhiloxStream st{f2u(bg[1]), f2u(bg[2]), f2u(bg[3]), f2u(bg[4])};
    const uint64_t k0 = (uint64_t)n * (uint64_t)sp.d;
    const float v = eval_row<0, STEP0>(st, k0, sp.d, (int)(k0 & 3u), loc_s + sp.off,
                                       scale_s + sp.off, t_loc + sp.off, t_scale + sp.off,
                                       lognorm + sp.off, STEP0 ? nullptr : best + sp.off, logtab);
    atomicMax(&keys[g], (unsigned long long)argmax_key(v, n));
  };
  int q = 0;  // wave-uniform queue length
  for (int64_t gb = ((int64_t)blockIdx.x * 4 + wv) * 64; gb < nb; gb += nwaves * 64) {
    const int64_t g = gb + lane;
    uint32_t cnt = 0, keep = 0;  // listed slots; bit s: slot s survives
    if (g < nb && grp[g].x != 0.0f) {  // exact blocks are scored below
      const uint32_t c = scnt[kSmallHdr * g];
      const uint32_t ns = c < CWQ_SLIST_PER_BLOCK ? c : CWQ_SLIST_PER_BLOCK;
      const float tau = unord_f32(gtau[g * CWQ_CSR_GTAU_STRIDE]);
      for (uint32_t sl = 0; sl < ns; ++sl)
        if (u2f(slist[CWQ_SLIST_PER_BLOCK * g + sl].y) >= tau) {
          keep |= 1u << sl;
          ++cnt;
        }
    }
    // exclusive scan of the counts: this lane's first queue position
    uint32_t inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = (uint32_t)__shfl_up((int)inc, (unsigned)o, 64);
      if (lane >= (uint32_t)o) inc += t;
    }
    const uint32_t total = (uint32_t)__shfl((int)inc, 63, 64);
    uint32_t pos = (uint32_t)q + inc - cnt;
    for (uint32_t m = keep; m != 0u; m &= m - 1u) {
      const uint32_t sl = (uint32_t)__builtin_ctz(m);
      q_g[wv][pos] = g;
      q_n[wv][pos] = slist[CWQ_SLIST_PER_BLOCK * g + sl].x;
      ++pos;
    }
    q += (int)total;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    while (q >= 64) {  // a full batch: the queue's last 64 entries
      q -= 64;
      const int64_t qg = q_g[wv][q + (int)lane];
      const uint32_t qn = q_n[wv][q + (int)lane];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      score(qg, qn);
    }
    // blocks k_small_screen did not screen (constants failed the gate, or
    // their survivor slots overflowed): every candidate exactly, the wave per block
    for (uint64_t m = __ballot(g < nb && grp[g].x == 0.0f); m != 0ull; m &= m - 1ull) {
      const int64_t ge = gb + (int64_t)__builtin_ctzll(m);
      const BlockSpan sp = block_span(block_off, ud, ge);
      const float* bg = bpre + kSmallHdr * ge;
      const PhiloxStream st{f2u(bg[1]), f2u(bg[2]), f2u(bg[3]), f2u(bg[4])};
      uint64_t bestk = 0;
      for (int r = 0; r < 4; ++r) {  // rows n = r (mod 4): one alignment class per pass
        const int align = (int)(((uint64_t)r * (uint64_t)sp.d) & 3u);
        for (int64_t n = r + 4 * (int64_t)lane; n < n_cand; n += 256) {
          const float v = eval_row<0, STEP0>(st, (uint64_t)n * (uint64_t)sp.d, sp.d, align,
                                             loc_s + sp.off, scale_s + sp.off, t_loc + sp.off,
                                             t_scale + sp.off, lognorm + sp.off,
                                             STEP0 ? nullptr : best + sp.off, logtab);
          const uint64_t k = argmax_key(v, (uint32_t)n);
          bestk = k > bestk ? k : bestk;
        }
      }
      bestk = wave_max_u64(bestk);
      if (lane == 0 && bestk) atomicMax(&keys[ge], (unsigned long long)bestk);
    }
  }
  if ((int)lane < q) score(q_g[wv][lane], q_n[wv][lane]);
}

// ---------------------------------------------------------------------------
// The small-candidate shapes (64 <= 2^b < 4096 candidates, blocks of d <=
// CWQ_FUSED_DMAX): shared pieces of the small pipeline below (k_small_*).
// Round 4 ran these shapes as one kernel (k_small_fused: a wave per four
// blocks doing constants, screen, exact survivors and finalize); round 5
// split it (see "The small-candidate step as a pipeline").
// ---------------------------------------------------------------------------
#ifndef CWQ_FUSED_DMAX
#define CWQ_FUSED_DMAX 64  // longest block of the small pipeline
#endif
#ifndef CWQ_FUSED_LIST
#define CWQ_FUSED_LIST 64  // listed rows per block
#endif
#ifndef CWQ_FUSED_STAGE
#define CWQ_FUSED_STAGE 256  // (row, dim) values per exact batch
#endif
#ifndef CWQ_FUSED_WAVES
#define CWQ_FUSED_WAVES 8
#endif
static_assert(CWQ_FUSED_STAGE >= CWQ_FUSED_DMAX, "an exact batch holds at least one row");
static_assert(CWQ_FUSED_LIST <= 64, "one listed row per lane");

// Exact normal k of a block's stream: its Philox block and the one
// Box-Muller pair that holds it (normal4_dev's element k & 3, bit for bit).
#ifndef CWQ_EXACT_NOINLINE
#define CWQ_EXACT_NOINLINE 0  // inline (k_small_one has no loop to hoist its constants out of)
#endif
#if CWQ_EXACT_NOINLINE
__device__ __noinline__
#else
__device__ __forceinline__
#endif
float exact_normal(const PhiloxStream& st, uint64_t k, const double* logtab) {
  const U4 x = philox_block_dev(st, k >> 2);
  const bool hi = (k & 2u) != 0;
  float f0, f1;
  box_muller_dev(hi ? x.z : x.x, hi ? x.w : x.y, logtab, f0, f1);
  return (k & 1u) ? f1 : f0;
}

// LDS written by some lanes of a wave and read by others: order the wave's
// accesses (no workgroup barrier: a wave's LDS is its own)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {  // set lanes of m below this one
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// A block for quad_exact_block: its first dim, length and step stream
struct QuadBlk {
  int64_t off;
  uint32_t d, k0, k1, c2, c3;
};
// a block's state in the small pipeline (SmallRec q0.w, then k_small_one's)
constexpr uint32_t kQuadKnown = 0;   // idx decided (empty block, or a single listed row)
constexpr uint32_t kQuadListed = 1;  // screened; listed rows scored exactly
constexpr uint32_t kQuadExact = 2;   // every candidate scored exactly

#ifndef CWQ_FUSED_NOINLINE
#define CWQ_FUSED_NOINLINE 1  // the rare whole-block exact path out of line (its registers)
#endif
#if CWQ_FUSED_NOINLINE
#define CWQ_RARE __device__ __noinline__
#else
#define CWQ_RARE __device__ __forceinline__
#endif
// Every candidate of a block exactly (eval_row, a lane per row): k_small_one's
// fallback for blocks outside the screening gate or with a full list.
// Returns the wave's best argmax key.
template <bool STEP0>
CWQ_RARE unsigned long long quad_exact_block(const QuadBlk r, const float* __restrict__ t_loc,
                                             const float* __restrict__ t_scale,
                                             const float* __restrict__ loc_s,
                                             const float* __restrict__ scale_s,
                                             const float* __restrict__ lognorm,
                                             const float* __restrict__ best, int64_t n_cand,
                                             const double* logtab) {
  const uint32_t lane = threadIdx.x & 63u;
  const PhiloxStream se{r.k0, r.k1, r.c2, r.c3};
  const int64_t ob = r.off;
  const int db = (int)r.d;
  uint64_t bestk = 0;
  for (int rr = 0; rr < 4; ++rr) {  // rows n = rr (mod 4): one alignment class per pass
    const int align = (int)(((uint64_t)rr * (uint64_t)db) & 3u);
    for (int64_t n = rr + 4 * (int64_t)lane; n < n_cand; n += 256) {
      const float v = eval_row<0, STEP0>(se, (uint64_t)n * (uint64_t)db, db, align, loc_s + ob,
                                         scale_s + ob, t_loc + ob, t_scale + ob, lognorm + ob,
                                         STEP0 ? nullptr : best + ob, logtab);
      const uint64_t kk = argmax_key(v, (uint32_t)n);
      bestk = kk > bestk ? kk : bestk;
    }
  }
  return wave_max_u64(bestk);
}

#ifdef CWQ_QUAD_TIMES
// timing builds only (tools/quad_times.py --one): per block of k_small_one the
// wall clock (s_memrealtime, 100 MHz) at its start [0], after its screen [1]
// and at its end [2..5]; info = HW_ID, XCC_ID, listed rows scored exactly,
// exact-block flag | d << 8
constexpr int kQuadTimes = 1 << 16;
__device__ unsigned long long g_quad_t[kQuadTimes][6];
__device__ unsigned int g_quad_info[kQuadTimes][4];
#endif

// ---------------------------------------------------------------------------
// The small-candidate step as a pipeline (round 5): blocks of d <= 64,
// 64 <= 2^b < 4096 candidates (C2/C3's 8-bit groups).  tools/quad_times.py
// showed where k_small_fused's time went on C2 (41.5k groups, 10.4k quads):
// the quads ran at the chip's issue rate while 8 waves shared each SIMD, but
// every quad took ~29 us, so the launch drained for ~35 us of its 62-69 us
// at falling occupancy, and 35% of a quad's time went to its constants phase
// (per-block f64 sums and bounds on 16-lane rows, DPP reductions, the stream
// key).  Here the per-block work runs lane-parallel before the screen, and
// the screen runs a wave per block:
//   k_small_prep1     a workgroup per CWQ_PREP1_BLOCKS blocks, a thread per
//                     dim: the shard constants (step 0, k_prep_dims'
//                     arithmetic) and each dim's screening constants
//                     (csr_dim), summed per block in LDS; then a thread per
//                     block: bounds, stream key -> a 64-byte record; the
//                     dim -> block map
//   k_small_one       a wave per block: screen, exact survivors -> index
//                     (variants measured in DESIGN.md 5e: more blocks per
//                     wave or per workgroup, a striding grid, a second kernel
//                     for the exact paths, the finalize fused in: all slower)
//   k_small_finalize  a thread per dim: best += the winning row (:63), and
//                     at the last step the destandardised sample (:292)
// ---------------------------------------------------------------------------
struct SmallRec {  // 4 x uint4: q0 = (off lo, off hi, d, state), q1 = stream key,
  uint4 q0, q1;    // q2 = (bf, c1, c2, As), q3 = (Pq, -, -, -)
  uint4 q2, q3;
};
static_assert(sizeof(SmallRec) <= 8 * CWQ_SLIST_PER_BLOCK, "a record per block in slist");
// blocks per k_small_prep1 workgroup of CWQ_PREP1_THREADS threads: C2's 41.5k
// blocks make 650 workgroups (with 256 per workgroup 163 of them ran 20 us,
// latency-bound)
#ifndef CWQ_PREP1_BLOCKS
#define CWQ_PREP1_BLOCKS 64
#endif
#ifndef CWQ_PREP1_THREADS
#define CWQ_PREP1_THREADS 256
#endif
constexpr int kSmallPrepBlocks = CWQ_PREP1_BLOCKS;
static_assert(CWQ_PREP1_BLOCKS <= CWQ_PREP1_THREADS, "a thread per block in the block phase");

// The dims of a launch's blocks: [block_off[0], block_off[nb]) (absolute: a
// forked part of a launch passes block_off + g0), or [0, nb ud) for uniform blocks
__device__ __forceinline__ void dims_of(const int64_t* __restrict__ block_off, int64_t ud,
                                        int64_t nb, int64_t& d0, int64_t& d1) {
  d0 = block_off ? block_off[0] : 0;
  d1 = block_off ? block_off[nb] : nb * ud;
}

// FIRST (step 0): also the shard constants and best = 0 (k_prep_dims).  The
// block sums are LDS atomics in no fixed order, which the bounds' slack (far
// above double rounding) covers, so the screen stays exact-safe.
template <bool FIRST>
__global__ void __launch_bounds__(CWQ_PREP1_THREADS) k_small_prep1(
    const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ p_loc, const float* __restrict__ p_scale, float nst, float sdiv,
    float rho, float* __restrict__ loc_s, float* __restrict__ scale_s,
    float* __restrict__ lognorm, float* __restrict__ best, const int64_t* __restrict__ block_off,
    int64_t ud, int64_t nb, SeedSpec sd, int32_t step, float2* __restrict__ pre_ab,
    SmallRec* __restrict__ rec, uint32_t* __restrict__ dmap) {
  constexpr int B = kSmallPrepBlocks;
  constexpr int T = CWQ_PREP1_THREADS;
  __shared__ int64_t boff[B + 1];
  __shared__ double acc[5][B];  // sum M, sum |M|, sum |M| + M, sum A^2, sum C
  __shared__ uint32_t amx[B], abad[B];
  const int t = threadIdx.x;
  const int64_t g0 = (int64_t)blockIdx.x * B;
  const int n = (int)(nb - g0 < B ? nb - g0 : B);
  for (int k = t; k <= n; k += T) boff[k] = block_off ? block_off[g0 + k] : (g0 + k) * ud;
  if (t < B) {
    for (int k = 0; k < 5; ++k) acc[k][t] = 0.0;
    amx[t] = 0u;
    abad[t] = 0u;
  }
  __syncthreads();
  const int64_t i0 = boff[0], i1 = boff[n];
  for (int64_t i = i0 + t; i < i1; i += T) {
    int lo = 0, hi = n;  // boff[lo] <= i < boff[hi] (empty blocks are skipped)
    while (hi - lo > 1) {
      const int m = (lo + hi) >> 1;
      if (boff[m] <= i) lo = m; else hi = m;
    }
    float ls, ss, c;
    const float sg = t_scale[i];
    if (FIRST) {  // k_prep_dims' arithmetic, bit for bit
      ls = p_loc[i] / nst;
      ss = (rho * p_scale[i]) / sdiv;
      c = kHalfLog2Pi + logf_full(sg, kLogTabConst);
      loc_s[i] = ls;
      scale_s[i] = ss;
      lognorm[i] = c;
    } else {
      ls = loc_s[i];
      ss = scale_s[i];
      c = lognorm[i];
    }
    const CsrDim o = csr_dim<FIRST>(ls, ss, t_loc[i], sg, c, FIRST ? 0.0f : best[i]);
    pre_ab[i] = float2{o.sa, o.sb};
    atomicAdd(&acc[0][lo], o.M);
    atomicAdd(&acc[1][lo], __builtin_fabs(o.M));
    atomicAdd(&acc[2][lo], __builtin_fabs(o.M) + o.M);
    atomicAdd(&acc[3][lo], (double)o.A * (double)o.A);
    atomicAdd(&acc[4][lo], (double)o.C);
    atomicMax(&amx[lo], f2u(o.A));  // A >= 0: float order is uint order
    if (!o.ok) atomicOr(&abad[lo], 1u);
    dmap[i] = (uint32_t)(g0 + lo);
  }
  __syncthreads();
  if (t >= n) return;
  const int64_t g = g0 + t;
  const int64_t off = boff[t];
  const int d = (int)(boff[t + 1] - off);
  const double sm = acc[0][t], sa = acc[1][t], sk = acc[2][t], s2 = acc[3][t], cs = acc[4][t];
  const double mx = (double)u2f(amx[t]);
  // the screening bound's block constants (round 4's k_small_fused, term for term)
  const double h_s = (double)d, h_e = (double)d / 8.0 + 8.0;
  const double gam = 1.01 * ((h_s > h_e ? h_s : h_e) + 1.0) * 0x1p-24;
  const double sl = (3.0 * gam + 0x1p-20) * (__builtin_fabs(sm) + sa + sk) + 0x1p-126;
  const float bf = round_up_f32(sm + cs * (1.0 + 0x1p-20) + sl);
  const float c1 = round_dn_f32(1.0 - 3.0 * gam - 0x1p-22);
  const float c2 = round_up_f32(1.0 + 3.0 * gam + 0x1p-14);
  const float as = round_dn_f32(sm - sl - 1.01 * s2 * (1.0 + 0x1p-11));
  const float pq = round_up_f32(2.01 * mx * __builtin_sqrt((double)(d > 0 ? d : 1)) *
                                (1.0 + 0x1p-11));
  const bool screen = abad[t] == 0u && d > 0 && d <= CWQ_FUSED_DMAX && as - as == 0.0f &&
                      pq - pq == 0.0f && bf - bf == 0.0f && mx - mx == 0.0;
  const PhiloxStream st = generate_key(step_seed(sd.of(g), step), 42);
  SmallRec r;
  r.q0 = uint4{(uint32_t)off, (uint32_t)((uint64_t)off >> 32), (uint32_t)d,
               d == 0 ? kQuadKnown : (screen ? kQuadListed : kQuadExact)};
  r.q1 = uint4{st.k0, st.k1, st.c2, st.c3};
  r.q2 = uint4{f2u(bf), f2u(c1), f2u(c2), f2u(as)};
  r.q3 = uint4{f2u(pq), 0u, 0u, 0u};
  rec[g] = r;
}

// The exact values of a block's listed rows (k_small_one), lane-parallel over
// (row, dim): each lane computes one normal exactly (its Philox block and the
// one Box-Muller pair holding it) and its log-density into lpv; a lane per row
// then sums in the Eigen order (eval_row's values bit for bit).  Returns the
// wave's best argmax key.  Out of line: its f64 Box-Muller constants would
// otherwise occupy k_small_one's registers for the whole kernel.
template <bool STEP0>
CWQ_RARE unsigned long long small_listed_exact(
    int64_t off, int db, const PhiloxStream sb, uint32_t used, const uint32_t* ln, float* lpv,
    const double* logtab, const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ loc_s, const float* __restrict__ scale_s,
    const float* __restrict__ lognorm, const float* __restrict__ best) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t du = (uint32_t)db;
  const uint32_t per = (uint32_t)CWQ_FUSED_STAGE / du;  // rows per batch (>= 1: d <= 64)
  uint64_t bestk = 0;
  for (uint32_t e0 = 0; e0 < used; e0 += per) {
    const uint32_t e1 = e0 + per < used ? e0 + per : used;
    const uint32_t i1 = (e1 - e0) * du;
    for (uint32_t it = lane; it < i1; it += 64) {
      const uint32_t e = e0 + it / du;
      const uint32_t j = it - (e - e0) * du;
      const int64_t ei = off + j;
      const float zz = exact_normal(sb, (uint64_t)ln[e] * (uint64_t)du + j, logtab);
      float sv = scale_s[ei] * zz;  // misc.py:14
      sv = loc_s[ei] + sv;          // misc.py:15
      const float tv = STEP0 ? sv : best[ei] + sv;  // :57
      lpv[it] = log_prob(tv, t_loc[ei], t_scale[ei], lognorm[ei]);
    }
    wave_lds_sync();
    const uint32_t e = e0 + lane;
    if (e < e1) {  // a lane per row: the Eigen-order sum (eval_row_f)
      const float* x = lpv + (e - e0) * du;
      const int vec = db & ~7;
      float p[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int jj = 0; jj < vec; jj += 8) {
#pragma unroll
        for (int l = 0; l < 8; ++l) p[l] = p[l] + x[jj + l];
      }
      float sum = 0.0f;
      for (int jj = vec; jj < db; ++jj) sum = sum + x[jj];
      const float r0 = p[0] + p[4], r1 = p[1] + p[5], r2 = p[2] + p[6], r3 = p[3] + p[7];
      const uint64_t k = argmax_key(sum + ((r0 + r2) + (r1 + r3)), ln[e]);
      bestk = k > bestk ? k : bestk;
    }
    wave_lds_sync();
  }
  return wave_max_u64(bestk);
}

// A wave (a 64-thread workgroup) per block: the screen (k_small_screen's spans)
// and the exact scoring of the listed rows; writes the index (out_idx).  The
// dispatcher hands a slot to the next wave as soon as one ends.  Measured
// alternatives on C2
// (tools/quad_times.py --one): persistent waves drawing blocks from one
// atomic counter, 474 us (41.5k same-address atomics serialise at ~11 ns);
// two blocks per wave in a loop, 69 us against 47 (the loop's spills), or
// as straight-line copies (2 or 4 blocks, 6-8 waves/SIMD): no gain on C2 or
// C3 (C3's scoring 1.11-1.20 ms per step in all five);
// longest blocks first (a counting sort by d), 41 us against 47 but the sort
// cost a launch and a histogram that needed zeroing.
template <bool STEP0>
__global__ void __launch_bounds__(64, CWQ_FUSED_WAVES) k_small_one(
    const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ loc_s, const float* __restrict__ scale_s,
    const float* __restrict__ lognorm, const float* __restrict__ best,
    const SmallRec* __restrict__ rec, const float2* __restrict__ pre_ab, int64_t nb, int64_t u0,
    int64_t n_cand, int32_t step, int n_steps, int32_t* __restrict__ out_idx) {
  __shared__ double logtab[32];
  // the block's (sA, sB) repeated 4 times: a lane's span of 4 rows is 4 d
  // normals, so Philox block b covers abx[4 b .. 4 b + 3] (two b128 reads,
  // issued ahead of the Philox rounds that hide their latency)
  __shared__ float4 abx[2 * CWQ_FUSED_DMAX];
  __shared__ uint32_t ln[CWQ_FUSED_LIST];
  __shared__ float lu[CWQ_FUSED_LIST];
  __shared__ float lpv[CWQ_FUSED_STAGE];
  __shared__ unsigned long long kmax;
  const uint32_t lane = threadIdx.x & 63u;
  if (lane < 32) logtab[lane] = kLogTabConst[lane];
  auto ufirst = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
  auto ffirst = [&](uint32_t v) { return u2f(ufirst(v)); };
  const int64_t g = u0 + blockIdx.x;
  {
#ifdef CWQ_QUAD_TIMES  // tools/quad_times.py --one: per block start, after the screen, end
    if (lane == 0u && g < kQuadTimes) g_quad_t[g][0] = __builtin_amdgcn_s_memrealtime();
#endif
    const uint4 q0 = rec[g].q0, q1 = rec[g].q1;
    const int64_t off = (int64_t)(((uint64_t)ufirst(q0.y) << 32) | ufirst(q0.x));
    const int db = (int)ufirst(q0.z);
    uint32_t state = ufirst(q0.w);
    PhiloxStream sb;
    sb.k0 = ufirst(q1.x);
    sb.k1 = ufirst(q1.y);
    sb.c2 = ufirst(q1.z);
    sb.c3 = ufirst(q1.w);
    uint32_t idx = 0u;
    uint32_t used = 0;
    if (lane == 0) kmax = 0ull;
    wave_lds_sync();
    if (state == kQuadListed) {
      const uint4 q2 = rec[g].q2;
      const float bfb = ffirst(q2.x), c1b = ffirst(q2.y), c2b = ffirst(q2.z);
      const float asb = ffirst(q2.w), pqb = ffirst(rec[g].q3.x);
      if ((int)lane < db) {  // d <= 64 (launch_small)
        const float2 e = pre_ab[off + lane];
        float2* ax = (float2*)abx;
        for (int r = 0; r < 4; ++r) ax[r * db + (int)lane] = e;
      }
      wave_lds_sync();
      const PhiloxLo K = philox_lo_key(sb);  // n_cand * d / 4 < 2^32 (d <= 64, < 4096 rows)
      float tau = -__builtin_inff();
      bool over = false;
      for (int64_t m0 = 0; 256 * m0 < n_cand; ++m0) {
        const int64_t ns = 4 * ((int64_t)lane + 64 * m0);
        const uint32_t b0 = (uint32_t)((uint64_t)ns * (uint64_t)db / 4u);
        float rs[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        float cur = 0.0f;
        int j = 0, qd = 0;
        for (int b = 0; b < db; ++b) {
          const float4 e01 = abx[2 * b], e23 = abx[2 * b + 1];
          const U4 x = philox10_lo(b0 + (uint32_t)b, K, sb.k0, sb.k1);
          float z[4];
          box_muller_screen(x.x, x.y, z[0], z[1]);
          box_muller_screen(x.z, x.w, z[2], z[3]);
          const float2 ev[4] = {float2{e01.x, e01.y}, float2{e01.z, e01.w},
                                float2{e23.x, e23.y}, float2{e23.z, e23.w}};
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) {
            const float2 e = ev[tt];  // = (sA, sB) of dim j
            const float a = __builtin_fmaf(e.x, z[tt], e.y);
            cur = __builtin_fmaf(-a, a, cur);
            if (++j == db) {  // wave-uniform: a row of the span is complete
              if (qd == 0) rs[0] = cur;
              else if (qd == 1) rs[1] = cur;
              else if (qd == 2) rs[2] = cur;
              else rs[3] = cur;
              cur = 0.0f;
              j = 0;
              ++qd;
            }
          }
        }
        // tau from the lane's best valid row (the lower bound is monotone in s)
        float smax = -__builtin_inff();
        bool any = false;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          if (ns + qq < n_cand) {
            smax = fmaxf(smax, rs[qq]);
            any = true;
          }
        const float lower = any ? __builtin_fmaf(smax, c2b, asb) -
                                      pqb * __builtin_amdgcn_sqrtf(-smax)
                                : -__builtin_inff();
        tau = fmaxf(tau, wave_max_f32(lower));
        uint64_t m[4];
        uint32_t cnt = 0;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          m[qq] = __ballot(ns + qq < n_cand && __builtin_fmaf(rs[qq], c1b, bfb) >= tau);
          cnt += (uint32_t)__builtin_popcountll(m[qq]);
        }
        if (cnt == 0) continue;
        if (used + cnt > CWQ_FUSED_LIST) {  // drop the rows the raised tau excludes
          const bool have = lane < used;
          const uint32_t nl = have ? ln[lane] : 0u;
          const float ul = have ? lu[lane] : 0.0f;
          const uint64_t keep = __ballot(have && ul >= tau);
          if ((keep >> lane) & 1ull) {
            const uint32_t r = lane_rank(keep);
            ln[r] = nl;
            lu[r] = ul;
          }
          used = (uint32_t)__builtin_popcountll(keep);
          wave_lds_sync();
        }
        if (used + cnt > CWQ_FUSED_LIST) {  // list full (near-ties): score the block exactly
          over = true;
          break;
        }
        uint32_t at = used;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const uint64_t mq = m[qq];
          if ((mq >> lane) & 1ull) {
            const uint32_t slot_i = at + lane_rank(mq);
            ln[slot_i] = (uint32_t)(ns + qq);
            lu[slot_i] = __builtin_fmaf(rs[qq], c1b, bfb);
          }
          at += (uint32_t)__builtin_popcountll(mq);
        }
        used = at;
        wave_lds_sync();
      }
      if (over) {
        state = kQuadExact;
        used = 0;
      } else {
        // keep the rows whose upper bound reaches the block's final tau
        const bool have = lane < used;
        const uint32_t nl = have ? ln[lane] : 0u;
        const uint64_t keep = __ballot(have && lu[have ? lane : 0] >= tau);
        const uint32_t nk = (uint32_t)__builtin_popcountll(keep);
        if (nk == 1u) {  // the single listed row is the argmax: no exact value needed
          idx = ufirst((uint32_t)__builtin_amdgcn_readlane((int)nl, __builtin_ctzll(keep)));
          state = kQuadKnown;
          used = 0;
        } else {
          if ((keep >> lane) & 1ull) ln[lane_rank(keep)] = nl;
          used = nk;
          if (nk == 0u) state = kQuadExact;  // (never: the best lower bound's row is listed)
        }
        wave_lds_sync();
      }
    }
#ifdef CWQ_QUAD_TIMES
    if (lane == 0u && g < kQuadTimes) {
      g_quad_t[g][1] = __builtin_amdgcn_s_memrealtime();
      g_quad_info[g][0] = (uint32_t)__builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
      g_quad_info[g][1] = (uint32_t)__builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));
      g_quad_info[g][2] = used;
      g_quad_info[g][3] = (state == kQuadExact ? 1u : 0u) | ((uint32_t)db << 8);
    }
#endif
    if (state == kQuadListed && used > 0) {  // rare (C2: 0.6% of the blocks): out of line
      const unsigned long long bk = small_listed_exact<STEP0>(
          off, db, sb, used, ln, lpv, logtab, t_loc, t_scale, loc_s, scale_s, lognorm, best);
      if (lane == 0) kmax = bk;
      wave_lds_sync();
    }
    if (state == kQuadExact) {  // every candidate exactly (constants outside the gate, list full)
      QuadBlk r;
      r.off = off;
      r.d = (uint32_t)db;
      r.k0 = sb.k0;
      r.k1 = sb.k1;
      r.c2 = sb.c2;
      r.c3 = sb.c3;
      const unsigned long long bk = quad_exact_block<STEP0>(r, t_loc, t_scale, loc_s, scale_s,
                                                             lognorm, best, n_cand, logtab);
      if (lane == 0) kmax = bk;
      wave_lds_sync();
    }
    if (state != kQuadKnown) {  // ArgMaxTupleReducer: a key at the clamp level is index 0
      const unsigned long long kb = kmax;
      idx = (kb >> 32) > kArgmaxClampOrd ? argmax_key_index(kb) : 0u;
    }
    if (lane == 0) out_idx[g * n_steps + step] = (int32_t)idx;
#ifdef CWQ_QUAD_TIMES
    if (lane == 0u && g < kQuadTimes)
      g_quad_t[g][2] = g_quad_t[g][3] = g_quad_t[g][4] = g_quad_t[g][5] =
          __builtin_amdgcn_s_memrealtime();
#endif
  }
}

// A thread per dim of [d0, d0 + n): best += the winning row of its block (:63)
template <bool STEP0>
__global__ void __launch_bounds__(256) k_small_finalize(
    const float* __restrict__ loc_s, const float* __restrict__ scale_s,
    const SmallRec* __restrict__ rec, const uint32_t* __restrict__ dmap,
    const int32_t* __restrict__ out_idx, int32_t step, int n_steps,
    const int64_t* __restrict__ block_off, int64_t ud, int64_t nb, float* __restrict__ best,
    float* __restrict__ ds_out, const float* __restrict__ ds_loc,
    const float* __restrict__ ds_scale) {
  __shared__ double logtab[32];
  fill_logtab(logtab);
  int64_t d0, d1;
  dims_of(block_off, ud, nb, d0, d1);
  for (int64_t i = d0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < d1;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t g = dmap[i];
    const uint4 q0 = rec[g].q0, q1 = rec[g].q1;
    const int64_t off = (int64_t)(((uint64_t)q0.y << 32) | q0.x);
    const uint32_t d = q0.z, j = (uint32_t)(i - off);
    const PhiloxStream st{q1.x, q1.y, q1.z, q1.w};
    const uint32_t idx = (uint32_t)out_idx[(int64_t)g * n_steps + step];  // k_small_one's
    const float zz = exact_normal(st, (uint64_t)idx * (uint64_t)d + j, logtab);
    float sv = scale_s[i] * zz;  // misc.py:14
    sv = loc_s[i] + sv;          // misc.py:15
    const float b = (STEP0 ? 0.0f : best[i]) + sv;
    best[i] = b;
    if (ds_out) {  // :292 destandardise (k_destandardise's arithmetic)
      const float m = ds_scale[i] * b;
      ds_out[i] = m + ds_loc[i];
    }
  }
}

// ---------------------------------------------------------------------------
// Encoder, end of a step: index -> out_idx; best += winning candidate (:63).
// General shapes (CSR groups, uniform d the float4 kernel does not take): one
// thread per flat dim i, which finds its block by binary search in block_off
// and regenerates its own word of the winning row; threads t < nb also write
// block t's index.  Work is spread evenly whatever the group sizes (a few
// 4095-dim groups or 10^5 tiny ones).  The dims covered are
// [block_off[0], block_off[nb]) (absolute: a forked part of a launch passes
// block_off + g0).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t block_of_dim(const int64_t* __restrict__ off, int64_t nb,
                                                int64_t i) {
  int64_t lo = 0, hi = nb;  // off[lo] <= i < off[hi]; empty blocks are skipped
  while (hi - lo > 1) {
    const int64_t m = (lo + hi) >> 1;
    if (off[m] <= i) lo = m; else hi = m;
  }
  return lo;
}

__device__ __forceinline__ uint32_t key_index(uint64_t key) {
  // ArgMaxTupleReducer starts at (index 0, lowest()) and only a value strictly
  // above lowest() replaces it: a winning key at the clamp level means index 0
  return (key >> 32) > kArgmaxClampOrd ? argmax_key_index(key) : 0u;
}

__global__ void __launch_bounds__(256) k_encode_finalize(
    const float* __restrict__ loc_s, const float* __restrict__ scale_s,
    const int64_t* __restrict__ block_off, int64_t ud, int64_t nb, SeedSpec sd, int32_t step,
    int n_steps,
    const unsigned long long* __restrict__ keys, int32_t* __restrict__ out_idx,
    float* __restrict__ out_sample) {
  __shared__ double logtab[32];
  fill_logtab(logtab);
  const int64_t d0 = block_off ? block_off[0] : 0;
  const int64_t d1 = block_off ? block_off[nb] : nb * ud;
  const int64_t nt = (d1 - d0) > nb ? (d1 - d0) : nb;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nt;
       t += (int64_t)gridDim.x * blockDim.x) {
    if (t < nb) out_idx[t * n_steps + step] = (int32_t)key_index(keys[t]);
    const int64_t i = d0 + t;
    if (i >= d1) continue;
    const int64_t g = block_off ? block_of_dim(block_off, nb, i) : i / ud;
    const int64_t off = block_off ? block_off[g] : g * ud;
    const int64_t d = block_off ? block_off[g + 1] - off : ud;
    const uint32_t idx = key_index(keys[g]);
    const PhiloxStream st =
        generate_key(step_seed(sd.of(g), step), 42);
    const uint64_t k = (uint64_t)idx * (uint64_t)d + (uint64_t)(i - off);
    const F4 z = normal4_dev(st, k >> 2, logtab);
    const uint32_t w = (uint32_t)(k & 3u);
    const float zz = w == 0 ? z.a : (w == 1 ? z.b : (w == 2 ? z.c : z.d));
    float sv = scale_s[i] * zz;
    sv = loc_s[i] + sv;
    out_sample[i] = out_sample[i] + sv;
  }
}

// Uniform blocks with d % 4 == 0, d <= 256: every row n*d starts on a Philox
// block, so one lane owns Philox block q of its block's winning row and with
// it dims 4q..4q+3 -- one Philox + two Box-Muller pairs per 4 dims, float4
// loads and stores.  A wave holds 64 / (d/4) whole blocks (lane -> (block,
// q) is fixed per lane: no 64-bit division in the loop); its chunks of blocks
// are strided over the grid's waves.
struct Q4Lane {
  bool active;
  uint32_t lb, q;  // block within the wave's chunk, Philox block within the row
};
__device__ __forceinline__ Q4Lane q4_lane(uint32_t qpb, uint32_t bpw) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lb = lane / qpb;
  return Q4Lane{lb < bpw, lb, lane - lb * qpb};
}

__global__ void __launch_bounds__(256) k_encode_finalize_q4(
    const float4* __restrict__ loc_s, const float4* __restrict__ scale_s, uint32_t qpb,
    uint32_t bpw, int64_t nb, SeedSpec sd, int32_t step, int n_steps,
    const unsigned long long* __restrict__ keys, int32_t* __restrict__ out_idx,
    float4* __restrict__ out_sample) {
  __shared__ double logtab[32];
  fill_logtab(logtab);
  const Q4Lane L = q4_lane(qpb, bpw);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t c = (int64_t)blockIdx.x * 4 + wave_id(); c * bpw < nb; c += nwaves) {
    const int64_t g = c * bpw + L.lb;
    if (!L.active || g >= nb) continue;
    const int64_t t = g * qpb + L.q;
    const uint64_t key = keys[g];
    const uint32_t idx = (key >> 32) > kArgmaxClampOrd ? argmax_key_index(key) : 0u;
    if (L.q == 0) out_idx[g * n_steps + step] = (int32_t)idx;
    const PhiloxStream st =
        generate_key(step_seed(sd.of(g), step), 42);
    const F4 z = normal4_dev(st, (uint64_t)idx * qpb + L.q, logtab);
    const float4 l = loc_s[t], sc = scale_s[t];
    float4 b = out_sample[t];
    float s;
    s = sc.x * z.a; s = l.x + s; b.x = b.x + s;
    s = sc.y * z.b; s = l.y + s; b.y = b.y + s;
    s = sc.z * z.c; s = l.z + s; b.z = b.z + s;
    s = sc.w * z.d; s = l.w + s; b.w = b.w + s;
    out_sample[t] = b;
  }
}

// ---------------------------------------------------------------------------
// Decoder (coded_greedy_sampler.py:93-167), O(n_steps * d) per block: only the
// selected row of each step is regenerated.  General shapes: one thread per
// flat dim, block found as in k_encode_finalize.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_decode(
    const int32_t* __restrict__ idx, const float* __restrict__ p_loc,
    const float* __restrict__ p_scale, const int64_t* __restrict__ block_off, int64_t ud,
    int64_t nb, int n_steps, int64_t n_cand, float nst, float sdiv, float rho, int32_t seed,
    int64_t block_id_base, float* __restrict__ out_sample) {
  __shared__ double logtab[32];
  fill_logtab(logtab);
  const int64_t d0 = block_off ? block_off[0] : 0;
  const int64_t d1 = block_off ? block_off[nb] : nb * ud;
  for (int64_t i = d0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < d1;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = block_off ? block_of_dim(block_off, nb, i) : i / ud;
    const int64_t off = block_off ? block_off[g] : g * ud;
    const int64_t d = block_off ? block_off[g + 1] - off : ud;
    const int32_t sg = block_seed(seed, block_id_base + g);
    const float ls = p_loc[i] / nst;
    const float rs = rho * p_scale[i];
    const float ss = rs / sdiv;
    float v = 0.0f;  // sample = tf.zeros (:143)
    for (int s = 0; s < n_steps; ++s) {
      const int64_t n = idx[g * n_steps + s];
      if (n < 0 || n >= n_cand) {
        v = __builtin_nanf("");
        continue;
      }
      const PhiloxStream st = generate_key(step_seed(sg, s), 42);
      const uint64_t k = (uint64_t)n * (uint64_t)d + (uint64_t)(i - off);
      const F4 z = normal4_dev(st, k >> 2, logtab);
      const uint32_t w = (uint32_t)(k & 3u);
      const float zz = w == 0 ? z.a : (w == 1 ? z.b : (w == 2 ? z.c : z.d));
      float sv = ss * zz;
      sv = ls + sv;
      v = v + sv;  // :153 tile(sample) + samples, row indices[i]
    }
    out_sample[i] = v;
  }
}

// Decoder for uniform blocks with d % 4 == 0, d <= 256 (the C4/C5 shapes):
// one lane per Philox block of the selected row -- dims 4q..4q+3 of block g,
// the same dims at every step because n*d is a multiple of 4 -- so each lane
// runs one Philox + two Box-Muller pairs per step, and p_loc / p_scale / the
// sample move as float4 (coalesced across the wave).  Lanes map to blocks as
// in k_encode_finalize_q4.  With n_steps == 1 the shard divisions are by 1.0f
// (exact identities; skipped on a uniform branch).
// A wave decodes a group of B = bpw * qpb blocks (<= 64) as qpb chunks of
// bpw blocks, one lane per Philox block of a row (float4 I/O, coalesced).
// Single-step codes: lane i computes the stream key of the group's block i
// once (TF GenerateKey is itself a Philox-10 call, as costly as a row's
// block) and each chunk takes its blocks' keys by lane shuffle, so a group
// pays one key call per block instead of one per lane.  The next chunk's
// inputs are loaded before the current chunk's arithmetic, so HBM reads stay
// in flight while the exact Box-Muller runs.
#ifndef CWQ_DECODE_MIN_WAVES
#define CWQ_DECODE_MIN_WAVES 1  // waves/SIMD the decoder's registers must allow (tuning)
#endif
#ifndef CWQ_DECODE_PROBE
#define CWQ_DECODE_PROBE 0  // tuning builds: 1 = loads/stores only, 2 = arithmetic only
#endif
#ifndef CWQ_DECODE_NT
#define CWQ_DECODE_NT 1  // non-temporal float4 streams: 3-4% faster on C4 (tools/decode_variants.sh)
#endif
__global__ void __launch_bounds__(256, CWQ_DECODE_MIN_WAVES) k_decode_q4(
    const int32_t* __restrict__ idx, const float4* __restrict__ p_loc,
    const float4* __restrict__ p_scale, uint32_t qpb, uint32_t bpw, int64_t nb, int n_steps,
    int64_t n_cand, float nst, float sdiv, float rho, int32_t seed, int64_t block_id_base,
    float4* __restrict__ out_sample) {
  __shared__ double logtab[32];
  fill_logtab(logtab);
  const Q4Lane L = q4_lane(qpb, bpw);
  const uint32_t lane = threadIdx.x & 63u;
  const int64_t B = (int64_t)bpw * qpb;
  const int64_t ngroups = (nb + B - 1) / B;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const bool unit = n_steps == 1;  // nst == sdiv == 1.0f
  for (int64_t grp = (int64_t)blockIdx.x * 4 + wave_id(); grp < ngroups; grp += nwaves) {
    const int64_t gb0 = grp * B;
    PhiloxStream kl{0u, 0u, 0u, 0u};
    if (unit)  // lanes past the group (or nb) compute an unused key
      kl = generate_key(step_seed(block_seed(seed, block_id_base + gb0 + lane), 0), 42);
    // chunk inputs: the current ones and the next chunk's, loaded one ahead
    float4 pl = float4{0.f, 0.f, 0.f, 0.f}, ps = pl;
    int32_t n1 = 0;  // single-step index
    auto load = [&](uint32_t j, float4& a, float4& b, int32_t& n) {
      const int64_t g = gb0 + (int64_t)(j * bpw + L.lb);
      if (CWQ_DECODE_PROBE == 2) {  // timing probe only: arithmetic without the loads
        a = float4{0.1f, 0.2f, 0.3f, (float)g};
        b = float4{1.0f, 1.1f, 1.2f, 1.3f};
        n = (int32_t)(g * 7919u) & 0xffff;
        return;
      }
      if (L.active && g < nb) {
        const int64_t t = g * qpb + L.q;
#if CWQ_DECODE_NT  // streamed once: non-temporal loads (tuning builds)
        typedef float nt4 __attribute__((ext_vector_type(4)));
        const nt4 va = __builtin_nontemporal_load(reinterpret_cast<const nt4*>(p_loc) + t);
        const nt4 vb = __builtin_nontemporal_load(reinterpret_cast<const nt4*>(p_scale) + t);
        a = float4{va.x, va.y, va.z, va.w};
        b = float4{vb.x, vb.y, vb.z, vb.w};
#else
        a = p_loc[t];
        b = p_scale[t];
#endif
        if (unit) n = idx[g];
      }
    };
    load(0u, pl, ps, n1);
    for (uint32_t j = 0; j < qpb; ++j) {
      const uint32_t src = j * bpw + L.lb;  // the lane holding this block's key
      const int64_t g = gb0 + (int64_t)src;
      const PhiloxStream ku{(uint32_t)__shfl((int)kl.k0, (int)src, 64),
                            (uint32_t)__shfl((int)kl.k1, (int)src, 64),
                            (uint32_t)__shfl((int)kl.c2, (int)src, 64),
                            (uint32_t)__shfl((int)kl.c3, (int)src, 64)};
      const float4 cl = pl, cs = ps;
      const int32_t cn = n1;
      if (j + 1 < qpb) load(j + 1, pl, ps, n1);
      if (!L.active || g >= nb) continue;
      float ls[4] = {cl.x, cl.y, cl.z, cl.w};
      float ss[4] = {rho * cs.x, rho * cs.y, rho * cs.z, rho * cs.w};
      if (!unit) {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          ls[w] = ls[w] / nst;
          ss[w] = ss[w] / sdiv;
        }
      }
      float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // sample = tf.zeros (:143)
      const int32_t sg = block_seed(seed, block_id_base + g);
      for (int i = 0; i < n_steps; ++i) {
        const int64_t n = unit ? (int64_t)cn : (int64_t)idx[g * n_steps + i];
        if (n < 0 || n >= n_cand) {
          v[0] = v[1] = v[2] = v[3] = __builtin_nanf("");
          continue;
        }
        const PhiloxStream st = unit ? ku : generate_key(step_seed(sg, i), 42);
#if CWQ_DECODE_PROBE == 1  // timing probe only: memory traffic without the arithmetic
        const F4 z{__builtin_bit_cast(float, st.k0 ^ (uint32_t)n), 1.0f, 1.0f, 1.0f};
#else
        const F4 z = normal4_dev(st, (uint64_t)n * qpb + L.q, logtab);
#endif
        const float zz[4] = {z.a, z.b, z.c, z.d};
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          float sv = ss[w] * zz[w];
          sv = ls[w] + sv;
          v[w] = v[w] + sv;  // :153 tile(sample) + samples, row indices[i]
        }
      }
#if CWQ_DECODE_NT
      typedef float nt4 __attribute__((ext_vector_type(4)));
      const nt4 vo = {v[0], v[1], v[2], v[3]};
      __builtin_nontemporal_store(vo, reinterpret_cast<nt4*>(out_sample) + g * qpb + L.q);
#else
      out_sample[g * qpb + L.q] = make_float4(v[0], v[1], v[2], v[3]);
#endif
    }
  }
}

// Single-step decode with the chunks' inputs streamed into LDS by LDS-DMA
// (global_load_lds, 16 B per lane; round 4).  The same group / chunk mapping
// as k_decode_q4, but chunk j + 2's p_loc / p_scale / index rows are in
// flight while chunk j's exact Box-Muller runs: the loads hold no VGPRs, so
// the ~90-VGPR arithmetic no longer caps how many are outstanding.  A ring of
// three slots per wave; a counted `s_waitcnt vmcnt` retires chunk j (the
// count covers only the younger chunks' loads, so the stores issued in
// between can only make it wait longer).  All LDS is one array (logf table
// first): a second __shared__ object makes hipcc wait vmcnt(0) before every
// LDS read (cdna_hip_programming.md, "three .s-level traps").
#ifndef CWQ_DECODE_GLDS
#define CWQ_DECODE_GLDS 1  // 0: the register-prefetch decoder for single-step codes too
#endif
#ifndef CWQ_GLDS_SLOTS
#define CWQ_GLDS_SLOTS 2  // ring slots per wave (chunks in flight: slots - 1)
#endif
constexpr int kGldsSlots = CWQ_GLDS_SLOTS;
static_assert(kGldsSlots == 2 || kGldsSlots == 3, "1 or 2 chunks ahead");
constexpr int kGldsSlot = 1024 + 1024 + 256;  // p_loc, p_scale (64 x 16 B), index (64 x 4 B)
#ifndef CWQ_GLDS_MIN_WAVES
#define CWQ_GLDS_MIN_WAVES 7  // 69 VGPRs, 2 x 2.3 KB ring per wave (tools/variants.sh glds*)
#endif
__global__ void __launch_bounds__(256, CWQ_GLDS_MIN_WAVES) k_decode_q4_glds(
    const int32_t* __restrict__ idx, const float4* __restrict__ p_loc,
    const float4* __restrict__ p_scale, uint32_t qpb, uint32_t bpw, int64_t nb, int64_t n_cand,
    float rho, int32_t seed, int64_t block_id_base, float4* __restrict__ out_sample) {
  __shared__ __attribute__((aligned(16))) char lds[256 + 4 * kGldsSlots * kGldsSlot];
  double* logtab = reinterpret_cast<double*>(lds);
  if (threadIdx.x < 32) logtab[threadIdx.x] = kLogTabConst[threadIdx.x];
  __syncthreads();
  const Q4Lane L = q4_lane(qpb, bpw);
  const uint32_t lane = threadIdx.x & 63u;
  char* ring = lds + 256 + wave_id() * (kGldsSlots * kGldsSlot);
  const int64_t B = (int64_t)bpw * qpb;
  const int64_t ngroups = (nb + B - 1) / B;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t grp = (int64_t)blockIdx.x * 4 + wave_id(); grp < ngroups; grp += nwaves) {
    const int64_t gb0 = grp * B;
    const PhiloxStream kl = generate_key(step_seed(block_seed(seed, block_id_base + gb0 + lane), 0), 42);
    const uint32_t J = qpb;
    // chunk j's rows: lane -> block gb0 + j bpw + lb, Philox block q (contiguous
    // float4s); lanes past nb or the group read row 0 (valid memory, unused)
    auto issue = [&](uint32_t j) {
      char* slot = ring + (j % kGldsSlots) * kGldsSlot;
      const int64_t g = gb0 + (int64_t)(j * bpw + L.lb);
      const bool ok = L.active && g < nb;
      const int64_t t = ok ? g * qpb + L.q : 0;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(p_loc + t),
                                       (__attribute__((address_space(3))) void*)(slot),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(p_scale + t),
                                       (__attribute__((address_space(3))) void*)(slot + 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(idx + (ok ? g : 0)),
                                       (__attribute__((address_space(3))) void*)(slot + 2048),
                                       4, 0, 0);
    };
    constexpr uint32_t kAhead = kGldsSlots - 1;
    for (uint32_t j = 0; j < kAhead && j < J; ++j) issue(j);
    for (uint32_t j = 0; j < J; ++j) {
      if (j + kAhead < J) issue(j + kAhead);
      // retire chunk j: at most the younger chunks' loads (3 each) may stay in flight
      const uint32_t younger = (J - 1 - j) < kAhead ? (J - 1 - j) : kAhead;
      if (younger >= 2)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (younger == 1)
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // the slot's rows by inline-asm LDS reads: hipcc would put a vmcnt(0)
      // (every chunk in flight) in front of ordinary reads of DMA-written LDS
      char* slot = ring + (j % kGldsSlots) * kGldsSlot;
      const uint32_t a16 =
          (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(slot) + lane * 16u;
      const uint32_t a4 =
          (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(slot + 2048) + lane * 4u;
      float4 cl, cs;
      int32_t n;
      asm volatile(
          "ds_read_b128 %0, %3\n\t"
          "ds_read_b128 %1, %3 offset:1024\n\t"
          "ds_read_b32 %2, %4\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(cl), "=&v"(cs), "=&v"(n)
          : "v"(a16), "v"(a4)
          : "memory");
      const uint32_t src = j * bpw + L.lb;  // the lane holding this block's key
      const PhiloxStream ku{(uint32_t)__shfl((int)kl.k0, (int)src, 64),
                            (uint32_t)__shfl((int)kl.k1, (int)src, 64),
                            (uint32_t)__shfl((int)kl.c2, (int)src, 64),
                            (uint32_t)__shfl((int)kl.c3, (int)src, 64)};
      const int64_t g = gb0 + (int64_t)src;
      if (L.active && g < nb) {
        float v[4];
        if (n < 0 || n >= n_cand) {
          v[0] = v[1] = v[2] = v[3] = __builtin_nanf("");
        } else {
          const F4 z = normal4_dev(ku, (uint64_t)n * qpb + L.q, logtab);
          const float zz[4] = {z.a, z.b, z.c, z.d};
          const float ls[4] = {cl.x, cl.y, cl.z, cl.w};
          const float ss[4] = {rho * cs.x, rho * cs.y, rho * cs.z, rho * cs.w};
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            float sv = ss[w] * zz[w];
            sv = ls[w] + sv;
            v[w] = 0.0f + sv;  // :153 tile(sample) + samples, from tf.zeros (:143)
          }
        }
        typedef float nt4 __attribute__((ext_vector_type(4)));
        const nt4 vo = {v[0], v[1], v[2], v[3]};
        __builtin_nontemporal_store(vo, reinterpret_cast<nt4*>(out_sample) + g * qpb + L.q);
      }
      // the slot is rewritten by issue(j + 3) next iteration: this wave's reads are done
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    }
  }
}

// ---------------------------------------------------------------------------
// misc.py:3-17 materialised: out[n*d+j] = loc[j] + scale[j] * (z*1 + 0).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_stateless_normal_sample(
    const float* __restrict__ loc, const float* __restrict__ scale, int64_t d, int64_t total,
    int32_t seed, float* __restrict__ out) {
  __shared__ double logtab[32];
  fill_logtab(logtab);
  const PhiloxStream st = generate_key(seed, 42);
  const int64_t ngrp = (total + 3) >> 2;
  for (int64_t G = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; G < ngrp;
       G += (int64_t)gridDim.x * blockDim.x) {
    const F4 z = normal4_dev(st, (uint64_t)G, logtab);
    const float zz[4] = {z.a, z.b, z.c, z.d};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int64_t f = 4 * G + w;
      if (f < total) {
        const int64_t j = f % d;
        const float r = zz[w] * 1.0f + 0.0f;  // rnd * stddev + mean
        const float s = scale[j] * r;
        out[f] = loc[j] + s;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Grouped-wrapper elementwise pieces.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_standardise(
    const float* __restrict__ q_loc, const float* __restrict__ q_scale,
    const float* __restrict__ p_loc, const float* __restrict__ p_scale, int64_t n,
    float* __restrict__ t_loc, float* __restrict__ t_scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float dl = q_loc[i] - p_loc[i];
    t_loc[i] = dl / p_scale[i];
    t_scale[i] = q_scale[i] / p_scale[i];
  }
}

__device__ __forceinline__ float kl_normal_normal_1(float a_loc, float a_scale, float b_loc,
                                                    float b_scale) {
  const float sa2 = a_scale * a_scale;
  const float sb2 = b_scale * b_scale;
  const float ratio = sa2 / sb2;
  const float dl = a_loc - b_loc;
  const float t1 = (dl * dl) / (2.0f * sb2);
  const float t2 = 0.5f * ((ratio - 1.0f) - logf_full(ratio, kLogTabConst));
  return t1 + t2;
}

__global__ void __launch_bounds__(256) k_kl_normal_normal(
    const float* __restrict__ a_loc, const float* __restrict__ a_scale,
    const float* __restrict__ b_loc, const float* __restrict__ b_scale, int64_t n,
    float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = kl_normal_normal_1(a_loc[i], a_scale[i], b_loc[i], b_scale[i]);
}

// The grouped coder's first launch (coded_greedy_sampler.py:193-201): the
// standardised target (k_standardise's expressions), the per-dim KL
// (k_kl_normal_normal's), the standard prior's zeros and ones, and zeroed
// partition counters (nz u64 at zinfo), in one pass over the inputs.
__global__ void __launch_bounds__(256) k_grouped_prep(
    const float* __restrict__ q_loc, const float* __restrict__ q_scale,
    const float* __restrict__ p_loc, const float* __restrict__ p_scale, int64_t n,
    float* __restrict__ t_loc, float* __restrict__ t_scale, float* __restrict__ kl,
    float* __restrict__ zeros, float* __restrict__ ones, unsigned long long* __restrict__ zinfo,
    int nz) {
  if (blockIdx.x == 0 && (int)threadIdx.x < nz) zinfo[threadIdx.x] = 0ull;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float ql = q_loc[i], qs = q_scale[i], pl = p_loc[i], ps = p_scale[i];
    const float dl = ql - pl;
    t_loc[i] = dl / ps;
    t_scale[i] = qs / ps;
    kl[i] = kl_normal_normal_1(ql, qs, pl, ps);
    zeros[i] = 0.0f;
    ones[i] = 1.0f;
  }
}

// The grouped importance coder's first launch (coded_importance_sampler.py:
// 137-148, 150, 160-163) in one pass: the standardised target (k_standardise's
// expressions), the per-dim KL (k_kl_normal_normal's) and the outlier test
// (k_imp_outliers': bits = kl / np.float32(log 2) <= limit, NaN an outlier,
// outliers standardised to N(0, 1)), the standard prior's zeros and ones, the
// KL of the (masked) standardised target against N(0, 1), which is what the
// partition and the plan read, and, for the outlier dims only, the target draw
// q_loc + q_scale z (:150; z element j of stateless_normal([1, D], [seed - 1,
// 42]), k_stateless_normal_sample's expressions).  A batch of
// items (item_off: device [n_items + 1], seed1: device [n_items] of
// seed - 1) numbers each item's dims from 0 in its own stream; item_off ==
// nullptr: one item with seed - 1 = seed1_one.
__global__ void __launch_bounds__(256) k_imp_grouped_prep(
    const float* __restrict__ q_loc, const float* __restrict__ q_scale,
    const float* __restrict__ p_loc, const float* __restrict__ p_scale, int64_t n, float limit,
    const int64_t* __restrict__ item_off, const int32_t* __restrict__ seed1, int64_t n_items,
    int32_t seed1_one, float* __restrict__ t_loc, float* __restrict__ t_scale,
    uint8_t* __restrict__ keep, float* __restrict__ zeros, float* __restrict__ ones,
    float* __restrict__ kl2, float* __restrict__ tsamp) {
  __shared__ double logtab[32];
  fill_logtab(logtab);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float ql = q_loc[i], qs = q_scale[i], pl = p_loc[i], ps = p_scale[i];
    const float dl = ql - pl;
    float tl = dl / ps;
    float ts = qs / ps;
    const float kl = kl_normal_normal_1(ql, qs, pl, ps);
    const float bits = kl / 0.6931472f;
    const bool k = bits <= limit;
    if (!k) {
      tl = 0.0f;
      ts = 1.0f;
      int64_t j = i;
      int32_t sd = seed1_one;
      if (item_off) {  // item of dim i: last it with item_off[it] <= i
        int64_t lo = 0, hi = n_items;
        while (hi - lo > 1) {
          const int64_t mid = (lo + hi) >> 1;
          if (item_off[mid] <= i) lo = mid; else hi = mid;
        }
        j = i - item_off[lo];
        sd = seed1[lo];
      }
      const F4 z = normal4_dev(generate_key(sd, 42), (uint64_t)j >> 2, logtab);
      const uint32_t w = (uint32_t)j & 3u;
      const float zz = w == 0 ? z.a : (w == 1 ? z.b : (w == 2 ? z.c : z.d));
      const float r = zz * 1.0f + 0.0f;  // rnd * stddev + mean
      const float sm = qs * r;           // misc.py:14
      tsamp[i] = ql + sm;                // misc.py:15
    }
    t_loc[i] = tl;
    t_scale[i] = ts;
    keep[i] = k ? 1 : 0;
    zeros[i] = 0.0f;
    ones[i] = 1.0f;
    kl2[i] = kl_normal_normal_1(tl, ts, 0.0f, 1.0f);
  }
}

__global__ void __launch_bounds__(256) k_destandardise(const float* sample,
                                                       const float* __restrict__ p_loc,
                                                       const float* __restrict__ p_scale,
                                                       int64_t n, float* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float m = p_scale[i] * sample[i];
    out[i] = m + p_loc[i];
  }
}

// ---------------------------------------------------------------------------
// Diagnostics: device transcendentals over explicit inputs.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_selftest_bm(uint32_t m0, int64_t count,
                                                     float* __restrict__ rad,
                                                     float* __restrict__ sn,
                                                     float* __restrict__ cs) {
  __shared__ double logtab[32];
  fill_logtab(logtab);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t m = m0 + (uint32_t)i;
    rad[i] = bm_radius_dev(m, logtab);
    float s, c;
    sincosf_pos(bm_angle_dev(m), s, c);
    sn[i] = s;
    cs[i] = c;
  }
}

__global__ void __launch_bounds__(256) k_selftest_screen(uint32_t m0, int64_t count,
                                                         float* __restrict__ rad,
                                                         float* __restrict__ sn,
                                                         float* __restrict__ cs) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t m = m0 + (uint32_t)i;
    rad[i] = bm_qradius_screen(m);  // r~ / sqrt(2 ln 2)
    float s, c;
    bm_sincos_screen(m, s, c);
    sn[i] = s;
    cs[i] = c;
  }
}

// out[w] = max over the 64 inputs of wave w (wave_max_f32, the DPP reduction
// the pruned kernel shares tau with)
__global__ void __launch_bounds__(256) k_selftest_wave_max(const float* __restrict__ x, int64_t nw,
                                                           float* __restrict__ out) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const float v = w < nw ? x[w * 64 + (threadIdx.x & 63)] : -__builtin_inff();
  const float m = wave_max_f32(v);
  if (w < nw && (threadIdx.x & 63) == 0) out[w] = m;
}

__global__ void __launch_bounds__(256) k_selftest_logf(const float* __restrict__ x, int64_t n,
                                                       float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = logf_full(x[i], kLogTabConst);
}

__global__ void __launch_bounds__(256) k_selftest_div(const float* __restrict__ a,
                                                      const float* __restrict__ b, int64_t n,
                                                      float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float y = 1.0f / b[i];
    out[i] = div_rn_markstein(a[i], b[i], y);
  }
}

// ---------------------------------------------------------------------------
// Host-side launchers.
// ---------------------------------------------------------------------------

static SeedSpec seeds_of(const EncodeArgs& a) {
  return SeedSpec{a.seed, a.block_id_base, a.seeds};
}

// The float4 lane-per-Philox-block kernels: uniform d % 4 == 0, d <= 256.
static bool q4_shape(const int64_t* block_off, int64_t ud) {
  return block_off == nullptr && ud > 0 && ud % 4 == 0 && ud <= 256;
}
// float4 access needs 16-byte aligned bases (callers may pass offset views)
static bool aligned16(const void* a, const void* b, const void* c) {
  return (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) & 15u) == 0;
}

hipError_t launch_prep_dims(const float* t_scale, const float* p_loc, const float* p_scale,
                            int64_t n, int n_steps, float rho, float* loc_s, float* scale_s,
                            float* lognorm, float* out_sample, unsigned long long* keys,
                            int64_t nb, hipStream_t stream) {
  if (n <= 0 && nb <= 0) return hipSuccess;
  const float nst = (float)n_steps;
  const float sdiv = (float)__builtin_sqrt((double)n_steps);
  hipLaunchKernelGGL(k_prep_dims, dim3(grid_for(n > nb ? n : nb, 256, 65536)), dim3(256), 0,
                     stream, t_scale, p_loc, p_scale, n, nst, sdiv, rho, loc_s, scale_s, lognorm,
                     out_sample, keys, nb);
  return hipGetLastError();
}

template <int DC, bool STEP0>
static void launch_eval_t(const EncodeArgs& a, int step, hipStream_t stream) {
  const int64_t ntiles = a.nb * a.tiles_per_block;
  const unsigned grid = (unsigned)(ntiles < (1LL << 30) ? ntiles : (1LL << 30));
  hipLaunchKernelGGL((k_encode_eval<DC, STEP0>), dim3(grid), dim3(256), 0, stream, a.t_loc,
                     a.t_scale, a.loc_s, a.scale_s, a.lognorm, a.out_sample, a.block_off, a.ud,
                     ntiles, a.tiles_per_block, a.cand_per_tile, a.n_cand, seeds_of(a),
                     step, a.keys);
}

template <int D, bool STEP0>
static void launch_prune_t(const EncodeArgs& a, int step, hipStream_t stream) {
  // grid of 256 CUs x 6 resident workgroups x 256; each workgroup loops over
  // its tiles (C4: 2.5 each).  Many more workgroups than resident slots keep
  // the SIMDs busy while a workgroup sets up its next tile: 1,536 (exactly
  // resident) was 15% slower on C4, 12,288 2%, 98,304 0.5%; one tile per
  // workgroup (1M) 0.5% (tools/variants.sh pg*)
#ifndef CWQ_PRUNE_GRID
#define CWQ_PRUNE_GRID (256 * 6 * 256)
#endif
  constexpr int64_t kPruneGrid = CWQ_PRUNE_GRID;
  const int64_t ntiles = a.nb * a.tiles_per_block;
#ifndef CWQ_TILE_INTERLEAVE
#define CWQ_TILE_INTERLEAVE 1
#endif
  // tau seeding: when a block spans several tiles, most of them
  // run at once and each would warm its threshold up from -inf.  A first launch
  // scores the block's first 2^CWQ_SEED_LOG2 candidates in small tiles; their
  // exact best keys land in keys[g], and every tile of the main launch starts
  // from that value (an actual row's exact value, so never above the block's
  // best).  The sample's rows are scored again by the main launch: its keys
  // are exact, so the final argmax is unchanged.
#ifndef CWQ_SEED_LOG2
#define CWQ_SEED_LOG2 0  // off: measured no gain
#endif
#ifndef CWQ_SEED_TILE
#define CWQ_SEED_TILE 4096
#endif
#ifndef CWQ_SEED_MIN_TPB
#define CWQ_SEED_MIN_TPB 2
#endif
  const int64_t seed_n = CWQ_SEED_LOG2 > 0 ? ((int64_t)1 << CWQ_SEED_LOG2) : 0;
  const bool seeded = CWQ_TILE_INTERLEAVE && seed_n > 0 && a.tiles_per_block >= CWQ_SEED_MIN_TPB &&
                      a.n_cand >= 4 * seed_n;
  if (seeded) {
    const int64_t cpt_s = seed_n < CWQ_SEED_TILE ? (seed_n > 0 ? seed_n : 1) : CWQ_SEED_TILE;
    const int64_t nt_s = a.nb * (seed_n / cpt_s);
    hipLaunchKernelGGL((k_encode_prune<D, STEP0, true>),
                       dim3((unsigned)(nt_s < kPruneGrid ? nt_s : kPruneGrid)), dim3(256), 0,
                       stream, a.t_loc, a.t_scale, a.loc_s, a.scale_s, a.lognorm, a.out_sample,
                       nt_s, seed_n / cpt_s, cpt_s, seed_n, seeds_of(a), step,
                       a.prune >= 2 ? 1 : 0, a.keys, seed_n / cpt_s, 1, nullptr);
  }
  // tile queue (k_encode_prune): a persistent grid of CWQ_QUEUE_GRID workgroups
  // draws tiles from a counter in the workspace, zeroed here before the launch
#ifndef CWQ_TILE_QUEUE
#define CWQ_TILE_QUEUE 1
#endif
#ifndef CWQ_QUEUE_GRID
#define CWQ_QUEUE_GRID 1536
#endif
  // Only for tiles of real work: with tiny tiles (C1: 16 candidates) the memset
  // and a counter round trip per tile cost more than the slots they keep busy
  // (C1 0.039 -> 0.065 ms with the queue)
#ifndef CWQ_QUEUE_MIN_CPT
#define CWQ_QUEUE_MIN_CPT 4096
#endif
  uint32_t* tq = nullptr;
  if (CWQ_TILE_QUEUE && a.tq != nullptr && ntiles < (1LL << 31) &&
      a.cand_per_tile >= CWQ_QUEUE_MIN_CPT && ntiles > CWQ_QUEUE_GRID) {
    if (hipMemsetAsync(a.tq, 0, sizeof(uint32_t), stream) == hipSuccess) tq = a.tq;
  }
  auto qgrid = [&](int64_t nt) -> unsigned {
    const int64_t cap = tq ? (int64_t)CWQ_QUEUE_GRID : kPruneGrid;
    return (unsigned)(nt < cap ? nt : cap);
  };
  if (CWQ_TILE_INTERLEAVE && (a.tiles_per_block > 1 || seeded)) {
    // tail: the last tile of each block's few last tiles split in CWQ_TAIL_SPLIT,
    // about two resident rounds (1,536 workgroups) of short tiles at the end
#ifndef CWQ_TAIL_SPLIT
#define CWQ_TAIL_SPLIT 4
#endif
    const int64_t tpb = a.tiles_per_block;
    int64_t from = tpb, div = 1;
    if (CWQ_TAIL_SPLIT > 1 && tpb >= 2 && a.cand_per_tile % (256 * CWQ_TAIL_SPLIT) == 0) {
      div = CWQ_TAIL_SPLIT;
      int64_t L = (2 * 1536 + div * a.nb - 1) / (div * a.nb);
      L = L < tpb / 2 ? L : tpb / 2;
      from = tpb - L;
    }
    const int64_t tpb2 = from + (tpb - from) * div;
    const int64_t nt2 = a.nb * tpb2;
    hipLaunchKernelGGL((k_encode_prune<D, STEP0, true>),
                       dim3(qgrid(nt2)), dim3(256), 0,
                       stream, a.t_loc, a.t_scale, a.loc_s, a.scale_s, a.lognorm, a.out_sample,
                       nt2, tpb2, a.cand_per_tile, a.n_cand, seeds_of(a), step,
                       a.prune >= 2 ? 1 : 0, a.keys, from, (int)div, tq);
  } else {
    hipLaunchKernelGGL((k_encode_prune<D, STEP0, false>), dim3(qgrid(ntiles)), dim3(256), 0,
                       stream, a.t_loc, a.t_scale, a.loc_s, a.scale_s, a.lognorm, a.out_sample,
                       ntiles, a.tiles_per_block, a.cand_per_tile, a.n_cand, seeds_of(a), step,
                       a.prune >= 2 ? 1 : 0, a.keys, a.tiles_per_block, 1, tq);
  }
}

template <bool STEP0>
static void launch_prune_csr(const EncodeArgs& a, int step, hipStream_t stream) {

  // own tiling: ~8192 tiles of >= 1024 candidates; tiles of a block share tau
  // through gtau, and later tiles start from it.  With few rows per lane (a
  // few large groups: the whole chip holds 1536 x 256 lanes) long rows are
  // walked cooperatively by 16 lanes instead, in tiles of >= 128 candidates.
  const int64_t kLanes = 1536 * 256;
  const int64_t rows = a.nb * a.n_cand;
  const bool coop = rows < CWQ_CSR_COOP_ROWS_PER_LANE * kLanes;
  int64_t tpb, max_tpb;
  if (coop) {
    tpb = (CWQ_CSR_COOP_TILES + a.nb - 1) / a.nb;
    max_tpb = a.n_cand / CWQ_CSR_COOP_TILE > 1 ? a.n_cand / CWQ_CSR_COOP_TILE : 1;
  } else {
    tpb = (CWQ_CSR_TILES + a.nb - 1) / a.nb;
    max_tpb = a.n_cand / CWQ_CSR_TILE > 1 ? a.n_cand / CWQ_CSR_TILE : 1;
  }
  tpb = tpb < max_tpb ? tpb : max_tpb;
  const int64_t cpt = (a.n_cand + tpb - 1) / tpb;
  tpb = (a.n_cand + cpt - 1) / cpt;  // no tile may start at or past n_cand
#if CWQ_COOP_CLASS_TILES
  // one-class tiles come in fours (the kernel skips a residue tile that gets
  // no row of a short last chunk)
  if (coop && tpb >= 4) tpb = (tpb + 3) & ~(int64_t)3;
#endif
  const int64_t ntiles = a.nb * tpb;
  const int64_t coop_min_d = coop ? (int64_t)CWQ_CSR_COOP_MIN_D : INT64_MAX;
#ifndef CWQ_PREP_SPLIT_MAX_NB
#define CWQ_PREP_SPLIT_MAX_NB 256
#endif
  // few blocks: one workgroup per class
  const unsigned cls_wgs = a.nb <= CWQ_PREP_SPLIT_MAX_NB ? 4 : 1;
  hipLaunchKernelGGL((k_csr_prep<STEP0>), dim3(grid_for(a.nb, 1, 65536), cls_wgs), dim3(256), 0,
                     stream, a.t_loc, a.t_scale, a.loc_s, a.scale_s, a.lognorm, a.out_sample,
                     a.block_off, a.ud, a.nb, a.sab, a.cdim, a.bpre, a.ordu, a.grp, a.gtau,
                     a.abp, (int64_t)CWQ_CSR_LDS_DIMS, coop_min_d);
  constexpr int64_t kGrid = 1 << 20;
  const unsigned grid = (unsigned)(ntiles < kGrid ? ntiles : kGrid);
  if (coop)
    hipLaunchKernelGGL((k_encode_prune_csr<STEP0, true>), dim3(grid), dim3(256), 0, stream,
                       a.t_loc, a.t_scale, a.loc_s, a.scale_s, a.lognorm, a.out_sample,
                       a.block_off, a.ud, ntiles, tpb, cpt, a.n_cand, seeds_of(a),
                       step, (const float2*)a.sab, (const float*)a.bpre,
                       (const uint32_t*)a.ordu, (const float4*)a.grp, a.gtau, a.keys,
                       coop_min_d, (const float4*)a.abp);
  else
    hipLaunchKernelGGL((k_encode_prune_csr<STEP0, false>), dim3(grid), dim3(256), 0, stream,
                       a.t_loc, a.t_scale, a.loc_s, a.scale_s, a.lognorm, a.out_sample,
                       a.block_off, a.ud, ntiles, tpb, cpt, a.n_cand, seeds_of(a),
                       step, (const float2*)a.sab, (const float*)a.bpre,
                       (const uint32_t*)a.ordu, (const float4*)a.grp, a.gtau, a.keys,
                       coop_min_d, (const float4*)a.abp);
}

#ifndef CWQ_SMALL_FUSED
#define CWQ_SMALL_FUSED 1  // 0: the three-kernel path for every block length (d <= 64 too)
#endif
// true: the launches also wrote the step's indices and sample (the small pipeline)
#ifndef CWQ_SMALL_PIPE
#define CWQ_SMALL_PIPE 1  // 0: the three-kernel path for these shapes too
#endif
// launch_eval_dc's choices, shared with launch_encode (which leaves step 0's
// prep to k_small_prep1 when the small pipeline runs)
static bool takes_uniform_pruned(const EncodeArgs& a) {
  // pruned path: uniform D % 8 == 0, D <= 64, Philox block index n*D/4 < 2^32
  return a.block_off == nullptr && a.prune && a.ud % 8 == 0 && a.ud >= 8 && a.ud <= 64 &&
         a.n_cand * (a.ud / 4) <= (1LL << 32);
}
static bool takes_small_path(const EncodeArgs& a) {  // launch_small's d <= 64 shapes
  return !takes_uniform_pruned(a) && !(a.prune >= 2 && a.sab != nullptr && a.n_cand >= 4096) &&
         a.prune >= 2 && a.sab != nullptr && a.slist != nullptr && a.ordu != nullptr &&
         a.n_cand >= CWQ_SMALL_MIN_CAND && CWQ_SMALL_FUSED && a.max_d >= 0 &&
         a.max_d <= CWQ_FUSED_DMAX && a.n_cand < 4096;
}
static bool small_pipe_ok(const EncodeArgs& a) {  // ... and the pipeline's arrays are there
  return a.sdmap && a.sab && a.slist && a.nb < (1LL << 32);
}
static bool takes_small_pipe(const EncodeArgs& a) {
  return CWQ_SMALL_PIPE && takes_small_path(a) && small_pipe_ok(a);
}

template <bool STEP0>
static bool launch_small(const EncodeArgs& a, int step, hipStream_t stream) {
  if (CWQ_SMALL_PIPE && CWQ_SMALL_FUSED && a.max_d >= 0 && a.max_d <= CWQ_FUSED_DMAX &&
      a.n_cand < 4096 && small_pipe_ok(a)) {
    // the small pipeline (k_small_*): constants, persistent screen, finalize
    SmallRec* rec = (SmallRec*)a.slist;
    float2* pab = const_cast<float2*>(a.pre_ab);  // by absolute dim (launch_encode)
    const float nst = (float)a.n_steps;
    const float sdiv = (float)__builtin_sqrt((double)a.n_steps);
    const unsigned pgrid = grid_for(a.nb, kSmallPrepBlocks, 1u << 31);
    if (STEP0)
      hipLaunchKernelGGL(k_small_prep1<true>, dim3(pgrid), dim3(CWQ_PREP1_THREADS), 0, stream, a.t_loc,
                         a.t_scale, a.p_loc, a.p_scale, nst, sdiv, a.rho, a.loc_s, a.scale_s,
                         a.lognorm, a.out_sample, a.block_off, a.ud, a.nb, seeds_of(a), step,
                         pab, rec, a.sdmap);
    else
      hipLaunchKernelGGL(k_small_prep1<false>, dim3(pgrid), dim3(CWQ_PREP1_THREADS), 0, stream, a.t_loc,
                         a.t_scale, a.p_loc, a.p_scale, nst, sdiv, a.rho, a.loc_s, a.scale_s,
                         a.lognorm, a.out_sample, a.block_off, a.ud, a.nb, seeds_of(a), step,
                         pab, rec, a.sdmap);
    const int64_t nu = a.nb;
    for (int64_t u0 = 0; u0 < nu; u0 += (int64_t)1 << 30)
      hipLaunchKernelGGL((k_small_one<STEP0>),
                         dim3((unsigned)(nu - u0 < (1LL << 30) ? nu - u0 : (1LL << 30))),
                         dim3(64), 0, stream, a.t_loc, a.t_scale, a.loc_s, a.scale_s, a.lognorm,
                         a.out_sample, rec, a.pre_ab, a.nb, u0, a.n_cand, step, a.n_steps,
                         a.out_idx);
    const unsigned dgrid = grid_for(a.total_dims > a.nb ? a.total_dims : a.nb, 256, 16384);
    hipLaunchKernelGGL((k_small_finalize<STEP0>), dim3(dgrid), dim3(256), 0, stream, a.loc_s,
                       a.scale_s, rec, a.sdmap, a.out_idx, step, a.n_steps, a.block_off, a.ud,
                       a.nb, a.out_sample, step == a.n_steps - 1 ? a.ds_out : nullptr, a.ds_loc,
                       a.ds_scale);
    return true;
  }
  const int64_t ntiles = a.nb * a.tiles_per_block;
  hipLaunchKernelGGL((k_small_prep<STEP0>), dim3(grid_for(a.nb, 4 * 64, 16384)), dim3(256), 0,
                     stream, a.t_loc, a.t_scale, a.loc_s, a.scale_s, a.lognorm, a.out_sample,
                     a.block_off, a.ud, a.nb, seeds_of(a), step, a.sab, a.bpre, a.grp, a.gtau,
                     a.ordu);
  hipLaunchKernelGGL((k_small_screen<STEP0>), dim3(grid_for(ntiles, 4, 1u << 20)),
                     dim3(256), 0, stream, a.block_off, a.ud, ntiles, a.tiles_per_block,
                     a.cand_per_tile, a.n_cand, seeds_of(a), step, (const float2*)a.sab,
                     (const float*)a.bpre, a.grp, a.gtau, a.ordu, a.slist);
  hipLaunchKernelGGL((k_small_survivors<STEP0>), dim3(grid_for(a.nb, 4 * 64, 4096)),
                     dim3(256), 0, stream, a.t_loc, a.t_scale, a.loc_s, a.scale_s, a.lognorm,
                     a.out_sample, a.block_off, a.ud, a.nb, a.n_cand, seeds_of(a), step,
                     (const float4*)a.grp, (const uint32_t*)a.gtau, (const uint32_t*)a.ordu,
                     (const uint2*)a.slist, (const float*)a.bpre, a.keys);
  return false;
}

// Scoring launches of one step; true when they also finalized it (indices and
// sample written), false when k_encode_finalize must follow.
template <bool STEP0>
static bool launch_eval_dc(const EncodeArgs& a, int step, hipStream_t stream) {
  if (takes_uniform_pruned(a)) {
    switch (a.ud) {
      case 8: return launch_prune_t<8, STEP0>(a, step, stream), false;
      case 16: return launch_prune_t<16, STEP0>(a, step, stream), false;
      case 24: return launch_prune_t<24, STEP0>(a, step, stream), false;
      case 32: return launch_prune_t<32, STEP0>(a, step, stream), false;
      case 40: return launch_prune_t<40, STEP0>(a, step, stream), false;
      case 48: return launch_prune_t<48, STEP0>(a, step, stream), false;
      case 56: return launch_prune_t<56, STEP0>(a, step, stream), false;
      case 64: return launch_prune_t<64, STEP0>(a, step, stream), false;
      default: break;
    }
  }
  // general pruned path (screening): CSR or other uniform d, >= 4096 candidates
  if (a.prune >= 2 && a.sab != nullptr && a.n_cand >= 4096)
    return launch_prune_csr<STEP0>(a, step, stream), false;
  // screened small-candidate path (k_small_*): few candidates per block
  if (a.prune >= 2 && a.sab != nullptr && a.slist != nullptr && a.ordu != nullptr &&
      a.n_cand >= CWQ_SMALL_MIN_CAND)
    return launch_small<STEP0>(a, step, stream);
  if (a.block_off == nullptr) {
    switch (a.ud) {
      case 8: return launch_eval_t<8, STEP0>(a, step, stream), false;
      case 16: return launch_eval_t<16, STEP0>(a, step, stream), false;
      case 32: return launch_eval_t<32, STEP0>(a, step, stream), false;
      default: break;
    }
  }
  launch_eval_t<0, STEP0>(a, step, stream);
  return false;
}

// The step loop of one block range on one stream: reset the argmax keys, score
// the candidates, finalize (index + best) -- steps are sequential per block.
static hipError_t encode_steps(const EncodeArgs& a, hipStream_t stream, bool events) {
  hipError_t e;
  // the general finalize covers max(nb, dims of this block range) threads
#ifndef CWQ_FIN_MAX_WGS
#define CWQ_FIN_MAX_WGS 16384
#endif
  const unsigned fgrid_dims =
      grid_for(a.total_dims > a.nb ? a.total_dims : a.nb, 256, CWQ_FIN_MAX_WGS);
  for (int s = 0; s < a.n_steps; ++s) {
    // step 0's keys were zeroed by k_prep_dims (launch_encode); the small
    // pipeline keeps its argmax in registers and LDS and never reads keys
    if (s > 0 && !takes_small_pipe(a) &&
        (e = hipMemsetAsync(a.keys, 0, (size_t)a.nb * sizeof(unsigned long long), stream)) !=
            hipSuccess)
      return e;
    if (events && s == 0 && a.ev_start) {
      e = hipEventRecord((hipEvent_t)a.ev_start, stream);
      if (e != hipSuccess) return e;
    }
    const bool finalized =
        s == 0 ? launch_eval_dc<true>(a, s, stream) : launch_eval_dc<false>(a, s, stream);
    if (events && s == a.n_steps - 1 && a.ev_stop) {
      e = hipEventRecord((hipEvent_t)a.ev_stop, stream);
      if (e != hipSuccess) return e;
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (finalized) continue;
    if (q4_shape(a.block_off, a.ud) && aligned16(a.loc_s, a.scale_s, a.out_sample)) {
      const uint32_t qpb = (uint32_t)(a.ud / 4), bpw = 64u / qpb;
      hipLaunchKernelGGL(k_encode_finalize_q4, dim3(grid_for(a.nb, 4 * (int64_t)bpw, 1u << 20)),
                         dim3(256), 0, stream, (const float4*)a.loc_s, (const float4*)a.scale_s,
                         qpb, bpw, a.nb, seeds_of(a), s, a.n_steps, a.keys,
                         a.out_idx, (float4*)a.out_sample);
    } else {
      hipLaunchKernelGGL(k_encode_finalize, dim3(fgrid_dims), dim3(256), 0, stream, a.loc_s,
                         a.scale_s, a.block_off, a.ud, a.nb, seeds_of(a), s,
                         a.n_steps, a.keys, a.out_idx, a.out_sample);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Two library streams per device (created once per host thread) onto which a
// multi-step CSR encode forks: the two halves of the block range run their
// step loops concurrently, so one half's end-of-step tail (the last tiles of
// a step, and the finalize/prep launches between steps) overlaps the other
// half's work.  Fork and join are events on the caller's stream, so the call
// stays stream-ordered (and capturable) for the caller.
#ifndef CWQ_ENCODE_SPLIT
#define CWQ_ENCODE_SPLIT 3  // most parts a multi-step CSR encode forks into
#endif
namespace {
constexpr int kMaxSplit = CWQ_ENCODE_SPLIT > 3 ? CWQ_ENCODE_SPLIT : 3;
constexpr int kMaxDevices = 16;
struct ForkStreams {
  bool ok = false;
  hipStream_t s[kMaxSplit] = {};
  hipStream_t cp[2] = {};  // copy streams of the pipelined batch coder (D2H, H2D)
  hipEvent_t fork = nullptr, join[kMaxSplit] = {};
  ~ForkStreams() {  // thread exit (the process's main thread: exit(), before HIP's teardown)
    if (!ok) return;
    for (int i = 0; i < kMaxSplit; ++i) {
      (void)hipStreamDestroy(s[i]);
      (void)hipEventDestroy(join[i]);
    }
    for (int i = 0; i < 2; ++i) (void)hipStreamDestroy(cp[i]);
    (void)hipEventDestroy(fork);
  }
};
thread_local ForkStreams tl_fork[kMaxDevices];
// The helper streams of the device the caller's stream belongs to (not the
// thread's current device: a caller may enqueue onto another GPU's stream).
ForkStreams* fork_streams(hipStream_t stream) {
  int dev = 0;
  if (hipStreamGetDevice(stream, &dev) != hipSuccess || dev < 0 || dev >= kMaxDevices)
    return nullptr;
  ForkStreams& f = tl_fork[dev];
  if (!f.ok) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    bool good = true;
    int made_s = 0, made_e = 0, made_c = 0;
    for (int i = 0; i < kMaxSplit && good; ++i) {
      good = hipStreamCreateWithFlags(&f.s[i], hipStreamNonBlocking) == hipSuccess;
      made_s += good;
      good = good && hipEventCreateWithFlags(&f.join[i], hipEventDisableTiming) == hipSuccess;
      made_e += good;
    }
    for (int i = 0; i < 2 && good; ++i) {
      good = hipStreamCreateWithFlags(&f.cp[i], hipStreamNonBlocking) == hipSuccess;
      made_c += good;
    }
    good = good && hipEventCreateWithFlags(&f.fork, hipEventDisableTiming) == hipSuccess;
    if (!good) {  // nothing half-made stays behind; the caller runs unsplit
      for (int i = 0; i < made_s; ++i) (void)hipStreamDestroy(f.s[i]);
      for (int i = 0; i < made_e; ++i) (void)hipEventDestroy(f.join[i]);
      for (int i = 0; i < made_c; ++i) (void)hipStreamDestroy(f.cp[i]);
    }
    if (cur != dev) (void)hipSetDevice(cur);
    if (!good) return nullptr;
    f.ok = true;
  }
  return &f;
}
}  // namespace

hipStream_t copy_stream(hipStream_t stream, int which) {
  ForkStreams* f = fork_streams(stream);
  return f && which >= 0 && which < 2 ? f->cp[which] : nullptr;
}

hipError_t launch_encode(const EncodeArgs& a_in, hipStream_t stream) {
  hipError_t e;
  EncodeArgs a = a_in;
  // the small pipeline's per-dim screening constants, by absolute dim offset: a
  // view of sab (the other paths' scratch) taken before a fork shifts it per part
  a.pre_ab = a.sab;
  if (takes_small_pipe(a))
    e = hipSuccess;  // its step 0 does k_prep_dims' work in k_small_prep1
  else
    e = launch_prep_dims(a.t_scale, a.p_loc, a.p_scale, a.total_dims, a.n_steps, a.rho, a.loc_s,
                         a.scale_s, a.lognorm, a.out_sample, a.keys, a.nb, stream);
  if (e != hipSuccess) return e;
  if (a.nb == 0) return hipSuccess;
  // :292 destandardise after the last step: the small pipeline's finalize
  // does it, anything else one k_destandardise on the caller's stream
  const bool ds_after = a.ds_out != nullptr && !takes_small_pipe(a);
  auto ds = [&]() -> hipError_t {
    if (!ds_after) return hipSuccess;
    return launch_destandardise(a.out_sample, a.ds_loc, a.ds_scale, a.total_dims, a.ds_out,
                                stream);
  };
  ForkStreams* f = (CWQ_ENCODE_SPLIT > 1 && a.block_off != nullptr && a.n_steps > 1 &&
                    a.nb >= 2)
                       ? fork_streams(stream)
                       : nullptr;
  if (f == nullptr) {
    if ((e = encode_steps(a, stream, true)) != hipSuccess) return e;
    return ds();
  }
  // k parts of the block range: block-indexed arrays move by g0, the padded
  // per-block regions of the general kernel by 8 g0 / 12 g0 (their layout is
  // off + 8 g / off + 12 g with absolute dim offsets off).  Launches of few
  // long rows (the cooperative mode) overlap best in three parts, others in two
  // (tools/stream_overlap.py).
  const bool few_rows = a.nb * a.n_cand < (int64_t)CWQ_CSR_COOP_ROWS_PER_LANE * 1536 * 256;
#ifndef CWQ_SPLIT_FEW
#define CWQ_SPLIT_FEW 3  // parts of a cooperative (few long rows) launch
#endif
  int k = few_rows ? CWQ_SPLIT_FEW : 2;
  k = k < CWQ_ENCODE_SPLIT ? k : CWQ_ENCODE_SPLIT;
  k = (int64_t)k < a.nb ? k : (int)a.nb;
  if (a.ev_start && (e = hipEventRecord((hipEvent_t)a.ev_start, stream)) != hipSuccess) return e;
  if ((e = hipEventRecord(f->fork, stream)) != hipSuccess) return e;
  int forked = 0;
  for (int i = 0; i < k && e == hipSuccess; ++i) {
    const int64_t g0 = a.nb * i / k, g1 = a.nb * (i + 1) / k;
    EncodeArgs p = a;
    p.block_off = a.block_off + g0;
    p.nb = g1 - g0;
    p.block_id_base = a.block_id_base + g0;
    if (a.seeds) p.seeds = a.seeds + g0;
    p.keys = a.keys + g0;
    if (a.tq) p.tq = a.tq + i;  // its own tile queue counter
    p.out_idx = a.out_idx + g0 * a.n_steps;
    if (a.sab) p.sab = a.sab + 8 * g0;
    if (a.bpre) p.bpre = a.bpre + 12 * g0;
    if (a.ordu) p.ordu = a.ordu + 12 * g0;
    if (a.grp) p.grp = a.grp + g0;
    if (a.gtau) p.gtau = a.gtau + g0 * CWQ_CSR_GTAU_STRIDE;
    // abp is indexed by absolute dim offset alone (csr_rec_base): unshifted
    if (a.slist) p.slist = a.slist + CWQ_SLIST_PER_BLOCK * g0;
    // sdmap is indexed by absolute dim offset (its values: the part's block numbers)
    if ((e = hipStreamWaitEvent(f->s[i], f->fork, 0)) != hipSuccess) break;
    forked = i + 1;
    e = encode_steps(p, f->s[i], false);
  }
  // join every stream that was forked, also after an error: the caller's
  // stream must not run ahead of (or free buffers under) work already queued
  for (int i = 0; i < forked; ++i) {
    hipError_t ej = hipEventRecord(f->join[i], f->s[i]);
    if (ej == hipSuccess) ej = hipStreamWaitEvent(stream, f->join[i], 0);
    if (ej != hipSuccess) {
      (void)hipStreamSynchronize(f->s[i]);  // last resort: drain it on the host
      if (e == hipSuccess) e = ej;
    }
  }
  if (e != hipSuccess) return e;
  if (a.ev_stop && (e = hipEventRecord((hipEvent_t)a.ev_stop, stream)) != hipSuccess) return e;
  return ds();
}

hipError_t launch_decode(const int32_t* idx, const float* p_loc, const float* p_scale,
                         const int64_t* block_off, int64_t ud, int64_t nb, int64_t total_dims,
                         int n_bits,
                         int n_steps, int32_t seed, float rho, int64_t block_id_base,
                         float* out_sample, hipStream_t stream) {
  if (nb <= 0) return hipSuccess;
  const float nst = (float)n_steps;
  const float sdiv = (float)__builtin_sqrt((double)n_steps);
  if (q4_shape(block_off, ud) && aligned16(p_loc, p_scale, out_sample)) {
    const uint32_t qpb = (uint32_t)(ud / 4), bpw = 64u / qpb;
    const int64_t ngroups = (nb + (int64_t)bpw * qpb - 1) / ((int64_t)bpw * qpb);
    if (CWQ_DECODE_GLDS && n_steps == 1) {
      hipLaunchKernelGGL(k_decode_q4_glds, dim3(grid_for(ngroups, 4, 1u << 20)), dim3(256), 0,
                         stream, idx, (const float4*)p_loc, (const float4*)p_scale, qpb, bpw, nb,
                         (int64_t)1 << n_bits, rho, seed, block_id_base, (float4*)out_sample);
      return hipGetLastError();
    }
    hipLaunchKernelGGL(k_decode_q4, dim3(grid_for(ngroups, 4, 1u << 20)), dim3(256), 0,
                       stream, idx, (const float4*)p_loc, (const float4*)p_scale, qpb, bpw, nb,
                       n_steps, (int64_t)1 << n_bits, nst, sdiv, rho, seed, block_id_base,
                       (float4*)out_sample);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_decode, dim3(grid_for(total_dims, 256, 16384)), dim3(256), 0, stream, idx,
                     p_loc, p_scale, block_off, ud, nb, n_steps, (int64_t)1 << n_bits, nst, sdiv,
                     rho, seed, block_id_base, out_sample);
  return hipGetLastError();
}

hipError_t launch_stateless_normal_sample(const float* loc, const float* scale, int64_t d,
                                          int64_t num_samples, int32_t seed, float* out,
                                          hipStream_t stream) {
  const int64_t total = d * num_samples;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_stateless_normal_sample, dim3(grid_for((total + 3) / 4, 256, 65536)),
                     dim3(256), 0, stream, loc, scale, d, total, seed, out);
  return hipGetLastError();
}

hipError_t launch_standardise(const float* q_loc, const float* q_scale, const float* p_loc,
                              const float* p_scale, int64_t n, float* t_loc, float* t_scale,
                              hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_standardise, dim3(grid_for(n, 256, 65536)), dim3(256), 0, stream, q_loc,
                     q_scale, p_loc, p_scale, n, t_loc, t_scale);
  return hipGetLastError();
}

hipError_t launch_kl(const float* q_loc, const float* q_scale, const float* p_loc,
                     const float* p_scale, int64_t n, float* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_kl_normal_normal, dim3(grid_for(n, 256, 65536)), dim3(256), 0, stream,
                     q_loc, q_scale, p_loc, p_scale, n, out);
  return hipGetLastError();
}

hipError_t launch_grouped_prep(const float* q_loc, const float* q_scale, const float* p_loc,
                               const float* p_scale, int64_t n, float* t_loc, float* t_scale,
                               float* kl, float* zeros, float* ones, unsigned long long* zinfo,
                               int nz, hipStream_t stream) {
  if (n <= 0 && nz <= 0) return hipSuccess;
  if (nz < 0 || nz > 256 || (nz > 0 && !zinfo)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_grouped_prep, dim3(n > 0 ? grid_for(n, 256, 65536) : 1u), dim3(256), 0,
                     stream, q_loc, q_scale, p_loc, p_scale, n, t_loc, t_scale, kl, zeros, ones,
                     zinfo, nz);
  return hipGetLastError();
}

hipError_t launch_imp_grouped_prep(const float* q_loc, const float* q_scale, const float* p_loc,
                                   const float* p_scale, int64_t n, float limit,
                                   const int64_t* item_off, const int32_t* seed1, int64_t n_items,
                                   int32_t seed1_one, float* t_loc, float* t_scale, uint8_t* keep,
                                   float* zeros, float* ones, float* kl2, float* tsamp,
                                   hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_imp_grouped_prep, dim3(grid_for(n, 256, 65536)), dim3(256), 0, stream,
                     q_loc, q_scale, p_loc, p_scale, n, limit, item_off, seed1, n_items, seed1_one,
                     t_loc, t_scale, keep, zeros, ones, kl2, tsamp);
  return hipGetLastError();
}

hipError_t launch_destandardise(const float* sample, const float* p_loc, const float* p_scale,
                                int64_t n, float* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_destandardise, dim3(grid_for(n, 256, 65536)), dim3(256), 0, stream,
                     sample, p_loc, p_scale, n, out);
  return hipGetLastError();
}

hipError_t launch_selftest_bm(uint32_t m0, int64_t count, float* rad, float* sn, float* cs,
                              hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_selftest_bm, dim3(grid_for(count, 256, 65536)), dim3(256), 0, stream, m0,
                     count, rad, sn, cs);
  return hipGetLastError();
}

hipError_t launch_selftest_screen(uint32_t m0, int64_t count, float* rad, float* sn, float* cs,
                                  hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_selftest_screen, dim3(grid_for(count, 256, 65536)), dim3(256), 0, stream,
                     m0, count, rad, sn, cs);
  return hipGetLastError();
}

int tile_times(unsigned long long* t0, unsigned long long* t1, unsigned int* wg, int n) {
#ifdef CWQ_TILE_TIMES
  if (n > kTileTimes) n = kTileTimes;
  if (hipMemcpyFromSymbol(t0, HIP_SYMBOL(g_tile_t0), (size_t)n * 8) != hipSuccess ||
      hipMemcpyFromSymbol(t1, HIP_SYMBOL(g_tile_t1), (size_t)n * 8) != hipSuccess ||
      hipMemcpyFromSymbol(wg, HIP_SYMBOL(g_tile_wg), (size_t)n * 4) != hipSuccess)
    return -1;
  return n;
#else
  (void)t0; (void)t1; (void)wg; (void)n;
  return 0;
#endif
}

int quad_times(unsigned long long* t, unsigned int* info, int n) {
#ifdef CWQ_QUAD_TIMES
  if (n > kQuadTimes) n = kQuadTimes;
  if (hipMemcpyFromSymbol(t, HIP_SYMBOL(g_quad_t), (size_t)n * 6 * 8) != hipSuccess ||
      hipMemcpyFromSymbol(info, HIP_SYMBOL(g_quad_info), (size_t)n * 4 * 4) != hipSuccess)
    return -1;
  return n;
#else
  (void)t; (void)info; (void)n;
  return 0;
#endif
}

int prune_stats(unsigned long long* out72, int reset) {
#ifdef CWQ_PRUNE_STATS
  if (hipMemcpyFromSymbol(out72, HIP_SYMBOL(g_prune_stats), sizeof(unsigned long long) * 72) !=
      hipSuccess)
    return -1;
  if (reset & 6) {
    const int v = (reset & 2) ? 1 : 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_seed_tau), &v, sizeof(int)) != hipSuccess) return -1;
  }
  if (reset & 1) {
    static const unsigned long long zero[72] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prune_stats), zero, sizeof(zero)) != hipSuccess) return -1;
  }
  return 1;
#else
  for (int i = 0; i < 72; ++i) out72[i] = 0;
  (void)reset;
  return 0;
#endif
}

hipError_t launch_selftest_wave_max(const float* x, int64_t nw, float* out, hipStream_t stream) {
  if (nw <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_selftest_wave_max, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, stream, x,
                     nw, out);
  return hipGetLastError();
}

hipError_t launch_selftest_div(const float* a, const float* b, int64_t n, float* out,
                               hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_selftest_div, dim3(grid_for(n, 256, 65536)), dim3(256), 0, stream, a, b, n,
                     out);
  return hipGetLastError();
}

hipError_t launch_selftest_logf(const float* x, int64_t n, float* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_selftest_logf, dim3(grid_for(n, 256, 65536)), dim3(256), 0, stream, x, n,
                     out);
  return hipGetLastError();
}

}  // namespace cwq
