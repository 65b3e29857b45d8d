// cwq_partition.hip -- the grouped coder's greedy partition on the device
// (coded_greedy_sampler.py:223-252), bit-identical to the sequential loop.
//
// The loop walks the dims once, carrying (float32 group KL, group size), and
// starts a group at idx when size >= size_threshold, or kl + kl[idx] >= the
// threshold, or idx == D - 1.  The carried state restarts at every group
// start, so the loop is a walk through the functional graph
//     nxt(i) = the next start after a start at i
// from node 0: the starts are 0, nxt(0), nxt(nxt(0)), ... up to D - 1 (always a
// start), preceded by the reference's [0] and, when dim 0 alone already trips
// the test ("dup"), a second 0 (an empty first group).  The launches:
//   k_part_next   every nxt(i) (a thread per dim scanning forward; a scan
//                 longer than kPartMaxJump dims marks the input "long" and
//                 the caller partitions on the host);
//   k_part_exit   per chunk of kPartW dims: for every dim i of the chunk
//                 ex(i) = the first node at or past the chunk's end on the
//                 walk from i (pointer jumping in LDS).  The walk enters chunk
//                 c at some node within [b_c, M_c], M_c the farthest nxt(s)
//                 of a dim s before b_c; when every candidate entry leads to
//                 the same exit the chunk is "converged" and its exit does not
//                 depend on which one it is (walks merge at a shared start);
//   k_part_mark   per chunk: its entry (the exit of the nearest converged
//                 chunk before it, followed through at most kPartRun others
//                 by their stored ex of the entry), then the walk's nodes in
//                 the chunk marked by pointer jumping in LDS, counted and
//                 compacted;
//   k_part_emit   per chunk: the global rank of its first node (the sum of
//                 the earlier chunks' counts; past kPartDirect chunks the
//                 earlier superchunks' sums from k_part_sup plus the earlier
//                 chunks of its own superchunk of kPartSuper, so the total
//                 work stays linear in the chunk count), the walk's nodes in
//                 rank order (one
//                 item: straight into its start list, with its largest group,
//                 and the two launches below are skipped);
//   k_part_ihdr / k_part_ibody  per item: its nodes (a rank range found by
//                 binary search) as its own start list, group count and
//                 largest group.
// Several items (the batch coder's latent sets) are one walk: an item's last
// dim is a forced start whose group is that dim alone, so nxt of it is the
// next item's first dim, which is therefore on the walk too.
// Inputs the scheme does not cover (a group longer than kPartMaxJump, walks
// that do not merge within kPartRun chunks) set info[2]; the caller then runs
// the host loop, so the result never depends on which path ran.
// ---------------------------------------------------------------------------
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cwq_kernels.h"

namespace cwq {

#ifndef CWQ_PART_UNROLL
#define CWQ_PART_UNROLL 4  // k_part_next's dims per threshold test (C3: 51 -> 44.5 us)
#endif
constexpr int kPartW = 1024;        // dims per chunk
constexpr int kPartMaxJump = 512;   // longest group the device path takes
constexpr int kPartRun = 8;         // non-converged chunks a walk may cross
constexpr int kPartThreads = 256;
constexpr int kPartLdsItems = 1024;  // batches up to this many items search offsets in LDS
constexpr int kPartSuper = 256;      // chunks per superchunk (k_part_sup's sums)
// up to this many chunks k_part_emit sums the earlier counts directly (at most
// 64 loads per thread; C3's 4,660 chunks: 18): an atomic per chunk into the
// superchunk sums instead cost C3's k_part_mark 33 us (37 -> 70 us)
constexpr int64_t kPartDirect = 16384;

// info[0] nodes on the walk, info[2] fallback flag, info[4] a jump nxt(i) - i
// above kPartMaxJump (the fallback; 0 when there is none).  Per item k: iinfo[2k] its starts (G + 1),
// iinfo[2k + 1] its largest group.
__device__ __forceinline__ int64_t item_end(const int64_t* __restrict__ item_off, int64_t n_items,
                                            int64_t D, int64_t i) {
  if (!item_off) return D;
  int64_t lo = 0, hi = n_items;  // item_off[lo] <= i < item_off[hi]
  while (hi - lo > 1) {
    const int64_t m = (lo + hi) >> 1;
    if (item_off[m] <= i) lo = m; else hi = m;
  }
  // empty items share their offset with the next one: skip to the last match
  return item_off[hi];
}

template <class T>
__device__ __forceinline__ T block_max(T v, T* red);

__global__ void __launch_bounds__(256) k_part_next(const float* __restrict__ kl, int64_t D,
                                                   const int64_t* __restrict__ item_off,
                                                   int64_t n_items, int64_t T, float thr,
                                                   int32_t* __restrict__ nxt,
                                                   unsigned long long* __restrict__ info) {
  __shared__ int32_t red[256];
  // the workgroup's 256 dims and the kPartMaxJump after them, staged in LDS
  // (coalesced): each thread's scan then reads LDS instead of a chain of
  // dependent global loads (C3's 9.6M dims: 72 us -> a few)
  __shared__ float skl[256 + kPartMaxJump + 1];
  __shared__ int64_t soff[kPartLdsItems + 1];
  const int64_t b = (int64_t)blockIdx.x * blockDim.x;
  const int64_t i = b + threadIdx.x;
  for (int t = threadIdx.x; t < 256 + kPartMaxJump + 1; t += 256)
    skl[t] = b + t < D ? kl[b + t] : 0.0f;
  // a batch's item offsets in LDS too (the binary search per dim is a chain of
  // dependent loads: 66 us of C3's 9.6M dims from global memory)
  const bool lds_off = item_off && n_items <= kPartLdsItems;
  if (lds_off)
    for (int t = threadIdx.x; t <= n_items; t += 256) soff[t] = item_off[t];
  __syncthreads();
  int32_t jump = 0;
  if (i < D) {
    const int64_t iend = item_end(lds_off ? soff : item_off, n_items, D, i);
    // the loop from a start at i (kl[i], size 1) accepts dim i + k while the
    // float32 running sum stays below the threshold (:233, :243), and stops at
    // size T (size == k), at the item's last dim (a forced start, :234), or one
    // past kPartMaxJump (longer than the device path takes: the fallback).
    // Folding those three limits into klim leaves one add and one compare per
    // dim (C3's low-KL stretches scan hundreds of dims from every start).
    int32_t k = 1;
    if (i < iend - 1) {
      int64_t klim = iend - 1 - i;
      klim = klim < T ? klim : T;
      klim = klim < kPartMaxJump + 1 ? klim : kPartMaxJump + 1;
      const int32_t kl32 = (int32_t)klim;
      const float* row = skl + (i - b);  // row[k] = kl[i + k]; i + k - b <= 255 + 512
      float cur = row[0];
      // CWQ_PART_UNROLL dims per test while none of them trips it (the same
      // running sums); the dims from the first test that trips are redone one
      // by one
      for (; k + CWQ_PART_UNROLL - 1 < kl32; k += CWQ_PART_UNROLL) {
        float sv = cur;
        bool trip = false;
#pragma unroll
        for (int u = 0; u < CWQ_PART_UNROLL; ++u) {
          sv = sv + row[k + u];
          trip |= sv >= thr;
        }
        if (trip) break;
        cur = sv;
      }
      for (; k < kl32; ++k) {
        const float s = cur + row[k];
        if (s >= thr) break;
        cur = s;
      }
    }  // i == iend - 1: the item's last group is that dim; the walk goes on at iend
    jump = k;  // > kPartMaxJump: not covered
    nxt[i] = (int32_t)(i + k);
  }
  const int32_t mj = block_max(jump, red);  // one atomic per workgroup
  // only a jump past kPartMaxJump matters (the fallback): an atomic from every
  // workgroup on one address serialised C3's 37.6k workgroups (~60 us)
  if (threadIdx.x == 0 && mj > kPartMaxJump) atomicMax(&info[4], (unsigned long long)mj);
}

template <class T>
__device__ __forceinline__ T block_max(T v, T* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int w = kPartThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = red[threadIdx.x] > red[threadIdx.x + w]
                                                     ? red[threadIdx.x]
                                                     : red[threadIdx.x + w];
    __syncthreads();
  }
  const T r = red[0];
  __syncthreads();
  return r;
}

// p[l] := the first node >= lim (the chunk's end, or D) on the walk from
// b + l (in place: every update replaces a node of the walk by a later one,
// never past the exit)
__device__ __forceinline__ void part_jump(int32_t* p, int64_t b, int32_t lim, int n) {
  for (int r = 0; r < 11; ++r) {  // 2^11 > kPartW
    for (int l = threadIdx.x; l < n; l += kPartThreads) {
      const int32_t v = p[l];
      if (v < lim) p[l] = p[v - b];
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) k_part_exit(const int32_t* __restrict__ nxt, int64_t D,
                                                   int32_t* __restrict__ exg,
                                                   int32_t* __restrict__ conv,
                                                   const unsigned long long* __restrict__ info) {
  __shared__ int32_t p[kPartW];
  __shared__ int32_t red[kPartThreads];
  if (info[4] > (unsigned long long)kPartMaxJump) return;  // host path
  const int64_t c = blockIdx.x;
  if (c >= (D + kPartW - 1) / kPartW) return;  // a grid past the chunks (launch_partition checks)
  const int64_t b = c * kPartW;
  const int n = (int)(D - b < kPartW ? D - b : kPartW);
  const int32_t lim = (int32_t)(b + n);  // the chunk's end (the last chunk: D)
  for (int l = threadIdx.x; l < n; l += kPartThreads) p[l] = nxt[b + l];
  __syncthreads();
  // M_c: the farthest node a dim before the chunk jumps to (chunk 0: entry 0)
  int32_t m = (int32_t)b;
  if (c > 0)
    for (int64_t s = b - kPartMaxJump + threadIdx.x; s < b; s += kPartThreads)
      if (s >= 0) m = nxt[s] > m ? nxt[s] : m;
  const int32_t mc = block_max(m, red);
  part_jump(p, b, lim, n);
  // candidate entries [b, mc]: their exits, and whether they agree
  const int ne = (int)(mc - b) + 1 < n ? (int)(mc - b) + 1 : n;
  const int32_t e0 = p[0];
  int32_t diff = 0;
  for (int l = threadIdx.x; l < ne; l += kPartThreads) {
    exg[b + l] = p[l];
    diff |= p[l] != e0 ? 1 : 0;
  }
  const int32_t any = block_max(diff, red);
  if (threadIdx.x == 0) conv[c] = any ? 0 : 1;
}

__global__ void __launch_bounds__(256) k_part_mark(const int32_t* __restrict__ nxt, int64_t D,
                                                   const int32_t* __restrict__ exg,
                                                   const int32_t* __restrict__ conv,
                                                   int32_t* __restrict__ node,
                                                   int32_t* __restrict__ cnt,
                                                   unsigned long long* __restrict__ info) {
  __shared__ int32_t ja[kPartW], jb[kPartW];
  __shared__ uint8_t mark[kPartW];
  __shared__ int32_t red[kPartThreads];
  __shared__ int32_t s_entry;
  if (info[4] > (unsigned long long)kPartMaxJump) return;
  const int64_t c = blockIdx.x;
  if (c >= (D + kPartW - 1) / kPartW) return;
  const int64_t b = c * kPartW;
  const int n = (int)(D - b < kPartW ? D - b : kPartW);
  const int32_t lim = (int32_t)(b + n);
  if (threadIdx.x == 0) {
    // the entry: the exit of the nearest converged chunk k < c (chunk 0 enters
    // at node 0), followed through the chunks between by their stored exits
    int32_t e = 0;
    if (c > 0) {
      int64_t k = c - 1;
      int run = 0;
      while (k > 0 && !conv[k] && run < kPartRun) {
        --k;
        ++run;
      }
      if (k > 0 && !conv[k]) {
        info[2] = 1ull;  // walks that do not merge: host path
        e = -1;
      } else {
        e = exg[k * kPartW];  // converged (or chunk 0): its exit, from its first dim
        for (int64_t k2 = k + 1; k2 < c && e >= 0; ++k2) e = exg[e];  // e in [b_k2, M_k2]
      }
    }
    s_entry = e;
  }
  for (int l = threadIdx.x; l < n; l += kPartThreads) {
    ja[l] = nxt[b + l];
    mark[l] = 0;
  }
  __syncthreads();
  const int32_t e = s_entry;
  if (e < 0) return;
  if (e < lim) {
    if (threadIdx.x == 0) mark[e - b] = 1;
    __syncthreads();
    // pointer jumping: after round r every node within 2^(r+1) - 1 steps of
    // the entry is marked (J_r = nxt^(2^r), double-buffered)
    int32_t* J = ja;
    int32_t* J2 = jb;
    for (int r = 0; r < 11; ++r) {
      for (int l = threadIdx.x; l < n; l += kPartThreads) {
        const int32_t v = J[l];
        if (mark[l] && v < lim) mark[v - b] = 1;
      }
      __syncthreads();
      for (int l = threadIdx.x; l < n; l += kPartThreads) {
        const int32_t v = J[l];
        J2[l] = v < lim ? J[v - b] : v;
      }
      __syncthreads();
      int32_t* t = J;
      J = J2;
      J2 = t;
    }
  }
  // compact the marked nodes in order: per-thread runs of 4 consecutive dims
  constexpr int kPer = kPartW / kPartThreads;
  int mine = 0;
  for (int q = 0; q < kPer; ++q) {
    const int l = threadIdx.x * kPer + q;
    mine += (l < n && mark[l]) ? 1 : 0;
  }
  red[threadIdx.x] = mine;
  __syncthreads();
  for (int o = 1; o < kPartThreads; o <<= 1) {  // inclusive scan
    const int32_t t = (int)threadIdx.x >= o ? red[threadIdx.x - o] : 0;
    __syncthreads();
    red[threadIdx.x] += t;
    __syncthreads();
  }
  int at = red[threadIdx.x] - mine;
  for (int q = 0; q < kPer; ++q) {
    const int l = threadIdx.x * kPer + q;
    if (l < n && mark[l]) node[b + at++] = (int32_t)(b + l);
  }
  if (threadIdx.x == kPartThreads - 1) cnt[c] = red[threadIdx.x];
}

// Superchunk sums of the chunk counts (launched past kPartDirect chunks): a
// workgroup per kPartSuper chunks
__global__ void __launch_bounds__(256) k_part_sup(const int32_t* __restrict__ cnt, int64_t nch,
                                                  int32_t* __restrict__ sup,
                                                  const unsigned long long* __restrict__ info) {
  __shared__ int64_t red[kPartThreads];
  if (info[4] > (unsigned long long)kPartMaxJump || info[2]) return;
  const int64_t k0 = (int64_t)blockIdx.x * kPartSuper;
  if (k0 >= nch) return;  // a grid past the superchunks
  int64_t v = 0;
  for (int64_t k = k0 + threadIdx.x; k < k0 + kPartSuper && k < nch; k += kPartThreads) v += cnt[k];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int w = kPartThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) sup[blockIdx.x] = (int32_t)red[0];
}

// SINGLE (one item, no item_off): the chunk's nodes go straight to the start
// list (st[dup + rank]; the last chunk adds st[0] = 0 and st[dup + total] = D)
// and the largest group to iinfo[1], so k_part_ihdr / k_part_ibody are not run.
template <bool SINGLE>
__global__ void __launch_bounds__(256) k_part_emit(int64_t nchunks,
                                                   const int32_t* __restrict__ node,
                                                   const int32_t* __restrict__ cnt,
                                                   const int32_t* __restrict__ sup,
                                                   int32_t* __restrict__ gnode,
                                                   unsigned long long* __restrict__ info,
                                                   const float* __restrict__ kl, int64_t D,
                                                   int64_t T, float thr,
                                                   const int32_t* __restrict__ nxt,
                                                   int64_t* __restrict__ starts,
                                                   int64_t* __restrict__ iinfo) {
  __shared__ int64_t red[kPartThreads];
  __shared__ int32_t redm[kPartThreads];
  if (info[4] > (unsigned long long)kPartMaxJump || info[2]) return;
  const int64_t c = blockIdx.x;
  if (c >= nchunks) return;  // a grid past the chunks
  const int64_t b = c * kPartW;
  // rank of the chunk's first node: the earlier chunks' counts (past
  // kPartDirect chunks: the earlier superchunks' sums, then the earlier chunks
  // of its own superchunk)
  const int64_t c0 = nchunks > kPartDirect ? c - c % kPartSuper : 0;
  int64_t s = 0;
  if (nchunks > kPartDirect)
    for (int64_t k = threadIdx.x; k < c / kPartSuper; k += kPartThreads) s += sup[k];
  for (int64_t k = c0 + threadIdx.x; k < c; k += kPartThreads) s += cnt[k];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = kPartThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const int64_t r0 = red[0];
  const int nc = cnt[c];
  if (!SINGLE) {
    for (int q = threadIdx.x; q < nc; q += kPartThreads) gnode[r0 + q] = node[b + q];
    if (threadIdx.x == 0 && c == nchunks - 1) info[0] = (unsigned long long)(r0 + nc);
    return;
  }
  // as k_part_ihdr's dup: dim 0 alone trips the test (:232-233), or D == 1
  const int64_t dup = (T <= 0 || kl[0] >= thr || D == 1) ? 1 : 0;
  int32_t mx = 0;
  for (int q = threadIdx.x; q < nc; q += kPartThreads) {
    const int32_t v = node[b + q];
    starts[dup + r0 + q] = v;  // rank 0 is dim 0
    const int32_t gsz = nxt[v] - v;
    mx = gsz > mx ? gsz : mx;
  }
  const int32_t m = block_max(mx, redm);
  if (threadIdx.x == 0) {
    if (m > 0) atomicMax((unsigned long long*)&iinfo[1], (unsigned long long)m);
    if (c == nchunks - 1) {
      const int64_t total = r0 + nc;
      starts[0] = 0;
      starts[dup + total] = D;
      iinfo[0] = dup + total + 1;
      info[0] = (unsigned long long)total;
    }
  }
}

__device__ __forceinline__ int64_t lower_bound_i32(const int32_t* __restrict__ a, int64_t n,
                                                   int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if ((int64_t)a[m] < v) lo = m + 1; else hi = m;
  }
  return lo;
}

// Item k's start list (coded_greedy_sampler.py:207-252 on its dims alone) at
// starts + item_off[k] + 2 k: [0], a second 0 when its first dim alone trips
// the test (:232-233 from the loop's initial (size 0, kl 0)), its walk nodes
// relative to its first dim, then its dim count (:252).  k_part_ihdr: a thread
// per item (its rank range by binary search, the ends of its list, its count);
// k_part_ibody: a thread per walk node (its entry and group size).
// iinfo: [2k] the item's starts (G + 1), [2k + 1] its largest group; scratch
// [2n + 2k] its first node's rank, [2n + 2k + 1] dup.
__global__ void __launch_bounds__(256) k_part_ihdr(const float* __restrict__ kl, int64_t D,
                                                   const int64_t* __restrict__ item_off,
                                                   int64_t n_items, int64_t T, float thr,
                                                   const int32_t* __restrict__ gnode,
                                                   int64_t* __restrict__ starts,
                                                   int64_t* __restrict__ iinfo,
                                                   const unsigned long long* __restrict__ info) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_items || info[4] > (unsigned long long)kPartMaxJump || info[2]) return;
  const int64_t a = item_off ? item_off[k] : 0;
  const int64_t e = item_off ? item_off[k + 1] : D;
  const int64_t Dk = e - a;
  int64_t* st = starts + a + 2 * k;
  iinfo[2 * k + 1] = 0;
  if (Dk == 0) {  // the loop never runs: [0, 0]
    st[0] = 0;
    st[1] = 0;
    iinfo[2 * k] = 2;
    return;
  }
  const int64_t total = (int64_t)info[0];
  const int64_t r0 = lower_bound_i32(gnode, total, a);
  const int64_t cnt = lower_bound_i32(gnode, total, e) - r0;
  const int64_t dup = (T <= 0 || kl[a] >= thr || Dk == 1) ? 1 : 0;
  st[0] = 0;           // the reference's initial [0] (and the empty first group's)
  st[dup + cnt] = Dk;  // :252
  iinfo[2 * k] = dup + cnt + 1;
  iinfo[2 * n_items + 2 * k] = r0;
  iinfo[2 * n_items + 2 * k + 1] = dup;
}

__global__ void __launch_bounds__(256) k_part_ibody(int64_t D, const int64_t* __restrict__ item_off,
                                                    int64_t n_items,
                                                    const int32_t* __restrict__ nxt,
                                                    const int32_t* __restrict__ gnode,
                                                    int64_t* __restrict__ starts,
                                                    int64_t* __restrict__ iinfo,
                                                    const unsigned long long* __restrict__ info) {
  __shared__ int32_t red[kPartThreads];
  __shared__ int64_t s_k0;
  __shared__ int64_t soff[kPartLdsItems + 1];
  if (info[4] > (unsigned long long)kPartMaxJump || info[2]) return;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)info[0];
  // the grid covers D (the node count is known on the device only): the
  // workgroups past the last node leave at once (C3: ~90% of them)
  if ((int64_t)blockIdx.x * blockDim.x >= total) return;
  const bool lds_off = item_off && n_items <= kPartLdsItems;
  if (lds_off)
    for (int t = threadIdx.x; t <= n_items; t += kPartThreads) soff[t] = item_off[t];
  __syncthreads();
  const int64_t* __restrict__ io = lds_off ? soff : item_off;
  int64_t k = -1;
  int32_t gsz = 0;
  if (r < total) {
    const int32_t v = gnode[r];
    k = 0;
    if (item_off) {  // the item holding dim v (empty items share offsets: the last match)
      int64_t lo = 0, hi = n_items;
      while (hi - lo > 1) {
        const int64_t m = (lo + hi) >> 1;
        if (io[m] <= v) lo = m; else hi = m;
      }
      k = lo;
    }
    const int64_t a = item_off ? io[k] : 0;
    const int64_t r0 = iinfo[2 * n_items + 2 * k], dup = iinfo[2 * n_items + 2 * k + 1];
    starts[a + 2 * k + dup + (r - r0)] = v - a;  // st[dup + rank] (rank 0: the first dim)
    gsz = nxt[v] - v;
  }
  // the largest group per item: one atomic for the block's first item, own ones
  // for the (rare) nodes of other items
  if (threadIdx.x == 0) s_k0 = k;
  __syncthreads();
  const int64_t k0 = s_k0;
  // (an atomic only when it can raise the value: few workgroups of an item
  // contend for its address)
  unsigned long long* im = (unsigned long long*)iinfo;
  if (k >= 0 && k != k0 && (unsigned long long)gsz > __atomic_load_n(&im[2 * k + 1], __ATOMIC_RELAXED))
    atomicMax(&im[2 * k + 1], (unsigned long long)gsz);
  const int32_t m0 = block_max(k == k0 ? gsz : 0, red);
  if (threadIdx.x == 0 && k0 >= 0 &&
      (unsigned long long)m0 > __atomic_load_n(&im[2 * k0 + 1], __ATOMIC_RELAXED))
    atomicMax(&im[2 * k0 + 1], (unsigned long long)m0);
}

__global__ void __launch_bounds__(256) k_batch_layout(const BatchItem* __restrict__ items,
                                                      const int64_t* __restrict__ dstarts,
                                                      int64_t* __restrict__ offs,
                                                      int32_t* __restrict__ seeds,
                                                      int64_t* __restrict__ pstarts) {
  const BatchItem it = items[blockIdx.x];  // item blockIdx.x, slice blockIdx.y of its groups
  const int64_t step = (int64_t)blockDim.x * gridDim.y;
  for (int64_t g = (int64_t)blockIdx.y * blockDim.x + threadIdx.x; g < it.G; g += step) {
    offs[it.go + g] = it.rel + dstarts[it.src + g];
    seeds[it.gs + g] = (int32_t)((uint32_t)it.seed + (uint32_t)g);  // :282, int32 wrap
  }
  if (pstarts)
    for (int64_t g = (int64_t)blockIdx.y * blockDim.x + threadIdx.x; g < it.ns; g += step)
      pstarts[it.pk + g] = dstarts[it.src + g];
  if (blockIdx.y == 0 && threadIdx.x == 0 && it.term >= 0) offs[it.term] = it.dc;
}

hipError_t launch_batch_layout(const BatchItem* items, int64_t n_items, const int64_t* dstarts,
                               int64_t* offs, int32_t* seeds, int64_t* pstarts,
                               hipStream_t stream) {
  if (n_items <= 0) return hipSuccess;
  // enough workgroups to fill the chip whatever the item count (48 C3 items: 16 each)
  const unsigned ys = n_items >= 2048 ? 1u : (unsigned)((2048 + n_items - 1) / n_items);
  hipLaunchKernelGGL(k_batch_layout, dim3((unsigned)n_items, ys > 64 ? 64u : ys), dim3(256), 0,
                     stream, items, dstarts, offs, seeds, pstarts);
  return hipGetLastError();
}

size_t partition_workspace_size(int64_t D) {
  const int64_t nch = (D + kPartW - 1) / kPartW;
  const int64_t nsup = (nch + kPartSuper - 1) / kPartSuper;
  const size_t b = (size_t)(4 * (D + 64) + 2 * (nch + 64) + (nsup + 64)) * 4 + 64 * 8;
  return (b + 255) & ~(size_t)255;  // callers place 8-byte words right after it
}

bool partition_fell_back(const unsigned long long* info) {
  return info[4] > (unsigned long long)kPartMaxJump || info[2] != 0ull || info[0] == 0ull;
}

bool partition_applies(int64_t D, int64_t size_threshold) {
  return D >= 2 && D < (1LL << 30) && size_threshold >= 1;
}

hipError_t launch_partition(const float* kl, int64_t D, const int64_t* item_off, int64_t n_items,
                            int64_t size_threshold, float thr, int64_t* starts, int64_t* iinfo,
                            void* ws, unsigned long long* info, hipStream_t stream,
                            bool info_zeroed) {
  // every per-chunk kernel indexes its chunk's counters, nodes and starts by
  // blockIdx.x: its grid is exactly the chunk (superchunk) count (round 5: a
  // work-in-progress launch of 256 workgroups over one chunk stored past the
  // start list; the kernels now also return past the last chunk)
  if (D < 1 || D >= (1LL << 30) || n_items < 1) return hipErrorInvalidValue;
  const int64_t nch = (D + kPartW - 1) / kPartW;
  int32_t* nxt = (int32_t*)ws;
  int32_t* exg = nxt + (D + 64);
  int32_t* node = exg + (D + 64);
  int32_t* gnode = node + (D + 64);
  int32_t* conv = gnode + (D + 64);
  int32_t* cnt = conv + (nch + 64);
  int32_t* sup = cnt + (nch + 64);
  const int64_t nsup = (nch + kPartSuper - 1) / kPartSuper;
  const dim3 gch((unsigned)nch), gsup((unsigned)nsup);
  if ((int64_t)gch.x != nch || (int64_t)gsup.x != nsup || nch < 1 || nsup < 1)
    return hipErrorInvalidValue;
  const bool single = item_off == nullptr && n_items == 1;
  if (!info_zeroed) {
    hipError_t e = hipMemsetAsync(info, 0, 8 * sizeof(unsigned long long), stream);
    if (e == hipSuccess && single) e = hipMemsetAsync(iinfo, 0, 2 * sizeof(int64_t), stream);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_part_next, dim3((unsigned)((D + 255) / 256)), dim3(256), 0, stream, kl, D,
                     item_off, n_items, size_threshold, thr, nxt, info);
  hipLaunchKernelGGL(k_part_exit, gch, dim3(kPartThreads), 0, stream, nxt, D, exg, conv, info);
  hipLaunchKernelGGL(k_part_mark, gch, dim3(kPartThreads), 0, stream, nxt, D, exg, conv, node, cnt,
                     info);
  if (nch > kPartDirect)
    hipLaunchKernelGGL(k_part_sup, gsup, dim3(kPartThreads), 0, stream, cnt, nch, sup, info);
  if (single) {
    hipLaunchKernelGGL(k_part_emit<true>, gch, dim3(kPartThreads), 0, stream, nch,
                       node, cnt, sup, gnode, info, kl, D, size_threshold, thr, nxt, starts, iinfo);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_part_emit<false>, gch, dim3(kPartThreads), 0, stream, nch,
                     node, cnt, sup, gnode, info, kl, D, size_threshold, thr, nxt, starts, iinfo);
  hipLaunchKernelGGL(k_part_ihdr, dim3((unsigned)((n_items + 255) / 256)), dim3(256), 0, stream,
                     kl, D, item_off, n_items, size_threshold, thr, gnode, starts, iinfo, info);
  hipLaunchKernelGGL(k_part_ibody, dim3((unsigned)((D + 255) / 256)), dim3(kPartThreads), 0, stream,
                     D, item_off, n_items, nxt, gnode, starts, iinfo, info);
  return hipGetLastError();
}

}  // namespace cwq
