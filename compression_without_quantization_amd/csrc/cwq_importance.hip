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
// grid find each tile's group by binary search (no host round trip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cwq_device.h"
#include "cwq_kernels.h"

namespace cwq {

constexpr int64_t kImpCandPerTile = 4096;

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

// tprefix[g] = sum_{h<g} ceil(max(N_h,1) / cpt); tprefix[nb] = total tiles.
__global__ void __launch_bounds__(1024) k_imp_tiles(const int64_t* __restrict__ n_samples,
                                                    int64_t nb, int64_t cpt,
                                                    int64_t* __restrict__ tprefix) {
  __shared__ int64_t part[1024];
  const int64_t chunk = (nb + 1023) / 1024;
  const int64_t g0 = threadIdx.x * chunk;
  const int64_t g1 = (g0 + chunk < nb) ? g0 + chunk : nb;
  int64_t sum = 0;
  for (int64_t g = g0; g < g1; ++g) {
    const int64_t n = n_samples[g] > 1 ? n_samples[g] : 1;
    sum += (n + cpt - 1) / cpt;
  }
  part[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int i = 0; i < 1024; ++i) {
      const int64_t v = part[i];
      part[i] = run;
      run += v;
    }
    tprefix[nb] = run;
  }
  __syncthreads();
  int64_t run = part[threadIdx.x];
  for (int64_t g = g0; g < g1; ++g) {
    tprefix[g] = run;
    const int64_t n = n_samples[g] > 1 ? n_samples[g] : 1;
    run += (n + cpt - 1) / cpt;
  }
}

__global__ void __launch_bounds__(256) k_imp_eval(
    const float* __restrict__ t_loc, const float* __restrict__ t_scale,
    const float* __restrict__ p_loc, const float* __restrict__ p_scale,
    const float* __restrict__ lnt, const float* __restrict__ lnp,
    const int64_t* __restrict__ block_off, const int64_t* __restrict__ n_samples, int64_t nb,
    const int64_t* __restrict__ tprefix, int64_t cpt, int32_t seed, int64_t block_id_base,
    unsigned long long* __restrict__ keys) {
  __shared__ double logtab[32];
  __shared__ unsigned long long wkey[4];
  fill_logtab(logtab);
  const uint32_t wv = wave_id();
  const uint32_t lane = threadIdx.x & 63u;
  const int64_t total = tprefix[nb];

  for (int64_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
    // group of this tile: last g with tprefix[g] <= tile
    int64_t lo = 0, hi = nb;  // tprefix[lo] <= tile < tprefix[hi]
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (tprefix[mid] <= tile) lo = mid; else hi = mid;
    }
    const int64_t g = lo;
    const int64_t off = block_off[g];
    const int64_t d = block_off[g + 1] - off;
    const int64_t N = n_samples[g] > 1 ? n_samples[g] : 1;
    const int64_t n0 = (tile - tprefix[g]) * cpt;
    const int64_t n1 = (n0 + cpt < N) ? n0 + cpt : N;
    const PhiloxStream st = generate_key(block_seed(seed, block_id_base + g), 42);
    const int align = (int)(((uint64_t)(n0 + wv) * (uint64_t)d) & 3u);
    const float* tl = t_loc + off;
    const float* ts = t_scale + off;
    const float* pl = p_loc + off;
    const float* ps = p_scale + off;
    const float* ct = lnt + off;
    const float* cp = lnp + off;

    uint64_t bestk = 0;
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

// Row `index` of group g's candidate stream: p_loc + p_scale * z (misc.py:14-15).
// With keys != nullptr the index comes from the argmax key (encoder), else
// from index_in (decoder, coded_importance_sampler.py:82-109).
__global__ void __launch_bounds__(256) k_imp_rows(
    const unsigned long long* __restrict__ keys, const int64_t* __restrict__ index_in,
    const float* __restrict__ p_loc, const float* __restrict__ p_scale,
    const int64_t* __restrict__ block_off, int64_t nb, int32_t seed, int64_t block_id_base,
    int64_t* __restrict__ index_out, float* __restrict__ out_sample) {
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
    const PhiloxStream st = generate_key(block_seed(seed, block_id_base + g), 42);
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
      out_sample[off + j] = v;
    }
  }
}

size_t importance_workspace_size(int64_t nb, int64_t total_dims) {
  auto up = [](size_t v) { return (v + 255) / 256 * 256; };
  return up((size_t)nb * 8) + up((size_t)(nb + 1) * 8) + 2 * up((size_t)total_dims * 4);
}

hipError_t launch_importance_encode(const float* t_loc, const float* t_scale, const float* p_loc,
                                    const float* p_scale, const int64_t* block_off,
                                    const int64_t* n_samples, int64_t nb, int64_t total_dims,
                                    int32_t seed, int64_t block_id_base, int64_t* out_index,
                                    float* out_sample, void* workspace, hipStream_t stream) {
  if (nb <= 0) return hipSuccess;
  auto up = [](size_t v) { return (v + 255) / 256 * 256; };
  char* w = (char*)workspace;
  unsigned long long* keys = (unsigned long long*)w;
  int64_t* tprefix = (int64_t*)(w + up((size_t)nb * 8));
  float* lnt = (float*)(w + up((size_t)nb * 8) + up((size_t)(nb + 1) * 8));
  float* lnp = lnt + up((size_t)total_dims * 4) / 4;
  hipError_t e = hipMemsetAsync(keys, 0, (size_t)nb * 8, stream);
  if (e != hipSuccess) return e;
  if (total_dims > 0)
    hipLaunchKernelGGL(k_imp_prep, dim3(grid_for(total_dims, 256, 65536)), dim3(256), 0, stream,
                       t_scale, p_scale, total_dims, lnt, lnp);
  hipLaunchKernelGGL(k_imp_tiles, dim3(1), dim3(1024), 0, stream, n_samples, nb,
                     kImpCandPerTile, tprefix);
  hipLaunchKernelGGL(k_imp_eval, dim3(256 * 16), dim3(256), 0, stream, t_loc, t_scale, p_loc,
                     p_scale, lnt, lnp, block_off, n_samples, nb, tprefix, kImpCandPerTile, seed,
                     block_id_base, keys);
  hipLaunchKernelGGL(k_imp_rows, dim3(grid_for(nb, 4, 65536)), dim3(256), 0, stream,
                     (const unsigned long long*)keys, (const int64_t*)nullptr, p_loc, p_scale,
                     block_off, nb, seed, block_id_base, out_index, out_sample);
  return hipGetLastError();
}

hipError_t launch_importance_decode(const int64_t* index, const float* p_loc,
                                    const float* p_scale, const int64_t* block_off, int64_t nb,
                                    int32_t seed, int64_t block_id_base, float* out_sample,
                                    hipStream_t stream) {
  if (nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_imp_rows, dim3(grid_for(nb, 4, 65536)), dim3(256), 0, stream,
                     (const unsigned long long*)nullptr, index, p_loc, p_scale, block_off, nb,
                     seed, block_id_base, (int64_t*)nullptr, out_sample);
  return hipGetLastError();
}

}  // namespace cwq
