// cwq_pln.hip -- the latent plumbing of the PLN image codec around the coders
// (code/pln.py:150-203, 213-627, 638-817).
//
// The convolutional transforms run as library convolutions (MIOpen through
// PyTorch); what sits between them and the coders is elementwise / gather
// work on the latent tensors, done here in one pass each:
//   * k_pln_posterior: the ladder's precision-weighted combination of the
//     level-1 likelihood (AnalysisTransform_1) with the level-1 prior
//     (SynthesisTransform_2), pln.py:165-185, float32 in the reference's
//     operation order;
//   * k_permute_gather: flatten an NCHW latent tensor in the reference's NHWC
//     order (tf.reshape(x, [-1]) of an NHWC tensor, pln.py:264-273) and apply
//     tfp.bijectors.Permute.forward (y[i] = x[perm[i]], pln.py:316-324);
//   * k_permute_scatter: the inverse (Permute.inverse + reshape back to the
//     latent shape, pln.py:394-397, :770-772, :801-803), written NCHW.
// All three are HBM-bound streams (8-16 B per latent).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cwq.h"
#include "cwq_kernels.h"

namespace cwq {
namespace {

__global__ void __launch_bounds__(256) k_pln_posterior(
    const float* __restrict__ lik_loc, const float* __restrict__ lik_scale,
    const float* __restrict__ pri_loc, const float* __restrict__ pri_scale, int64_t n, float eps,
    float* __restrict__ loc, float* __restrict__ scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float ls = lik_scale[i], ps = pri_scale[i];
    const float lv = ls * ls;                   // :169 tf.square
    const float pv = ps * ps;                   // :170
    const float lp = 1.0f / (lv + eps);         // :172
    const float pp = 1.0f / (pv + eps);         // :173
    const float cv = 1.0f / (lp + pp);          // :176
    const float cl0 = lik_loc[i] * pp;          // :180
    const float cl1 = cl0 + pri_loc[i] * lp;    // :181
    scale[i] = __builtin_sqrtf(cv);             // :177 (correctly rounded)
    loc[i] = cl1 * cv;                          // :182
  }
}

// out[i] = x_nhwc[f], f = perm[i] (identity when perm is null), where
// x_nhwc[(h W + w) C + c] = x_nchw[c HW + h W + w].
__global__ void __launch_bounds__(256) k_permute_gather(const float* __restrict__ src, int64_t C,
                                                        int64_t HW, const int32_t* __restrict__ perm,
                                                        float* __restrict__ out) {
  const int64_t n = C * HW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = perm ? (int64_t)perm[i] : i;
    const int64_t hw = f / C;
    const int64_t c = f - hw * C;
    out[i] = src[c * HW + hw];
  }
}

// x_nchw[c HW + hw] = src[i] for f = perm[i] = hw C + c: the inverse of
// k_permute_gather (a permutation, so every output is written once).
__global__ void __launch_bounds__(256) k_permute_scatter(const float* __restrict__ src, int64_t C,
                                                         int64_t HW,
                                                         const int32_t* __restrict__ perm,
                                                         float* __restrict__ out) {
  const int64_t n = C * HW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = perm ? (int64_t)perm[i] : i;
    const int64_t hw = f / C;
    const int64_t c = f - hw * C;
    out[c * HW + hw] = src[i];
  }
}

unsigned grid_1d(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (unsigned)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

}  // namespace
}  // namespace cwq

extern "C" {

int cwq_pln_posterior(const float* lik_loc, const float* lik_scale, const float* prior_loc,
                      const float* prior_scale, int64_t n, float eps, float* loc, float* scale,
                      void* stream) {
  if (n < 0) return cwq::set_error(CWQ_ERR_INVALID, "cwq_pln_posterior: negative size");
  if (n == 0) return cwq::set_error(CWQ_OK, "");
  if (!lik_loc || !lik_scale || !prior_loc || !prior_scale || !loc || !scale)
    return cwq::set_error(CWQ_ERR_INVALID, "cwq_pln_posterior: null pointer");
  hipLaunchKernelGGL(cwq::k_pln_posterior, dim3(cwq::grid_1d(n)), dim3(256), 0,
                     (hipStream_t)stream, lik_loc, lik_scale, prior_loc, prior_scale, n, eps, loc,
                     scale);
  if (hipGetLastError() != hipSuccess)
    return cwq::set_error(CWQ_ERR_HIP, "cwq_pln_posterior: launch failed");
  return cwq::set_error(CWQ_OK, "");
}

int cwq_permute_gather(const float* src, int64_t C, int64_t HW, const int32_t* perm, float* out,
                       void* stream) {
  if (C < 0 || HW < 0 || (C > 0 && HW > INT32_MAX / C))
    return cwq::set_error(CWQ_ERR_INVALID, "cwq_permute_gather: bad shape");
  if (C * HW == 0) return cwq::set_error(CWQ_OK, "");
  if (!src || !out) return cwq::set_error(CWQ_ERR_INVALID, "cwq_permute_gather: null pointer");
  hipLaunchKernelGGL(cwq::k_permute_gather, dim3(cwq::grid_1d(C * HW)), dim3(256), 0,
                     (hipStream_t)stream, src, C, HW, perm, out);
  if (hipGetLastError() != hipSuccess)
    return cwq::set_error(CWQ_ERR_HIP, "cwq_permute_gather: launch failed");
  return cwq::set_error(CWQ_OK, "");
}

int cwq_permute_scatter(const float* src, int64_t C, int64_t HW, const int32_t* perm, float* out,
                        void* stream) {
  if (C < 0 || HW < 0 || (C > 0 && HW > INT32_MAX / C))
    return cwq::set_error(CWQ_ERR_INVALID, "cwq_permute_scatter: bad shape");
  if (C * HW == 0) return cwq::set_error(CWQ_OK, "");
  if (!src || !out) return cwq::set_error(CWQ_ERR_INVALID, "cwq_permute_scatter: null pointer");
  hipLaunchKernelGGL(cwq::k_permute_scatter, dim3(cwq::grid_1d(C * HW)), dim3(256), 0,
                     (hipStream_t)stream, src, C, HW, perm, out);
  if (hipGetLastError() != hipSuccess)
    return cwq::set_error(CWQ_ERR_HIP, "cwq_permute_scatter: launch failed");
  return cwq::set_error(CWQ_OK, "");
}

}  // extern "C"
