/* capi_demo.c -- the C ABI (include/cwq.h) from plain C, no Python or torch:
 * what a non-Python host (cgo, JNI, a C++ service) binds.  Encodes nb blocks of
 * dimension d at b bits per block (one step, seed + g per block, as
 * code_grouped_greedy_sample's groups), decodes them from the indices alone,
 * checks decode(encode(x)) == the encoder's sample bit for bit, and prints the
 * indices' checksum so tests/test_gpu.py can compare with the Python path.
 *
 *   examples/capi_demo NB D BITS SEED
 * Inputs: t_loc[i] = u(i) - 0.5, t_scale[i] = 0.3 + 0.6 u(i + n), p_loc = 0,
 * p_scale = 1, u(k) = ((k * 2654435761) mod 2^32) / 2^32 (float32). */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cwq.h"

static float u01(uint64_t k) {
  return (float)((uint32_t)(k * 2654435761u)) * (float)(1.0 / 4294967296.0);
}

#define CHECK_HIP(x)                                                          \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 2;                                                               \
    }                                                                         \
  } while (0)
#define CHECK_CWQ(x)                                                          \
  do {                                                                        \
    int64_t r_ = (x);                                                         \
    if (r_ < 0) {                                                             \
      fprintf(stderr, "%s: %lld %s\n", #x, (long long)r_, cwq_last_error());  \
      return 3;                                                               \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  const int64_t nb = argc > 1 ? atoll(argv[1]) : 1000;
  const int64_t d = argc > 2 ? atoll(argv[2]) : 32;
  const int bits = argc > 3 ? atoi(argv[3]) : 12;
  const int32_t seed = argc > 4 ? atoi(argv[4]) : 42;
  const int64_t n = nb * d;
  float* h = (float*)malloc((size_t)n * 4 * sizeof(float));
  float *tl = h, *ts = h + n, *pl = h + 2 * n, *ps = h + 3 * n;
  for (int64_t i = 0; i < n; ++i) {
    tl[i] = u01((uint64_t)i) - 0.5f;
    ts[i] = 0.3f + 0.6f * u01((uint64_t)(i + n));
    pl[i] = 0.0f;
    ps[i] = 1.0f;
  }
  float *d_in, *d_sample, *d_dec;
  int32_t* d_idx;
  void* d_ws;
  const size_t ws = cwq_greedy_encode_uniform_workspace_size(nb, d);
  CHECK_HIP(hipMalloc((void**)&d_in, (size_t)n * 4 * sizeof(float)));
  CHECK_HIP(hipMalloc((void**)&d_sample, (size_t)n * sizeof(float)));
  CHECK_HIP(hipMalloc((void**)&d_dec, (size_t)n * sizeof(float)));
  CHECK_HIP(hipMalloc((void**)&d_idx, (size_t)nb * sizeof(int32_t)));
  CHECK_HIP(hipMalloc(&d_ws, ws > 0 ? ws : 1));
  CHECK_HIP(hipMemcpy(d_in, h, (size_t)n * 4 * sizeof(float), hipMemcpyHostToDevice));
  hipStream_t st;
  CHECK_HIP(hipStreamCreate(&st));
  CHECK_CWQ(cwq_greedy_encode_uniform(d_in, d_in + n, d_in + 2 * n, d_in + 3 * n, nb, d, bits, 1,
                                      seed, 1.0f, 0, d_idx, d_sample, d_ws, ws, NULL, st));
  CHECK_CWQ(cwq_greedy_decode_uniform(d_idx, d_in + 2 * n, d_in + 3 * n, nb, d, bits, 1, seed,
                                      1.0f, 0, d_dec, st));
  CHECK_HIP(hipStreamSynchronize(st));
  int32_t* idx = (int32_t*)malloc((size_t)nb * sizeof(int32_t));
  uint32_t* a = (uint32_t*)malloc((size_t)n * 4);
  uint32_t* b = (uint32_t*)malloc((size_t)n * 4);
  CHECK_HIP(hipMemcpy(idx, d_idx, (size_t)nb * sizeof(int32_t), hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(a, d_sample, (size_t)n * 4, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(b, d_dec, (size_t)n * 4, hipMemcpyDeviceToHost));
  int64_t bad = 0;
  for (int64_t i = 0; i < n; ++i) bad += a[i] != b[i];
  uint64_t sum = 0;
  for (int64_t g = 0; g < nb; ++g) sum = sum * 1000003u + (uint32_t)idx[g];
  printf("blocks %lld d %lld bits %d idx0 %d checksum %llu roundtrip_mismatch %lld\n",
         (long long)nb, (long long)d, bits, idx[0], (unsigned long long)sum, (long long)bad);
  hipStreamDestroy(st);
  hipFree(d_in);
  hipFree(d_sample);
  hipFree(d_dec);
  hipFree(d_idx);
  hipFree(d_ws);
  free(h);
  free(idx);
  free(a);
  free(b);
  return bad == 0 ? 0 : 1;
}
