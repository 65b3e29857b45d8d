// Instruction-throughput microbenchmarks for gfx950 (development aid, not product).
// Each kernel runs 8 independent dependency chains per lane; we time many waves.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096
#define CH 8

__global__ void k_fma_f32(float* out, float a) {
  float x[CH]; for (int i = 0; i < CH; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) x[i] = __builtin_fmaf(x[i], a, 0.5f);
  float s = 0; for (int i = 0; i < CH; ++i) s += x[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_pk_fma_f32(float* out, float a) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 x[CH]; for (int i = 0; i < CH; ++i) x[i] = f2{(float)threadIdx.x, (float)i};
  f2 av = {a, a}, bv = {0.5f, 0.5f};
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) x[i] = __builtin_elementwise_fma(x[i], av, bv);
  float s = 0; for (int i = 0; i < CH; ++i) s += x[i].x + x[i].y; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma_f64(double* out, double a) {
  double x[CH]; for (int i = 0; i < CH; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) x[i] = __builtin_fma(x[i], a, 0.5);
  double s = 0; for (int i = 0; i < CH; ++i) s += x[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mad_u64(uint32_t* out, uint32_t m) {
  uint32_t x[CH]; for (int i = 0; i < CH; ++i) x[i] = threadIdx.x * 7 + i;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) { uint64_t p = (uint64_t)x[i] * m; x[i] = (uint32_t)(p >> 32) ^ (uint32_t)p; }
  uint32_t s = 0; for (int i = 0; i < CH; ++i) s ^= x[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mulhi_u32(uint32_t* out, uint32_t m) {
  uint32_t x[CH]; for (int i = 0; i < CH; ++i) x[i] = threadIdx.x * 7 + i;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) x[i] = __umulhi(x[i], m) + 0x12345u;
  uint32_t s = 0; for (int i = 0; i < CH; ++i) s ^= x[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mullo_u32(uint32_t* out, uint32_t m) {
  uint32_t x[CH]; for (int i = 0; i < CH; ++i) x[i] = threadIdx.x * 7 + i;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) x[i] = x[i] * m + 0x12345u;
  uint32_t s = 0; for (int i = 0; i < CH; ++i) s ^= x[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_xor(uint32_t* out, uint32_t m) {
  uint32_t x[CH]; for (int i = 0; i < CH; ++i) x[i] = threadIdx.x * 7 + i;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) x[i] = (x[i] ^ m) + (x[i] >> 3);
  uint32_t s = 0; for (int i = 0; i < CH; ++i) s ^= x[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_sqrt_f32(float* out, float a) {
  float x[CH]; for (int i = 0; i < CH; ++i) x[i] = threadIdx.x + i + 1;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) x[i] = __builtin_amdgcn_sqrtf(x[i]) + a;
  float s = 0; for (int i = 0; i < CH; ++i) s += x[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_cvt_f64(float* out, float a) {
  float x[CH]; for (int i = 0; i < CH; ++i) x[i] = threadIdx.x + i + 1;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) x[i] = (float)((double)x[i]);
  float s = 0; for (int i = 0; i < CH; ++i) s += x[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

#define UNARY_KERNEL(NAME, EXPR)                                                        \
  __global__ void NAME(float* out, float a) {                                           \
    float x[CH]; for (int i = 0; i < CH; ++i) x[i] = (threadIdx.x + i + 1) * 1e-3f;     \
    for (int it = 0; it < ITERS; ++it)                                                  \
      _Pragma("unroll") for (int i = 0; i < CH; ++i) { float v = x[i]; x[i] = (EXPR) + a; } \
    float s = 0; for (int i = 0; i < CH; ++i) s += x[i];                                \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                     \
  }
UNARY_KERNEL(k_log_f32, __builtin_amdgcn_logf(v))
UNARY_KERNEL(k_sin_f32, __builtin_amdgcn_sinf(v))
UNARY_KERNEL(k_cos_f32, __builtin_amdgcn_cosf(v))
UNARY_KERNEL(k_rsq_f32, __builtin_amdgcn_rsqf(v))
UNARY_KERNEL(k_exp_f32, __builtin_amdgcn_exp2f(v))
// one v_sin per 4 independent f32 FMAs: does the transcendental overlap?
__global__ void k_sin_mix(float* out, float a) {
  float x[CH], y[CH];
  for (int i = 0; i < CH; ++i) { x[i] = (threadIdx.x + i + 1) * 1e-3f; y[i] = x[i] + 1.f; }
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      x[i] = __builtin_amdgcn_sinf(x[i]);
      y[i] = __builtin_fmaf(y[i], a, 0.5f);
      y[i] = __builtin_fmaf(y[i], a, 0.25f);
      y[i] = __builtin_fmaf(y[i], a, 0.125f);
      y[i] = __builtin_fmaf(y[i], a, 0.0625f);
    }
  float s = 0; for (int i = 0; i < CH; ++i) s += x[i] + y[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// one v_mad_u64_u32 (+ the xor that keeps the chain) per 4 independent f32
// FMAs: do plain ops issue in the multiply's shadow?
__global__ void k_mad_mix(uint32_t* out, uint32_t m) {
  uint32_t x[CH]; float y[CH];
  for (int i = 0; i < CH; ++i) { x[i] = threadIdx.x * 7 + i; y[i] = (float)x[i]; }
  const float a = __uint_as_float(0x3f7ff000u);
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      uint64_t p = (uint64_t)x[i] * m; x[i] = (uint32_t)(p >> 32) ^ (uint32_t)p;
      y[i] = __builtin_fmaf(y[i], a, 0.5f);
      y[i] = __builtin_fmaf(y[i], a, 0.25f);
      y[i] = __builtin_fmaf(y[i], a, 0.125f);
      y[i] = __builtin_fmaf(y[i], a, 0.0625f);
    }
  uint32_t s = 0; for (int i = 0; i < CH; ++i) s ^= x[i] ^ __float_as_uint(y[i]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// the screening unit's quarter-rate mix alone: 9 v_mad_u64_u32 (+ xor) and 4
// transcendentals per chain-iteration, then the same with 25 plain f32 ops
template <int PLAIN>
__global__ void k_unit_mix(uint32_t* out, uint32_t m) {
  uint32_t x[CH]; float y[CH], t[CH];
  for (int i = 0; i < CH; ++i) { x[i] = threadIdx.x * 7 + i; y[i] = (float)x[i]; t[i] = 0.5f; }
  const float a = __uint_as_float(0x3f7ff000u);
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < CH; ++i) {
#pragma unroll
      for (int r = 0; r < 9; ++r) {
        uint64_t p = (uint64_t)x[i] * m; x[i] = (uint32_t)(p >> 32) ^ (uint32_t)p;
      }
      const float u = __uint_as_float((x[i] & 0x7fffffu) | 0x3f800000u);
      t[i] += __builtin_amdgcn_sinf(u) + __builtin_amdgcn_cosf(u) + __builtin_amdgcn_logf(u) +
              __builtin_amdgcn_sqrtf(u);
#pragma unroll
      for (int r = 0; r < PLAIN; ++r) y[i] = __builtin_fmaf(y[i], a, 0.5f);
    }
  uint32_t s = 0;
  for (int i = 0; i < CH; ++i) s ^= x[i] ^ __float_as_uint(y[i]) ^ __float_as_uint(t[i]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K, typename T>
void run(const char* name, K k, T arg, int ops_per_iter_per_chain) {
  void* out; hipMalloc(&out, 256 * 8192 * 8);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  int grid = 256 * 16;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, (decltype(arg)*)nullptr == nullptr ? (T*)out : (T*)out, arg);
  hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, (T*)out, arg);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double lane_ops = (double)grid * 256 * ITERS * CH * ops_per_iter_per_chain;
  printf("%-14s %8.3f ms  %8.3f Tlane-ops/s  (%5.2f of 7.86e13)\n", name, ms, lane_ops / ms / 1e9,
         lane_ops / (ms * 1e-3) / 7.86e13);
  hipFree(out);
}

int main() {
  run("fma_f32", k_fma_f32, 1.0001f, 1);
  run("pk_fma_f32", k_pk_fma_f32, 1.0001f, 2);
  run("fma_f64", k_fma_f64, 1.0001, 1);
  run("mad_u64+xor", k_mad_u64, 0xD2511F53u, 2);
  run("mulhi+add", k_mulhi_u32, 0xD2511F53u, 2);
  run("mullo+add", k_mullo_u32, 0xD2511F53u, 2);
  run("xor+shr+add", k_xor, 0xD2511F53u, 3);
  run("sqrt+add", k_sqrt_f32, 1.0f, 2);
  run("cvt64+cvt32", k_cvt_f64, 1.0f, 2);
  run("log+add", k_log_f32, 1.0f, 2);
  run("sin+add", k_sin_f32, 0.001f, 2);
  run("cos+add", k_cos_f32, 0.001f, 2);
  run("rsq+add", k_rsq_f32, 1.0f, 2);
  run("exp2+add", k_exp_f32, -1.0f, 2);
  run("sin+4fma", k_sin_mix, 0.999f, 5);
  run("mad+xor+4fma", k_mad_mix, 0xD2511F53u, 6);
  // unit mix: counted as "instructions" (9 mad + 9 xor + 4 trans + 3 add + 2 and/or + PLAIN)
  run("unit_mix+0", k_unit_mix<0>, 0xD2511F53u, 27);
  run("unit_mix+12", k_unit_mix<12>, 0xD2511F53u, 39);
  run("unit_mix+25", k_unit_mix<25>, 0xD2511F53u, 52);
  run("unit_mix+50", k_unit_mix<50>, 0xD2511F53u, 77);
  return 0;
}
