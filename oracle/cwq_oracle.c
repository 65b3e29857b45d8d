/*
 * cwq_oracle.c -- CPU ORACLE for the greedy coded sampling loop.
 *
 *   *** TEST INFRASTRUCTURE ONLY. ***
 *   Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 *   load this library, and only as the checker / the reported CPU baseline.
 *   The product path (compression_without_quantization_amd) never links it.
 *
 * What it restates (plain C, glibc libm, -O2 -ffp-contract=off):
 *   - code/coded_greedy_sampler.py:29-89   code_greedy_sample (encoder loop)
 *   - code/coded_greedy_sampler.py:93-167  decode_greedy_sample
 *   - code/coded_greedy_sampler.py:170-296 the grouped wrapper's numeric parts
 *     (standardisation :193-199, KL :201, grouping :207-244, seed+g :282,
 *     de-standardisation :292)
 *   - code/misc.py:3-17                    stateless_normal_sample
 *   - third-party semantics the reference calls into (SURVEY.md Appendix A,
 *     recalled from TF/TFP/Eigen public sources, NOT verifiable offline):
 *       A.1 Philox4x32-10, A.2 TF GenerateKey, A.3 FillPhiloxRandom layout,
 *       A.4 BoxMullerFloat (glibc logf/sqrtf/sincosf), A.5 TFP<=0.7
 *       Normal.log_prob, A.6 Eigen 3.3 AVX inner-dim sum order,
 *       A.7 argmax lowest-index-on-ties, A.9 TFP<=0.7 KL(Normal||Normal).
 *
 * Parity status: the reference (TF1 graph code) cannot be imported or run in
 * this environment (TF/TFP absent; building/importing anything
 * from /root/reference was refused).  This oracle is pinned by
 *   (1) published Random123 Philox4x32-10 known-answer vectors (tests/golden),
 *   (2) the bit-string examples readable in code/binary_io.py:41-67,
 *   (3) the host glibc 2.35 libm itself (logf, sincosf, sqrtf are called
 *       directly here, so the Box-Muller transcendentals ARE the declared
 *       semantics, not a restatement of them).
 * Everything that depends on TF/TFP/Eigen internals is declared semantics:
 * PARITY AGAINST THE REFERENCE IS UNPINNED beyond those pins.
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define CWQO_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* A.1 Philox4x32-10 (TF random::PhiloxRandom; same round as Random123).     */
/* ------------------------------------------------------------------------ */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

CWQO_API void cwqo_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2],
                                 uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
    uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n1 = lo1;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    uint32_t n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    if (r < 9) { k0 += PHILOX_W0; k1 += PHILOX_W1; }
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* n independent blocks: out[4i..] = Philox4x32-10(ctr[4i..], key[2i..]) (pin tests) */
CWQO_API void cwqo_philox4x32_10_many(const uint32_t* ctr, const uint32_t* key, int64_t n,
                                      uint32_t* out) {
  for (int64_t i = 0; i < n; ++i) cwqo_philox4x32_10(ctr + 4 * i, key + 2 * i, out + 4 * i);
}

/* A.2 TF stateless seed scrambling (stateless_random_ops.cc GenerateKey).
 * seed = [s0, s1] int32 (misc.py:11 passes [1000*seed+i, 42]); each is
 * sign-extended to 64 bits. */
CWQO_API void cwqo_generate_key(int32_t s0, int32_t s1, uint32_t key[2], uint32_t ctr[4]) {
  uint64_t seed0 = (uint64_t)(int64_t)s0;
  uint64_t seed1 = (uint64_t)(int64_t)s1;
  uint32_t k[2] = {0x3ec8f720u, 0x02461e29u};
  uint32_t c[4] = {(uint32_t)seed0, (uint32_t)(seed0 >> 32), (uint32_t)seed1,
                   (uint32_t)(seed1 >> 32)};
  uint32_t mix[4];
  cwqo_philox4x32_10(c, k, mix);
  key[0] = mix[0];
  key[1] = mix[1];
  ctr[0] = 0;
  ctr[1] = 0;
  ctr[2] = mix[2];
  ctr[3] = mix[3];
}

/* 128-bit counter skip (PhiloxRandom::Skip). */
static void philox_skip(const uint32_t base[4], uint64_t count, uint32_t out[4]) {
  uint32_t lo = (uint32_t)count, hi = (uint32_t)(count >> 32);
  out[0] = base[0] + lo;
  if (out[0] < lo) ++hi;
  out[1] = base[1] + hi;
  out[2] = base[2];
  out[3] = base[3];
  if (out[1] < hi) {
    if (++out[2] == 0) ++out[3];
  }
}

/* ------------------------------------------------------------------------ */
/* A.4 BoxMullerFloat with TF Uint32ToFloat, glibc transcendentals.          */
/* ------------------------------------------------------------------------ */
static inline float uint32_to_float(uint32_t x) {
  uint32_t val = (127u << 23) | (x & 0x7fffffu);
  float f;
  memcpy(&f, &val, 4);
  return f - 1.0f;
}

CWQO_API float cwqo_bm_radius(uint32_t x0) {
  float u1 = uint32_to_float(x0);
  if (u1 < 1.0e-7f) u1 = 1.0e-7f;
  return sqrtf(-2.0f * logf(u1));
}

CWQO_API float cwqo_bm_angle(uint32_t x1) {
  /* `2.0f * M_PI * Uint32ToFloat(x1)` is evaluated in double (M_PI is a
   * double literal) and then narrowed to float. */
  return (float)(2.0f * M_PI * (double)uint32_to_float(x1));
}

CWQO_API void cwqo_bm_sincos(uint32_t x1, float* s, float* c) {
  float v1 = cwqo_bm_angle(x1);
  sincosf(v1, s, c);
}

CWQO_API void cwqo_box_muller(uint32_t x0, uint32_t x1, float* f0, float* f1) {
  float u2 = cwqo_bm_radius(x0);
  float s, c;
  cwqo_bm_sincos(x1, &s, &c);
  *f0 = s * u2;
  *f1 = c * u2;
}

/* Philox group `grp` of stream (key, ctr) -> 4 normals (NormalDistribution). */
static void normal_group(const uint32_t key[2], const uint32_t ctr[4], uint64_t grp,
                         float z[4]) {
  uint32_t c[4], x[4];
  philox_skip(ctr, grp, c);
  cwqo_philox4x32_10(c, key, x);
  cwqo_box_muller(x[0], x[1], &z[0], &z[1]);
  cwqo_box_muller(x[2], x[3], &z[2], &z[3]);
}

/* tf.random.stateless_normal(shape=[n], seed=[s0,s1]) flattened, including the
 * python wrapper's `rnd * stddev + mean` with stddev=1, mean=0 (A.3, A.4). */
CWQO_API void cwqo_stateless_normal(int32_t s0, int32_t s1, int64_t n, float* out) {
  uint32_t key[2], ctr[4];
  cwqo_generate_key(s0, s1, key, ctr);
  float z[4];
  for (int64_t k = 0; k < n; ++k) {
    if ((k & 3) == 0) normal_group(key, ctr, (uint64_t)k >> 2, z);
    out[k] = z[k & 3] * 1.0f + 0.0f;
  }
}

/* misc.py:3-17 stateless_normal_sample(loc, scale, num_samples, seed) for a
 * rank-1 loc/scale of length d: out[n*d+j] = loc[j] + scale[j]*Z[n*d+j]. */
CWQO_API void cwqo_stateless_normal_sample(const float* loc, const float* scale, int64_t d,
                                           int64_t num_samples, int32_t seed, float* out) {
  cwqo_stateless_normal(seed, 42, num_samples * d, out);
  for (int64_t n = 0; n < num_samples; ++n)
    for (int64_t j = 0; j < d; ++j) {
      float s = scale[j] * out[n * d + j]; /* misc.py:14 */
      out[n * d + j] = loc[j] + s;         /* misc.py:15 */
    }
}

/* ------------------------------------------------------------------------ */
/* A.5 TFP (<=0.7) Normal.log_prob; A.6 Eigen inner-dim sum; A.7 argmax.     */
/* ------------------------------------------------------------------------ */
/* 0.5*math.log(2.*math.pi) converted to float32 by TF. */
static float half_log_2pi_f32(void) { return (float)(0.5 * log(2.0 * M_PI)); }

CWQO_API float cwqo_log_normalization(float scale) {
  return half_log_2pi_f32() + logf(scale);
}

static inline float log_prob_c(float x, float loc, float scale, float lognorm) {
  float z = (x - loc) / scale;      /* _z(x) */
  float u = -0.5f * (z * z);        /* _log_unnormalized_prob: -0.5*square(z) */
  return u - lognorm;               /* minus _log_normalization() */
}

CWQO_API float cwqo_normal_log_prob(float x, float loc, float scale) {
  return log_prob_c(x, loc, scale, cwqo_log_normalization(scale));
}

/* Eigen 3.3 InnerMostDimReducer<SumReducer>, Packet8f (AVX): 8 lane partials,
 * predux((p0+p4,p1+p5,p2+p6,p3+p7)) = (q0+q2)+(q1+q3), scalar tail, t + r. */
CWQO_API float cwqo_eigen_rowsum(const float* x, int64_t d) {
  int64_t vec = (d / 8) * 8;
  float p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t j = 0; j < vec; j += 8)
    for (int l = 0; l < 8; ++l) p[l] = p[l] + x[j + l];
  float t = 0.0f;
  for (int64_t j = vec; j < d; ++j) t = t + x[j];
  float q0 = p[0] + p[4], q1 = p[1] + p[5], q2 = p[2] + p[6], q3 = p[3] + p[7];
  float r = (q0 + q2) + (q1 + q3);
  return t + r;
}

static inline int32_t step_seed(int32_t seed, int32_t i) {
  /* `1000 * seed + i` in int32 (wraps, as TF int32 arithmetic does). */
  return (int32_t)((uint32_t)1000u * (uint32_t)seed + (uint32_t)i);
}

/* Per-block proposal shard constants (coded_greedy_sampler.py:42-45). */
static void shard_params(const float* p_loc, const float* p_scale, int64_t d, int n_steps,
                         float rho, float* loc_s, float* scale_s) {
  float nst = (float)n_steps;
  float sdiv = (float)sqrt((double)n_steps); /* np.sqrt(n_steps) -> float32 */
  for (int64_t j = 0; j < d; ++j) {
    loc_s[j] = p_loc[j] / nst;
    float rs = rho * p_scale[j];
    scale_s[j] = rs / sdiv;
  }
}

/* Streaming evaluation of candidate rows: the reference materialises the
 * [2^b, d] tensors; the values computed per element are identical. */
typedef struct {
  uint32_t key[2], ctr[4];
  uint64_t cur_grp;
  int have;
  float z[4];
} normal_stream;

static inline float stream_normal(normal_stream* st, uint64_t k) {
  uint64_t g = k >> 2;
  if (!st->have || st->cur_grp != g) {
    normal_group(st->key, st->ctr, g, st->z);
    st->cur_grp = g;
    st->have = 1;
  }
  return st->z[k & 3] * 1.0f + 0.0f;
}

/* code_greedy_sample for ONE block of d dims (coded_greedy_sampler.py:29-89).
 * out_idx[n_steps], out_sample[d].  Returns 0 on success.  log_scale: NULL
 * (the declared normaliser, glibc logf of t_scale) or the log(sigma_j) to use
 * instead (normaliser sensitivity, tools/normaliser_sensitivity.py). */
static int code_greedy_sample_impl(const float* t_loc, const float* t_scale,
                                   const float* p_loc, const float* p_scale, int64_t d,
                                   int n_bits_per_step, int n_steps, int32_t seed, float rho,
                                   const float* log_scale, int32_t* out_idx, float* out_sample,
                                   double* out_gap);

CWQO_API int cwqo_code_greedy_sample(const float* t_loc, const float* t_scale,
                                     const float* p_loc, const float* p_scale, int64_t d,
                                     int n_bits_per_step, int n_steps, int32_t seed, float rho,
                                     int32_t* out_idx, float* out_sample) {
  return code_greedy_sample_impl(t_loc, t_scale, p_loc, p_scale, d, n_bits_per_step, n_steps,
                                 seed, rho, NULL, out_idx, out_sample, NULL);
}

static int code_greedy_sample_impl(const float* t_loc, const float* t_scale,
                                   const float* p_loc, const float* p_scale, int64_t d,
                                   int n_bits_per_step, int n_steps, int32_t seed, float rho,
                                   const float* log_scale, int32_t* out_idx, float* out_sample,
                                   double* out_gap) {
  if (n_bits_per_step < 0 || n_bits_per_step > 30 || n_steps < 1 || d < 0) return -1;
  int64_t n_samples = (int64_t)1 << n_bits_per_step;
  size_t db = (size_t)(d > 0 ? d : 1) * sizeof(float);
  float* loc_s = (float*)malloc(db);
  float* scale_s = (float*)malloc(db);
  float* lognorm = (float*)malloc(db);
  float* row = (float*)malloc(db);
  if (!loc_s || !scale_s || !lognorm || !row) {
    free(loc_s); free(scale_s); free(lognorm); free(row);
    return -2;
  }
  shard_params(p_loc, p_scale, d, n_steps, rho, loc_s, scale_s);
  for (int64_t j = 0; j < d; ++j)
    lognorm[j] = log_scale ? half_log_2pi_f32() + log_scale[j]
                           : cwqo_log_normalization(t_scale[j]);
  for (int64_t j = 0; j < d; ++j) out_sample[j] = 0.0f; /* tf.zeros */

  for (int i = 0; i < n_steps; ++i) {
    normal_stream st;
    memset(&st, 0, sizeof(st));
    cwqo_generate_key(step_seed(seed, i), 42, st.key, st.ctr);
    int64_t best_idx = 0;
    float best_val = -FLT_MAX; /* ArgMaxTupleReducer initial accumulator */
    float second_val = -FLT_MAX; /* diagnostics only (out_gap) */
    for (int64_t n = 0; n < n_samples; ++n) {
      for (int64_t j = 0; j < d; ++j) {
        float z = stream_normal(&st, (uint64_t)(n * d + j));
        float s = scale_s[j] * z;       /* misc.py:14 */
        s = loc_s[j] + s;               /* misc.py:15 */
        float tv = out_sample[j] + s;   /* coded_greedy_sampler.py:57 */
        row[j] = log_prob_c(tv, t_loc[j], t_scale[j], lognorm[j]); /* :59 */
      }
      float v = cwqo_eigen_rowsum(row, d); /* :59 reduce_sum axis=1 */
      if (v > best_val) { second_val = best_val; best_val = v; best_idx = n; } /* :61 argmax */
      else if (v > second_val) second_val = v;
    }
    if (out_gap) out_gap[i] = (double)best_val - (double)second_val;
    /* :63 best_sample = test_samples[index, :] */
    for (int64_t j = 0; j < d; ++j) {
      float z = stream_normal(&st, (uint64_t)(best_idx * d + j));
      float s = scale_s[j] * z;
      s = loc_s[j] + s;
      row[j] = out_sample[j] + s;
    }
    memcpy(out_sample, row, (size_t)d * sizeof(float));
    out_idx[i] = (int32_t)best_idx;
  }
  free(loc_s); free(scale_s); free(lognorm); free(row);
  return 0;
}

/* decode_greedy_sample for ONE block (coded_greedy_sampler.py:93-167). */
CWQO_API int cwqo_decode_greedy_sample(const int32_t* idx, const float* p_loc,
                                       const float* p_scale, int64_t d, int n_bits_per_step,
                                       int n_steps, int32_t seed, float rho, float* out_sample) {
  if (n_bits_per_step < 0 || n_bits_per_step > 30 || n_steps < 1 || d < 0) return -1;
  size_t db = (size_t)(d > 0 ? d : 1) * sizeof(float);
  float* loc_s = (float*)malloc(db);
  float* scale_s = (float*)malloc(db);
  if (!loc_s || !scale_s) { free(loc_s); free(scale_s); return -2; }
  shard_params(p_loc, p_scale, d, n_steps, rho, loc_s, scale_s);
  for (int64_t j = 0; j < d; ++j) out_sample[j] = 0.0f;
  for (int i = 0; i < n_steps; ++i) {
    normal_stream st;
    memset(&st, 0, sizeof(st));
    cwqo_generate_key(step_seed(seed, i), 42, st.key, st.ctr);
    int64_t n = idx[i];
    if (n < 0 || n >= ((int64_t)1 << n_bits_per_step)) { free(loc_s); free(scale_s); return -3; }
    for (int64_t j = 0; j < d; ++j) {
      float z = stream_normal(&st, (uint64_t)(n * d + j));
      float s = scale_s[j] * z;
      s = loc_s[j] + s;
      out_sample[j] = out_sample[j] + s; /* :151-158 samples = tile(sample) + ... */
    }
  }
  free(loc_s); free(scale_s);
  return 0;
}

/* code_greedy_sample for ONE block and ONE step with the candidate rows split
 * over OpenMP threads (the per-block coder above is serial over rows): each
 * thread scans a contiguous row range with the reference's argmax rule
 * (strictly greater replaces, from -FLT_MAX), and the ranges are merged in
 * row order with the same rule, so the first maximal row wins as in the serial
 * scan (coded_greedy_sampler.py:59-63).  For blocks too large for one core:
 * the tests of launches whose Philox block indices pass 2^32. */
CWQO_API int cwqo_code_greedy_sample_rows(const float* t_loc, const float* t_scale,
                                          const float* p_loc, const float* p_scale, int64_t d,
                                          int n_bits_per_step, int32_t seed, float rho,
                                          int32_t* out_idx, float* out_sample, int nthreads) {
  if (n_bits_per_step < 0 || n_bits_per_step > 30 || d < 1) return -1;
  const int64_t n_samples = (int64_t)1 << n_bits_per_step;
  const size_t db = (size_t)d * sizeof(float);
  float* loc_s = (float*)malloc(db);
  float* scale_s = (float*)malloc(db);
  float* lognorm = (float*)malloc(db);
  if (!loc_s || !scale_s || !lognorm) {
    free(loc_s); free(scale_s); free(lognorm);
    return -2;
  }
  shard_params(p_loc, p_scale, d, 1, rho, loc_s, scale_s);
  for (int64_t j = 0; j < d; ++j) lognorm[j] = cwqo_log_normalization(t_scale[j]);
  uint32_t key[2], ctr[4];
  cwqo_generate_key(step_seed(seed, 0), 42, key, ctr);
  const int64_t nchunk = 1024;
  float* cval = (float*)malloc(sizeof(float) * nchunk);
  int64_t* cidx = (int64_t*)malloc(sizeof(int64_t) * nchunk);
  int err = 0;
  if (!cval || !cidx) err = 1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
  for (int64_t ch = 0; ch < nchunk; ++ch) {
    if (!cval || !cidx) continue;
    float* row = (float*)malloc(db);
    if (!row) { err |= 1; continue; }
    normal_stream st;
    memset(&st, 0, sizeof(st));
    memcpy(st.key, key, sizeof(key));
    memcpy(st.ctr, ctr, sizeof(ctr));
    const int64_t n0 = n_samples * ch / nchunk, n1 = n_samples * (ch + 1) / nchunk;
    float bv = -FLT_MAX;
    int64_t bi = n0;
    for (int64_t n = n0; n < n1; ++n) {
      for (int64_t j = 0; j < d; ++j) {
        float z = stream_normal(&st, (uint64_t)(n * d + j));
        float s = scale_s[j] * z;
        s = loc_s[j] + s;
        float tv = 0.0f + s; /* step 0: best_sample is tf.zeros */
        row[j] = log_prob_c(tv, t_loc[j], t_scale[j], lognorm[j]);
      }
      float v = cwqo_eigen_rowsum(row, d);
      if (v > bv) { bv = v; bi = n; }
    }
    cval[ch] = bv;
    cidx[ch] = n1 > n0 ? bi : -1;
    free(row);
  }
  if (!err) {
    float best_val = -FLT_MAX;
    int64_t best_idx = 0;
    for (int64_t ch = 0; ch < nchunk; ++ch)
      if (cidx[ch] >= 0 && cval[ch] > best_val) { best_val = cval[ch]; best_idx = cidx[ch]; }
    normal_stream st;
    memset(&st, 0, sizeof(st));
    memcpy(st.key, key, sizeof(key));
    memcpy(st.ctr, ctr, sizeof(ctr));
    for (int64_t j = 0; j < d; ++j) {
      float z = stream_normal(&st, (uint64_t)(best_idx * d + j));
      float s = scale_s[j] * z;
      out_sample[j] = 0.0f + (loc_s[j] + s);
    }
    out_idx[0] = (int32_t)best_idx;
  }
  free(cval); free(cidx); free(loc_s); free(scale_s); free(lognorm);
  return err ? -2 : 0;
}

/* Batched (CSR) encoder: block g = dims [off[g], off[g+1]), seed + block_id_base + g
 * (coded_greedy_sampler.py:282 `seed_feed: seed + i`).  OpenMP over blocks.
 * nthreads <= 0 -> OpenMP default. */
CWQO_API int cwqo_greedy_encode(const float* t_loc, const float* t_scale, const float* p_loc,
                                const float* p_scale, const int64_t* block_off, int64_t nb,
                                int n_bits_per_step, int n_steps, int32_t seed, float rho,
                                int64_t block_id_base, int32_t* out_idx, float* out_sample,
                                int nthreads) {
  int err = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
  for (int64_t g = 0; g < nb; ++g) {
    int64_t o = block_off[g], d = block_off[g + 1] - block_off[g];
    int32_t sg = (int32_t)((uint32_t)seed + (uint32_t)(block_id_base + g));
    int rc = cwqo_code_greedy_sample(t_loc + o, t_scale + o, p_loc + o, p_scale + o, d,
                                     n_bits_per_step, n_steps, sg, rho,
                                     out_idx + g * n_steps, out_sample + o);
    if (rc) err |= 1;
  }
  return err ? -1 : 0;
}

/* cwqo_greedy_encode with the per-dim log(sigma) supplied (log_scale [D], or
 * NULL for logf) and, if out_gap is non-NULL, the gap between the best and the
 * second-best row value of every step: the normaliser sensitivity experiments
 * (DESIGN.md 2). */
CWQO_API int cwqo_greedy_encode_lsig(const float* t_loc, const float* t_scale,
                                     const float* p_loc, const float* p_scale,
                                     const int64_t* block_off, int64_t nb, int n_bits_per_step,
                                     int n_steps, int32_t seed, float rho, int64_t block_id_base,
                                     const float* log_scale, int32_t* out_idx, float* out_sample,
                                     double* out_gap, int nthreads) {
  int err = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
  for (int64_t g = 0; g < nb; ++g) {
    int64_t o = block_off[g], d = block_off[g + 1] - block_off[g];
    int32_t sg = (int32_t)((uint32_t)seed + (uint32_t)(block_id_base + g));
    int rc = code_greedy_sample_impl(t_loc + o, t_scale + o, p_loc + o, p_scale + o, d,
                                     n_bits_per_step, n_steps, sg, rho,
                                     log_scale ? log_scale + o : NULL, out_idx + g * n_steps,
                                     out_sample + o, out_gap ? out_gap + g * n_steps : NULL);
    if (rc) err |= 1;
  }
  return err ? -1 : 0;
}

/* ------------------------------------------------------------------------ */
/* Per-candidate semantics sensitivity (tools/semantics_        */
/* sensitivity.py).  The declared row value (A.5 TFP<=0.7 log_prob, A.6 Eigen */
/* 3.3 AVX order) is one of several a TF build could have computed; these    */
/* variants change every candidate's value by a different rounding, so they  */
/* are the choices that could move an argmax.  [ext] all recalled from the   */
/* libraries' public sources, unverifiable offline.                          */
/* ------------------------------------------------------------------------ */
#define SEM_NFORM 2 /* 0: TFP<=0.7 (declared), 1: TFP>=0.8 squared_difference */
#define SEM_NSUM 6  /* row-sum orders, see sem_rowsum */
/* RNG transcendentals (round 5): the declared form and order on
 * normals a TF build with another logf / sincosf (a non-glibc libm, TF-GPU's
 * device functions, Eigen numext) or another 2pi evaluation could have drawn:
 *   0 ulp_hash  every Box-Muller output one ulp away from glibc's, up or down
 *               by a hash of (stream, flat index): the proxy for a libm whose
 *               results differ in the last place at random;
 *   1 ulp_up    every output one ulp toward +inf;
 *   2 ulp_down  every output one ulp toward -inf;
 *   3 v1_f32    the angle in float, (2.0f * (float)M_PI) * U(x1), instead of
 *               TF's double 2.0f * M_PI (a build whose constant is a float). */
#define SEM_NRNG 4
#define SEM_NV (SEM_NFORM * SEM_NSUM + SEM_NRNG)

/* TFP >= 0.8 Normal._log_prob:
 *   -0.5 * squared_difference(x / scale, loc / scale) - (0.5 log 2pi + log scale)
 * squared_difference(a, b) = (a - b) * (a - b). */
static inline float log_prob_tfp08(float x, float loc, float scale, float lognorm) {
  float a = x / scale, b = loc / scale;
  float dd = a - b;
  float u = -0.5f * (dd * dd);
  return u - lognorm;
}

/* Eigen InnerMostDimReducer<SumReducer> packet orders:
 *  0 avx8   Packet8f (declared, cwqo_eigen_rowsum)
 *  1 sse4   Packet4f: 4 lane partials, predux (p0+p2)+(p1+p3), tail t, t + r
 *  2 avx8x2 Eigen 3.4 style: two Packet8f accumulators over packet pairs,
 *           leftover packet into the first, then p + p2, predux as avx8
 *  3 avx512 Packet16f (AVX512DQ predux): fold the 16 partials to 8 as
 *           l + (l + 8), then the avx8 predux
 *  4 seq    a scalar (non-vectorised) build: ((x0 + x1) + x2) + ...
 *  5 tree   pairwise halving: sum(x[0:h]) + sum(x[h:n]), h = n / 2 (a GPU-style
 *           tree, representative only) */
static float packet_sum(const float* x, int64_t d, int w, int npacc) {
  float p[2][16];
  memset(p, 0, sizeof(p));
  int64_t vec = (d / w) * w;
  int64_t np = vec / w, pairs = npacc == 2 ? (np / 2) * 2 : 0;
  int64_t k = 0;
  for (; k < pairs; k += 2)
    for (int a = 0; a < 2; ++a)
      for (int l = 0; l < w; ++l) p[a][l] = p[a][l] + x[(k + a) * w + l];
  for (; k < np; ++k)
    for (int l = 0; l < w; ++l) p[0][l] = p[0][l] + x[k * w + l];
  if (npacc == 2)
    for (int l = 0; l < w; ++l) p[0][l] = p[0][l] + p[1][l];
  float t = 0.0f;
  for (int64_t j = vec; j < d; ++j) t = t + x[j];
  float* q = p[0];
  if (w == 16) for (int l = 0; l < 8; ++l) q[l] = q[l] + q[l + 8];
  if (w >= 8) for (int l = 0; l < 4; ++l) q[l] = q[l] + q[l + 4];
  float r = (q[0] + q[2]) + (q[1] + q[3]);
  return t + r;
}

static float tree_sum(const float* x, int64_t n) {
  if (n <= 0) return 0.0f;
  if (n == 1) return x[0];
  int64_t h = n / 2;
  return tree_sum(x, h) + tree_sum(x + h, n - h);
}

static float sem_rowsum(const float* x, int64_t d, int order) {
  switch (order) {
    case 0: return cwqo_eigen_rowsum(x, d);
    case 1: return packet_sum(x, d, 4, 1);
    case 2: return packet_sum(x, d, 8, 2);
    case 3: return packet_sum(x, d, 16, 1);
    case 4: {
      float s = 0.0f;
      for (int64_t j = 0; j < d; ++j) s = s + x[j];
      return s;
    }
    default: return tree_sum(x, d);
  }
}

CWQO_API int cwqo_sem_num_variants(void) { return SEM_NV; }

static inline uint64_t mix64(uint64_t x) {  /* splitmix64 finaliser */
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

/* The normals of Philox group `grp` twice: z as declared (A.4) and zf with
 * the float angle (RNG variant v1_f32). */
static void normal_group_f32angle(const uint32_t key[2], const uint32_t ctr[4], uint64_t grp,
                                  float z[4], float zf[4]) {
  uint32_t c[4], x[4];
  philox_skip(ctr, grp, c);
  cwqo_philox4x32_10(c, key, x);
  for (int h = 0; h < 2; ++h) {
    const float u2 = cwqo_bm_radius(x[2 * h]);
    float sn, cs;
    cwqo_bm_sincos(x[2 * h + 1], &sn, &cs);
    z[2 * h] = sn * u2;
    z[2 * h + 1] = cs * u2;
    const float v1f = (2.0f * (float)M_PI) * uint32_to_float(x[2 * h + 1]);
    sincosf(v1f, &sn, &cs);
    zf[2 * h] = sn * u2;
    zf[2 * h + 1] = cs * u2;
  }
}

typedef struct {
  uint32_t key[2], ctr[4];
  uint64_t cur_grp, sid;
  int have;
  float z[4], zf[4];
} rng_stream;

/* normal k of the stream under the declared generator (v < 0) or RNG
 * variant v */
static inline float rng_normal(rng_stream* st, uint64_t k, int v) {
  const uint64_t g = k >> 2;
  if (!st->have || st->cur_grp != g) {
    normal_group_f32angle(st->key, st->ctr, g, st->z, st->zf);
    st->cur_grp = g;
    st->have = 1;
  }
  const float z = st->z[k & 3] * 1.0f + 0.0f;
  switch (v) {
    case 0: return nextafterf(z, (mix64(st->sid ^ mix64(k)) & 1u) ? INFINITY : -INFINITY);
    case 1: return nextafterf(z, INFINITY);
    case 2: return nextafterf(z, -INFINITY);
    case 3: return st->zf[k & 3] * 1.0f + 0.0f;
    default: return z;
  }
}
CWQO_API float cwqo_sem_rowsum(const float* x, int64_t d, int order) {
  return sem_rowsum(x, d, order);
}

/* The encoder of code_greedy_sample_impl with every candidate row also scored
 * under the SEM_NV variants v = form * SEM_NSUM + order (v = 0 is the declared
 * semantics).  The chain of best samples follows the declared argmax, so
 * out_vidx[(g * n_steps + i) * SEM_NV + v] is the index variant v would emit
 * at step i given the same history: a conditional per-index flip test.
 * out_gap[g * n_steps + i]: declared best minus second-best row value;
 * out_dev[(g * n_steps + i) * SEM_NV + v] (optional): variant v's value of the
 * declared best row minus the declared value (how far each choice moves a row). */
CWQO_API int cwqo_greedy_encode_semvar(const float* t_loc, const float* t_scale,
                                       const float* p_loc, const float* p_scale,
                                       const int64_t* block_off, int64_t nb,
                                       int n_bits_per_step, int n_steps, int32_t seed,
                                       float rho, int64_t block_id_base, int32_t* out_vidx,
                                       float* out_sample, double* out_gap, float* out_dev,
                                       int nthreads) {
  if (n_bits_per_step < 0 || n_bits_per_step > 30 || n_steps < 1) return -1;
  int err = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
  for (int64_t g = 0; g < nb; ++g) {
    const int64_t o = block_off[g], d = block_off[g + 1] - block_off[g];
    const int32_t sg = (int32_t)((uint32_t)seed + (uint32_t)(block_id_base + g));
    const float *tl = t_loc + o, *ts = t_scale + o;
    float* best = out_sample + o;
    const size_t db = (size_t)(d > 0 ? d : 1) * sizeof(float);
    float* loc_s = (float*)malloc(db);
    float* scale_s = (float*)malloc(db);
    float* lognorm = (float*)malloc(db);
    float* row = (float*)malloc((2 + SEM_NRNG) * db);
    if (!loc_s || !scale_s || !lognorm || !row) {
      free(loc_s); free(scale_s); free(lognorm); free(row);
      err |= 1;
      continue;
    }
    float* row8 = row + (d > 0 ? d : 1);
    float* rowr = row8 + (d > 0 ? d : 1);  /* [SEM_NRNG][d]: the RNG variants' rows */
    shard_params(p_loc + o, p_scale + o, d, n_steps, rho, loc_s, scale_s);
    for (int64_t j = 0; j < d; ++j) lognorm[j] = cwqo_log_normalization(ts[j]);
    for (int64_t j = 0; j < d; ++j) best[j] = 0.0f;
    const int64_t n_samples = (int64_t)1 << n_bits_per_step;
    for (int i = 0; i < n_steps; ++i) {
      rng_stream st;
      memset(&st, 0, sizeof(st));
      cwqo_generate_key(step_seed(sg, i), 42, st.key, st.ctr);
      st.sid = mix64(((uint64_t)st.key[0] << 32 | st.key[1]) ^
                     mix64((uint64_t)st.ctr[2] << 32 | st.ctr[3]));
      float bv[SEM_NV], bdev[SEM_NV];
      int64_t bi[SEM_NV];
      for (int v = 0; v < SEM_NV; ++v) { bv[v] = -FLT_MAX; bi[v] = 0; }
      float second = -FLT_MAX;
      for (int v = 0; v < SEM_NV; ++v) bdev[v] = 0.0f;
      for (int64_t n = 0; n < n_samples; ++n) {
        for (int64_t j = 0; j < d; ++j) {
          const uint64_t k = (uint64_t)(n * d + j);
          float z = rng_normal(&st, k, -1);
          float s = scale_s[j] * z;
          s = loc_s[j] + s;
          float tv = best[j] + s;
          row[j] = log_prob_c(tv, tl[j], ts[j], lognorm[j]);
          row8[j] = log_prob_tfp08(tv, tl[j], ts[j], lognorm[j]);
          for (int r = 0; r < SEM_NRNG; ++r) {
            float sr = scale_s[j] * rng_normal(&st, k, r);
            sr = loc_s[j] + sr;
            rowr[r * d + j] = log_prob_c(best[j] + sr, tl[j], ts[j], lognorm[j]);
          }
        }
        float vals[SEM_NV];
        for (int v = 0; v < SEM_NV; ++v) {
          const int f = v < SEM_NFORM * SEM_NSUM ? v / SEM_NSUM : 0;
          const int ord = v < SEM_NFORM * SEM_NSUM ? v % SEM_NSUM : 0;
          const float* rv = v < SEM_NFORM * SEM_NSUM ? (f ? row8 : row)
                                                     : rowr + (v - SEM_NFORM * SEM_NSUM) * d;
          const float val = sem_rowsum(rv, d, ord);
          vals[v] = val;
          if (v == 0) {
            if (val > bv[0]) second = bv[0];
            else if (val > second) second = val;
          }
          if (val > bv[v]) { bv[v] = val; bi[v] = n; }
        }
        if (bi[0] == n) /* the declared best row so far: each variant's deviation on it */
          for (int v = 0; v < SEM_NV; ++v) bdev[v] = vals[v] - vals[0];
      }
      if (out_gap) out_gap[g * n_steps + i] = (double)bv[0] - (double)second;
      for (int v = 0; v < SEM_NV; ++v) {
        out_vidx[(g * n_steps + i) * SEM_NV + v] = (int32_t)bi[v];
        if (out_dev) out_dev[(g * n_steps + i) * SEM_NV + v] = bdev[v];
      }
      for (int64_t j = 0; j < d; ++j) {
        float z = rng_normal(&st, (uint64_t)(bi[0] * d + j), -1);
        float s = scale_s[j] * z;
        s = loc_s[j] + s;
        best[j] = best[j] + s;
      }
    }
    free(loc_s); free(scale_s); free(lognorm); free(row);
  }
  return err ? -1 : 0;
}

/* Eigen 3.3 plog<Packet8f> (Eigen/src/Core/arch/AVX/MathFunctions.h, the
 * Cephes single-precision log) on one lane -- [ext] restated from Eigen's
 * published source, not from /root/reference: TF's CPU kernel evaluates
 * log(scale) with it for full 8-wide packets.  fma != 0 uses
 * fused pmadd (an -mfma build); 0 the mul + add of a plain -mavx build (TF 1.x
 * pip wheels).  Used only by the normaliser sensitivity experiment. */
static inline float madd(float a, float b, float c, int fma) {
  return fma ? fmaf(a, b, c) : a * b + c;
}
CWQO_API float cwqo_eigen_plog(float x0, int fma) {
  if (!(x0 >= 0.0f)) return NAN;      /* invalid_mask (also NaN) */
  if (x0 == 0.0f) return -INFINITY;   /* iszero_mask */
  float x = x0 < 1.17549435e-38f ? 1.17549435e-38f : x0;  /* pmax(x, min_norm_pos) */
  uint32_t u;
  memcpy(&u, &x, 4);
  float e = (float)(int32_t)(u >> 23) - 126.0f;
  u = (u & ~0x7f800000u) | 0x3f000000u;  /* mantissa in [0.5, 1) */
  memcpy(&x, &u, 4);
  const int lt = x < 0.707106781186547524f;
  const float tmp0 = lt ? x : 0.0f;
  x = x - 1.0f;
  e = e - (lt ? 1.0f : 0.0f);
  x = x + tmp0;
  const float x2 = x * x;
  const float x3 = x2 * x;
  float y = madd(7.0376836292E-2f, x, -1.1514610310E-1f, fma);
  float y1 = madd(-1.2420140846E-1f, x, +1.4249322787E-1f, fma);
  float y2 = madd(+2.0000714765E-1f, x, -2.4999993993E-1f, fma);
  y = madd(y, x, 1.1676998740E-1f, fma);
  y1 = madd(y1, x, -1.6668057665E-1f, fma);
  y2 = madd(y2, x, +3.3333331174E-1f, fma);
  y = madd(y, x3, y1, fma);
  y = madd(y, x3, y2, fma);
  y = y * x3;
  y1 = e * -2.12194440e-4f;
  const float tmp = x2 * 0.5f;
  y = y + y1;
  x = x - tmp;
  y2 = e * 0.693359375f;
  x = x + y;
  x = x + y2;
  return x;
}

CWQO_API void cwqo_eigen_plog_table(const float* x, int64_t n, int fma, float* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = cwqo_eigen_plog(x[i], fma);
}

CWQO_API int cwqo_greedy_decode(const int32_t* idx, const float* p_loc, const float* p_scale,
                                const int64_t* block_off, int64_t nb, int n_bits_per_step,
                                int n_steps, int32_t seed, float rho, int64_t block_id_base,
                                float* out_sample, int nthreads) {
  int err = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16) reduction(| : err)
#endif
  for (int64_t g = 0; g < nb; ++g) {
    int64_t o = block_off[g], d = block_off[g + 1] - block_off[g];
    int32_t sg = (int32_t)((uint32_t)seed + (uint32_t)(block_id_base + g));
    int rc = cwqo_decode_greedy_sample(idx + g * n_steps, p_loc + o, p_scale + o, d,
                                       n_bits_per_step, n_steps, sg, rho, out_sample + o);
    if (rc) err |= 1;
  }
  return err ? -1 : 0;
}

/* ------------------------------------------------------------------------ */
/* Grouped wrapper numerics (coded_greedy_sampler.py:193-244, 292).          */
/* ------------------------------------------------------------------------ */
/* :198-199 standardise the target by the proposal (float32 ops). */
CWQO_API void cwqo_standardise(const float* q_loc, const float* q_scale, const float* p_loc,
                               const float* p_scale, int64_t n, float* t_loc, float* t_scale) {
  for (int64_t i = 0; i < n; ++i) {
    float dl = q_loc[i] - p_loc[i];
    t_loc[i] = dl / p_scale[i];
    t_scale[i] = q_scale[i] / p_scale[i];
  }
}

/* A.9 TFP (<=0.7) _kl_normal_normal(a=target, b=proposal), float32. */
CWQO_API void cwqo_kl_normal_normal(const float* a_loc, const float* a_scale,
                                    const float* b_loc, const float* b_scale, int64_t n,
                                    float* out) {
  for (int64_t i = 0; i < n; ++i) {
    float sa2 = a_scale[i] * a_scale[i];
    float sb2 = b_scale[i] * b_scale[i];
    float ratio = sa2 / sb2;
    float dl = a_loc[i] - b_loc[i];
    float t1 = (dl * dl) / (2.0f * sb2);
    float t2 = 0.5f * ((ratio - 1.0f) - logf(ratio));
    out[i] = t1 + t2;
  }
}

/* :207-244 greedy grouping.  size_threshold = smallest s with
 * np.log(s+1)/np.log(2) >= max_group_size_bits (computed by the caller with
 * NumPy, exactly as the reference evaluates it).  The running group KL is a
 * float32 (numpy float32 scalar arithmetic); the comparison is done in float64
 * against n_nats = n_bits_per_group*np.log(2) - 1.
 * Writes starts[0..n_starts) = [0, ...boundaries..., D]; returns n_starts or
 * -1 if cap is too small. */
CWQO_API int64_t cwqo_group_starts(const float* kl, int64_t D, int64_t size_threshold,
                                   double n_nats, int64_t* starts, int64_t cap) {
  int64_t ns = 0;
  if (cap < 1) return -1;
  starts[ns++] = 0;
  int64_t cur_size = 0;
  float cur_kl = 0.0f;
  for (int64_t idx = 0; idx < D; ++idx) {
    float s = cur_kl + kl[idx];
    if (cur_size >= size_threshold || (double)s >= n_nats || idx == D - 1) {
      if (ns >= cap) return -1;
      starts[ns++] = idx;
      cur_size = 1;
      cur_kl = kl[idx];
    } else {
      cur_kl = s;
      cur_size += 1;
    }
  }
  if (ns >= cap) return -1;
  starts[ns++] = D; /* :252 group_start_indices += [num_dimensions] */
  return ns;
}

/* :292 sample = proposal.scale * sample + proposal.loc (float32, two roundings) */
CWQO_API void cwqo_destandardise(const float* sample, const float* p_loc, const float* p_scale,
                                 int64_t n, float* out) {
  for (int64_t i = 0; i < n; ++i) {
    float m = p_scale[i] * sample[i];
    out[i] = m + p_loc[i];
  }
}

CWQO_API int cwqo_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ------------------------------------------------------------------------ */
/* Batch tables for exhaustive transcendental checks (glibc = declared       */
/* semantics).  m is the 23-bit mantissa field of the Philox word.           */
/* ------------------------------------------------------------------------ */
CWQO_API void cwqo_bm_radius_table(uint32_t m0, int64_t count, float* out) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (int64_t i = 0; i < count; ++i) out[i] = cwqo_bm_radius((uint32_t)(m0 + i));
}

CWQO_API void cwqo_bm_sincos_table(uint32_t m0, int64_t count, float* s, float* c) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (int64_t i = 0; i < count; ++i) cwqo_bm_sincos((uint32_t)(m0 + i), &s[i], &c[i]);
}

CWQO_API void cwqo_logf_table(const float* x, int64_t n, float* out) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (int64_t i = 0; i < n; ++i) out[i] = logf(x[i]);
}

/* ------------------------------------------------------------------------ */
/* Importance sampler (code/coded_importance_sampler.py).                    */
/* ------------------------------------------------------------------------ */
/* :48-51 num_samples = int32(ceil(exp(reduce_sum(KL(target || proposal)))))
 * (float32 KL per dim, Eigen-order sum, glibc expf, ceilf). */
CWQO_API int64_t cwqo_importance_num_samples(const float* t_loc, const float* t_scale,
                                             const float* p_loc, const float* p_scale,
                                             int64_t d) {
  float* kl = (float*)malloc((size_t)(d > 0 ? d : 1) * sizeof(float));
  if (!kl) return -1;
  cwqo_kl_normal_normal(t_loc, t_scale, p_loc, p_scale, d, kl);
  float total = cwqo_eigen_rowsum(kl, d);
  free(kl);
  float e = ceilf(expf(total));
  return (int64_t)(int32_t)e;
}

/* Given per-dim KLs and group starts (group g = [s[g], s[g+1])), the same
 * count per group from the precomputed KLs. */
CWQO_API void cwqo_importance_plan(const float* kl, const int64_t* starts, int64_t ng,
                                   int64_t* n_samples) {
  for (int64_t g = 0; g < ng; ++g) {
    float total = cwqo_eigen_rowsum(kl + starts[g], starts[g + 1] - starts[g]);
    n_samples[g] = (int64_t)(int32_t)ceilf(expf(total));
  }
}

/* code_importance_sample for ONE block (:29-79): samples = stateless_normal_sample(
 * p_loc, p_scale, num_samples, seed) (note: `seed` itself, not 1000*seed+i);
 * weights = reduce_sum(target.log_prob(x) - proposal.log_prob(x), axis=1);
 * index = argmax.  Writes the 0-based index and best_sample [d]. */
CWQO_API int cwqo_importance_encode_block(const float* t_loc, const float* t_scale,
                                          const float* p_loc, const float* p_scale, int64_t d,
                                          int32_t seed, int64_t n_samples, int64_t* out_index,
                                          float* out_sample) {
  if (d < 0 || n_samples < 1) return -1;
  size_t db = (size_t)(d > 0 ? d : 1) * sizeof(float);
  float* ct = (float*)malloc(db);
  float* cp = (float*)malloc(db);
  float* row = (float*)malloc(db);
  if (!ct || !cp || !row) { free(ct); free(cp); free(row); return -2; }
  for (int64_t j = 0; j < d; ++j) {
    ct[j] = cwqo_log_normalization(t_scale[j]);
    cp[j] = cwqo_log_normalization(p_scale[j]);
  }
  normal_stream st;
  memset(&st, 0, sizeof(st));
  cwqo_generate_key(seed, 42, st.key, st.ctr);
  int64_t best_idx = 0;
  float best_val = -FLT_MAX;
  for (int64_t n = 0; n < n_samples; ++n) {
    for (int64_t j = 0; j < d; ++j) {
      float z = stream_normal(&st, (uint64_t)(n * d + j));
      float x = p_scale[j] * z;  /* misc.py:14 */
      x = p_loc[j] + x;          /* misc.py:15 */
      float lt = log_prob_c(x, t_loc[j], t_scale[j], ct[j]);
      float lp = log_prob_c(x, p_loc[j], p_scale[j], cp[j]);
      row[j] = lt - lp;          /* :60 */
    }
    float v = cwqo_eigen_rowsum(row, d);
    if (v > best_val) { best_val = v; best_idx = n; }
  }
  for (int64_t j = 0; j < d; ++j) {
    float z = stream_normal(&st, (uint64_t)(best_idx * d + j));
    float x = p_scale[j] * z;
    out_sample[j] = p_loc[j] + x; /* :63 samples[index] */
  }
  *out_index = best_idx;
  free(ct); free(cp); free(row);
  return 0;
}

/* decode_importance_sample (:82-109): the last of index+1 samples = row index. */
CWQO_API void cwqo_importance_decode_block(int64_t index, const float* p_loc,
                                           const float* p_scale, int64_t d, int32_t seed,
                                           float* out_sample) {
  normal_stream st;
  memset(&st, 0, sizeof(st));
  cwqo_generate_key(seed, 42, st.key, st.ctr);
  for (int64_t j = 0; j < d; ++j) {
    float z = stream_normal(&st, (uint64_t)(index * d + j));
    float x = p_scale[j] * z;
    out_sample[j] = p_loc[j] + x;
  }
}

/* Batched over CSR groups with per-group counts; group g uses seed+base+g (:243). */
CWQO_API int cwqo_importance_encode(const float* t_loc, const float* t_scale, const float* p_loc,
                                    const float* p_scale, const int64_t* block_off, int64_t nb,
                                    const int64_t* n_samples, int32_t seed,
                                    int64_t block_id_base, int64_t* out_index,
                                    float* out_sample, int nthreads) {
  int err = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
  for (int64_t g = 0; g < nb; ++g) {
    int64_t o = block_off[g], d = block_off[g + 1] - block_off[g];
    int32_t sg = (int32_t)((uint32_t)seed + (uint32_t)(block_id_base + g));
    if (cwqo_importance_encode_block(t_loc + o, t_scale + o, p_loc + o, p_scale + o, d, sg,
                                     n_samples[g], out_index + g, out_sample + o))
      err |= 1;
  }
  return err ? -1 : 0;
}

/* tf.quantization.quantize(x, -30, 30, tf.quint16) (MIN_COMBINED, unsigned fast
 * path): cast<uint16>((clamp(x) - min) * scale + 0.5f), scale = float(65535/60). */
CWQO_API void cwqo_quantize_quint16(const float* x, int64_t n, float mn, float mx,
                                    uint16_t* out) {
  float scale = (float)((65535.0 - 0.0) / ((double)mx - (double)mn));
  for (int64_t i = 0; i < n; ++i) {
    if (x[i] != x[i]) { /* NaN: code 0, as x86's truncating conversion */
      out[i] = 0;
      continue;
    }
    float v = x[i] < mx ? x[i] : mx;   /* cwiseMin(max_range) */
    v = v > mn ? v : mn;               /* cwiseMax(min_range) */
    float t = (v - mn) * scale;
    t = t + 0.5f;
    out[i] = (uint16_t)t;
  }
}

/* tf.quantization.dequantize(q, -30, 30) for quint16 (MIN_COMBINED):
 * q * ((max - min) / 65535) + min, float32. */
CWQO_API void cwqo_dequantize_quint16(const uint16_t* q, int64_t n, float mn, float mx,
                                      float* out) {
  float sf = (mx - mn) / 65535.0f;
  for (int64_t i = 0; i < n; ++i) {
    float t = (float)q[i] * sf;
    out[i] = t + mn;
  }
}
