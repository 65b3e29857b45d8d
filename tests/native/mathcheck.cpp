// Host build of the product's device-math restatement (csrc/cwq_math.h), used
// by tests/test_math_exhaustive.py to compare it with the host glibc over the
// full Box-Muller input domains.  Test-only shim; not part of the product.
#include <stdint.h>
#include "../../compression_without_quantization_amd/csrc/cwq_math.h"

static const double kTab[32] = CWQ_LOGF_TAB_INIT;

extern "C" {
void mc_bm_radius_table(uint32_t m0, int64_t count, float* out) {
  for (int64_t i = 0; i < count; ++i) out[i] = cwq::bm_radius((uint32_t)(m0 + i), kTab);
}
void mc_bm_sincos_table(uint32_t m0, int64_t count, float* s, float* c) {
  for (int64_t i = 0; i < count; ++i) cwq::sincosf_pos(cwq::bm_angle((uint32_t)(m0 + i)), s[i], c[i]);
}
void mc_bm_angle_table(uint32_t m0, int64_t count, float* out) {
  for (int64_t i = 0; i < count; ++i) out[i] = cwq::bm_angle((uint32_t)(m0 + i));
}
void mc_logf_table(const float* x, int64_t n, float* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = cwq::logf_full(x[i], kTab);
}
void mc_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
  cwq::U4 r = cwq::philox10(ctr[0], ctr[1], ctr[2], ctr[3], key[0], key[1]);
  out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
}
void mc_philox_many(const uint32_t* ctr, const uint32_t* key, int64_t n, uint32_t* out) {
  for (int64_t i = 0; i < n; ++i) mc_philox(ctr + 4 * i, key + 2 * i, out + 4 * i);
}
}
