// Test shim (not product code): ROCm's own Philox4x32-10, the rocRAND SDK
// header /opt/rocm/include/rocrand/rocrand_philox4x32_10.h (ten_rounds,
// single_round, bumpkey at :270-302; constants :62-65), compiled for the host.
// It is an implementation independent of both the oracle (oracle/cwq_oracle.c)
// and the product header (csrc/cwq_math.h); tests/test_oracle.py compares all
// three on 10^6 random (counter, key) pairs (SURVEY.md 8(c) pin 1).
#include <rocrand/rocrand_philox4x32_10.h>
#include <stdint.h>

namespace {
// ten_rounds is protected in the engine class; a subclass exposes it as is
struct Pin : rocrand_device::philox4x32_10_engine {
  using philox4x32_10_engine::ten_rounds;
};
}  // namespace

extern "C" void rr_philox_many(const uint32_t* ctr, const uint32_t* key, int64_t n,
                               uint32_t* out) {
  Pin e;
  for (int64_t i = 0; i < n; ++i) {
    const uint4 c = {ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]};
    const uint2 k = {key[2 * i], key[2 * i + 1]};
    const uint4 r = e.ten_rounds(c, k);
    out[4 * i] = r.x;
    out[4 * i + 1] = r.y;
    out[4 * i + 2] = r.z;
    out[4 * i + 3] = r.w;
  }
}
