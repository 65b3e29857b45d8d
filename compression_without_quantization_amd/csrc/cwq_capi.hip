// cwq_capi.hip -- the C ABI declared in include/cwq.h.
//
// Thin: validates arguments, carves the caller's workspace, picks the tiling
// and enqueues the kernels on the caller's stream.  Never allocates, never
// synchronises, never throws.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>
#include <math.h>
#include <string.h>
#include <time.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <sched.h>
#include <unistd.h>
#include <stdlib.h>
#include <thread>
#include <vector>

#include "../../include/cwq.h"
#include "cwq_debug.h"
#include "cwq_kernels.h"

namespace {

thread_local char g_err[512] = {0};

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int ok() {
  g_err[0] = 0;
  return CWQ_OK;
}

int hip_fail(hipError_t e, const char* where) {
  return fail(CWQ_ERR_HIP, "%s: %s", where, hipGetErrorString(e));
}

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

struct WsLayout {
  size_t keys, tq, loc_s, scale_s, lognorm, sab, cdim, bpre, ordu, grp, gtau, abp, slist;
  size_t sdmap, total;
  bool csr;   // has the general pruned kernel's arrays
  bool recs;  // ... and the visit-order records of blocks longer than CWQ_CSR_LDS_DIMS
};

// Blocks the uniform fast pruned kernel takes (d % 8 == 0, 8 <= d <= 64) need
// only keys + the per-dim shard constants; everything else (CSR, other d) also
// gets the general pruned kernel's screening constants and the screened small-candidate
// path's survivor slots and the small-candidate pipeline's arrays (24 B/dim + 244 B/block),
// and, when some block may exceed CWQ_CSR_LDS_DIMS dims, the visit-order
// records of the long blocks (32 B/dim + 384 B per CWQ_CSR_LDS_DIMS + 1 dims,
// csr_rec_entries: short blocks take no room, so a grouped call sized for
// D + 1 possible groups does not pay 384 B for each).
bool uniform_fast(int64_t d) { return d % 8 == 0 && d >= 8 && d <= 64; }

WsLayout ws_layout(int64_t nb, int64_t total_dims, bool csr, bool recs) {
  WsLayout l;
  size_t o = 0;
  l.keys = o;
  o = align_up(o + (size_t)nb * 8, 256);
  l.tq = o;  // k_encode_prune's tile queue counters
  o = align_up(o + (size_t)cwq::kTileQueueSlots * 4, 256);
  l.loc_s = o;
  o = align_up(o + (size_t)total_dims * 4, 256);
  l.scale_s = o;
  o = align_up(o + (size_t)total_dims * 4, 256);
  l.lognorm = o;
  o = align_up(o + (size_t)total_dims * 4, 256);
  l.csr = csr;
  l.recs = csr && recs;
  l.sab = l.cdim = l.bpre = l.ordu = l.grp = l.gtau = l.abp = l.slist = o;
  l.sdmap = o;
  if (csr) {
    l.slist = o;  // the screened small-candidate path's survivor slots (8 B each)
    o = align_up(o + (size_t)nb * CWQ_SLIST_PER_BLOCK * 8, 256);
    l.sab = o;
    o = align_up(o + (size_t)(total_dims + 8 * nb + 4) * 8, 256);  // + 4 zeros (pad unit)
    l.cdim = o;
    o = align_up(o + (size_t)total_dims * 4, 256);
    l.bpre = o;
    o = align_up(o + (size_t)(total_dims + 12 * nb) * 4, 256);
    l.ordu = o;
    o = align_up(o + (size_t)(total_dims + 12 * nb) * 4, 256);
    l.grp = o;
    o = align_up(o + (size_t)nb * 16, 256);
    l.gtau = o;
    o = align_up(o + (size_t)nb * 4 * CWQ_CSR_GTAU_STRIDE, 256);
    l.sdmap = o;  // the small-candidate pipeline's dim -> block map
    o = align_up(o + (size_t)total_dims * 4, 256);
    if (l.recs) {
      l.abp = o;
      o = align_up(o + (size_t)cwq::csr_rec_entries(total_dims) * 32, 256);
    }
  }
  l.total = o;
  return l;
}
// CSR blocks of at most max_block_dim dims
WsLayout ws_layout_csr(int64_t nb, int64_t total_dims, int64_t max_block_dim) {
  return ws_layout(nb, total_dims, true, max_block_dim > CWQ_CSR_LDS_DIMS);
}
WsLayout ws_layout_uniform(int64_t nb, int64_t d) {
  const bool csr = nb > 0 && !uniform_fast(d);
  return ws_layout(nb, nb * d, csr, d > CWQ_CSR_LDS_DIMS);
}

#ifndef CWQ_TARGET_TILES
#define CWQ_TARGET_TILES 16384  // tiles per launch the tiling aims for (tuning builds)
#endif
void choose_tiling(int64_t nb, int64_t n_cand, int64_t* tiles_per_block, int64_t* cand_per_tile) {
  const int64_t kTargetTiles = CWQ_TARGET_TILES;
  int64_t want = nb > 0 ? (kTargetTiles + nb - 1) / nb : 1;
  int64_t max_split = (n_cand + 255) / 256;  // at least one candidate per lane
  if (want > max_split) want = max_split;
  if (want < 1) want = 1;
  int64_t cpt = (n_cand + want - 1) / want;
  cpt = (cpt + 255) / 256 * 256;
  if (cpt < 256) cpt = 256;
  *cand_per_tile = cpt;
  *tiles_per_block = (n_cand + cpt - 1) / cpt;
}

// Eigen 3.3 AVX inner-dim sum order, host side.
float eigen_sum(const float* x, int64_t d) {
  const int64_t vec = (d / 8) * 8;
  float p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t j = 0; j < vec; j += 8)
    for (int l = 0; l < 8; ++l) p[l] = p[l] + x[j + l];
  float t = 0.0f;
  for (int64_t j = vec; j < d; ++j) t = t + x[j];
  const float q0 = p[0] + p[4], q1 = p[1] + p[5], q2 = p[2] + p[6], q3 = p[3] + p[7];
  return t + ((q0 + q2) + (q1 + q3));
}

// Branch-free float32 grouping scan over kl[i0, i1) (see group_starts_impl),
// appending group starts to starts[ns...].
void scan_sse(const float* kl, int64_t i0, int64_t i1, float thr, int64_t size_threshold,
              int64_t* starts, int64_t& ns) {
  // Loop-carried state in SSE registers: running float32 sum, group size (as
  // float: exact below 2^24, size_threshold <= 2^24 here), and the reset
  // mask; the selects are and/andnot/or, so nothing branches on data.
  const __m128 vthr = _mm_set_ss(thr);
  const __m128 vthr_size = _mm_set_ss((float)size_threshold);
  const __m128 one = _mm_set_ss(1.0f);
  __m128 cur = _mm_setzero_ps();
  __m128 size = _mm_setzero_ps();
  for (int64_t i = i0; i < i1; ++i) {
    const __m128 k = _mm_load_ss(kl + i);
    const __m128 sum = _mm_add_ss(cur, k);  // float32 + float32
    const __m128 m = _mm_or_ps(_mm_cmpge_ss(size, vthr_size), _mm_cmpge_ss(sum, vthr));
    starts[ns] = i;
    ns += _mm_movemask_ps(m) & 1;
    cur = _mm_or_ps(_mm_and_ps(m, k), _mm_andnot_ps(m, sum));
    size = _mm_or_ps(_mm_and_ps(m, one), _mm_andnot_ps(m, _mm_add_ss(size, one)));
  }
}

// The smallest float32 thr with (double)thr >= n_nats (> when strict): the
// reference's float64 comparison of a float32 sum s is then s >= thr.
float group_thr(double n_nats, bool strict) {
  auto cond = [&](float f) { return strict ? ((double)f > n_nats) : ((double)f >= n_nats); };
  float thr = (float)n_nats;
  while (!cond(thr) && thr < __builtin_inff()) thr = nextafterf(thr, __builtin_inff());
  while (cond(nextafterf(thr, -__builtin_inff())) && thr > -__builtin_inff())
    thr = nextafterf(thr, -__builtin_inff());
  return thr;
}

// coded_greedy_sampler.py:207-252 (strict=false) and
// coded_importance_sampler.py:178-203 (strict=true).
int64_t group_starts_impl(const float* kl, int64_t D, int64_t size_threshold, double n_nats,
                          int64_t* starts, int64_t cap, bool strict) {
  if (D < 0 || (D > 0 && !kl) || !starts || cap < 2)
    return fail(CWQ_ERR_INVALID, "group starts: bad arguments");
  if (cap < D + 2 || size_threshold > (1 << 24)) {
    // exact but slower: the branch-free scan below writes one slot per dim and
    // carries the group size in float32
    int64_t ns = 0;
    starts[ns++] = 0;
    int64_t cur_size = 0;
    float cur_kl = 0.0f;
    for (int64_t i = 0; i < D; ++i) {
      const float s = cur_kl + kl[i];
      const bool over = strict ? ((double)s > n_nats) : ((double)s >= n_nats);
      if (cur_size >= size_threshold || over || i == D - 1) {
        if (ns >= cap) return fail(CWQ_ERR_INVALID, "group starts: cap too small");
        starts[ns++] = i;
        cur_size = 1;
        cur_kl = kl[i];
      } else {
        cur_kl = s;
        cur_size += 1;
      }
    }
    if (ns >= cap) return fail(CWQ_ERR_INVALID, "group starts: cap too small");
    starts[ns++] = D;
    ok();
    return ns;
  }
  // The reference compares the float32 running sum in float64 (`>=`, or `>`
  // when strict).  For a float s that equals s >= thr with thr the smallest
  // float satisfying the comparison, so the scan stays in float32, and it is
  // branch-free (group boundaries are data-dependent: a branch mispredicts).
  const float thr = group_thr(n_nats, strict);
  if (D < 8 * 1024) {
    int64_t ns = 1;
    starts[0] = 0;
    scan_sse(kl, 0, D - 1, thr, size_threshold, starts, ns);
    if (D > 0) starts[ns++] = D - 1;  // idx == D - 1 always starts a group (:232)
    starts[ns++] = D;
    ok();
    return ns;
  }
  // Long inputs: 8 chunks scanned at once (two 4-lane SSE chains), chunk l > 0
  // starting speculatively from a fresh group; then a sequential fix-up runs
  // the exact scan into each chunk from its true state until both scans start
  // a group at the same index -- from there on they are identical (a group
  // start resets the state), so the speculative rest of the chunk is taken.
  constexpr int L = 8;
  const int64_t n = D - 1;  // indices scanned before the forced last group
  const int64_t len = n / L;
  int64_t b[L + 1];
  for (int l = 0; l < L; ++l) b[l] = (int64_t)l * len;
  b[L] = n;
  thread_local std::vector<int64_t> spec;
  spec.resize((size_t)(n + L));
  int64_t* sp[L];
  int64_t cnt[L];
  for (int l = 0; l < L; ++l) {
    sp[l] = spec.data() + b[l] + l;
    cnt[l] = 0;
  }
  const __m128 vthr = _mm_set1_ps(thr);
  const __m128 vthr_size = _mm_set1_ps((float)size_threshold);
  const __m128 one = _mm_set1_ps(1.0f);
  __m128 cur0 = _mm_setzero_ps(), size0 = _mm_setzero_ps();
  __m128 cur1 = _mm_setzero_ps(), size1 = _mm_setzero_ps();
  for (int64_t t = 0; t < len; ++t) {
    const __m128 k0 = _mm_setr_ps(kl[b[0] + t], kl[b[1] + t], kl[b[2] + t], kl[b[3] + t]);
    const __m128 k1 = _mm_setr_ps(kl[b[4] + t], kl[b[5] + t], kl[b[6] + t], kl[b[7] + t]);
    const __m128 s0 = _mm_add_ps(cur0, k0), s1 = _mm_add_ps(cur1, k1);
    const __m128 m0 = _mm_or_ps(_mm_cmpge_ps(size0, vthr_size), _mm_cmpge_ps(s0, vthr));
    const __m128 m1 = _mm_or_ps(_mm_cmpge_ps(size1, vthr_size), _mm_cmpge_ps(s1, vthr));
    const int bits = _mm_movemask_ps(m0) | (_mm_movemask_ps(m1) << 4);
    for (int l = 0; l < L; ++l) {
      sp[l][cnt[l]] = b[l] + t;
      cnt[l] += (bits >> l) & 1;
    }
    cur0 = _mm_or_ps(_mm_and_ps(m0, k0), _mm_andnot_ps(m0, s0));
    cur1 = _mm_or_ps(_mm_and_ps(m1, k1), _mm_andnot_ps(m1, s1));
    size0 = _mm_or_ps(_mm_and_ps(m0, one), _mm_andnot_ps(m0, _mm_add_ps(size0, one)));
    size1 = _mm_or_ps(_mm_and_ps(m1, one), _mm_andnot_ps(m1, _mm_add_ps(size1, one)));
  }
  float ecur[L], esize[L];
  _mm_storeu_ps(ecur, cur0);
  _mm_storeu_ps(ecur + 4, cur1);
  _mm_storeu_ps(esize, size0);
  _mm_storeu_ps(esize + 4, size1);
  // fix-up, chunk by chunk
  int64_t ns = 1;
  starts[0] = 0;
  for (int64_t q = 0; q < cnt[0]; ++q) starts[ns++] = sp[0][q];  // chunk 0 is exact
  float cur = ecur[0];
  int64_t csz = (int64_t)esize[0];
  for (int l = 1; l < L; ++l) {
    const int64_t e = (l == L - 1) ? n : b[l + 1];
    const int64_t spec_end = b[l] + len;  // the speculative scan covered [b[l], b[l] + len)
    int64_t p = 0;
    int64_t i = b[l];
    bool synced = false;
    for (; i < spec_end; ++i) {
      const float k = kl[i];
      const float sm = cur + k;
      const bool reset = (csz >= size_threshold) | (sm >= thr);
      if (reset) {
        starts[ns++] = i;
        cur = k;
        csz = 1;
        while (p < cnt[l] && sp[l][p] < i) ++p;
        if (p < cnt[l] && sp[l][p] == i) {  // same group start: identical from here on
          for (++p; p < cnt[l]; ++p) starts[ns++] = sp[l][p];
          cur = ecur[l];
          csz = (int64_t)esize[l];
          i = spec_end;
          synced = true;
          break;
        }
      } else {
        cur = sm;
        csz += 1;
      }
    }
    (void)synced;
    for (; i < e; ++i) {  // the last chunk's remainder past the common length
      const float k = kl[i];
      const float sm = cur + k;
      if ((csz >= size_threshold) | (sm >= thr)) {
        starts[ns++] = i;
        cur = k;
        csz = 1;
      } else {
        cur = sm;
        csz += 1;
      }
    }
  }
  starts[ns++] = D - 1;  // idx == D - 1 always starts a group (:232)
  starts[ns++] = D;
  ok();
  return ns;
}

// cwq_options (NULL = CWQ_OPTIONS_INIT), validated.
int read_options(const cwq_options* opts, cwq_options* out) {
  const cwq_options def = CWQ_OPTIONS_INIT;
  *out = opts ? *opts : def;
  if (out->prune_mode < 0 || out->prune_mode > 2)
    return fail(CWQ_ERR_INVALID, "cwq_options.prune_mode=%d outside [0, 2]", out->prune_mode);
  if (out->reserved != 0) return fail(CWQ_ERR_INVALID, "cwq_options.reserved must be 0");
  if ((out->eval_start_event == nullptr) != (out->eval_stop_event == nullptr))
    return fail(CWQ_ERR_INVALID, "cwq_options: give both eval events or neither");
  return CWQ_OK;
}

int check_common(int n_bits, int n_steps, int64_t nb) {
  if (n_bits < 0 || n_bits > CWQ_MAX_BITS_PER_STEP)
    return fail(CWQ_ERR_INVALID, "n_bits_per_step=%d outside [0, %d]", n_bits,
                CWQ_MAX_BITS_PER_STEP);
  if (n_steps < 1) return fail(CWQ_ERR_INVALID, "n_steps=%d must be >= 1", n_steps);
  if (nb < 0) return fail(CWQ_ERR_INVALID, "nb=%lld must be >= 0", (long long)nb);
  return CWQ_OK;
}

int encode_impl(const float* t_loc, const float* t_scale, const float* p_loc,
                const float* p_scale, const int64_t* block_off, int64_t ud, int64_t nb,
                int64_t total_dims, int64_t max_block_dim, int n_bits, int n_steps, int32_t seed, float rho,
                int64_t block_id_base, int32_t* out_idx, float* out_sample, void* workspace,
                size_t workspace_bytes, const cwq_options* opts, void* stream,
                const int32_t* block_seeds = nullptr, float* ds_out = nullptr,
                const float* ds_loc = nullptr, const float* ds_scale = nullptr) {
  int rc = check_common(n_bits, n_steps, nb);
  if (rc) return rc;
  cwq_options o;
  if ((rc = read_options(opts, &o))) return rc;
  if (total_dims < 0) return fail(CWQ_ERR_INVALID, "total_dims must be >= 0");
  if (nb > 0 && (!out_idx)) return fail(CWQ_ERR_INVALID, "out_idx is null");
  if (total_dims > 0 && (!t_loc || !t_scale || !p_loc || !p_scale || !out_sample))
    return fail(CWQ_ERR_INVALID, "null input/output pointer");
  // required: cwq_greedy_encode_workspace_size (CSR: always the general pruned
  // kernel's arrays) or cwq_greedy_encode_uniform_workspace_size
  const WsLayout l =
      block_off ? ws_layout_csr(nb, total_dims, max_block_dim) : ws_layout_uniform(nb, ud);
  if (workspace_bytes < l.total || (l.total && !workspace))
    return fail(CWQ_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes,
                l.total);
  cwq::EncodeArgs a;
  a.t_loc = t_loc;
  a.t_scale = t_scale;
  a.p_loc = p_loc;
  a.p_scale = p_scale;
  a.block_off = block_off;
  a.ud = ud;
  a.nb = nb;
  a.total_dims = total_dims;
  a.max_d = block_off ? max_block_dim : ud;
  a.n_cand = (int64_t)1 << n_bits;
  choose_tiling(nb, a.n_cand, &a.tiles_per_block, &a.cand_per_tile);
  a.n_steps = n_steps;
  a.prune = o.prune_mode;
  a.seed = seed;
  a.rho = rho;
  a.block_id_base = block_id_base;
  a.seeds = block_seeds;
  a.out_idx = out_idx;
  a.out_sample = out_sample;
  char* w = (char*)workspace;
  a.keys = (unsigned long long*)(w + l.keys);
  a.tq = (uint32_t*)(w + l.tq);
  a.loc_s = (float*)(w + l.loc_s);
  a.scale_s = (float*)(w + l.scale_s);
  a.lognorm = (float*)(w + l.lognorm);
  a.sab = l.csr ? (float2*)(w + l.sab) : nullptr;
  a.cdim = l.csr ? (float*)(w + l.cdim) : nullptr;
  a.bpre = l.csr ? (float*)(w + l.bpre) : nullptr;
  a.ordu = l.csr ? (uint32_t*)(w + l.ordu) : nullptr;
  a.grp = l.csr ? (float4*)(w + l.grp) : nullptr;
  a.gtau = l.csr ? (uint32_t*)(w + l.gtau) : nullptr;
#ifdef CWQ_NO_RECS
  a.abp = nullptr;
#else
  a.abp = l.recs ? (float4*)(w + l.abp) : nullptr;
#endif
  a.slist = l.csr ? (uint2*)(w + l.slist) : nullptr;
  a.sdmap = l.csr ? (uint32_t*)(w + l.sdmap) : nullptr;
  a.ev_start = o.eval_start_event;
  a.ev_stop = o.eval_stop_event;
  a.ds_out = ds_out;
  a.ds_loc = ds_loc;
  a.ds_scale = ds_scale;
  hipError_t e = cwq::launch_encode(a, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_greedy_encode");
  return ok();
}

}  // namespace

namespace cwq {
int set_error(int code, const char* msg) { return fail(code, "%s", msg); }
}  // namespace cwq

extern "C" {

int cwq_version(void) { return CWQ_ABI_VERSION; }

const char* cwq_last_error(void) { return g_err; }

int cwq_stateless_normal_sample(const float* loc, const float* scale, int64_t d,
                                int64_t num_samples, int32_t seed, float* out, void* stream) {
  if (d < 0 || num_samples < 0) return fail(CWQ_ERR_INVALID, "negative size");
  if (d * num_samples > 0 && (!loc || !scale || !out))
    return fail(CWQ_ERR_INVALID, "null pointer");
  hipError_t e =
      cwq::launch_stateless_normal_sample(loc, scale, d, num_samples, seed, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_stateless_normal_sample");
  return ok();
}

size_t cwq_greedy_encode_workspace_size(int64_t nb, int64_t total_dims, int64_t max_block_dim) {
  if (nb < 0 || total_dims < 0 || max_block_dim < 0) return 0;
  return ws_layout_csr(nb, total_dims, max_block_dim).total;
}

size_t cwq_greedy_encode_uniform_workspace_size(int64_t nb, int64_t d) {
  if (nb < 0 || d < 0 || (d > 0 && nb > INT64_MAX / d)) return 0;
  return ws_layout_uniform(nb, d).total;
}

int cwq_greedy_encode(const float* t_loc, const float* t_scale, const float* p_loc,
                      const float* p_scale, const int64_t* block_off, int64_t nb,
                      int64_t total_dims, int64_t max_block_dim, int n_bits_per_step,
                      int n_steps, int32_t seed, float rho, int64_t block_id_base,
                      int32_t* out_idx, float* out_sample, void* workspace,
                      size_t workspace_bytes, const cwq_options* opts, void* stream) {
  if (nb > 0 && !block_off) return fail(CWQ_ERR_INVALID, "block_off is null");
  if (max_block_dim < 0) return fail(CWQ_ERR_INVALID, "max_block_dim must be >= 0");
  return encode_impl(t_loc, t_scale, p_loc, p_scale, block_off, 0, nb, total_dims, max_block_dim,
                     n_bits_per_step, n_steps, seed, rho, block_id_base, out_idx, out_sample,
                     workspace, workspace_bytes, opts, stream);
}

int cwq_greedy_encode_uniform(const float* t_loc, const float* t_scale, const float* p_loc,
                              const float* p_scale, int64_t nb, int64_t d,
                              int n_bits_per_step, int n_steps, int32_t seed, float rho,
                              int64_t block_id_base, int32_t* out_idx, float* out_sample,
                              void* workspace, size_t workspace_bytes, const cwq_options* opts,
                              void* stream) {
  if (d < 0) return fail(CWQ_ERR_INVALID, "d must be >= 0");
  if (nb < 0 || (d > 0 && nb > INT64_MAX / d)) return fail(CWQ_ERR_INVALID, "bad nb");
  return encode_impl(t_loc, t_scale, p_loc, p_scale, nullptr, d, nb, nb * d, d, n_bits_per_step,
                     n_steps, seed, rho, block_id_base, out_idx, out_sample, workspace,
                     workspace_bytes, opts, stream);
}

int cwq_greedy_decode(const int32_t* idx, const float* p_loc, const float* p_scale,
                      const int64_t* block_off, int64_t nb, int64_t total_dims,
                      int64_t max_block_dim, int n_bits_per_step, int n_steps, int32_t seed,
                      float rho, int64_t block_id_base, float* out_sample, void* stream) {
  int rc = check_common(n_bits_per_step, n_steps, nb);
  if (rc) return rc;
  if (nb > 0 && (!block_off || !idx)) return fail(CWQ_ERR_INVALID, "null pointer");
  if (total_dims > 0 && (!p_loc || !p_scale || !out_sample))
    return fail(CWQ_ERR_INVALID, "null pointer");
  (void)max_block_dim;
  hipError_t e = cwq::launch_decode(idx, p_loc, p_scale, block_off, 0, nb, total_dims,
                                    n_bits_per_step,
                                    n_steps, seed, rho, block_id_base, out_sample,
                                    (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_greedy_decode");
  return ok();
}

int cwq_greedy_decode_uniform(const int32_t* idx, const float* p_loc, const float* p_scale,
                              int64_t nb, int64_t d, int n_bits_per_step, int n_steps,
                              int32_t seed, float rho, int64_t block_id_base, float* out_sample,
                              void* stream) {
  int rc = check_common(n_bits_per_step, n_steps, nb);
  if (rc) return rc;
  if (d < 0) return fail(CWQ_ERR_INVALID, "d must be >= 0");
  if (nb > 0 && !idx) return fail(CWQ_ERR_INVALID, "null pointer");
  if (nb * d > 0 && (!p_loc || !p_scale || !out_sample))
    return fail(CWQ_ERR_INVALID, "null pointer");
  hipError_t e = cwq::launch_decode(idx, p_loc, p_scale, nullptr, d, nb, nb * d,
                                    n_bits_per_step,
                                    n_steps, seed, rho, block_id_base, out_sample,
                                    (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_greedy_decode_uniform");
  return ok();
}

int cwq_standardise(const float* q_loc, const float* q_scale, const float* p_loc,
                    const float* p_scale, int64_t n, float* t_loc, float* t_scale, void* stream) {
  if (n < 0) return fail(CWQ_ERR_INVALID, "negative size");
  if (n > 0 && (!q_loc || !q_scale || !p_loc || !p_scale || !t_loc || !t_scale))
    return fail(CWQ_ERR_INVALID, "null pointer");
  hipError_t e = cwq::launch_standardise(q_loc, q_scale, p_loc, p_scale, n, t_loc, t_scale,
                                         (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_standardise");
  return ok();
}

int cwq_kl_normal_normal(const float* q_loc, const float* q_scale, const float* p_loc,
                         const float* p_scale, int64_t n, float* out, void* stream) {
  if (n < 0) return fail(CWQ_ERR_INVALID, "negative size");
  if (n > 0 && (!q_loc || !q_scale || !p_loc || !p_scale || !out))
    return fail(CWQ_ERR_INVALID, "null pointer");
  hipError_t e = cwq::launch_kl(q_loc, q_scale, p_loc, p_scale, n, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_kl_normal_normal");
  return ok();
}

int cwq_destandardise(const float* sample, const float* p_loc, const float* p_scale, int64_t n,
                      float* out, void* stream) {
  if (n < 0) return fail(CWQ_ERR_INVALID, "negative size");
  if (n > 0 && (!sample || !p_loc || !p_scale || !out))
    return fail(CWQ_ERR_INVALID, "null pointer");
  hipError_t e =
      cwq::launch_destandardise(sample, p_loc, p_scale, n, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_destandardise");
  return ok();
}

// ---------------------------------------------------------------------------
// The whole grouped greedy coder of one latent tensor in one call
// (coded_greedy_sampler.py:170-296): device standardise + KL, host grouping,
// device encode + destandardise, host bitcode.  Two host<->device round trips
// per call instead of one per Python step.
// ---------------------------------------------------------------------------
namespace {
struct GroupedWs {
  size_t t_loc, t_scale, kl, zeros, ones, sample, out, offs, idx, part, pinfo, enc, total;
};
// D dims in at most max_groups groups (a partition of D dims has at most D + 1:
// the reference's forced boundary at D - 1 can leave an empty first group)
GroupedWs grouped_ws(int64_t D, int n_steps, int64_t max_groups) {
  GroupedWs l;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align_up(o + bytes, 256);
    return at;
  };
  const size_t fd = (size_t)(D > 0 ? D : 0) * 4;
  l.t_loc = take(fd);
  l.t_scale = take(fd);
  l.kl = take(fd);
  l.zeros = take(fd);
  l.ones = take(fd);
  l.sample = take(fd);
  l.out = take(fd);
  const int64_t G = max_groups > 1 ? max_groups : 1;
  l.offs = take((size_t)(G + 1) * 8);
  l.idx = take((size_t)G * (size_t)(n_steps > 0 ? n_steps : 1) * 4);
  l.part = take(cwq::partition_workspace_size(D > 0 ? D : 0));  // device partition scratch
  l.pinfo = take(16 * sizeof(unsigned long long));  // partition info[8] + item info[2]
  l.enc = take(ws_layout_csr(G, D, D).total);
  l.total = o;
  return l;
}
// Events of one call, created on the stream's device and destroyed with it.
// Events of one call on the stream's device, from a per-thread pool (creating
// and destroying a few dozen events per call cost ~0.3 ms on the batch
// coder); returned to the pool with the call, destroyed at thread exit.
struct EventPool {
  std::vector<hipEvent_t> free_ev[16][2];  // [device][timing]
  ~EventPool() {
    for (auto& d : free_ev)
      for (auto& v : d)
        for (hipEvent_t e : v) (void)hipEventDestroy(e);
  }
};
thread_local EventPool tl_events;
struct CallEvents {
  std::vector<hipEvent_t> ev;
  int dev = -1, timing = 0;
  bool made(int n, hipStream_t s, unsigned flags) {
    if (hipStreamGetDevice(s, &dev) != hipSuccess || dev < 0 || dev >= 16) return false;
    timing = (flags & hipEventDisableTiming) ? 0 : 1;
    std::vector<hipEvent_t>& pool = tl_events.free_ev[dev][timing];
    while (n > 0 && !pool.empty()) {
      ev.push_back(pool.back());
      pool.pop_back();
      --n;
    }
    if (n == 0) return true;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return false;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return false;
    bool ok = true;
    for (int i = 0; i < n && ok; ++i) {
      hipEvent_t e = nullptr;
      ok = hipEventCreateWithFlags(&e, flags) == hipSuccess;
      if (ok) ev.push_back(e);
    }
    if (cur != dev) (void)hipSetDevice(cur);
    return ok;
  }
  ~CallEvents() {  // the call has synchronised (or never used them): reusable
    if (dev >= 0 && dev < 16)
      for (hipEvent_t e : ev) tl_events.free_ev[dev][timing].push_back(e);
  }
};
// Waits for an event by polling (the batch coder's host threads wait on
// copies of a few hundred microseconds: a blocking wait's wake-up latency is
// of the same order), falling back to the blocking wait after ~2 ms.
hipError_t wait_event(hipEvent_t e) {
  for (int i = 0; i < 20000; ++i) {
    const hipError_t q = hipEventQuery(e);
    if (q != hipErrorNotReady) return q;
    _mm_pause();
  }
  return hipEventSynchronize(e);
}
thread_local std::vector<float> g_kl_host;
thread_local std::vector<int32_t> g_idx_host;
// the device partition's info[8], then item 0's (G + 1, largest): pinned, so the
// copy is a direct DMA (pageable memory is staged), per thread
// A thread's page-locked buffer, freed when the thread ends (the main
// thread's at exit, before the HIP runtime's own teardown)
struct PinnedTl {
  void* p = nullptr;
  size_t n = 0;
  void* get(size_t bytes, size_t want) {
    if (n < bytes) {
      if (p) (void)hipHostFree(p);
      p = nullptr;
      n = 0;
      if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
        p = nullptr;
        return nullptr;
      }
      n = want;
    }
    return p;
  }
  ~PinnedTl() {
    if (p) (void)hipHostFree(p);
  }
};
unsigned long long* part_info_host() {
  thread_local PinnedTl b;
  constexpr size_t kBytes = 16 * sizeof(unsigned long long);
  return (unsigned long long*)b.get(kBytes, kBytes);
}
// CWQ_HOST_PARTITION=1: the host partition loop even where the device one
// applies (A/B timing; the results are identical)
bool device_partition_enabled() {
  static const bool on = [] {
    const char* e = getenv("CWQ_HOST_PARTITION");
    return !(e && e[0] == '1');
  }();
  return on;
}
// The single grouped call's device partition pays off from this many dims: below
// it the host loop over the copied KL (one round trip instead of seven chained
// launches and two) is faster (tools/single_call_laps.py: 2,304 dims 120 ->
// 90 us a call).  CWQ_DEV_PART_MIN_D overrides it (A/B timing; results never
// depend on the path).
int64_t dev_partition_min_dims() {
  static const int64_t v = [] {
    const char* e = getenv("CWQ_DEV_PART_MIN_D");
    return e && *e ? (int64_t)atoll(e) : (int64_t)16384;
  }();
  return v;
}
// :81-87, :288 (and binary_io.py:41-53) each of n indices as n_bits LSB-first
// '0'/'1' chars; returns n * n_bits, or CWQ_ERR_INVALID for an index that does
// not fit (to_bit_string raises there).
// BMI2 form (runtime-dispatched): a byte of the index becomes its 8 chars with
// one pdep (bit k -> the low bit of byte k, LSB first) and an OR with '0'x8;
// C2's 41.5k 8-bit indices: ~16 us against ~31 us through the table.
__attribute__((target("bmi2"))) int64_t write_bitcode_pdep(const int32_t* idx, int64_t n,
                                                           int n_bits, char* o) {
  constexpr uint64_t kLow = 0x0101010101010101ull, kZero = 0x3030303030303030ull;
  const int full = n_bits >> 3, rem = n_bits & 7;
  const uint64_t rmask = kLow & ((1ull << (8 * rem)) - 1);  // rem < 8: the first rem bytes
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t v = (uint32_t)idx[i];
    if (n_bits < 31 && (v >> n_bits) != 0)
      return fail(CWQ_ERR_INVALID, "index %u does not fit %d bits", v, n_bits);
    for (int k = 0; k < full; ++k) {
      const uint64_t w = _pdep_u64((v >> (8 * k)) & 0xffu, kLow) | kZero;
      memcpy(o, &w, 8);
      o += 8;
    }
    if (rem) {
      const uint64_t w = _pdep_u64(v >> (8 * full), rmask) | (kZero & ((1ull << (8 * rem)) - 1));
      memcpy(o, &w, (size_t)rem);
      o += rem;
    }
  }
  return n * n_bits;
}
int64_t write_bitcode(const int32_t* idx, int64_t n, int n_bits, char* o) {
  static const bool bmi2 = __builtin_cpu_supports("bmi2");
  if (bmi2) return write_bitcode_pdep(idx, n, n_bits, o);
  static const struct ByteChars {  // byte value -> its 8 LSB-first '0'/'1' chars
    uint64_t c[256];
    ByteChars() {
      for (int v = 0; v < 256; ++v) {
        uint64_t w = 0;
        for (int b = 0; b < 8; ++b) w |= (uint64_t)('0' + ((v >> b) & 1)) << (8 * b);
        c[v] = w;
      }
    }
  } kByteChars;
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t v = (uint32_t)idx[i];
    if (n_bits < 31 && (v >> n_bits) != 0)
      return fail(CWQ_ERR_INVALID, "index %u does not fit %d bits", v, n_bits);
    int b = 0;
    for (; b + 8 <= n_bits; b += 8) {
      memcpy(o, &kByteChars.c[(v >> b) & 0xffu], 8);
      o += 8;
    }
    for (; b < n_bits; ++b) *o++ = (char)('0' + ((v >> b) & 1u));
  }
  return n * n_bits;
}
}  // namespace

size_t cwq_code_grouped_greedy_workspace_size(int64_t D, int n_steps) {
  if (D < 0 || n_steps < 0) return 0;
  return grouped_ws(D, n_steps, D + 1).total;
}

namespace {
// cwq_code_grouped_greedy up to its last copies: standardise, KL, host
// partition (starts_host), the encode, destandardisation, and the copies of
// the G * n_steps indices to idx_host and the sample to sample_host, all
// enqueued on the stream.  Returns G.  tev (eval_ms_out only): its two
// timing events, recorded around the encode.  bits_cap >= 0: the bitcode
// capacity, checked once G is known, before the encode.
int64_t grouped_begin(const float* q_loc, const float* q_scale, const float* p_loc,
                      const float* p_scale, int64_t D, int n_steps, int n_bits_per_step,
                      int32_t seed, float rho, int64_t size_threshold, double n_nats,
                      float* sample_host, int32_t* idx_host, int64_t idx_cap,
                      int64_t* starts_host, int64_t starts_cap, double* kl_sum_out,
                      void* workspace, size_t workspace_bytes, const cwq_options* opts,
                      const cwq_options& o, CallEvents* tev, int n_bits_cap_check,
                      int64_t bits_cap, void* stream, const char* who) {
  if (D < 0 || n_steps < 1 || n_bits_per_step < 0 || n_bits_per_step > CWQ_MAX_BITS_PER_STEP)
    return fail(CWQ_ERR_INVALID, "%s: bad sizes", who);
  if (D > 0 && (!q_loc || !q_scale || !p_loc || !p_scale || !sample_host))
    return fail(CWQ_ERR_INVALID, "%s: null pointer", who);
  if (!starts_host || starts_cap < D + 2)
    return fail(CWQ_ERR_CAPACITY, "%s: starts_cap must be >= D + 2", who);
  const GroupedWs l = grouped_ws(D, n_steps, D + 1);
  if (workspace_bytes < l.total || !workspace)
    return fail(CWQ_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes,
                l.total);
  hipStream_t s = (hipStream_t)stream;
#ifdef CWQ_PHASE_TIMES  // tuning builds: per-phase host wall times to stderr
  struct timespec ts0, ts1;
  clock_gettime(CLOCK_MONOTONIC, &ts0);
  auto lap = [&](const char* what) {
    clock_gettime(CLOCK_MONOTONIC, &ts1);
    fprintf(stderr, "[cwq] %-10s %8.1f us\n", what,
            (ts1.tv_sec - ts0.tv_sec) * 1e6 + (ts1.tv_nsec - ts0.tv_nsec) * 1e-3);
    ts0 = ts1;
  };
#else
  auto lap = [](const char*) {};
#endif
  char* w = (char*)workspace;
  float* t_loc = (float*)(w + l.t_loc);
  float* t_scale = (float*)(w + l.t_scale);
  float* kl = (float*)(w + l.kl);
  float* zeros = (float*)(w + l.zeros);
  float* ones = (float*)(w + l.ones);
  float* sample = (float*)(w + l.sample);
  float* out = (float*)(w + l.out);
  int64_t* offs = (int64_t*)(w + l.offs);
  int32_t* idx = (int32_t*)(w + l.idx);
  hipError_t e = hipSuccess;
  int rc;
  // :207-252 the partition: on the device when it applies (cwq_partition.hip,
  // bit-identical to the loop; no KL round trip), else the host loop
  bool dev_part = false;
  int64_t n = 0, maxd = 0;
  bool kl_on_host = false;
  CallEvents pev;  // the partition info's and the starts' copies
  if (D > 0) {
    // :193-199 standardise; :201, :210 per-dim KL(target || proposal); the
    // standard prior (zeros, ones) and the partition's counters, one launch
    unsigned long long* g_part_info = part_info_host();
    const bool try_dev = device_partition_enabled() && D >= dev_partition_min_dims() &&
                         cwq::partition_applies(D, size_threshold) && g_part_info != nullptr;
    unsigned long long* info_d = (unsigned long long*)(w + l.pinfo);
    if ((e = cwq::launch_grouped_prep(q_loc, q_scale, p_loc, p_scale, D, t_loc, t_scale, kl, zeros,
                                      ones, info_d, try_dev ? 16 : 0, s)) != hipSuccess)
      return hip_fail(e, "standardise / KL");
    if (try_dev) {
      if ((e = cwq::launch_partition(kl, D, nullptr, 1, size_threshold, group_thr(n_nats, false),
                                     offs, (int64_t*)(info_d + 8), w + l.part, info_d, s,
                                     true)) != hipSuccess ||
          (e = hipMemcpyAsync(g_part_info, info_d, 16 * sizeof(unsigned long long),
                              hipMemcpyDeviceToHost, s)) != hipSuccess)
        return hip_fail(e, "device partition");
      if (kl_sum_out) {  // the log line's total KL only
        g_kl_host.resize((size_t)D);
        if ((e = hipMemcpyAsync(g_kl_host.data(), kl, (size_t)D * 4, hipMemcpyDeviceToHost, s)) !=
            hipSuccess)
          return hip_fail(e, "KL to host");
        kl_on_host = true;
      }
      // a polled event: the blocking wait's wake-up is of the order of the
      // partition itself
      if (!pev.made(1, s, hipEventDisableTiming) || hipEventRecord(pev.ev[0], s) != hipSuccess)
        return fail(CWQ_ERR_HIP, "%s: events failed", who);
      if ((e = wait_event(pev.ev[0])) != hipSuccess) return hip_fail(e, "sync");
      if (!cwq::partition_fell_back(g_part_info)) {
        dev_part = true;
        n = (int64_t)g_part_info[8];
        maxd = (int64_t)g_part_info[9];
      }
    }
    if (!dev_part && !kl_on_host) {
      g_kl_host.resize((size_t)D);
      if ((e = hipMemcpyAsync(g_kl_host.data(), kl, (size_t)D * 4, hipMemcpyDeviceToHost, s)) !=
          hipSuccess)
        return hip_fail(e, "KL to host");
      if (pev.ev.empty() && !pev.made(1, s, hipEventDisableTiming))
        return fail(CWQ_ERR_HIP, "%s: events failed", who);
      if ((e = hipEventRecord(pev.ev[0], s)) != hipSuccess || (e = wait_event(pev.ev[0])) != hipSuccess)
        return hip_fail(e, "sync");
      kl_on_host = true;
    }
  }
  lap("kl");
  if (kl_sum_out) {  // log line only: four independent accumulators
    double t[4] = {0.0, 0.0, 0.0, 0.0};
    int64_t i = 0;
    for (; i + 4 <= D; i += 4)
      for (int q = 0; q < 4; ++q) t[q] += (double)g_kl_host[(size_t)(i + q)];
    for (; i < D; ++i) t[0] += (double)g_kl_host[(size_t)i];
    *kl_sum_out = (t[0] + t[2]) + (t[1] + t[3]);
  }
  if (!dev_part) {
    // :207-252 the sequential partition (host, exact reference semantics)
    n = group_starts_impl(D > 0 ? g_kl_host.data() : nullptr, D, size_threshold, n_nats,
                          starts_host, starts_cap, false);
    if (n < 0) return n;
    for (int64_t g = 0; g + 1 < n; ++g) {
      const int64_t dg = starts_host[g + 1] - starts_host[g];
      maxd = dg > maxd ? dg : maxd;
    }
  }
  const int64_t G = n - 1;
  lap("group");
  if (n_bits_cap_check && bits_cap < G * (int64_t)n_steps * n_bits_per_step)
    return fail(CWQ_ERR_CAPACITY, "%s: bits_cap %lld < %lld", who, (long long)bits_cap,
                (long long)(G * (int64_t)n_steps * n_bits_per_step));
  if (G <= 0) return G < 0 ? 0 : G;
  if (idx_cap < G * (int64_t)n_steps || !idx_host)
    return fail(CWQ_ERR_CAPACITY, "%s: index buffer %lld < %lld", who, (long long)idx_cap,
                (long long)(G * n_steps));
  if (!dev_part &&
      (e = hipMemcpyAsync(offs, starts_host, (size_t)(G + 1) * 8, hipMemcpyHostToDevice, s)) !=
          hipSuccess)
    return hip_fail(e, "offsets to device");
  // device partition: the group starts go to the caller (who reads them before
  // _end) on a copy stream, queued before the encode's own copies so they do
  // not wait behind it; the partition has completed (synchronised above)
  hipStream_t d2h_starts = nullptr;
  if (dev_part) {
    d2h_starts = cwq::copy_stream(s, 0);
    if (!d2h_starts) d2h_starts = s;
    if ((e = hipMemcpyAsync(starts_host, offs, (size_t)(G + 1) * 8, hipMemcpyDeviceToHost,
                            d2h_starts)) != hipSuccess)
      return hip_fail(e, "starts to host");
    if (pev.ev.size() != 1 || !pev.made(1, s, hipEventDisableTiming) ||
        (e = hipEventRecord(pev.ev[1], d2h_starts)) != hipSuccess) {
      (void)hipStreamSynchronize(d2h_starts);
      return fail(CWQ_ERR_HIP, "%s: events failed", who);
    }
  }
  // :273-284 one greedy coder per group, seed + g.  eval_ms_out: this call's
  // two events go to the encoder as its eval events, so they bracket the
  // candidate-scoring launches and not the destandardisation after them
  cwq_options oe = o;
  if (o.eval_ms_out && !o.eval_start_event) {
    if (!tev->made(2, s, hipEventDefault))
      return fail(CWQ_ERR_HIP, "%s: timing events failed", who);
    oe.eval_start_event = tev->ev[0];
    oe.eval_stop_event = tev->ev[1];
  }
  oe.eval_ms_out = nullptr;
  // (and :292 destandardise into out, folded into the encoder's last launch)
  if ((rc = encode_impl(t_loc, t_scale, zeros, ones, offs, 0, G, D, maxd, n_bits_per_step,
                        n_steps, seed, rho, 0, idx, sample, w + l.enc, workspace_bytes - l.enc,
                        &oe, stream, nullptr, out, p_loc, p_scale)) < 0)
    return rc;
  if ((e = hipMemcpyAsync(idx_host, idx, (size_t)(G * n_steps) * 4, hipMemcpyDeviceToHost, s)) !=
      hipSuccess)
    return hip_fail(e, "indices to host");
  if ((e = hipMemcpyAsync(sample_host, out, (size_t)D * 4, hipMemcpyDeviceToHost, s)) !=
      hipSuccess)
    return hip_fail(e, "sample to host");
  if (d2h_starts && (e = wait_event(pev.ev[1])) != hipSuccess) {
    (void)hipStreamSynchronize(s);
    return hip_fail(e, "starts to host");
  }
  lap("enqueued");
  return G;
}

// :81-87, :288 each of the G * n_steps indices as n_bits_per_step LSB-first
// chars, steps then groups
int64_t grouped_bits(const int32_t* idx_host, int64_t G, int n_steps, int n_bits_per_step,
                     char* bits_host, int64_t bits_cap, const char* who) {
  const int64_t nbits = G * (int64_t)n_steps * n_bits_per_step;
  if (bits_cap < nbits || (nbits > 0 && !bits_host))
    return fail(CWQ_ERR_CAPACITY, "%s: bits_cap %lld < %lld", who, (long long)bits_cap,
                (long long)nbits);
  if (G <= 0) return 0;
  return write_bitcode(idx_host, G * n_steps, n_bits_per_step, bits_host);
}
}  // namespace

int64_t cwq_code_grouped_greedy(const float* q_loc, const float* q_scale, const float* p_loc,
                                const float* p_scale, int64_t D, int n_steps,
                                int n_bits_per_step, int32_t seed, float rho,
                                int64_t size_threshold, double n_nats, float* sample_host,
                                char* bits_host, int64_t bits_cap, int64_t* starts_host,
                                int64_t starts_cap, double* kl_sum_out, void* workspace,
                                size_t workspace_bytes, const cwq_options* opts, void* stream) {
  static const char* const who = "cwq_code_grouped_greedy";
  cwq_options o;
  {
    const int rc0 = read_options(opts, &o);
    if (rc0) return rc0;
  }
  if (D < 0 || n_steps < 1 || D > (INT64_MAX / 8) / n_steps)
    return fail(CWQ_ERR_INVALID, "%s: D %lld, n_steps %d", who, (long long)D, n_steps);
  CallEvents tev;
  try {
    g_idx_host.resize((size_t)((D + 1) * n_steps));
  } catch (...) {
    return fail(CWQ_ERR_ALLOC, "%s: host index buffer of %lld entries", who,
                (long long)((D + 1) * n_steps));
  }
  const int64_t G = grouped_begin(q_loc, q_scale, p_loc, p_scale, D, n_steps, n_bits_per_step,
                                  seed, rho, size_threshold, n_nats, sample_host,
                                  g_idx_host.data(), (int64_t)g_idx_host.size(), starts_host,
                                  starts_cap, kl_sum_out, workspace, workspace_bytes, opts, o,
                                  &tev, 1, bits_cap, stream, who);
  if (G < 0) {
    // work grouped_begin queued (the encode, the copies into g_idx_host and
    // starts_host) may still be in flight: drain it before g_idx_host or the
    // events are reused
    (void)hipStreamSynchronize((hipStream_t)stream);
    if (hipStream_t c = cwq::copy_stream((hipStream_t)stream, 0)) (void)hipStreamSynchronize(c);
    return G;
  }
  hipError_t e;
  if (G > 0 && (e = hipStreamSynchronize((hipStream_t)stream)) != hipSuccess)
    return hip_fail(e, "sync");
  if (G > 0 && o.eval_ms_out &&
      (e = hipEventElapsedTime(o.eval_ms_out, tev.ev[0], tev.ev[1])) != hipSuccess)
    return hip_fail(e, "event time");
  const int64_t nw = grouped_bits(g_idx_host.data(), G, n_steps, n_bits_per_step, bits_host,
                                  bits_cap, who);
  if (nw < 0) return nw;
  cwq::set_error(CWQ_OK, "");
  return G;
}

int64_t cwq_code_grouped_greedy_begin(const float* q_loc, const float* q_scale,
                                      const float* p_loc, const float* p_scale, int64_t D,
                                      int n_steps, int n_bits_per_step, int32_t seed, float rho,
                                      int64_t size_threshold, double n_nats, float* sample_host,
                                      int32_t* idx_host, int64_t idx_cap, int64_t* starts_host,
                                      int64_t starts_cap, double* kl_sum_out, void* workspace,
                                      size_t workspace_bytes, const cwq_options* opts,
                                      void* stream) {
  static const char* const who = "cwq_code_grouped_greedy_begin";
  cwq_options o;
  {
    const int rc0 = read_options(opts, &o);
    if (rc0) return rc0;
  }
  if (o.eval_ms_out)
    return fail(CWQ_ERR_INVALID, "%s: eval_ms_out needs the synchronous call (use the events)",
                who);
  const int64_t G = grouped_begin(q_loc, q_scale, p_loc, p_scale, D, n_steps, n_bits_per_step,
                                  seed, rho, size_threshold, n_nats, sample_host, idx_host,
                                  idx_cap, starts_host, starts_cap, kl_sum_out, workspace,
                                  workspace_bytes, opts, o, nullptr, 0, 0, stream, who);
  if (G < 0) {  // nothing queued may outlive an error
    (void)hipStreamSynchronize((hipStream_t)stream);
    if (hipStream_t c = cwq::copy_stream((hipStream_t)stream, 0)) (void)hipStreamSynchronize(c);
    return G;
  }
  cwq::set_error(CWQ_OK, "");
  return G;
}

int64_t cwq_code_grouped_greedy_end(const int32_t* idx_host, int64_t G, int n_steps,
                                    int n_bits_per_step, char* bits_host, int64_t bits_cap,
                                    void* stream) {
  static const char* const who = "cwq_code_grouped_greedy_end";
  if (G < 0 || n_steps < 1 || n_bits_per_step < 0 || n_bits_per_step > CWQ_MAX_BITS_PER_STEP)
    return fail(CWQ_ERR_INVALID, "%s: bad sizes", who);
  hipError_t e;
  // a polled event rather than a blocking stream wait (its wake-up cost ~20 us
  // a call)
  {
    CallEvents ev;
    if (!ev.made(1, (hipStream_t)stream, hipEventDisableTiming) ||
        hipEventRecord(ev.ev[0], (hipStream_t)stream) != hipSuccess) {
      if ((e = hipStreamSynchronize((hipStream_t)stream)) != hipSuccess) return hip_fail(e, "sync");
    } else if ((e = wait_event(ev.ev[0])) != hipSuccess) {
      return hip_fail(e, "sync");
    }
  }
  if (G > 0 && !idx_host) return fail(CWQ_ERR_INVALID, "%s: null pointer", who);
  const int64_t nw = grouped_bits(idx_host, G, n_steps, n_bits_per_step, bits_host, bits_cap, who);
  if (nw < 0) return nw;
  cwq::set_error(CWQ_OK, "");
  return nw;
}

// ---------------------------------------------------------------------------
// A batch of independent code_grouped_greedy_sample calls (the images of a
// dataset, or both ladder levels of several images) in one call.  Item i is
// dims [item_off[i], item_off[i+1]) of the concatenated inputs and is coded
// exactly as cwq_code_grouped_greedy on that slice with seed seeds[i]: its
// partition is its own (:207-252), its groups are numbered from 0 and group g
// is coded with seeds[i] + g (:273-284).  All items share one
// standardisation, one KL copy, ONE encode launch over every item's groups
// (per-block seeds) and one destandardisation, so a batch of small items
// fills the chip instead of paying a launch sequence and two host round trips
// each.
// ---------------------------------------------------------------------------
namespace {
// Device workspace of the batch: the grouped layout for D dims, with the
// per-chunk regions of the group-indexed arrays (chunk c of a call owns
// [a_c + i0_c, ...) of them, a_c its first dim and i0_c its first item, so
// chunks never share a slot however their group counts come out): offsets
// D + 2 n + 1 entries, indices / seeds D + n.
struct BatchWs {
  GroupedWs g;
  size_t seeds, ioff, dstarts, iinfo, itab, pstarts, total;
};
BatchWs batch_ws(int64_t D, int64_t n_items, int n_steps) {
  BatchWs l;
  const int64_t n = n_items > 0 ? n_items : 0;
  l.g = grouped_ws(D, n_steps, D + 2 * n + 1);
  l.seeds = l.g.total;
  // the device partition: item offsets, the items' start lists (the host
  // layout: item i at item_off[i] + 2 i), per-item counts, the layout table
  l.ioff = align_up(l.seeds + (size_t)(D + n + 1) * 4, 256);
  l.dstarts = align_up(l.ioff + (size_t)(n + 1) * 8, 256);
  l.iinfo = align_up(l.dstarts + (size_t)(D + 2 * n + 1) * 8, 256);
  l.itab = align_up(l.iinfo + (size_t)(4 * n + 4) * 8, 256);
  // the start lists packed back to back (at most D_i + 2 entries each)
  l.pstarts = align_up(l.itab + (size_t)(n + 1) * sizeof(cwq::BatchItem), 256);
  l.total = align_up(l.pstarts + (size_t)(D + 2 * n + 1) * 8, 256);
  return l;
}
// Host staging of the batch (the caller's pinned memory, or thread-local
// vectors): per-dim KL, then the offsets / seeds / indices regions as above.
struct BatchHostWs {
  size_t kl, offs, seeds, idx, total;
};
BatchHostWs batch_host_ws(int64_t D, int64_t n_items, int n_steps) {
  BatchHostWs h;
  const int64_t n = n_items > 0 ? n_items : 0;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align_up(o + bytes, 256);
    return at;
  };
  h.kl = take((size_t)D * 4);
  h.offs = take((size_t)(D + 2 * n + 1) * 8);
  h.seeds = take((size_t)(D + n + 1) * 4);
  h.idx = take((size_t)(D + n + 1) * (size_t)(n_steps > 0 ? n_steps : 1) * 4);
  h.total = o;
  return h;
}
// Host threads for the per-chunk host phases: CWQ_HOST_THREADS if set, else the
// CPUs this process may run on, at most 8.  (On the GPU boxes, whose cgroup
// quota is 16 CPUs, 12 or 16 threads sporadically ran C3 2.5x slower: the
// quota's throttling; 4 and 8 were steady at 9-10 ms per 24 images.)
int64_t host_threads() {
  static const int64_t n = [] {
    if (const char* e = getenv("CWQ_HOST_THREADS")) {
      const long v = strtol(e, nullptr, 10);
      if (v >= 1) return (int64_t)v;
    }
    cpu_set_t set;
    int64_t c = 0;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) c = CPU_COUNT(&set);
    if (c < 1) c = (int64_t)std::thread::hardware_concurrency();
    return std::max<int64_t>(1, std::min<int64_t>(8, c));
  }();
  return n;
}
// A process-wide pool of host worker threads for the batch call's per-item
// work (C3: 48 bitcodes), created on first use and kept: creating and joining
// seven threads per call sat on the call's critical path.  The pool object is
// never destroyed (its threads sleep on a condition variable through process
// exit).  run() executes f on up to n pool threads and the calling thread and
// returns once every one of them has returned; concurrent run()s queue.
#ifndef CWQ_POOL_WAIT_ALL
#define CWQ_POOL_WAIT_ALL 0  // 1: run() also waits for every started helper (A/B)
#endif
class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = new HostPool();
    return *p;
  }
  void run(int64_t n, const std::function<void()>& f) {
    std::lock_guard<std::mutex> one(run_m_);  // one job at a time
    int64_t started = 0;
    {
      std::unique_lock<std::mutex> lk(m_);
      if (pid_ != getpid()) {  // a forked child has none of the parent's threads
        pid_ = getpid();
        threads_ = 0;
      }
      while ((int64_t)threads_ < n) {
        try {
          std::thread(&HostPool::loop, this, threads_).detach();
        } catch (...) {
          break;  // no more threads (pids cgroup): fewer helpers
        }
        ++threads_;
      }
      started = std::min<int64_t>(n, (int64_t)threads_);
      job_ = &f;
      active_ = started;
      running_ = 0;
      left_ = started;
      ++gen_;
    }
    cv_.notify_all();
    f();
    // the caller's f() returns once the job's work is claimed (every user's f
    // claims work items until none is left): helpers that have not woken yet
    // skip the job instead of being waited for (a futex wake-up can take tens
    // of microseconds: I2's 24-item planning waited ~70 us for them); helpers
    // inside f() finish the items they hold
    std::unique_lock<std::mutex> lk(m_);
    if (CWQ_POOL_WAIT_ALL) done_.wait(lk, [&] { return left_ == 0; });  // A/B: the old rule
    job_ = nullptr;
    done_.wait(lk, [&] { return running_ == 0; });
  }

 private:
  void loop(int64_t id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void()>* f = nullptr;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (id >= active_ || !job_) continue;  // not needed, or the job has closed
        f = job_;
        ++running_;
      }
      (*f)();
      std::lock_guard<std::mutex> lk(m_);
      --left_;
      if (--running_ == 0 || left_ == 0) done_.notify_all();
    }
  }
  std::mutex run_m_, m_;
  std::condition_variable cv_, done_;
  const std::function<void()>* job_ = nullptr;
  pid_t pid_ = getpid();
  uint64_t gen_ = 0;
  int64_t threads_ = 0, active_ = 0, running_ = 0, left_ = 0;
};
// Chunks a batch is pipelined in (CWQ_BATCH_CHUNKS, default below): the host
// phases of one chunk run while the device codes another.
#ifndef CWQ_BATCH_CHUNKS
#define CWQ_BATCH_CHUNKS 6
#endif
int64_t batch_chunks() {
  static const int64_t n = [] {
    if (const char* e = getenv("CWQ_BATCH_CHUNKS")) {
      const long v = strtol(e, nullptr, 10);
      if (v >= 1) return (int64_t)v;
    }
    return (int64_t)CWQ_BATCH_CHUNKS;
  }();
  return n;
}
thread_local std::vector<char> g_batch_host;
// page-locked per-thread buffer of at least `bytes` (the batch partition's
// info; pageable memory would be staged), nullptr when allocation fails
void* pinned_tl(size_t bytes) {
  thread_local PinnedTl b;
  return b.get(bytes, bytes < 4096 ? 4096 : bytes * 2);
}
thread_local std::vector<cwq::BatchItem> g_batch_items;

constexpr int64_t kBatchFellBack = INT64_MIN;

// The batch call's result copies (indices, sample, start lists) on the GPU's
// SDMA engines (hsa_amd_memory_async_copy) instead of hipMemcpyAsync, which
// runs device-to-host copies as blit kernels on the CUs: beside C3's coding
// they took ~60 us of CU time from each chunk's screen (k_small_one 165 ->
// 227 us; without the copies the call took 0.15 ms less).  The host orders
// them: a copy is issued once its chunk's event has completed.  Each signal
// carries a token (1) until every copy of its slot is issued, plus one count
// per copy in flight, so a waiter sees 0 only when the slot's copies are done.
// CWQ_SDMA=0 keeps the HIP copies (A/B).
bool sdma_enabled() {
  static const bool on = [] {
    const char* e = getenv("CWQ_SDMA");
    if (e && e[0] == '0') return false;
    return hsa_init() == HSA_STATUS_SUCCESS;  // reference-counted: the HIP runtime holds one
  }();
  return on;
}
class SdmaCopies {
 public:
  // n slots; the buffers every copy will use must be HSA allocations (device
  // memory, page-locked host memory): false otherwise (use HIP copies)
  bool init(int n, std::initializer_list<const void*> bufs) {
    for (const void* p : bufs) {
      hsa_amd_pointer_info_t info;
      info.size = sizeof(info);
      if (!p || hsa_amd_pointer_info(p, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
          info.type == HSA_EXT_POINTER_TYPE_UNKNOWN)
        return false;
    }
    sig_.assign((size_t)n, hsa_signal_t{0});
    released_.assign((size_t)n, 0);
    for (int k = 0; k < n; ++k)
      if (hsa_signal_create(1, 0, nullptr, &sig_[(size_t)k]) != HSA_STATUS_SUCCESS) {
        sig_.resize((size_t)k);
        return false;
      }
    return true;
  }
  // device src -> host dst, counted on slot k (before its release)
  bool copy(int k, void* dst, const void* src, size_t bytes) {
    if (bytes == 0) return true;
    hsa_amd_pointer_info_t si, di;
    si.size = di.size = sizeof(si);
    if (hsa_amd_pointer_info(src, &si, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        hsa_amd_pointer_info(dst, &di, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS)
      return false;
    hsa_signal_add_relaxed(sig_[(size_t)k], 1);
    if (hsa_amd_memory_async_copy(dst, di.agentOwner, src, si.agentOwner, bytes, 0, nullptr,
                                  sig_[(size_t)k]) != HSA_STATUS_SUCCESS) {
      hsa_signal_subtract_relaxed(sig_[(size_t)k], 1);
      return false;
    }
    return true;
  }
  // every copy of slot k is issued (or never will be: failed marks an error)
  void release(int k, bool failed = false) {
    if (failed) failed_.store(true);
    released_[(size_t)k] = 1;
    hsa_signal_subtract_screlease(sig_[(size_t)k], 1);
  }
  // waits for slot k's copies; false on a copy error or a failed release
  bool wait(int k) {
    const hsa_signal_value_t v = hsa_signal_wait_scacquire(
        sig_[(size_t)k], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
    return v == 0 && !failed_.load();
  }
  ~SdmaCopies() {  // nothing issued may outlive the call (and its staging)
    for (size_t k = 0; k < sig_.size(); ++k) {
      if (released_[k]) (void)wait((int)k);
      hsa_signal_destroy(sig_[k]);
    }
  }

 private:
  std::vector<hsa_signal_t> sig_;
  std::vector<char> released_;
  std::atomic<bool> failed_{false};
};

// cwq_code_grouped_greedy_batch with every item's partition on the device
// (cwq_partition.hip) and the chunks' group layouts built there too
// (k_batch_layout): after one small copy of the items' group counts the host
// only enqueues the chunks' encodes and writes the bitcode, on its threads, as
// each chunk's indices arrive.  Returns kBatchFellBack (nothing written) when
// the device partition does not cover the batch; the caller then runs the host
// path.  Standardisation and KL are already queued on s.
int64_t batch_device_path(int64_t n_items, const int64_t* item_off, int64_t D, int n_steps,
                          int n_bits_per_step, const int32_t* seeds, float rho,
                          int64_t size_threshold, double n_nats, float* sample_host,
                          char* bits_host, int64_t bits_cap, int64_t* bits_off,
                          int64_t* starts_host, int64_t* n_starts, char* w, size_t workspace_bytes,
                          const BatchWs& bl, const cwq_options& o, const std::vector<int64_t>& ci,
                          const float* t_loc, const float* t_scale, const float* kl,
                          const float* zeros, const float* ones, float* sample, float* out,
                          int64_t* offs, int32_t* idx, int32_t* bseed, int32_t* idx_h,
                          CallEvents& evs, CallEvents& tev, const float* p_loc,
                          const float* p_scale, hipStream_t s, hipStream_t d2h, hipStream_t h2d,
                          hipEvent_t part_ev, int64_t* pstage) {
  const GroupedWs& l = bl.g;
  const int64_t K = (int64_t)ci.size() - 1;
#ifdef CWQ_PHASE_TIMES  // tuning builds: per-phase host wall times to stderr
  struct timespec ts_start;
  clock_gettime(CLOCK_MONOTONIC, &ts_start);
  auto lap = [&](const char* what) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    fprintf(stderr, "[cwq batch dev] %-14s at %8.1f us (monotonic %.1f us)\n", what,
            (t.tv_sec - ts_start.tv_sec) * 1e6 + (t.tv_nsec - ts_start.tv_nsec) * 1e-3,
            t.tv_sec * 1e6 + t.tv_nsec * 1e-3);
  };
  lap("entry");
#else
  auto lap = [](const char*) {};
#endif
  int64_t* ioff_d = (int64_t*)(w + bl.ioff);
  int64_t* dst = (int64_t*)(w + bl.dstarts);
  int64_t* iinfo_d = (int64_t*)(w + bl.iinfo);
  cwq::BatchItem* itab_d = (cwq::BatchItem*)(w + bl.itab);
  int64_t* pst_d = (int64_t*)(w + bl.pstarts);
  unsigned long long* info_d = (unsigned long long*)(w + l.pinfo);
  hipEvent_t* done_ev = evs.ev.data() + K;
  // (the host path's per-chunk KL / layout events are free here)
  hipEvent_t layout_ev = evs.ev[0], pst_ev = evs.ev[(size_t)(2 * K)];
  hipEvent_t* res_ev = evs.ev.data() + 3 * K;
  auto drain = [&]() {
    (void)hipStreamSynchronize(s);
    (void)hipStreamSynchronize(d2h);
    (void)hipStreamSynchronize(h2d);
  };
  hipError_t e;
  unsigned long long* hi =
      (unsigned long long*)pinned_tl((size_t)(8 + 2 * n_items) * sizeof(unsigned long long));
  if (!hi) return kBatchFellBack;
  // info[0..7] were zeroed by the caller's k_grouped_prep; the wait polls
  if ((e = hipMemcpyAsync(ioff_d, item_off, (size_t)(n_items + 1) * 8, hipMemcpyHostToDevice,
                          s)) != hipSuccess ||
      (e = cwq::launch_partition(kl, D, ioff_d, n_items, size_threshold, group_thr(n_nats, false),
                                 dst, iinfo_d, w + l.part, info_d, s, true)) != hipSuccess ||
      (e = hipMemcpyAsync(hi, info_d, 8 * 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
      (e = hipMemcpyAsync(hi + 8, iinfo_d, (size_t)(2 * n_items) * 8, hipMemcpyDeviceToHost, s)) !=
          hipSuccess ||
      (e = hipEventRecord(part_ev, s)) != hipSuccess || (e = wait_event(part_ev)) != hipSuccess) {
    drain();
    return hip_fail(e, "cwq_code_grouped_greedy_batch: device partition");
  }
  if (cwq::partition_fell_back(hi)) return kBatchFellBack;
  lap("partitioned");
  // the items' group counts; per chunk its groups, largest group and layout
  std::vector<int64_t> gl((size_t)n_items), chunk_of((size_t)n_items);
  std::vector<int64_t> cG((size_t)K, 0), cmaxd((size_t)K, 0);
  g_batch_items.resize((size_t)n_items);
  std::vector<int64_t> pk((size_t)n_items + 1, 0);  // packed start-list offsets
  for (int64_t c = 0; c < K; ++c) {
    const int64_t a = item_off[ci[(size_t)c]], gb = a + ci[(size_t)c];
    int64_t g = 0;
    for (int64_t i = ci[(size_t)c]; i < ci[(size_t)c + 1]; ++i) {
      n_starts[i] = (int64_t)hi[8 + 2 * i];
      pk[(size_t)i + 1] = pk[(size_t)i] + n_starts[i];
      const int64_t Gi = n_starts[i] - 1 > 0 ? n_starts[i] - 1 : 0;
      gl[(size_t)i] = g;
      chunk_of[(size_t)i] = c;
      cmaxd[(size_t)c] = std::max<int64_t>(cmaxd[(size_t)c], (int64_t)hi[9 + 2 * i]);
      cwq::BatchItem& it = g_batch_items[(size_t)i];
      it.src = item_off[i] + 2 * i;
      it.rel = item_off[i] - a;
      it.go = gb + c + g;
      it.gs = gb + g;
      it.G = Gi;
      it.seed = seeds[i];
      it.pad = 0;
      it.pk = pk[(size_t)i];
      it.ns = n_starts[i];
      it.term = -1;
      it.dc = 0;
      g += Gi;
      bits_off[i + 1] = bits_off[i] + Gi * (int64_t)n_steps * n_bits_per_step;
    }
    cG[(size_t)c] = g;
    cwq::BatchItem& last = g_batch_items[(size_t)(ci[(size_t)c + 1] - 1)];
    last.term = gb + c + g;  // the chunk's closing offset: its dims
    last.dc = item_off[ci[(size_t)c + 1]] - a;
  }
  if (bits_off[n_items] > bits_cap) {
    drain();
    return fail(CWQ_ERR_CAPACITY, "cwq_code_grouped_greedy_batch: bits_cap %lld < %lld",
                (long long)bits_cap, (long long)bits_off[n_items]);
  }
  if ((e = hipMemcpyAsync(itab_d, g_batch_items.data(), (size_t)n_items * sizeof(cwq::BatchItem),
                          hipMemcpyHostToDevice, s)) != hipSuccess ||
      (e = cwq::launch_batch_layout(itab_d, n_items, dst, offs, bseed, pst_d, s)) !=
          hipSuccess) {
    drain();
    return hip_fail(e, "cwq_code_grouped_greedy_batch: layout");
  }
  // the items' start lists go to the caller in one copy on d2h, queued behind
  // the first chunk's coding (one copy per item took ~21 us each, serialised
  // after the coding: ~1 ms of C3's 48 items; one copy ahead of the first
  // chunk delayed its coding by the copy's 145 us); the bitcode workers unpack
  const int64_t npk = pk[(size_t)n_items];
  if (npk > 0 && (e = hipEventRecord(layout_ev, s)) != hipSuccess) {
    drain();
    return hip_fail(e, "cwq_code_grouped_greedy_batch: layout event");
  }
  auto starts_copy = [&]() -> hipError_t {
    hipError_t r = hipSuccess;
    if (npk > 0 && ((r = hipStreamWaitEvent(d2h, layout_ev, 0)) != hipSuccess ||
                    (r = hipMemcpyAsync(pstage, pst_d, (size_t)npk * 8, hipMemcpyDeviceToHost,
                                        d2h)) != hipSuccess ||
                    (r = hipEventRecord(pst_ev, d2h)) != hipSuccess))
      return r;
    return hipSuccess;
  };
  // the result copies: SDMA when available (slot c: chunk c, slot K: the start
  // lists), else HIP copies on d2h
  SdmaCopies sd;
  const bool use_sdma =
      sdma_enabled() && sd.init((int)K + 1, {pstage, pst_d, idx_h, idx, sample_host, out});
  // the chunks: encode, destandardise, results to the host behind the next chunk
  int64_t Gtot = 0;
  int rc = CWQ_OK;
  int64_t c_done = 0;
  for (int64_t c = 0; c < K && rc == CWQ_OK; ++c) {
    const int64_t a = item_off[ci[(size_t)c]], Dc = item_off[ci[(size_t)c + 1]] - a;
    const int64_t gb = a + ci[(size_t)c], Gc = cG[(size_t)c];
    Gtot += Gc;
    if (o.eval_start_event && c == 0 &&
        (e = hipEventRecord((hipEvent_t)o.eval_start_event, s)) != hipSuccess)
      rc = hip_fail(e, "event");
    if (rc == CWQ_OK && Gc > 0) {
      // eval_ms_out: the chunk's events bracket its scoring launches (inside
      // the encoder, before the destandardisation)
      cwq_options oc = o;
      oc.eval_start_event = o.eval_ms_out ? tev.ev[(size_t)(2 * c)] : nullptr;
      oc.eval_stop_event = o.eval_ms_out ? tev.ev[(size_t)(2 * c + 1)] : nullptr;
      oc.eval_ms_out = nullptr;
      if (rc == CWQ_OK)  // :273-284 the chunk's groups in one launch sequence
        rc = encode_impl(t_loc + a, t_scale + a, zeros + a, ones + a, offs + gb + c, 0, Gc, Dc,
                         cmaxd[(size_t)c], n_bits_per_step, n_steps, 0, rho, 0,
                         idx + gb * n_steps, sample + a, w + l.enc, workspace_bytes - l.enc, &oc,
                         s, bseed + gb, out + a, p_loc + a, p_scale + a);  // + :292
    } else if (rc == CWQ_OK && Dc > 0 &&
               (e = hipMemsetAsync(out + a, 0, (size_t)Dc * 4, s)) != hipSuccess) {
      rc = hip_fail(e, "memset");
    }
    if (rc == CWQ_OK && o.eval_stop_event && c == K - 1 &&
        (e = hipEventRecord((hipEvent_t)o.eval_stop_event, s)) != hipSuccess)
      rc = hip_fail(e, "event");
    if (rc == CWQ_OK && c == 0 && !use_sdma && (e = starts_copy()) != hipSuccess)
      rc = hip_fail(e, "start lists to host");
    if (rc == CWQ_OK && (e = hipEventRecord(res_ev[c], s)) != hipSuccess)
      rc = hip_fail(e, "event");
    if (use_sdma) {  // the copies are issued from the host once res_ev[c] completes
      if (rc == CWQ_OK) c_done = c + 1;
      continue;
    }
    if (rc == CWQ_OK && (e = hipStreamWaitEvent(d2h, res_ev[c], 0)) != hipSuccess)
      rc = hip_fail(e, "event");
#ifndef CWQ_DIAG_NO_D2H  // diagnostic builds only: the results' copies left out (timing)
    if (rc == CWQ_OK && Gc > 0 &&
        (e = hipMemcpyAsync(idx_h + gb * n_steps, idx + gb * n_steps, (size_t)(Gc * n_steps) * 4,
                            hipMemcpyDeviceToHost, d2h)) != hipSuccess)
      rc = hip_fail(e, "indices to host");
    if (rc == CWQ_OK && Dc > 0 &&
        (e = hipMemcpyAsync(sample_host + a, out + a, (size_t)Dc * 4, hipMemcpyDeviceToHost,
                            d2h)) != hipSuccess)
      rc = hip_fail(e, "sample to host");
#endif
    if (rc == CWQ_OK && (e = hipEventRecord(done_ev[c], d2h)) != hipSuccess)
      rc = hip_fail(e, "event");
    if (rc == CWQ_OK) c_done = c + 1;
  }
  lap("enqueued");
  // bitcode (:81-87, :288) and start list item by item as its chunk's
  // indices arrive, on the host threads and the calling thread
  std::atomic<int64_t> next{0};
  std::atomic<int> err{0};
  std::atomic<bool> issuer{false};
  // SDMA: the first thread in issues every copy, in order (the start lists
  // once the layout is done, then each chunk's results once it is coded);
  // every slot is released, also on an error, so no waiter hangs
  // a copy the SDMA path refuses is made with a synchronous HIP copy instead
  // (the event has completed: the data is final)
  auto copy = [&](int k, void* dst, const void* src, size_t bytes) {
    return sd.copy(k, dst, src, bytes) ||
           (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, d2h) == hipSuccess &&
            hipStreamSynchronize(d2h) == hipSuccess);
  };
  auto issue = [&]() {
    bool ok = npk == 0 || (wait_event(layout_ev) == hipSuccess &&
                           copy((int)K, pstage, pst_d, (size_t)npk * 8));
    sd.release((int)K, !ok);
    for (int64_t c = 0; c < K; ++c) {
      if (ok && c < c_done) {
        const int64_t a = item_off[ci[(size_t)c]], Dc = item_off[ci[(size_t)c + 1]] - a;
        const int64_t gb = a + ci[(size_t)c], Gc = cG[(size_t)c];
        ok = wait_event(res_ev[c]) == hipSuccess &&
             copy((int)c, idx_h + gb * n_steps, idx + gb * n_steps,
                  (size_t)(Gc * n_steps) * 4) &&
             copy((int)c, sample_host + a, out + a, (size_t)Dc * 4);
      }
      sd.release((int)c, !ok);  // waiters see the failure: no slot is left held
    }
  };
  auto bits_worker = [&]() {
    if (use_sdma && !issuer.exchange(true)) issue();
    for (;;) {
      const int64_t i = next.fetch_add(1);
      if (i >= n_items || err.load()) return;
      const int64_t c = chunk_of[(size_t)i];
      if (c >= c_done) return;
      const bool copied = use_sdma ? ((npk == 0 || sd.wait((int)K)) && sd.wait((int)c))
                                   : ((npk == 0 || wait_event(pst_ev) == hipSuccess) &&
                                      wait_event(done_ev[c]) == hipSuccess);
      if (!copied) {
        int z = 0;
        err.compare_exchange_strong(z, fail(CWQ_ERR_HIP, "results copy failed"));
        return;
      }
      memcpy(starts_host + item_off[i] + 2 * i, pstage + pk[(size_t)i],
             (size_t)n_starts[i] * 8);
      const int64_t gb = item_off[ci[(size_t)c]] + ci[(size_t)c];
      const int64_t Gi = n_starts[i] - 1 > 0 ? n_starts[i] - 1 : 0;
      const int64_t nw = write_bitcode(idx_h + (gb + gl[(size_t)i]) * n_steps, Gi * n_steps,
                                       n_bits_per_step, bits_host + bits_off[i]);
      if (nw < 0) {
        int z = 0;
        err.compare_exchange_strong(z, (int)nw);
        return;
      }
      if (o.item_ready) __atomic_store_n(o.item_ready + i, 1, __ATOMIC_RELEASE);
    }
  };
  if (rc == CWQ_OK) {
    const int64_t nw = std::min<int64_t>(host_threads() - 1, n_items - 1);
    HostPool::get().run(nw > 0 ? nw : 0, bits_worker);
  }
  lap("bits written");
  drain();
  lap("drained");
  if (rc < 0) return rc;
  if (err.load() < 0) return err.load();
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(e, "sync");
  if (o.eval_ms_out) {
    float tot = 0.0f;
    for (int64_t c = 0; c < K; ++c) {
      if (cG[(size_t)c] <= 0) continue;
      float ms = 0.0f;
      if ((e = hipEventElapsedTime(&ms, tev.ev[(size_t)(2 * c)], tev.ev[(size_t)(2 * c + 1)])) !=
          hipSuccess)
        return hip_fail(e, "event time");
      tot += ms;
    }
    *o.eval_ms_out = tot;
  }
  cwq::set_error(CWQ_OK, "");
  return Gtot;
}

}  // namespace

size_t cwq_code_grouped_greedy_batch_workspace_size(int64_t D, int64_t n_items, int n_steps) {
  if (D < 0 || n_items < 0 || n_steps < 0) return 0;
  return batch_ws(D, n_items, n_steps).total;
}

size_t cwq_code_grouped_greedy_batch_host_workspace_size(int64_t D, int64_t n_items,
                                                         int n_steps) {
  if (D < 0 || n_items < 0 || n_steps < 0) return 0;
  return batch_host_ws(D, n_items, n_steps).total;
}

int64_t cwq_code_grouped_greedy_batch(
    int64_t n_items, const int64_t* item_off, const float* q_loc, const float* q_scale,
    const float* p_loc, const float* p_scale, int n_steps, int n_bits_per_step,
    const int32_t* seeds, float rho, int64_t size_threshold, double n_nats, float* sample_host,
    char* bits_host, int64_t bits_cap, int64_t* bits_off, int64_t* starts_host,
    int64_t starts_cap, int64_t* n_starts, void* workspace, size_t workspace_bytes,
    void* host_workspace, size_t host_workspace_bytes, const cwq_options* opts, void* stream) {
  cwq_options o;
  {
    const int rc0 = read_options(opts, &o);
    if (rc0) return rc0;
  }
  if (n_items < 0 || n_steps < 1 || n_bits_per_step < 0 ||
      n_bits_per_step > CWQ_MAX_BITS_PER_STEP)
    return fail(CWQ_ERR_INVALID, "cwq_code_grouped_greedy_batch: bad sizes");
  if (!item_off || !bits_off || !n_starts || (n_items > 0 && !seeds))
    return fail(CWQ_ERR_INVALID, "cwq_code_grouped_greedy_batch: null pointer");
  if (item_off[0] != 0) return fail(CWQ_ERR_INVALID, "item_off[0] must be 0");
  for (int64_t i = 0; i < n_items; ++i)
    if (item_off[i + 1] < item_off[i])
      return fail(CWQ_ERR_INVALID, "item_off must be non-decreasing");
  const int64_t D = item_off[n_items];
  if (D > 0 && (!q_loc || !q_scale || !p_loc || !p_scale || !sample_host))
    return fail(CWQ_ERR_INVALID, "cwq_code_grouped_greedy_batch: null pointer");
  if (!starts_host || starts_cap < D + 2 * n_items)
    return fail(CWQ_ERR_CAPACITY, "starts_cap must be >= D_total + 2 n_items");
  const BatchWs bl = batch_ws(D, n_items, n_steps);
  const GroupedWs& l = bl.g;
  if (workspace_bytes < bl.total || !workspace)
    return fail(CWQ_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes,
                bl.total);
  const BatchHostWs hl = batch_host_ws(D, n_items, n_steps);
  if (host_workspace && host_workspace_bytes < hl.total)
    return fail(CWQ_ERR_WORKSPACE, "host workspace %zu bytes < required %zu",
                host_workspace_bytes, hl.total);
  if (bits_cap > 0 && !bits_host)
    return fail(CWQ_ERR_INVALID, "cwq_code_grouped_greedy_batch: null bits_host");
  bits_off[0] = 0;
  if (n_items == 0) return ok();
  hipStream_t s = (hipStream_t)stream;
#ifdef CWQ_PHASE_TIMES  // tuning builds: per-phase host wall times to stderr
  struct timespec ts_start;
  clock_gettime(CLOCK_MONOTONIC, &ts_start);
  auto lap = [&](const char* what, int64_t c) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    fprintf(stderr, "[cwq batch] %-12s chunk %2lld at %8.1f us (monotonic %.1f us)\n", what,
            (long long)c,
            (t.tv_sec - ts_start.tv_sec) * 1e6 + (t.tv_nsec - ts_start.tv_nsec) * 1e-3,
            t.tv_sec * 1e6 + t.tv_nsec * 1e-3);
  };
  lap("entry", 0);
#else
  auto lap = [](const char*, int64_t) {};
#endif
  char* hw = (char*)host_workspace;
  if (!hw) {  // no pinned staging from the caller: pageable, thread-local
    g_batch_host.resize(hl.total);
    hw = g_batch_host.data();
  }
  float* kl_h = (float*)(hw + hl.kl);
  int64_t* offs_h = (int64_t*)(hw + hl.offs);
  int32_t* seed_h = (int32_t*)(hw + hl.seeds);
  int32_t* idx_h = (int32_t*)(hw + hl.idx);
  char* w = (char*)workspace;
  float* t_loc = (float*)(w + l.t_loc);
  float* t_scale = (float*)(w + l.t_scale);
  float* kl = (float*)(w + l.kl);
  float* zeros = (float*)(w + l.zeros);
  float* ones = (float*)(w + l.ones);
  float* sample = (float*)(w + l.sample);
  float* out = (float*)(w + l.out);
  int64_t* offs = (int64_t*)(w + l.offs);
  int32_t* idx = (int32_t*)(w + l.idx);
  int32_t* bseed = (int32_t*)(w + bl.seeds);

  // chunks of consecutive items (at least one each): the first about a quarter
  // the size of the middle ones, so the device starts after a short first host
  // phase
  std::vector<int64_t> ci;  // chunk c = items [ci[c], ci[c + 1])
  {
    const int64_t K = D < (1 << 16) ? 1 : std::min<int64_t>(batch_chunks(), n_items);
    // the first chunk a quarter share, so the device starts early, the last a
    // half share (C3, 9 x 600 calls: 2.5% faster per call than a quarter; an
    // eighth was 3-5% slower): boundary c (1 <= c < K) at
    // D (c - 1 + f) / (K - 2 + f + l) with f = kSh[0] / 4, l = kSh[1] / 4;
    // one chunk when K == 1
    ci.push_back(0);
    for (int64_t i = 1; i < n_items && K > 1; ++i) {
      const int64_t c = (int64_t)ci.size();
#ifndef CWQ_BATCH_SHARES  // 4 x (first, last) chunk shares (tuning builds may set others)
#define CWQ_BATCH_SHARES 1, 2
#endif
      constexpr int64_t kSh[2] = {CWQ_BATCH_SHARES};
      if (c < K && item_off[i] * (4 * K - 8 + kSh[0] + kSh[1]) >= D * (4 * c - 4 + kSh[0]) &&
          item_off[i] > item_off[ci.back()])
        ci.push_back(i);
    }
    ci.push_back(n_items);
  }
  const int64_t K = (int64_t)ci.size() - 1;
  auto a_of = [&](int64_t c) { return item_off[ci[(size_t)c]]; };
  auto gbase = [&](int64_t c) { return a_of(c) + ci[(size_t)c]; };  // group-array region

  // Streams: the coding on the caller's stream s; device-to-host copies (the
  // KL chunks, then each chunk's results) on d2h and the chunks' layouts on
  // h2d, library copy streams of s's device, so the copies overlap the coding.
  // Events: KL ready; per chunk its KL on the host, its layout on the device,
  // its results computed, its results on the host (+ 2 K timing events).
  hipStream_t d2h = cwq::copy_stream(s, 0), h2d = cwq::copy_stream(s, 1);
  if (!d2h || !h2d) d2h = h2d = s;
  CallEvents evs;
  if (!evs.made((int)(4 * K + 1), s, hipEventDisableTiming))
    return fail(CWQ_ERR_HIP, "cwq_code_grouped_greedy_batch: event creation failed");
  CallEvents tev;
  if (o.eval_ms_out && !tev.made((int)(2 * K), s, hipEventDefault))
    return fail(CWQ_ERR_HIP, "cwq_code_grouped_greedy_batch: event creation failed");
  hipEvent_t* kl_ev = evs.ev.data();
  hipEvent_t* done_ev = evs.ev.data() + K;
  hipEvent_t* h2d_ev = evs.ev.data() + 2 * K;
  hipEvent_t* res_ev = evs.ev.data() + 3 * K;
  hipEvent_t kl_ready = evs.ev[(size_t)(4 * K)];
  auto drain = [&]() {  // nothing this call queued may outlive it
    (void)hipStreamSynchronize(h2d);
    (void)hipStreamSynchronize(s);
    (void)hipStreamSynchronize(d2h);
  };

  hipError_t e = hipSuccess;
  int rc;
  // :193-210 for every item at once (elementwise), then the KL to the host chunk
  // by chunk, so the first chunk's partitions start before the rest arrives
  // (one launch: standardise, KL, the standard prior, the partition's counters)
  const bool try_dev = device_partition_enabled() && cwq::partition_applies(D, size_threshold);
  if ((e = cwq::launch_grouped_prep(q_loc, q_scale, p_loc, p_scale, D, t_loc, t_scale, kl, zeros,
                                    ones, (unsigned long long*)(w + l.pinfo), try_dev ? 8 : 0,
                                    s)) != hipSuccess)
    return hip_fail(e, "cwq_code_grouped_greedy_batch: standardise / KL");
  if (try_dev) {
    // :207-252 every item's partition on the device (cwq_partition.hip: one walk
    // over the batch, bit-identical to the host loop), then the chunks' group
    // layouts on the device too: the host only sequences launches and writes the
    // bitcode.  Falls through to the host path when the device one does not apply.
    lap("to device", 0);
    const int64_t r = batch_device_path(
        n_items, item_off, D, n_steps, n_bits_per_step, seeds, rho, size_threshold, n_nats,
        sample_host, bits_host, bits_cap, bits_off, starts_host, n_starts, w, workspace_bytes, bl,
        o, ci, t_loc, t_scale, kl, zeros, ones, sample, out, offs, idx, bseed, idx_h, evs, tev,
        p_loc, p_scale, s, d2h, h2d, kl_ready, offs_h);
    if (r != kBatchFellBack) return r;
  }
  if ((e = hipEventRecord(kl_ready, s)) == hipSuccess) e = hipStreamWaitEvent(d2h, kl_ready, 0);
  for (int64_t c = 0; c < K && e == hipSuccess; ++c) {
    const int64_t a = a_of(c), n = a_of(c + 1) - a;
    if (n > 0 &&
        (e = hipMemcpyAsync(kl_h + a, kl + a, (size_t)n * 4, hipMemcpyDeviceToHost, d2h)) !=
            hipSuccess)
      break;
    e = hipEventRecord(kl_ev[c], d2h);
  }
  if (e != hipSuccess) {
    drain();
    return hip_fail(e, "KL to host");
  }
  lap("kl queued", 0);

  // Host tasks, on worker threads (the calling thread sequences the device),
  // claimed in item order:
  //   part(i): item i's partition (:207-252; its starts at item_off[i] + 2 i)
  //            once its chunk's KL is on the host; the thread that finishes a
  //            chunk's last partition lays out the chunk's CSR offsets (local
  //            group numbers) and seeds seeds[i] + g (:282);
  //   bits(i): once item i's chunk is on the host, its LSB-first bitcode at
  //            bits_off[i] (:81-87, :288).
  // The calling thread runs any task no worker has taken when it needs it
  // (also when no worker thread could be started).
  struct ChunkState {
    std::atomic<int64_t> parts_left{0};
    std::atomic<int> failed{0};
    std::atomic<int> prepared{0};  // 1 laid out, -1 failed
    std::atomic<int> enqueued{0};  // 1 results on their way (bits_off known), -1 abandoned
    int64_t G = 0, maxd = 0;
  };
  std::vector<ChunkState> cs((size_t)K);
  std::vector<int64_t> chunk_of((size_t)n_items), imaxd((size_t)n_items, 0);
  for (int64_t c = 0; c < K; ++c) {
    cs[(size_t)c].parts_left.store(ci[(size_t)c + 1] - ci[(size_t)c]);
    for (int64_t i = ci[(size_t)c]; i < ci[(size_t)c + 1]; ++i) chunk_of[(size_t)i] = c;
  }
  std::unique_ptr<std::atomic<int>[]> part_claimed(new std::atomic<int>[(size_t)n_items]);
  std::unique_ptr<std::atomic<int>[]> bits_claimed(new std::atomic<int>[(size_t)n_items]);
  for (int64_t i = 0; i < n_items; ++i) {
    part_claimed[(size_t)i].store(0);
    bits_claimed[(size_t)i].store(0);
  }
  std::vector<int64_t> gloc((size_t)n_items + 1, 0);  // item's first group within its chunk
  std::atomic<int> err_rc{0};
  std::mutex mu;
  std::condition_variable cv;
  const float* klh = kl_h;
  auto record_err = [&](int r) {
    int z = 0;
    err_rc.compare_exchange_strong(z, r);
  };
  auto set_flag = [&](std::atomic<int>& f, int v) {
    {
      std::lock_guard<std::mutex> lk(mu);
      f.store(v);
    }
    cv.notify_all();
  };
  auto partition = [&](int64_t i) -> int {
    const int64_t c = chunk_of[(size_t)i];
    if (wait_event(kl_ev[c]) != hipSuccess) return fail(CWQ_ERR_HIP, "KL copy failed");
    lap("kl in", i);
    const int64_t ai = item_off[i], Di = item_off[i + 1] - ai;
    int64_t* st = starts_host + ai + 2 * i;
    const int64_t ns = group_starts_impl(Di > 0 ? klh + ai : nullptr, Di, size_threshold, n_nats,
                                         st, Di + 2, false);
    if (ns < 0) return (int)ns;
    n_starts[i] = ns;
    int64_t md = 0;
    for (int64_t g = 0; g + 1 < ns; ++g) md = std::max(md, st[g + 1] - st[g]);
    imaxd[(size_t)i] = md;
    lap("parted", i);
    return CWQ_OK;
  };
  auto layout = [&](int64_t c) {  // every item of chunk c is partitioned
    const int64_t a = a_of(c), gb = gbase(c);
    int64_t gl = 0, md = 0;
    for (int64_t i = ci[(size_t)c]; i < ci[(size_t)c + 1]; ++i) {
      const int64_t* st = starts_host + item_off[i] + 2 * i;
      const int64_t Gi = n_starts[i] - 1 > 0 ? n_starts[i] - 1 : 0;
      gloc[(size_t)i] = gl;
      int64_t* go = offs_h + gb + c + gl;  // offsets relative to the chunk's first dim
      int32_t* gs = seed_h + gb + gl;
      const int64_t rel = item_off[i] - a;
      for (int64_t g = 0; g < Gi; ++g) {
        go[g] = rel + st[g];
        gs[g] = (int32_t)((uint32_t)seeds[i] + (uint32_t)g);  // :282, int32 wrap
      }
      md = std::max(md, imaxd[(size_t)i]);
      gl += Gi;
    }
    offs_h[gb + c + gl] = a_of(c + 1) - a;
    cs[(size_t)c].G = gl;
    cs[(size_t)c].maxd = md;
  };
  auto run_part = [&](int64_t i) {
    const int64_t c = chunk_of[(size_t)i];
    const int r = err_rc.load() ? CWQ_OK : partition(i);
    if (r < 0) {
      record_err(r);
      cs[(size_t)c].failed.store(1);
    }
    if (cs[(size_t)c].parts_left.fetch_sub(1) == 1) {  // the chunk's last partition
      const bool bad = cs[(size_t)c].failed.load() || err_rc.load();
      if (!bad) layout(c);
      lap("prepared", c);
      set_flag(cs[(size_t)c].prepared, bad ? -1 : 1);
    }
  };
  auto run_bits = [&](int64_t i) {
    const int64_t c = chunk_of[(size_t)i];
    {  // bits_off of the chunk's items is known once the chunk is enqueued
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return cs[(size_t)c].enqueued.load() != 0; });
    }
    if (cs[(size_t)c].enqueued.load() < 0) return;
    if (wait_event(done_ev[c]) != hipSuccess) {
      record_err(fail(CWQ_ERR_HIP, "results copy failed"));
      return;
    }
    const int64_t Gi = n_starts[i] - 1 > 0 ? n_starts[i] - 1 : 0;
    const int64_t nw = write_bitcode(idx_h + (gbase(c) + gloc[(size_t)i]) * n_steps, Gi * n_steps,
                                     n_bits_per_step, bits_host + bits_off[i]);
    if (nw < 0) {
      record_err((int)nw);
      return;
    }
    if (o.item_ready) __atomic_store_n(o.item_ready + i, 1, __ATOMIC_RELEASE);
  };
  auto worker = [&]() {
    for (int64_t i = 0; i < n_items; ++i)
      if (!part_claimed[(size_t)i].exchange(1)) run_part(i);
    for (int64_t i = 0; i < n_items; ++i)
      if (!bits_claimed[(size_t)i].exchange(1)) run_bits(i);
  };
  std::vector<std::thread> pool;
  {
    // thread creation may fail (pids cgroup, RLIMIT_NPROC): the exception must
    // not cross the C ABI; the calling thread then runs the remaining tasks
    const int64_t nw = K > 1 ? std::min<int64_t>(host_threads() - 1, n_items) : 0;
    try {
      for (int64_t t = 0; t < nw; ++t) pool.emplace_back(worker);
    } catch (...) {
    }
  }
  // the calling thread: chunk by chunk, in order, enqueue the device work
  int64_t Gtot = 0;
  int64_t c_done = 0;  // chunks whose device work was enqueued
  for (int64_t c = 0; c < K && err_rc.load() == 0; ++c) {
    for (int64_t i = ci[(size_t)c]; i < ci[(size_t)c + 1]; ++i)
      if (!part_claimed[(size_t)i].exchange(1)) run_part(i);
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return cs[(size_t)c].prepared.load() != 0; });
    }
    if (cs[(size_t)c].prepared.load() < 0) break;
    const int64_t i0 = ci[(size_t)c], i1 = ci[(size_t)c + 1];
    for (int64_t i = i0; i < i1; ++i) {
      const int64_t Gi = n_starts[i] - 1 > 0 ? n_starts[i] - 1 : 0;
      bits_off[i + 1] = bits_off[i] + Gi * (int64_t)n_steps * n_bits_per_step;
    }
    if (bits_off[i1] > bits_cap) {
      record_err(fail(CWQ_ERR_CAPACITY, "cwq_code_grouped_greedy_batch: bits_cap %lld < %lld",
                      (long long)bits_cap, (long long)bits_off[i1]));
      break;
    }
    const ChunkState& ch = cs[(size_t)c];
    const int64_t a = a_of(c), Dc = a_of(c + 1) - a, gb = gbase(c);
    Gtot += ch.G;
    rc = CWQ_OK;
    // the caller's eval events span the chunks' encodes (device gaps between
    // chunks included); eval_ms_out sums the chunks' own spans
    if (o.eval_start_event && c == 0 &&
        (e = hipEventRecord((hipEvent_t)o.eval_start_event, s)) != hipSuccess)
      rc = hip_fail(e, "event");
    if (rc == CWQ_OK && ch.G > 0) {
      if ((e = hipMemcpyAsync(offs + gb + c, offs_h + gb + c, (size_t)(ch.G + 1) * 8,
                              hipMemcpyHostToDevice, h2d)) != hipSuccess ||
          (e = hipMemcpyAsync(bseed + gb, seed_h + gb, (size_t)ch.G * 4, hipMemcpyHostToDevice,
                              h2d)) != hipSuccess ||
          (e = hipEventRecord(h2d_ev[c], h2d)) != hipSuccess ||
          (e = hipStreamWaitEvent(s, h2d_ev[c], 0)) != hipSuccess)
        rc = hip_fail(e, "layout to device");
      // :273-284 the chunk's groups in one launch sequence; eval_ms_out: the
      // chunk's events bracket its scoring launches (inside the encoder, before
      // the destandardisation)
      cwq_options oc = o;
      oc.eval_start_event = o.eval_ms_out ? tev.ev[(size_t)(2 * c)] : nullptr;
      oc.eval_stop_event = o.eval_ms_out ? tev.ev[(size_t)(2 * c + 1)] : nullptr;
      oc.eval_ms_out = nullptr;
      if (rc == CWQ_OK)
        rc = encode_impl(t_loc + a, t_scale + a, zeros + a, ones + a, offs + gb + c, 0, ch.G, Dc,
                         ch.maxd, n_bits_per_step, n_steps, 0, rho, 0, idx + gb * n_steps,
                         sample + a, w + l.enc, workspace_bytes - l.enc, &oc, stream, bseed + gb,
                         out + a, p_loc + a, p_scale + a);  // + :292 destandardise
    } else if (rc == CWQ_OK && Dc > 0) {  // no groups (empty items only): the sample is zeros
      if ((e = hipMemsetAsync(out + a, 0, (size_t)Dc * 4, s)) != hipSuccess)
        rc = hip_fail(e, "memset");
    }
    if (rc == CWQ_OK && o.eval_stop_event && c == K - 1 &&
        (e = hipEventRecord((hipEvent_t)o.eval_stop_event, s)) != hipSuccess)
      rc = hip_fail(e, "event");
    // the chunk's results to the host on d2h, behind the coding of the next chunk
    if (rc == CWQ_OK && ((e = hipEventRecord(res_ev[c], s)) != hipSuccess ||
                         (e = hipStreamWaitEvent(d2h, res_ev[c], 0)) != hipSuccess))
      rc = hip_fail(e, "event");
    if (rc == CWQ_OK && ch.G > 0 &&
        (e = hipMemcpyAsync(idx_h + gb * n_steps, idx + gb * n_steps,
                            (size_t)(ch.G * n_steps) * 4, hipMemcpyDeviceToHost, d2h)) !=
            hipSuccess)
      rc = hip_fail(e, "indices to host");
    if (rc == CWQ_OK && Dc > 0 &&
        (e = hipMemcpyAsync(sample_host + a, out + a, (size_t)Dc * 4, hipMemcpyDeviceToHost,
                            d2h)) != hipSuccess)
      rc = hip_fail(e, "sample to host");
    if (rc == CWQ_OK && (e = hipEventRecord(done_ev[c], d2h)) != hipSuccess)
      rc = hip_fail(e, "event");
    if (rc < 0) {
      record_err(rc);
      break;
    }
    set_flag(cs[(size_t)c].enqueued, 1);
    c_done = c + 1;
    lap("enqueued", c);
  }
  // chunks never enqueued release the workers waiting for them; then the
  // calling thread takes the bitcode tasks no worker took
  for (int64_t i = 0; i < n_items; ++i)
    if (chunk_of[(size_t)i] >= c_done) part_claimed[(size_t)i].store(1);  // not started from now on
  for (int64_t c = c_done; c < K; ++c) set_flag(cs[(size_t)c].enqueued, -1);
  for (int64_t i = 0; i < n_items; ++i)
    if (!bits_claimed[(size_t)i].exchange(1)) run_bits(i);
  for (auto& th : pool) th.join();
  // no device work of this call may outlive it (also after an error); the
  // caller's stream is ordered after the copies
  if (c_done > 0 && (e = hipStreamWaitEvent(s, done_ev[c_done - 1], 0)) != hipSuccess &&
      err_rc.load() == 0) {
    drain();
    return hip_fail(e, "join");
  }
  drain();
  if ((e = hipStreamSynchronize(s)) != hipSuccess && err_rc.load() == 0)
    return hip_fail(e, "sync");
  if (err_rc.load() < 0) return err_rc.load();
  lap("bits done", K);
  if (o.eval_ms_out) {
    float tot = 0.0f;
    for (int64_t c = 0; c < K; ++c) {
      if (cs[(size_t)c].G <= 0) continue;
      float ms = 0.0f;
      if ((e = hipEventElapsedTime(&ms, tev.ev[(size_t)(2 * c)], tev.ev[(size_t)(2 * c + 1)])) !=
          hipSuccess)
        return hip_fail(e, "event time");
      tot += ms;
    }
    *o.eval_ms_out = tot;
  }
  cwq::set_error(CWQ_OK, "");
  return Gtot;
}

// ---------------------------------------------------------------------------
// code_grouped_importance_sample (coded_importance_sampler.py:112-274) for one
// item or a batch of items in one call: device standardisation, KL, outlier
// masking and the outliers' seeded target draw (one launch), the host
// partition and sample-count plan of every item, one encode launch over every
// item's groups (item i's group g seeded seeds[i] + g), device
// destandardisation.  Elias-delta strings and quint16 packing stay with the
// caller (host, cheap).
// ---------------------------------------------------------------------------
namespace {
struct GroupedImpWs {
  size_t t_loc, t_scale, zeros, ones, sample, res, d2h, plan, items, enc, total;
  size_t a4;  // align_up(4 D, 256): the stride inside the packed regions
};
// D dims in I items: at most D + I groups (an item's partition has at most
// D_i + 1 groups).  What crosses PCIe sits in packed regions, one copy each,
// laid out identically in the host staging: d2h = [KL | outlier draws | kept
// flags] (to the host after the preparation launch), res = [sample | indices]
// (to the host at the end), plan = [counts | offsets | seeds] (to the device;
// the offsets and seeds start at offsets set by the call's group count, see
// imp_plan_offsets), items = [item offsets | seeds - 1] (to the device, batches).
GroupedImpWs grouped_imp_ws(int64_t D, int64_t I) {
  GroupedImpWs l;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align_up(o + bytes, 256);
    return at;
  };
  const size_t n = (size_t)(D > 0 ? D : 0), ni = (size_t)(I > 0 ? I : 0), g = n + ni;
  l.a4 = align_up(n * 4, 256);
  l.t_loc = take(n * 4);
  l.t_scale = take(n * 4);
  l.zeros = take(n * 4);
  l.ones = take(n * 4);
  l.sample = take(n * 4);
  l.res = take(l.a4 + g * 8);
  l.d2h = take(2 * l.a4 + n);
  l.plan = take(align_up(g * 8, 256) + align_up((g + 1) * 8, 256) + g * 4);
  l.items = take(align_up((ni + 1) * 8, 256) + ni * 4);
  l.enc = take(cwq::importance_workspace_size((int64_t)g, (int64_t)n));
  l.total = o;
  return l;
}
// The plan region for G groups: counts at 0, offsets at *po, seeds at *pg;
// returns the bytes one copy moves (the seeds only with per-item seeds).
size_t imp_plan_offsets(int64_t G, bool seeds, size_t* po, size_t* pg) {
  *po = align_up((size_t)G * 8, 256);
  *pg = *po + align_up((size_t)(G + 1) * 8, 256);
  return seeds ? *pg + (size_t)G * 4 : *po + (size_t)(G + 1) * 8;
}
thread_local PinnedTl tl_imp_pin;             // the grouped importance calls' host staging
thread_local std::vector<char> tl_imp_pageable;  // ... when page-locked memory is unavailable

int64_t grouped_importance_impl(int64_t I, const int64_t* item_off, const float* q_loc,
                                const float* q_scale, const float* p_loc, const float* p_scale,
                                const int32_t* seeds, float dim_kl_bit_limit,
                                int64_t size_threshold, double n_nats, float* sample_host,
                                int64_t* index_host, int64_t* starts_host, int64_t starts_cap,
                                int64_t* n_starts, int64_t* outlier_idx_host,
                                float* outlier_val_host, int64_t* n_outliers,
                                double* kl_sum_out, void* workspace, size_t workspace_bytes,
                                const cwq_options* opts, void* stream, const char* who) {
  cwq_options oi;
  {
    const int rc0 = read_options(opts, &oi);
    if (rc0) return rc0;
  }
  if (I < 1 || !item_off || !seeds || !n_starts || !n_outliers)
    return fail(CWQ_ERR_INVALID, "%s: bad arguments", who);
  if (item_off[0] != 0) return fail(CWQ_ERR_INVALID, "%s: item_off[0] must be 0", who);
  for (int64_t i = 0; i < I; ++i)
    if (item_off[i + 1] < item_off[i]) return fail(CWQ_ERR_INVALID, "%s: item_off not sorted", who);
  const int64_t D = item_off[I];
  if (D > 0 && (!q_loc || !q_scale || !p_loc || !p_scale || !sample_host || !index_host ||
                !outlier_idx_host || !outlier_val_host))
    return fail(CWQ_ERR_INVALID, "%s: null pointer", who);
  if (!starts_host || starts_cap < D + 2 * I)
    return fail(CWQ_ERR_CAPACITY, "%s: starts_cap must be >= D + 2 n_items", who);
  const GroupedImpWs l = grouped_imp_ws(D, I);
  if (workspace_bytes < l.total || !workspace)
    return fail(CWQ_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, l.total);
  for (int64_t i = 0; i < I; ++i) {
    n_outliers[i] = 0;
    n_starts[i] = 1;
    starts_host[item_off[i] + 2 * i] = 0;
    if (kl_sum_out) kl_sum_out[i] = 0.0;
  }
  if (oi.eval_ms_out) *oi.eval_ms_out = 0.0f;
  if (D == 0) return ok();
  hipStream_t s = (hipStream_t)stream;
#ifdef CWQ_PHASE_TIMES  // tuning builds: per-phase host wall times to stderr
  struct timespec ts0, ts1;
  clock_gettime(CLOCK_MONOTONIC, &ts0);
  auto lap = [&](const char* what) {
    clock_gettime(CLOCK_MONOTONIC, &ts1);
    fprintf(stderr, "[cwq imp] %-10s %8.1f us\n", what,
            (ts1.tv_sec - ts0.tv_sec) * 1e6 + (ts1.tv_nsec - ts0.tv_nsec) * 1e-3);
    ts0 = ts1;
  };
#else
  auto lap = [](const char*) {};
#endif
  char* w = (char*)workspace;
  float* t_loc = (float*)(w + l.t_loc);
  float* t_scale = (float*)(w + l.t_scale);
  float* kl2 = (float*)(w + l.d2h);
  float* tsamp = (float*)(w + l.d2h + l.a4);
  uint8_t* keep = (uint8_t*)(w + l.d2h + 2 * l.a4);
  float* zeros = (float*)(w + l.zeros);
  float* ones = (float*)(w + l.ones);
  float* sample = (float*)(w + l.sample);
  float* out = (float*)(w + l.res);
  int64_t* idx = (int64_t*)(w + l.res + l.a4);
  int64_t* nsamp = (int64_t*)(w + l.plan);
  int64_t* items_d = (int64_t*)(w + l.items);
  int32_t* seed1_d = (int32_t*)(w + l.items + align_up((size_t)(I + 1) * 8, 256));
  // the host side's arrays in this thread's page-locked staging (pageable
  // memory is staged by the runtime: I1's 2.9 MB of copies took ~0.5 ms more),
  // waits polled on events (a blocking wait's wake-up cost I2's small calls
  // ~0.1 ms each)
  const size_t Dz = (size_t)D, Gz = (size_t)(D + I), Iz = (size_t)I;
  size_t ho = 0;
  auto htake = [&](size_t b) {
    const size_t at = ho;
    ho = align_up(ho + b, 256);
    return at;
  };
  // the packed regions (same layout as the device's) and the batch's per-item plans
  const size_t o_d2h = htake(2 * l.a4 + Dz), o_res = htake(l.a4 + Gz * 8),
               o_plan = htake(align_up(Gz * 8, 256) + align_up((Gz + 1) * 8, 256) + Gz * 4),
               o_items = htake(align_up((Iz + 1) * 8, 256) + Iz * 4),
               o_nst = htake(I > 1 ? Gz * 8 : 0);
  char* hp = (char*)tl_imp_pin.get(ho, ho + ho / 4);
  if (!hp) {  // no page-locked memory: pageable staging (slower copies)
    tl_imp_pageable.resize(ho);
    hp = tl_imp_pageable.data();
  }
  float* kl_h = (float*)(hp + o_d2h);
  float* ts_h = (float*)(hp + o_d2h + l.a4);
  uint8_t* keep_h = (uint8_t*)(hp + o_d2h + 2 * l.a4);
  float* out_h = (float*)(hp + o_res);
  int64_t* idx_h = (int64_t*)(hp + o_res + l.a4);
  int64_t* ns_h = (int64_t*)(hp + o_plan);
  int64_t* items_h = (int64_t*)(hp + o_items);
  int32_t* s1_h = (int32_t*)(hp + o_items + align_up((Iz + 1) * 8, 256));
  int64_t* nst_h = I > 1 ? (int64_t*)(hp + o_nst) : ns_h;  // item i's plan at item_off[i] + i
  hipError_t e = hipSuccess;
  // every failure after the first copy or launch drains the stream first: the
  // staging buffer may be reused (or reallocated) by this thread's next call
  auto drain_fail = [&](hipError_t err, const char* where) -> int64_t {
    (void)hipStreamSynchronize(s);
    return hip_fail(err, where);
  };
  auto drain_rc = [&](int64_t r) -> int64_t {
    (void)hipStreamSynchronize(s);
    return r;
  };
  CallEvents hev;
  if (!hev.made(2, s, hipEventDisableTiming))
    return fail(CWQ_ERR_HIP, "%s: event creation failed", who);
  // :137-138 standardise; :142 KL(target || proposal); :144-148 outliers; :150
  // the outlier dims' target draw, seeded [seed - 1, 42];
  // :160-163 KL of the standardised target against N(0, 1): one launch
  const int64_t* items_arg = nullptr;
  const int32_t* seed1_arg = nullptr;
  if (I > 1) {
    memcpy(items_h, item_off, (Iz + 1) * 8);
    for (int64_t i = 0; i < I; ++i) s1_h[i] = (int32_t)((uint32_t)seeds[i] - 1u);
    if ((e = hipMemcpyAsync(items_d, items_h, align_up((Iz + 1) * 8, 256) + Iz * 4,
                            hipMemcpyHostToDevice, s)) != hipSuccess)
      return drain_fail(e, "items to device");
    items_arg = items_d;
    seed1_arg = seed1_d;
  }
  if ((e = cwq::launch_imp_grouped_prep(q_loc, q_scale, p_loc, p_scale, D, dim_kl_bit_limit,
                                        items_arg, seed1_arg, I,
                                        (int32_t)((uint32_t)seeds[0] - 1u), t_loc, t_scale, keep,
                                        zeros, ones, kl2, tsamp, s)) != hipSuccess)
    return drain_fail(e, "standardise / KL / outliers");
  if ((e = hipMemcpyAsync(kl_h, kl2, 2 * l.a4 + Dz, hipMemcpyDeviceToHost, s)) != hipSuccess ||
      (e = hipEventRecord(hev.ev[0], s)) != hipSuccess)
    return drain_fail(e, "to host");
  lap("prep queued");
  if ((e = wait_event(hev.ev[0])) != hipSuccess) return drain_fail(e, "sync");
  lap("kl in");
  // per item: outliers, :164-203 the sequential partition (strict >), :48-51
  // ceil(exp(sum KL)) per group (a batch: items on the host pool's threads;
  // I2's 24 items took 240 us in one thread), then every group's global
  // offset, seed and count in order
  std::atomic<int64_t> next_item{0}, item_rc{0};
  auto plan_items = [&]() {
    for (int64_t i; (i = next_item.fetch_add(1)) < I && item_rc.load() == 0;) {
      const int64_t a = item_off[i], Di = item_off[i + 1] - a;
      int64_t no = 0;
      for (int64_t j = 0; j < Di; ++j)
        if (!keep_h[a + j]) {
          outlier_idx_host[a + no] = j;
          outlier_val_host[a + no] = ts_h[a + j];
          ++no;
        }
      n_outliers[i] = no;
      if (kl_sum_out) {  // log line only
        double t = 0.0;
        for (int64_t j = 0; j < Di; ++j) t += (double)kl_h[a + j];
        kl_sum_out[i] = t;
      }
      if (Di == 0) continue;
      int64_t* st = starts_host + a + 2 * i;
      const int64_t n = group_starts_impl(kl_h + a, Di, size_threshold, n_nats, st, Di + 2, true);
      int64_t r = n < 0 ? n : cwq_importance_plan(kl_h + a, st, n - 1, nst_h + a + (I > 1 ? i : 0));
      if (r < 0) {
        int64_t z = 0;
        item_rc.compare_exchange_strong(z, r);
        continue;
      }
      n_starts[i] = n;
    }
  };
  const int64_t nw = I > 1 ? std::min<int64_t>(host_threads() - 1, I - 1) : 0;
  if (nw > 0 && D >= 4096)
    HostPool::get().run(nw, plan_items);
  else
    plan_items();
  if (item_rc.load() < 0)
    return drain_rc(fail((int)item_rc.load(), "%s: item partition / plan failed", who));
  int64_t Gtot = 0;
  for (int64_t i = 0; i < I; ++i) Gtot += n_starts[i] - 1 > 0 ? n_starts[i] - 1 : 0;
  size_t po = 0, pg = 0;
  const size_t plan_bytes = imp_plan_offsets(Gtot, I > 1, &po, &pg);
  int64_t* offs_h = (int64_t*)(hp + o_plan + po);
  int32_t* gs_h = (int32_t*)(hp + o_plan + pg);
  int64_t* offs = (int64_t*)(w + l.plan + po);
  int32_t* gseed = (int32_t*)(w + l.plan + pg);
  Gtot = 0;
  for (int64_t i = 0; i < I; ++i) {
    const int64_t a = item_off[i], G = n_starts[i] - 1;
    const int64_t* st = starts_host + a + 2 * i;
    if (I > 1 && G > 0) memcpy(ns_h + Gtot, nst_h + a + i, (size_t)G * 8);
    for (int64_t g = 0; g < G; ++g) {
      offs_h[Gtot + g] = a + st[g];
      gs_h[Gtot + g] = (int32_t)((uint32_t)seeds[i] + (uint32_t)g);  // :243 seed + g
    }
    Gtot += G;
  }
  offs_h[Gtot] = D;
  lap("planned");
  int64_t tcand = 0;  // the launch's candidates (selects the encoder's instantiation)
  for (int64_t g = 0; g < Gtot; ++g) tcand += ns_h[g] > 1 ? ns_h[g] : 1;
  if (Gtot > 0) {
    if ((e = hipMemcpyAsync(nsamp, ns_h, plan_bytes, hipMemcpyHostToDevice, s)) != hipSuccess)
      return drain_fail(e, "plan to device");
    // :212-245 every group's importance coder; eval_ms_out: its launches timed
    // with events of this call (the call synchronises anyway)
    CallEvents tev;
    if (oi.eval_ms_out && !tev.made(2, s, hipEventDefault))
      return drain_rc(fail(CWQ_ERR_HIP, "%s: event creation failed", who));
    if ((oi.eval_ms_out && (e = hipEventRecord(tev.ev[0], s)) != hipSuccess) ||
        (e = cwq::launch_importance_encode(t_loc, t_scale, zeros, ones, offs, nsamp, Gtot, D,
                                           seeds[0], 0, I > 1 ? gseed : nullptr,
                                           oi.prune_mode >= 2 ? 1 : 0, idx, nullptr, w + l.enc,
                                           s, tcand, cwq::importance_tile_count(ns_h, Gtot, tcand),
                                           p_loc, p_scale, out)) != hipSuccess ||
        (oi.eval_ms_out && (e = hipEventRecord(tev.ev[1], s)) != hipSuccess))
      return drain_fail(e, "importance encode");
    if (oi.eval_ms_out) {
      if ((e = hipEventSynchronize(tev.ev[1])) != hipSuccess ||
          (e = hipEventElapsedTime(oi.eval_ms_out, tev.ev[0], tev.ev[1])) != hipSuccess)
        return drain_fail(e, "event time");
    }
  } else {  // (no groups: D == 0 returned above; kept for completeness)
    if ((e = hipMemsetAsync(sample, 0, Dz * 4, s)) != hipSuccess ||
        (e = cwq::launch_destandardise(sample, p_loc, p_scale, D, out, s)) != hipSuccess)
      return drain_fail(e, "destandardise");
  }
  // :265 rescale: in the encoder's row launch (every dim is in a group);
  // :267 outliers keep their target draw
  if ((e = hipMemcpyAsync(out_h, out, Gtot > 0 ? l.a4 + (size_t)Gtot * 8 : Dz * 4,
                          hipMemcpyDeviceToHost, s)) != hipSuccess ||
      (e = hipEventRecord(hev.ev[1], s)) != hipSuccess)
    return drain_fail(e, "to host");
  lap("enqueued");
  if ((e = wait_event(hev.ev[1])) != hipSuccess) return drain_fail(e, "sync");
  lap("done");
  int64_t gb = 0;
  for (int64_t i = 0; i < I; ++i) {
    const int64_t G = n_starts[i] - 1;
    if (G > 0) memcpy(index_host + item_off[i] + i, idx_h + gb, (size_t)G * 8);
    gb += G;
  }
  for (int64_t j = 0; j < D; ++j) sample_host[j] = keep_h[j] ? out_h[j] : ts_h[j];
  lap("out");
  cwq::set_error(CWQ_OK, "");
  return Gtot;
}
}  // namespace

size_t cwq_code_grouped_importance_workspace_size(int64_t D) {
  if (D < 0) return 0;
  return grouped_imp_ws(D, 1).total;
}

int64_t cwq_code_grouped_importance(const float* q_loc, const float* q_scale,
                                    const float* p_loc, const float* p_scale, int64_t D,
                                    int32_t seed, float dim_kl_bit_limit, int64_t size_threshold,
                                    double n_nats, float* sample_host, int64_t* index_host,
                                    int64_t* starts_host, int64_t starts_cap,
                                    int64_t* outlier_idx_host, float* outlier_val_host,
                                    int64_t* n_outliers, double* kl_sum_out, void* workspace,
                                    size_t workspace_bytes, const cwq_options* opts,
                                    void* stream) {
  if (D < 0) return fail(CWQ_ERR_INVALID, "cwq_code_grouped_importance: negative size");
  const int64_t item_off[2] = {0, D};
  int64_t n_starts = 0;
  return grouped_importance_impl(1, item_off, q_loc, q_scale, p_loc, p_scale, &seed,
                                 dim_kl_bit_limit, size_threshold, n_nats, sample_host,
                                 index_host, starts_host, starts_cap, &n_starts, outlier_idx_host,
                                 outlier_val_host, n_outliers, kl_sum_out, workspace,
                                 workspace_bytes, opts, stream, "cwq_code_grouped_importance");
}

size_t cwq_code_grouped_importance_batch_workspace_size(int64_t D_total, int64_t n_items) {
  if (D_total < 0 || n_items < 1) return 0;
  return grouped_imp_ws(D_total, n_items).total;
}

int64_t cwq_code_grouped_importance_batch(
    int64_t n_items, const int64_t* item_off, const float* q_loc, const float* q_scale,
    const float* p_loc, const float* p_scale, const int32_t* seeds, float dim_kl_bit_limit,
    int64_t size_threshold, double n_nats, float* sample_host, int64_t* index_host,
    int64_t* starts_host, int64_t starts_cap, int64_t* n_starts, int64_t* outlier_idx_host,
    float* outlier_val_host, int64_t* n_outliers, double* kl_sum_out, void* workspace,
    size_t workspace_bytes, const cwq_options* opts, void* stream) {
  return grouped_importance_impl(n_items, item_off, q_loc, q_scale, p_loc, p_scale, seeds,
                                 dim_kl_bit_limit, size_threshold, n_nats, sample_host,
                                 index_host, starts_host, starts_cap, n_starts, outlier_idx_host,
                                 outlier_val_host, n_outliers, kl_sum_out, workspace,
                                 workspace_bytes, opts, stream,
                                 "cwq_code_grouped_importance_batch");
}

int64_t cwq_group_starts(const float* kl, int64_t D, int64_t size_threshold, double n_nats,
                         int64_t* starts, int64_t cap) {
  return group_starts_impl(kl, D, size_threshold, n_nats, starts, cap, false);
}

int64_t cwq_importance_group_starts(const float* kl, int64_t D, int64_t size_threshold,
                                    double n_nats, int64_t* starts, int64_t cap) {
  return group_starts_impl(kl, D, size_threshold, n_nats, starts, cap, true);
}

int cwq_importance_plan(const float* kl, const int64_t* starts, int64_t ng, int64_t* n_samples) {
  if (ng < 0 || (ng > 0 && (!kl || !starts || !n_samples)))
    return fail(CWQ_ERR_INVALID, "cwq_importance_plan: bad arguments");
  for (int64_t g = 0; g < ng; ++g) {
    const int64_t a = starts[g], b = starts[g + 1];
    if (b < a) return fail(CWQ_ERR_INVALID, "cwq_importance_plan: starts not sorted");
    const float total = eigen_sum(kl + a, b - a);            // tf.reduce_sum(kls)
    const float e = ceilf(expf(total));                       // tf.math.ceil(tf.exp(.))
    n_samples[g] = (int64_t)(int32_t)(e == e && e < 2147483648.0f ? e : -2147483648.0f);
  }
  return ok();
}

size_t cwq_importance_workspace_size(int64_t nb, int64_t total_dims) {
  if (nb < 0 || total_dims < 0) return 0;
  return cwq::importance_workspace_size(nb, total_dims);
}

int cwq_importance_encode(const float* t_loc, const float* t_scale, const float* p_loc,
                          const float* p_scale, const int64_t* block_off,
                          const int64_t* n_samples, int64_t nb, int64_t total_dims, int32_t seed,
                          int64_t block_id_base, int64_t* out_index, float* out_sample,
                          void* workspace, size_t workspace_bytes, const cwq_options* opts,
                          void* stream) {
  if (nb < 0 || total_dims < 0) return fail(CWQ_ERR_INVALID, "negative size");
  cwq_options o;
  int rc = read_options(opts, &o);
  if (rc) return rc;
  if (nb > 0 && (!block_off || !n_samples || !out_index))
    return fail(CWQ_ERR_INVALID, "null pointer");
  if (total_dims > 0 && (!t_loc || !t_scale || !p_loc || !p_scale || !out_sample))
    return fail(CWQ_ERR_INVALID, "null pointer");
  const size_t need = cwq::importance_workspace_size(nb, total_dims);
  if (workspace_bytes < need || (need && !workspace))
    return fail(CWQ_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
  hipError_t e = hipSuccess;
  if (o.eval_start_event)  // the caller's timer around the candidate-scoring launches
    e = hipEventRecord((hipEvent_t)o.eval_start_event, (hipStream_t)stream);
  if (e == hipSuccess)
    e = cwq::launch_importance_encode(t_loc, t_scale, p_loc, p_scale, block_off, n_samples, nb,
                                      total_dims, seed, block_id_base, nullptr,
                                      o.prune_mode >= 2 ? 1 : 0,
                                      out_index, out_sample, workspace, (hipStream_t)stream);
  if (e == hipSuccess && o.eval_stop_event)
    e = hipEventRecord((hipEvent_t)o.eval_stop_event, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_importance_encode");
  return ok();
}

int cwq_importance_decode(const int64_t* index, const float* p_loc, const float* p_scale,
                          const int64_t* block_off, int64_t nb, int64_t total_dims, int32_t seed,
                          int64_t block_id_base, float* out_sample, void* stream) {
  if (nb < 0 || total_dims < 0) return fail(CWQ_ERR_INVALID, "negative size");
  if (nb > 0 && (!block_off || !index)) return fail(CWQ_ERR_INVALID, "null pointer");
  if (total_dims > 0 && (!p_loc || !p_scale || !out_sample))
    return fail(CWQ_ERR_INVALID, "null pointer");
  hipError_t e = cwq::launch_importance_decode(index, p_loc, p_scale, block_off, nb, seed,
                                               block_id_base, out_sample, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_importance_decode");
  return ok();
}

int cwq_selftest_bm_tables(uint32_t m0, int64_t count, float* radius, float* sin_out,
                           float* cos_out, void* stream) {
  if (count < 0 || (count > 0 && (!radius || !sin_out || !cos_out)))
    return fail(CWQ_ERR_INVALID, "cwq_selftest_bm_tables: bad arguments");
  hipError_t e = cwq::launch_selftest_bm(m0, count, radius, sin_out, cos_out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_selftest_bm_tables");
  return ok();
}

int cwq_selftest_screen_tables(uint32_t m0, int64_t count, float* radius, float* sin_out,
                               float* cos_out, void* stream) {
  if (count < 0 || (count > 0 && (!radius || !sin_out || !cos_out)))
    return fail(CWQ_ERR_INVALID, "cwq_selftest_screen_tables: bad arguments");
  hipError_t e =
      cwq::launch_selftest_screen(m0, count, radius, sin_out, cos_out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_selftest_screen_tables");
  return ok();
}

size_t cwq_debug_partition_workspace_size(int64_t D) {
  return D < 0 ? 0 : cwq::partition_workspace_size(D) + 16 * sizeof(unsigned long long);
}

int64_t cwq_debug_group_starts_device(const float* kl, int64_t D, int64_t size_threshold,
                                      double n_nats, int64_t* starts, void* workspace,
                                      size_t workspace_bytes, unsigned long long* info_host,
                                      void* stream) {
  if (!kl || !starts || !workspace || !info_host || D < 0)
    return fail(CWQ_ERR_INVALID, "cwq_debug_group_starts_device: bad arguments");
  if (!cwq::partition_applies(D, size_threshold)) return 0;
  if (workspace_bytes < cwq_debug_partition_workspace_size(D))
    return fail(CWQ_ERR_WORKSPACE, "cwq_debug_group_starts_device: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  unsigned long long* info_d =
      (unsigned long long*)((char*)workspace + cwq::partition_workspace_size(D));
  hipError_t e = cwq::launch_partition(kl, D, nullptr, 1, size_threshold, group_thr(n_nats, false),
                                       starts, (int64_t*)(info_d + 8), workspace, info_d, s);
  unsigned long long h[16];
  if (e == hipSuccess)
    e = hipMemcpyAsync(h, info_d, sizeof(h), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "cwq_debug_group_starts_device");
  ok();
  for (int i = 0; i < 8; ++i) info_host[i] = h[i];
  info_host[0] = h[8] - 1;  // G
  info_host[1] = h[9];      // largest group
  return cwq::partition_fell_back(h) ? 0 : (int64_t)h[8];
}

int cwq_debug_tile_times(unsigned long long* t0, unsigned long long* t1, unsigned int* wg,
                         int n) {
  if (!t0 || !t1 || !wg || n < 0) return fail(CWQ_ERR_INVALID, "cwq_debug_tile_times: bad args");
  const int r = cwq::tile_times(t0, t1, wg, n);
  if (r < 0) return fail(CWQ_ERR_HIP, "cwq_debug_tile_times: symbol copy failed");
  return r;
}

int cwq_debug_quad_times(unsigned long long* t, unsigned int* info, int n) {
  if (!t || !info || n < 0) return fail(CWQ_ERR_INVALID, "cwq_debug_quad_times: bad args");
  const int r = cwq::quad_times(t, info, n);
  if (r < 0) return fail(CWQ_ERR_HIP, "cwq_debug_quad_times: symbol copy failed");
  return r;
}

int cwq_debug_prune_stats(unsigned long long* out72, int flags) {
  if (!out72) return fail(CWQ_ERR_INVALID, "cwq_debug_prune_stats: null output");
  const int r = cwq::prune_stats(out72, flags);
  if (r < 0) return fail(CWQ_ERR_HIP, "cwq_debug_prune_stats: symbol copy failed");
  cwq::set_error(CWQ_OK, "");
  return r;
}

int cwq_selftest_wave_max(const float* x, int64_t n_waves, float* out, void* stream) {
  if (n_waves < 0 || n_waves > (1LL << 31) || (n_waves > 0 && (!x || !out)))
    return fail(CWQ_ERR_INVALID, "cwq_selftest_wave_max: bad arguments");
  hipError_t e = cwq::launch_selftest_wave_max(x, n_waves, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_selftest_wave_max");
  return ok();
}

int cwq_selftest_div(const float* a, const float* b, int64_t n, float* out, void* stream) {
  if (n < 0 || (n > 0 && (!a || !b || !out)))
    return fail(CWQ_ERR_INVALID, "cwq_selftest_div: bad arguments");
  hipError_t e = cwq::launch_selftest_div(a, b, n, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_selftest_div");
  return ok();
}

int cwq_selftest_logf(const float* x, int64_t n, float* out, void* stream) {
  if (n < 0 || (n > 0 && (!x || !out)))
    return fail(CWQ_ERR_INVALID, "cwq_selftest_logf: bad arguments");
  hipError_t e = cwq::launch_selftest_logf(x, n, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "cwq_selftest_logf");
  return ok();
}

}  // extern "C"
