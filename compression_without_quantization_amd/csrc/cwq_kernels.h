// cwq_kernels.h -- launchers shared between the kernels and the C ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cwq {

#ifndef CWQ_CSR_GTAU_STRIDE
#define CWQ_CSR_GTAU_STRIDE 1  // words between blocks' shared thresholds (tuning builds)
#endif

// Records `msg` for cwq_last_error() (thread-local) and returns `code`.
int set_error(int code, const char* msg);

#ifndef CWQ_CSR_LDS_DIMS
#define CWQ_CSR_LDS_DIMS 1024  // general pruned kernel: blocks up to this d keep their
                               // screening constants in LDS (longer: abp records)
#endif

// First entry of a long block's visit-order records (abp, 32 B per entry) for a
// block at absolute dim offset off.  Only blocks of more than CWQ_CSR_LDS_DIMS
// dims have records, and two of them start at least CWQ_CSR_LDS_DIMS + 1 dims
// apart, so each gets a disjoint region of d + 12 entries here and the array
// needs csr_rec_entries(total_dims) entries however many short blocks there are.
__host__ __device__ inline int64_t csr_rec_base(int64_t off) {
  return off + 12 * (off / (CWQ_CSR_LDS_DIMS + 1));
}
__host__ __device__ inline int64_t csr_rec_entries(int64_t total_dims) {
  return total_dims + 12 * (total_dims / (CWQ_CSR_LDS_DIMS + 1) + 1);
}

constexpr int kTileQueueSlots = 64;

struct EncodeArgs {
  const float* t_loc;
  const float* t_scale;
  const float* p_loc;
  const float* p_scale;
  const int64_t* block_off;  // nullptr -> uniform blocks of dimension ud
  int64_t ud;
  int64_t nb;
  int64_t total_dims;
  int64_t max_d;             // longest block (uniform: ud); -1: unknown
  int64_t n_cand;            // 2^n_bits_per_step
  int64_t tiles_per_block;
  int64_t cand_per_tile;     // multiple of 256
  int n_steps;
  int prune;                 // 1: use the pruned kernel where it applies
  int32_t seed;
  float rho;
  int64_t block_id_base;
  const int32_t* seeds;      // device [nb] per-block seeds, or nullptr: seed + block_id_base + g
  int32_t* out_idx;
  float* out_sample;
  // workspace
  unsigned long long* keys;  // [nb]
  // tile queue counters of k_encode_prune (kTileQueueSlots u32, one per fork
  // part; nullptr: static tile loop); zeroed by the launcher before each launch
  uint32_t* tq = nullptr;
  float* loc_s;              // [total_dims]
  float* scale_s;            // [total_dims]
  float* lognorm;            // [total_dims]
  // screening constants of the general pruned kernel (k_encode_prune_csr);
  // nullptr when the workspace was sized without them
  float2* sab;               // [total_dims + 8 nb] (sA, sB), 4 zero pads either side per block
  float* cdim;               // [total_dims] C_j of the screening bound (k_csr_prep scratch)
  float* bpre;               // [total_dims + 12 nb] drop bounds per visit position (k_csr_prep)
  uint32_t* ordu;            // [total_dims + 12 nb] unit visited at each position
  float4* grp;               // [nb] (c1, c2, As, Pq); c1 == 0: block not screened
  uint32_t* gtau;            // [nb] per-block shared threshold (ord)
  float4* abp;               // [2 (total_dims + 12 nb)] visit-order (sa, sb) records of the
                             // blocks longer than CWQ_CSR_LDS_DIMS; nullptr if none are
  uint2* slist;              // screened small-candidate path: CWQ_SLIST_PER_BLOCK
                             // (row, upper bits) survivor slots per block; the
                             // per-block counts live in ordu[off + 12 g]
  // optional profiling events around the eval launches (hipEvent_t)
  void* ev_start;
  void* ev_stop;
  // the small-candidate pipeline (k_small_*; nullptr: not sized for it):
  // per-dim screening constants (sA, sB) by absolute dim offset (a view of
  // sab, set by launch_encode) and the dim -> block map [total_dims]
  const float2* pre_ab = nullptr;
  uint32_t* sdmap = nullptr;
  // grouped pipelines (coded_greedy_sampler.py:292): also ds_out[i] =
  // ds_scale[i] * sample[i] + ds_loc[i] after the last step, folded into the
  // small pipeline's finalize where it runs, else one k_destandardise
  float* ds_out = nullptr;
  const float* ds_loc = nullptr;
  const float* ds_scale = nullptr;
};

#define CWQ_SLIST_PER_BLOCK 8

// Library copy streams (which = 0: device to host, 1: host to device) on the
// device of the caller's stream, created once per host thread; nullptr if they
// cannot be made.  Used by the pipelined batch coder to overlap its copies with
// the coding on the caller's stream.
hipStream_t copy_stream(hipStream_t stream, int which);
hipError_t launch_encode(const EncodeArgs& a, hipStream_t stream);
hipError_t launch_decode(const int32_t* idx, const float* p_loc, const float* p_scale,
                         const int64_t* block_off, int64_t ud, int64_t nb, int64_t total_dims,
                         int n_bits,
                         int n_steps, int32_t seed, float rho, int64_t block_id_base,
                         float* out_sample, hipStream_t stream);
hipError_t launch_stateless_normal_sample(const float* loc, const float* scale, int64_t d,
                                          int64_t num_samples, int32_t seed, float* out,
                                          hipStream_t stream);
hipError_t launch_standardise(const float* q_loc, const float* q_scale, const float* p_loc,
                              const float* p_scale, int64_t n, float* t_loc, float* t_scale,
                              hipStream_t stream);
hipError_t launch_kl(const float* q_loc, const float* q_scale, const float* p_loc,
                     const float* p_scale, int64_t n, float* out, hipStream_t stream);
hipError_t launch_destandardise(const float* sample, const float* p_loc, const float* p_scale,
                                int64_t n, float* out, hipStream_t stream);
// the grouped importance coder's standardise + KL + outliers + standard prior
// + KL against N(0, 1) + the outlier dims' target draw (seed - 1 per item:
// item_off / seed1 device arrays of a batch, or item_off == nullptr and
// seed1_one for one item), one launch (cwq_code_grouped_importance[_batch])
hipError_t launch_imp_grouped_prep(const float* q_loc, const float* q_scale, const float* p_loc,
                                   const float* p_scale, int64_t n, float limit,
                                   const int64_t* item_off, const int32_t* seed1, int64_t n_items,
                                   int32_t seed1_one, float* t_loc, float* t_scale, uint8_t* keep,
                                   float* zeros, float* ones, float* kl2, float* tsamp,
                                   hipStream_t stream);
// standardise + KL + the standard prior's zeros/ones + nz zeroed u64 at zinfo
// (nz <= 256), one launch (the grouped coder's first step)
hipError_t launch_grouped_prep(const float* q_loc, const float* q_scale, const float* p_loc,
                               const float* p_scale, int64_t n, float* t_loc, float* t_scale,
                               float* kl, float* zeros, float* ones, unsigned long long* zinfo,
                               int nz, hipStream_t stream);

// The grouped coder's greedy partition on the device (cwq_partition.hip), of
// one item (item_off == nullptr, n_items == 1) or of each item [item_off[k],
// item_off[k+1]) of a batch (device offsets): item k's starts at starts +
// item_off[k] + 2 k, iinfo[2k] their count (G + 1), iinfo[2k + 1] its largest
// group (iinfo holds 4 n_items entries: the rest is scratch).  partition_fell_back(info copied to the host): not covered, the caller
// runs the host loop (the results never depend on which path ran).
size_t partition_workspace_size(int64_t D);
bool partition_applies(int64_t D, int64_t size_threshold);
// One item of a batch in the device layout of its chunk's encode: its G groups
// go to offs[go ...] (block offsets relative to the chunk's first dim: rel +
// its starts at dstarts[src ...]) and seeds[gs ...] (seed + g, :282); term >= 0:
// offs[term] = dc, the chunk's closing offset (written with the chunk's last item).
struct BatchItem {
  int64_t src, rel, go, gs, G, term, dc;
  int64_t pk, ns;  // the item's start list: packed offset and length (pstarts)
  int32_t seed, pad;
};
// pstarts (may be nullptr): every item's start list packed back to back, for
// one device-to-host copy
hipError_t launch_batch_layout(const BatchItem* items, int64_t n_items, const int64_t* dstarts,
                               int64_t* offs, int32_t* seeds, int64_t* pstarts,
                               hipStream_t stream);
// info_zeroed: info[0..7] (and, single item, iinfo[0..1]) were zeroed on the
// stream by the caller (launch_grouped_prep); otherwise a memset does it
hipError_t launch_partition(const float* kl, int64_t D, const int64_t* item_off, int64_t n_items,
                            int64_t size_threshold, float thr, int64_t* starts, int64_t* iinfo,
                            void* ws, unsigned long long* info, hipStream_t stream,
                            bool info_zeroed = false);
bool partition_fell_back(const unsigned long long* info_host);

size_t importance_workspace_size(int64_t nb, int64_t total_dims);
hipError_t launch_imp_outliers(const float* kl, int64_t n, float limit, float* t_loc,
                               float* t_scale, uint8_t* keep, hipStream_t stream);
hipError_t launch_importance_encode(const float* t_loc, const float* t_scale, const float* p_loc,
                                    const float* p_scale, const int64_t* block_off,
                                    const int64_t* n_samples, int64_t nb, int64_t total_dims,
                                    int32_t seed, int64_t block_id_base,
                                    const int32_t* block_seeds, int allow_screen,
                                    int64_t* out_index, float* out_sample, void* workspace,
                                    hipStream_t stream, int64_t total_cands = -1,
                                    int64_t total_tiles = -1, const float* dst_loc = nullptr,
                                    const float* dst_scale = nullptr, float* dst_out = nullptr);
// The encode launch's k_imp_eval tile count from host copies of the plan
// (total_cands: sum of max(N_g, 1)); it only selects the tile hand-out.
int64_t importance_tile_count(const int64_t* n_samples_host, int64_t nb, int64_t total_cands);
hipError_t launch_importance_decode(const int64_t* index, const float* p_loc,
                                    const float* p_scale, const int64_t* block_off, int64_t nb,
                                    int32_t seed, int64_t block_id_base, float* out_sample,
                                    hipStream_t stream);

hipError_t launch_selftest_bm(uint32_t m0, int64_t count, float* rad, float* sn, float* cs,
                              hipStream_t stream);
hipError_t launch_selftest_screen(uint32_t m0, int64_t count, float* rad, float* sn, float* cs,
                                  hipStream_t stream);
int prune_stats(unsigned long long* out72, int reset);
int tile_times(unsigned long long* t0, unsigned long long* t1, unsigned int* wg, int n);
int quad_times(unsigned long long* t, unsigned int* info, int n);
hipError_t launch_selftest_wave_max(const float* x, int64_t nw, float* out, hipStream_t stream);
hipError_t launch_selftest_div(const float* a, const float* b, int64_t n, float* out,
                               hipStream_t stream);
hipError_t launch_selftest_logf(const float* x, int64_t n, float* out, hipStream_t stream);

}  // namespace cwq
