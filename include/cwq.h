/*
 * cwq.h -- C ABI of the MI355X (gfx950) greedy coded sampler (libcwq.so).
 *
 * Drop-in boundary for the reference's relative-entropy coding hot path.  The
 * reference has no native ABI (its sampler is a TF1 graph); each entry point
 * below replaces the graph op named next to it:
 *
 *   cwq_stateless_normal_sample  <- code/misc.py:3-17 stateless_normal_sample
 *                                   (tf.random.stateless_normal, seed=[seed,42],
 *                                   then scale*z and loc+ at misc.py:14-15)
 *   cwq_greedy_encode[_uniform]  <- code/coded_greedy_sampler.py:29-89
 *                                   code_greedy_sample, batched over the groups
 *                                   that code_grouped_greedy_sample (:170-296)
 *                                   feeds one sess.run at a time (:273-284);
 *                                   group g uses seed + block_id_base + g (:282)
 *   cwq_greedy_decode[_uniform]  <- code/coded_greedy_sampler.py:93-167
 *                                   decode_greedy_sample, batched the same way
 *                                   as decode_grouped_greedy_sample (:345-356)
 *   cwq_standardise              <- code/coded_greedy_sampler.py:193-199
 *   cwq_kl_normal_normal         <- code/coded_greedy_sampler.py:201
 *                                   (tfd.kl_divergence(target, proposal))
 *   cwq_destandardise            <- code/coded_greedy_sampler.py:292 / :362
 *   cwq_group_starts             <- code/coded_greedy_sampler.py:207-252
 *                                   (host-side sequential partition)
 *   cwq_code_grouped_greedy      <- code/coded_greedy_sampler.py:170-296
 *                                   (the whole grouped coder in one call)
 *   cwq_code_grouped_greedy_batch <- the same, once per item of a batch
 *
 * Conventions
 *   - All float/index pointers are DEVICE pointers (hipMalloc / torch cuda
 *     tensors) unless documented as host.  `stream` is a hipStream_t (NULL =
 *     default stream).  Calls are stream-ordered and asynchronous; no device
 *     memory is allocated and nothing synchronises (graph-capturable), except
 *     the host functions and the fused grouped pipelines documented as such.
 *     A multi-step CSR encode forks its two block halves onto two library
 *     streams (created once per host thread and device) and joins them back
 *     with events on the caller's stream.
 *   - Blocks ("groups" in the reference) are described in CSR form:
 *     block g covers dims [block_off[g], block_off[g+1]) of the flat arrays;
 *     block_off is a device int64 array of nb+1 entries.  The *_uniform
 *     variants take a fixed block dimension instead.
 *   - target = posterior q (t_loc, t_scale); proposal = prior p (p_loc,
 *     p_scale), as in the reference's argument order.
 *   - Return value: 0 on success, a negative CWQ_ERR_* code otherwise; the
 *     message is available from cwq_last_error() (thread-local).  Nothing
 *     throws across this ABI.
 */
#ifndef CWQ_H_
#define CWQ_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CWQ_OK 0
#define CWQ_ERR_INVALID (-1)   /* bad argument (sizes, bits, null pointer) */
#define CWQ_ERR_HIP (-2)       /* HIP runtime error (launch, memset) */
#define CWQ_ERR_WORKSPACE (-3) /* workspace too small */
#define CWQ_ERR_CAPACITY (-4)  /* output buffer too small (retry with a larger one) */
#define CWQ_ERR_ALLOC (-5)     /* host allocation failed */

#define CWQ_MAX_BITS_PER_STEP 30

/* ABI version, (major << 16) | minor.  Bindings must refuse a library whose
 * cwq_version() differs from the header they were written against.
 *   0.2  per-call cwq_options before the stream in the encoders, a
 *        max_block_dim argument to cwq_greedy_encode_workspace_size, no
 *        process-wide tuning setters;
 *   0.3  cwq_code_grouped_greedy_begin / _end;
 *   0.4  per-item ready flags of the batched grouped coder
 *        (cwq_options.item_ready);
 *   0.5  CWQ_ERR_ALLOC (host allocation failures are returned, never thrown);
 *        starts_host of the grouped _begin calls is read asynchronously;
 *   0.6  cwq_code_grouped_importance_batch. */
#define CWQ_ABI_VERSION ((0 << 16) | 6)
int cwq_version(void);

/* Thread-local description of the last error ("" if none). */
const char* cwq_last_error(void);

/* misc.py:3-17.  out[n*d + j] = loc[j] + scale[j] * Z[n*d + j] for
 * n < num_samples, j < d, where Z = tf.random.stateless_normal(
 * [num_samples, d], seed=[seed, 42]) (flat Philox4x32-10 + Box-Muller). */
int cwq_stateless_normal_sample(const float* loc, const float* scale, int64_t d,
                                int64_t num_samples, int32_t seed, float* out, void* stream);

/* Per-call options of the encoders (no process or thread state: every call
 * says what it wants; opts == NULL means the defaults below).
 *   prune_mode: 2 (default) = candidate pruning with the screening pass
 *               (DESIGN.md "screening bound") where a tile's constants allow
 *               it, exact pruning elsewhere; 1 = pruning on exact values only;
 *               0 = every candidate scored exactly.  Results never depend on
 *               it.  For the importance encoders, 2 turns on their screening
 *               pass, 0 and 1 score every candidate exactly.
 *   eval_start_event / eval_stop_event: hipEvent_t handles (both or neither)
 *               recorded on the call's stream right before the first
 *               candidate-scoring launch and right after the last one, so a
 *               caller can time the dominant kernel alone (bench.py).
 *   eval_ms_out: HOST float, or NULL.  The fused grouped calls
 *               (cwq_code_grouped_greedy[_batch], cwq_code_grouped_importance),
 *               which synchronise, write the summed milliseconds of their
 *               candidate-scoring launches (a pipelined batch codes in chunks:
 *               device gaps between them are excluded, unlike the event
 *               span).  Asynchronous entry points ignore it.
 *   item_ready: HOST int32 array of n_items flags, zeroed by the caller, or
 *               NULL.  cwq_code_grouped_greedy_batch sets flag i to 1 (a
 *               release store) as soon as item i's sample, bitcode, bits_off
 *               and starts are final in the host arrays, while later chunks
 *               still code; a caller running the call on another thread can
 *               consume the items as they complete (coded_greedy_sampler.py
 *               builds the bitcode strings this way).  The call itself still
 *               returns only when everything is done; on an error some flags
 *               stay 0.  Other entry points ignore it. */
typedef struct cwq_options {
  int32_t prune_mode;
  int32_t reserved; /* must be 0 */
  void* eval_start_event;
  void* eval_stop_event;
  float* eval_ms_out;
  int32_t* item_ready;
} cwq_options;
#define CWQ_OPTIONS_INIT {2, 0, NULL, NULL, NULL, NULL}

/* Workspace bytes needed by cwq_greedy_encode (CSR blocks) for nb blocks
 * holding total_dims dims in all, none longer than max_block_dim: the argmax
 * keys and per-dim shard constants plus the general pruned kernel's per-step
 * screening constants (24 B/dim + 244 B/block) and, when max_block_dim > 1024,
 * their visit-order copies for the long blocks (32 B/dim + 384 B per 1025
 * dims).  A
 * CSR call given less returns CWQ_ERR_WORKSPACE (it never silently falls back
 * to a slower kernel). */
size_t cwq_greedy_encode_workspace_size(int64_t nb, int64_t total_dims, int64_t max_block_dim);

/* Workspace bytes needed by cwq_greedy_encode_uniform for nb blocks of
 * dimension d: keys + shard constants only when d % 8 == 0, 8 <= d <= 64 (the
 * fast pruned kernel), the cwq_greedy_encode_workspace_size layout otherwise. */
size_t cwq_greedy_encode_uniform_workspace_size(int64_t nb, int64_t d);

/* Greedy coded sampling, encoder (coded_greedy_sampler.py:29-89) for nb
 * independent blocks.
 *   out_idx    [nb * n_steps] int32: the argmax index of every step (the
 *              reference emits these as LSB-first bit strings, :81-87)
 *   out_sample [total_dims] f32: best_sample of every block (:89)
 *   max_block_dim: an upper bound on the largest block's dimension (the same
 *              value the workspace was sized with).
 * Block g is coded with seed (seed + block_id_base + g) (int32 wrap), step i of
 * it with the stateless seed [1000*(that) + i, 42] (:55). */
int cwq_greedy_encode(const float* t_loc, const float* t_scale, const float* p_loc,
                      const float* p_scale, const int64_t* block_off, int64_t nb,
                      int64_t total_dims, int64_t max_block_dim, int n_bits_per_step,
                      int n_steps, int32_t seed, float rho, int64_t block_id_base,
                      int32_t* out_idx, float* out_sample, void* workspace,
                      size_t workspace_bytes, const cwq_options* opts, void* stream);

/* Same with every block of dimension d (block g = dims [g*d, (g+1)*d)). */
int cwq_greedy_encode_uniform(const float* t_loc, const float* t_scale, const float* p_loc,
                              const float* p_scale, int64_t nb, int64_t d,
                              int n_bits_per_step, int n_steps, int32_t seed, float rho,
                              int64_t block_id_base, int32_t* out_idx, float* out_sample,
                              void* workspace, size_t workspace_bytes, const cwq_options* opts,
                              void* stream);

/* Decoder (coded_greedy_sampler.py:93-167): sample = sum over steps of the
 * proposal-shard candidate idx[g*n_steps + i] of step i.  O(n_steps * d) per
 * block (only the selected row of the candidate stream is regenerated). */
int cwq_greedy_decode(const int32_t* idx, const float* p_loc, const float* p_scale,
                      const int64_t* block_off, int64_t nb, int64_t total_dims,
                      int64_t max_block_dim, int n_bits_per_step, int n_steps, int32_t seed,
                      float rho, int64_t block_id_base, float* out_sample, void* stream);

int cwq_greedy_decode_uniform(const int32_t* idx, const float* p_loc, const float* p_scale,
                              int64_t nb, int64_t d, int n_bits_per_step, int n_steps,
                              int32_t seed, float rho, int64_t block_id_base, float* out_sample,
                              void* stream);

/* coded_greedy_sampler.py:198-199: t_loc = (q_loc - p_loc) / p_scale,
 * t_scale = q_scale / p_scale (float32). */
int cwq_standardise(const float* q_loc, const float* q_scale, const float* p_loc,
                    const float* p_scale, int64_t n, float* t_loc, float* t_scale, void* stream);

/* coded_greedy_sampler.py:201: per-dim KL(q || p) of two diagonal Gaussians
 * (TFP <= 0.7 formula, float32). */
int cwq_kl_normal_normal(const float* q_loc, const float* q_scale, const float* p_loc,
                         const float* p_scale, int64_t n, float* out, void* stream);

/* coded_greedy_sampler.py:292: out = p_scale * sample + p_loc (float32, two
 * roundings).  out may alias sample. */
int cwq_destandardise(const float* sample, const float* p_loc, const float* p_scale, int64_t n,
                      float* out, void* stream);

/* HOST function (coded_greedy_sampler.py:207-252).  kl: HOST float32 [D].
 * size_threshold: the smallest group size s for which the reference's
 * `np.log(s + 1) / np.log(2) >= max_group_size_bits` holds.  n_nats:
 * n_bits_per_group * np.log(2) - 1 (float64).  Writes the reference's
 * group_start_indices (including the leading 0, the forced boundary at D-1 and
 * the trailing D) to starts[0..n) and returns n, or a negative error code if
 * cap is too small. */
int64_t cwq_group_starts(const float* kl, int64_t D, int64_t size_threshold, double n_nats,
                         int64_t* starts, int64_t cap);

/* code_grouped_greedy_sample (coded_greedy_sampler.py:170-296) in one call:
 * device standardisation and KL (:193-210), the host partition (:207-252, as
 * cwq_group_starts with size_threshold / n_nats), one greedy coder per group
 * with seed + g (:273-284), destandardisation (:292) and the LSB-first
 * bitcode (:81-87, :288).  q_* / p_*: DEVICE float32 [D] (target, proposal).
 * Outputs are HOST memory: sample_host [D] float32, bits_host ('0'/'1' chars,
 * groups x n_steps x n_bits_per_step of them), starts_host (the reference's
 * group_start_indices incl. the trailing D; starts_cap >= D + 2) and, if
 * non-NULL, kl_sum_out (sum of the per-dim KL in nats, for the reference's
 * log line).  Returns the number of groups, or a negative error code.
 * Synchronises the stream twice (after the KL, at the end). */
size_t cwq_code_grouped_greedy_workspace_size(int64_t D, int n_steps);
int64_t cwq_code_grouped_greedy(const float* q_loc, const float* q_scale, const float* p_loc,
                                const float* p_scale, int64_t D, int n_steps,
                                int n_bits_per_step, int32_t seed, float rho,
                                int64_t size_threshold, double n_nats, float* sample_host,
                                char* bits_host, int64_t bits_cap, int64_t* starts_host,
                                int64_t starts_cap, double* kl_sum_out, void* workspace,
                                size_t workspace_bytes, const cwq_options* opts, void* stream);

/* cwq_code_grouped_greedy in two halves, so the caller can work while the
 * device codes (the Python wrapper builds the reference's group_start_indices
 * list meanwhile).  _begin: the same inputs; waits for the partition (on the
 * device where it applies: its 128-byte result; else the KL copy and the host
 * loop), writes starts_host[0..G] and returns G (or a negative error code), with the
 * encode, the destandardisation and the copies of the G * n_steps indices to
 * idx_host (idx_cap >= G * n_steps; D + 1 groups at most) and of the sample to
 * sample_host still in flight on the stream: both must stay valid until _end,
 * and page-locked host memory keeps the copies asynchronous.  starts_host is
 * also the source of an asynchronous copy of the group offsets to the device:
 * it must stay valid and unchanged until _end too.
 * opts->eval_ms_out must be NULL (the caller's eval events work).  _end:
 * synchronises the stream and writes the bitcode of those indices; returns
 * the number of chars (G * n_steps * n_bits_per_step) or a negative code. */
int64_t cwq_code_grouped_greedy_begin(const float* q_loc, const float* q_scale,
                                      const float* p_loc, const float* p_scale, int64_t D,
                                      int n_steps, int n_bits_per_step, int32_t seed, float rho,
                                      int64_t size_threshold, double n_nats, float* sample_host,
                                      int32_t* idx_host, int64_t idx_cap, int64_t* starts_host,
                                      int64_t starts_cap, double* kl_sum_out, void* workspace,
                                      size_t workspace_bytes, const cwq_options* opts,
                                      void* stream);
int64_t cwq_code_grouped_greedy_end(const int32_t* idx_host, int64_t G, int n_steps,
                                    int n_bits_per_step, char* bits_host, int64_t bits_cap,
                                    void* stream);

/* A batch of independent code_grouped_greedy_sample calls (coded_greedy_sampler.py:170-296
 * once per item: the images of a dataset, or the ladder levels of several
 * images) in one call.  Item i is dims [item_off[i], item_off[i+1]) of the
 * concatenated DEVICE q_* / p_* (item_off: HOST int64 [n_items + 1], item_off[0]
 * == 0) and is coded exactly as cwq_code_grouped_greedy on that slice with seed
 * seeds[i] (HOST int32 [n_items]): its own partition (:207-252), its groups
 * numbered from 0 and coded with seeds[i] + g (:273-284).  One standardisation
 * and KL launch serve all items, and one device partition (cwq_partition.hip)
 * finds every item's groups (when the device scheme does not cover an input,
 * the host loop partitions chunk by chunk instead, with identical results).
 * The items are then pipelined in chunks of consecutive items
 * (CWQ_BATCH_CHUNKS, default 6; the first a quarter share, the last a half): one
 * encode launch sequence per chunk with per-block seeds, chunk c's results
 * copied to the host while chunk c + 1 codes, and each item's bitcode written
 * as soon as its chunk's indices arrive, on a pool of host threads (up to
 * CWQ_HOST_THREADS - 1, default min(8, CPUs) - 1) that the library creates on
 * the first batch call and keeps for the life of the process.
 * HOST outputs: sample_host [D_total]; item i's bitcode at
 * bits_host[bits_off[i], bits_off[i+1]) (bits_off: HOST int64 [n_items + 1],
 * written); item i's group_start_indices (local, incl. its trailing D_i):
 * n_starts[i] entries (HOST int64 [n_items], written) at starts_host +
 * item_off[i] + 2 i (starts_cap >= D_total + 2 n_items).  host_workspace:
 * HOST staging of host_workspace_bytes >=
 * cwq_code_grouped_greedy_batch_host_workspace_size (per-dim KL, group
 * offsets, seeds, indices), page-locked for asynchronous copies (hipHostMalloc,
 * or torch's pinned memory); NULL = library-owned pageable staging (slower
 * copies).  sample_host is best page-locked as well.  Returns the total number
 * of groups, or a negative error code.  Returns only after all of its device
 * work has finished (also on error). */
size_t cwq_code_grouped_greedy_batch_workspace_size(int64_t D_total, int64_t n_items,
                                                    int n_steps);
size_t cwq_code_grouped_greedy_batch_host_workspace_size(int64_t D_total, int64_t n_items,
                                                         int n_steps);
int64_t cwq_code_grouped_greedy_batch(
    int64_t n_items, const int64_t* item_off, const float* q_loc, const float* q_scale,
    const float* p_loc, const float* p_scale, int n_steps, int n_bits_per_step,
    const int32_t* seeds, float rho, int64_t size_threshold, double n_nats, float* sample_host,
    char* bits_host, int64_t bits_cap, int64_t* bits_off, int64_t* starts_host,
    int64_t starts_cap, int64_t* n_starts, void* workspace, size_t workspace_bytes,
    void* host_workspace, size_t host_workspace_bytes, const cwq_options* opts, void* stream);

/* ---- Importance sampler (code/coded_importance_sampler.py) ------------- */
/* Workspace bytes for cwq_importance_encode. */
size_t cwq_importance_workspace_size(int64_t nb, int64_t total_dims);

/* code_importance_sample (:29-79) for nb CSR groups at once.  Group g draws
 * n_samples[g] (device int64) candidates x = p_loc + p_scale*z from the
 * stateless stream with seed (seed + block_id_base + g) -- the group seed
 * itself (:55, :243) -- scores sum_j log q(x_j) - log p(x_j) (:60) and writes
 * the 0-based argmax out_index[g] (device int64; the reference codes
 * index + 1 with Elias-delta) and that candidate into out_sample. */
int cwq_importance_encode(const float* t_loc, const float* t_scale, const float* p_loc,
                          const float* p_scale, const int64_t* block_off,
                          const int64_t* n_samples, int64_t nb, int64_t total_dims, int32_t seed,
                          int64_t block_id_base, int64_t* out_index, float* out_sample,
                          void* workspace, size_t workspace_bytes, const cwq_options* opts,
                          void* stream);

/* decode_importance_sample (:82-109): the last of index+1 samples, i.e. row
 * `index` of group g's stream. */
int cwq_importance_decode(const int64_t* index, const float* p_loc, const float* p_scale,
                          const int64_t* block_off, int64_t nb, int64_t total_dims, int32_t seed,
                          int64_t block_id_base, float* out_sample, void* stream);

/* HOST (:178-203): the importance coder's partition; as cwq_group_starts but
 * with the reference's strict comparisons (`group_bits > max bits`,
 * `kl_sum > n_nats`).  size_threshold: the smallest s with
 * np.log(s + 1) / np.log(2) > max_group_size_bits. */
int64_t cwq_importance_group_starts(const float* kl, int64_t D, int64_t size_threshold,
                                    double n_nats, int64_t* starts, int64_t cap);

/* HOST (:48-51): n_samples[g] = int32(ceil(expf(sum of group g's float32 KLs in
 * Eigen inner-dim order))), for groups [starts[g], starts[g+1]) of HOST kl. */
int cwq_importance_plan(const float* kl, const int64_t* starts, int64_t ng, int64_t* n_samples);

/* coded_importance_sampler.py:112-274 code_grouped_importance_sample in one
 * call (the counterpart of cwq_code_grouped_greedy): device standardisation,
 * KL and outlier masking (kl / ln 2 > dim_kl_bit_limit, float32), the seeded
 * outlier target draw q_loc + q_scale z, z from [seed - 1, 42],
 * the host partition (size_threshold and n_nats as cwq_importance_group_starts)
 * and sample-count plan, one encode launch, device destandardisation.
 * Device inputs; HOST outputs: sample_host [D] (outlier dims hold the target
 * draw, :267), index_host [G] (argmax index, the reference codes index + 1),
 * starts_host (group starts incl. the trailing D; starts_cap >= D + 2), the
 * outlier dims and their unquantised draws (outlier_*_host, capacity D,
 * *n_outliers of them), and optionally (kl_sum_out) the total standardised KL
 * in nats for the reference's log line.  Returns G or a negative error code.
 * Blocks the host until the results are on it. */
size_t cwq_code_grouped_importance_workspace_size(int64_t D);
int64_t cwq_code_grouped_importance(const float* q_loc, const float* q_scale,
                                    const float* p_loc, const float* p_scale, int64_t D,
                                    int32_t seed, float dim_kl_bit_limit, int64_t size_threshold,
                                    double n_nats, float* sample_host, int64_t* index_host,
                                    int64_t* starts_host, int64_t starts_cap,
                                    int64_t* outlier_idx_host, float* outlier_val_host,
                                    int64_t* n_outliers, double* kl_sum_out, void* workspace,
                                    size_t workspace_bytes, const cwq_options* opts,
                                    void* stream);

/* A batch of independent code_grouped_importance_sample calls
 * (coded_importance_sampler.py:112-274 once per item: the level-2 latents of
 * a dataset's images, pln.py:350-359) in one call.  Item i is dims
 * [item_off[i], item_off[i+1]) of the concatenated DEVICE q_* / p_* (item_off:
 * HOST int64 [n_items + 1], item_off[0] == 0) and is coded exactly as
 * cwq_code_grouped_importance on that slice with seed seeds[i] (HOST int32
 * [n_items]): its own outliers and outlier draw ([seeds[i] - 1, 42] over its
 * own dims), its own partition and plan, its groups numbered from 0 and coded
 * with seeds[i] + g.  One preparation launch and one encode launch serve every
 * item.  HOST outputs, item i's at the offsets shown:
 *   sample_host [D_total] (item i's dims in place);
 *   index_host + item_off[i] + i: its G_i argmax indices (capacity D_total +
 *     n_items);
 *   starts_host + item_off[i] + 2 i: its group starts incl. its trailing D_i,
 *     n_starts[i] (= G_i + 1) of them (starts_cap >= D_total + 2 n_items);
 *   outlier_idx_host / outlier_val_host + item_off[i]: its n_outliers[i]
 *     outlier dims (local indices) and their unquantised draws;
 *   kl_sum_out [n_items] (optional): each item's standardised KL in nats.
 * opts->eval_ms_out receives the encode launches' milliseconds.  Returns the
 * total number of groups, or a negative error code.  Blocks the host until
 * the results are on it. */
size_t cwq_code_grouped_importance_batch_workspace_size(int64_t D_total, int64_t n_items);
int64_t cwq_code_grouped_importance_batch(
    int64_t n_items, const int64_t* item_off, const float* q_loc, const float* q_scale,
    const float* p_loc, const float* p_scale, const int32_t* seeds, float dim_kl_bit_limit,
    int64_t size_threshold, double n_nats, float* sample_host, int64_t* index_host,
    int64_t* starts_host, int64_t starts_cap, int64_t* n_starts, int64_t* outlier_idx_host,
    float* outlier_val_host, int64_t* n_outliers, double* kl_sum_out, void* workspace,
    size_t workspace_bytes, const cwq_options* opts, void* stream);

/* ---- Arithmetic coder (code/coding.pyx:27-310), HOST functions ---------- */
/* ArithmeticCoder(P, precision).encode(message): writes the code as '0'/'1'
 * chars to out_bits (if non-null, at most cap) and returns the number of bits
 * (or a negative error).  counts: P[K] (non-negative, sum > 0); message
 * symbols in [0, K) with non-zero counts (CWQ_ERR_INVALID otherwise: the
 * reference loops forever on a zero-count symbol) and, as the reference's
 * callers do, ending with the EOF symbol 0.  precision in [3, 62] (the
 * reference uses 32). */
int64_t cwq_ac_encode(const int64_t* counts, int64_t K, int precision, const int64_t* message,
                      int64_t n, char* out_bits, int64_t cap);

/* .decode / .decode_fast (:129-310): decodes until the EOF symbol 0 and
 * returns the number of symbols written to out_msg (EOF included),
 * CWQ_ERR_CAPACITY if cap is too small, or CWQ_ERR_INVALID for a corrupt code
 * (where the reference would loop forever). */
int64_t cwq_ac_decode(const int64_t* counts, int64_t K, int precision, const char* bits,
                      int64_t nbits, int64_t* out_msg, int64_t cap);

/* Elias-delta codes of the importance sampler's index + 1 values
 * (code/binary_io.py:7-39), concatenated.  Host memory.  encode writes the
 * '0'/'1' chars of x[0..n) to out (NULL: only count) and returns their
 * number; values must lie in [1, 2^30) (CWQ_ERR_INVALID otherwise, where the
 * reference's float64 log formulas may differ from the bit lengths).  decode
 * parses `count` codes from bits[0..nbits) into out and returns the chars
 * consumed (coded_importance_sampler.py:325-336). */
int64_t cwq_elias_delta_encode(const int64_t* x, int64_t n, char* out, int64_t cap);
int64_t cwq_elias_delta_decode(const char* bits, int64_t nbits, int64_t count, int64_t* out);

/* The greedy coder's bit parse (code/coded_greedy_sampler.py:107-126 and
 * :330-342, binary_io.py:55-67 from_bit_string of each num_bits substring):
 * count indices of num_bits LSB-first chars each from bits[0..nbits) into
 * out.  Chars past nbits read as '0' (the short substring tf.strings.substr
 * yields at the end of the string); any char other than '1' reads as 0.  Host
 * memory.  Returns count, or CWQ_ERR_INVALID (num_bits outside
 * [0, CWQ_MAX_BITS_PER_STEP], negative sizes, null pointers). */
int64_t cwq_bitcode_to_indices(const char* bits, int64_t nbits, int num_bits, int64_t count,
                               int32_t* out);

/* Diagnostics (used by the parity tests): evaluate the device restatement of
 * the Box-Muller transcendentals for the 23-bit mantissas m0 .. m0+count-1:
 *   radius[i] = sqrtf(-2 logf(max(m*2^-23, 1e-7f)))    (BoxMullerFloat u2)
 *   sin[i], cos[i] = sincosf((float)(2*pi * m*2^-23))   (BoxMullerFloat v1)
 * and logf(x[i]) for arbitrary floats (the per-dimension normaliser's log). */
int cwq_selftest_bm_tables(uint32_t m0, int64_t count, float* radius, float* sin_out,
                           float* cos_out, void* stream);
int cwq_selftest_logf(const float* x, int64_t n, float* out, void* stream);
/* The screening passes' approximations of the same three tables (hardware
 * v_log/v_sqrt/v_sin/v_cos); radius[i] holds r~ / sqrt(2 ln 2), the form the
 * kernels carry.  The tests bound their deviation from the exact tables by the
 * constants the screening bounds are built on. */
int cwq_selftest_screen_tables(uint32_t m0, int64_t count, float* radius, float* sin_out,
                               float* cos_out, void* stream);
/* out[i] = the device's fast correctly-rounded quotient a[i] / b[i]
 * (Markstein sequence with y = RN(1/b); only valid in the ranges documented in
 * DESIGN.md -- the test feeds it exactly those). */
int cwq_selftest_div(const float* a, const float* b, int64_t n, float* out, void* stream);
/* out[w] = max(x[64 w .. 64 w + 63]): the wave-wide DPP max the pruned encoder
 * shares its threshold with. */
int cwq_selftest_wave_max(const float* x, int64_t n_waves, float* out, void* stream);



/* ---- PLN image codec plumbing (csrc/cwq_pln.hip) ----
 * The ladder network's transforms are library convolutions; these three
 * stream kernels connect them to the coders.  Latent tensors are NCHW with
 * batch 1 (C channels, HW = H*W positions); the reference flattens them in
 * TF's NHWC order, index f = hw*C + c. */

/* pln.py:165-185: level-1 posterior = precision-weighted combination of the
 * likelihood N(lik_loc, lik_scale) (AnalysisTransform_1) and the prior
 * N(prior_loc, prior_scale) (SynthesisTransform_2), float32 in the
 * reference's order: lp = 1/(lik_scale^2 + eps), pp = 1/(prior_scale^2 + eps),
 * var = 1/(lp + pp), scale = sqrt(var), loc = (lik_loc*pp + prior_loc*lp)*var.
 * Elementwise over n values; any layout. */
int cwq_pln_posterior(const float* lik_loc, const float* lik_scale, const float* prior_loc,
                      const float* prior_scale, int64_t n, float eps, float* loc, float* scale,
                      void* stream);

/* pln.py:264-273 + :316-324: out[i] = src_nhwc[perm[i]] for i < C*HW, i.e.
 * tfp.bijectors.Permute(perm).forward(tf.reshape(x_nhwc, [-1])), reading the
 * NCHW tensor src.  perm: device int32 [C*HW] permutation, or NULL for the
 * identity (use_permutation=False). */
int cwq_permute_gather(const float* src, int64_t C, int64_t HW, const int32_t* perm, float* out,
                       void* stream);

/* pln.py:394-397, :770-772, :801-803: the inverse, Permute.inverse and the
 * reshape back to the latent shape, written NCHW: out_nchw[c*HW + hw] = src[i]
 * where perm[i] = hw*C + c. */
int cwq_permute_scatter(const float* src, int64_t C, int64_t HW, const int32_t* perm, float* out,
                        void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CWQ_H_ */
