/*
 * cwq_debug.h -- tools-only entry points of libcwq.so (not part of the C ABI in
 * include/cwq.h; used by tools/prune_stats.py and tools/csr_stats.py).
 */
#ifndef CWQ_DEBUG_H_
#define CWQ_DEBUG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Tuning counters of the pruned encoder, filled only by builds compiled with
 * -DCWQ_PRUNE_STATS (tools/prune_stats.py); returns 1 there, 0 (and zeros)
 * otherwise.  out72[k] = candidates finished after k units (k <= 64),
 * [65] completed rows, [66] survivors pushed, [67] tiles on the screening pass,
 * [68] survivors re-evaluated exactly at tile end, [69] in-loop exact evaluations.
 * flags: bit 0 resets the counters; bit 1 / bit 2 switch the "oracle tau"
 * experiment on / off (later launches start each tile at the best value the
 * last launch found for it). */
int cwq_debug_prune_stats(unsigned long long* out72, int flags);

/* Per-tile wall clock of the last k_encode_prune launch (s_memrealtime ticks,
 * 100 MHz) and the workgroup that ran each tile, filled only by builds compiled
 * with -DCWQ_TILE_TIMES (tools/tile_times.py); returns the entries copied (0 in
 * other builds). */
int cwq_debug_tile_times(unsigned long long* t0, unsigned long long* t1, unsigned int* wg, int n);

/* Per-quad wall clock of the last k_small_fused launch: t[6*q + i] is quad q's
 * s_memrealtime at its start (i = 0) and after its constants, screen, exact
 * rows, exact blocks and finalize (i = 1..5); info[4*q + ...] = HW_ID, XCC_ID,
 * listed rows scored exactly, exact blocks | dims << 8.  Filled only by builds
 * compiled with -DCWQ_QUAD_TIMES (tools/quad_times.py); returns the quads
 * copied (0 in other builds). */
int cwq_debug_quad_times(unsigned long long* t, unsigned int* info, int n);

/* The grouped coder's device partition (cwq_partition.hip) on a device KL
 * array: starts (device, D + 2 int64) as cwq_group_starts computes them on the
 * host.  Returns the number of starts, or 0 when the device path does not cover
 * the input (info_host[2] / info_host[4]: the caller uses the host loop), or a
 * negative code.  info_host: 8 entries (G, largest group, fallback, dup, longest
 * jump). */
size_t cwq_debug_partition_workspace_size(int64_t D);
int64_t cwq_debug_group_starts_device(const float* kl, int64_t D, int64_t size_threshold,
                                      double n_nats, int64_t* starts, void* workspace,
                                      size_t workspace_bytes, unsigned long long* info_host,
                                      void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CWQ_DEBUG_H_ */
