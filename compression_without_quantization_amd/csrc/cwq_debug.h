/*
 * cwq_debug.h -- tools-only entry points of libcwq.so (not part of the C ABI in
 * include/cwq.h; used by tools/prune_stats.py and tools/csr_stats.py).
 */
#ifndef CWQ_DEBUG_H_
#define CWQ_DEBUG_H_

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

#ifdef __cplusplus
}
#endif
#endif /* CWQ_DEBUG_H_ */
