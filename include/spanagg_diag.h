/*
 * spanagg_diag.h -- test and profiling entry points of libspanagg.
 *
 * These are not connector operations and replace nothing in the reference:
 * the parity tests use them to check single kernel stages (the exponential
 * bucket index, the group's device key union) against numpy / the oracle, and
 * the profiling tools read per-workgroup timestamps.  The drop-in boundary is
 * include/spanagg.h, which does not include this header; a collector binding
 *  never needs it.
 */
#ifndef SPANAGG_DIAG_H
#define SPANAGG_DIAG_H
#include "spanagg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostic: out[i] = the exponential bucket index of v[i] at scale[i] and
 * logs[i] = Go's math.Log(v[i]), both computed on the engine's GPU
 * (host arrays; n <= 2^20). */
int sa_expo_probe(sa_engine *e, const double *v, const int32_t *scale, uint64_t n, int32_t *out, double *logs);
/* Diagnostic: the bucket-index fast path the counting kernel uses.  For each
 * duration d_ns[i] > 0 at scale[i]: exact[i] = the Go-exact index of
 * d_ns / (1e6 or 1e9 by the engine's unit), fast[i] = the fast path's index
 * or INT32_MIN when it defers to the exact path (host arrays; n <= 2^20).
 * *log2_err (may be null) = max |v_log_f32(m) - log2(m)| over every float m
 * in [1, 2), the bound the fast path's margins assume. */
int sa_expo_fast_probe(sa_engine *e, const uint64_t *d_ns, const int32_t *scale, uint64_t n, int32_t *fast,
                       int32_t *exact, double *log2_err);

/* Diagnostic: the device key union the group flush builds (sa::key_union:
 * bucket sort by the top bits, bitonic per bucket, repeats and 0 dropped) on
 * the engine's GPU.  out[0 .. *n_out) = the distinct non-zero ids of
 * in[0 .. n) ascending (host arrays; out holds n; n <= 2^28). */
int sa_key_union_probe(sa_engine *e, const uint64_t *in, uint64_t n, uint64_t *out, uint64_t *n_out);

/* Diagnostic only: per-workgroup s_memrealtime stamps (100 MHz) of the last
 * small-table ingest launch, [G][136] = {start, after LDS setup, after the span
 * loop, after the slab flush, 0 x 4, then per wave 8 segment cycle sums};
 * filled only when the engine was created with SA_OPT_STAMPS (*n_out = 0
 * otherwise). */
int sa_debug_stamps(sa_engine *e, uint64_t *out, uint64_t cap, uint64_t *n_out);

#ifdef __cplusplus
}
#endif
#endif
