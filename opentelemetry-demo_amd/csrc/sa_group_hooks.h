// sa_group_hooks.h -- internal (not in the C-ABI): asynchronous forms of the
// engine's merge hooks for the engine group's flush (spanagg_group.cpp), so a
// flush of n members waits once per phase instead of once per member per
// call.  Host outputs must be page-locked (the copies are asynchronous);
// every call orders `s` after the engine's earlier work.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "spanagg.h"

namespace sa_grp {
// sa_export_keys without the wait: the resident keys with a non-zero delta
// into d_keys (capacity cap); *h_n (pinned) = their count and *h_dropped
// (pinned) = the engine's dropped-span counter, once `s` passes this point
int export_keys_async(sa_engine *e, uint64_t *d_keys, uint64_t cap, uint64_t *h_n, uint64_t *h_dropped,
                      hipStream_t s);
// the flush-time reclamation decision's key count: *h_n (pinned) = resident
// keys, once the engine stream passes this point
int count_keys_async(sa_engine *e, uint64_t *h_n);
// empties the key table on the engine stream (after its window error counts
// are folded into the count-min cells), without waiting: the reclamation
// sa_reclaim_keys does once count_keys_async's count is over the threshold
int reclaim_async(sa_engine *e);
// the reclamation threshold of this engine's table (sa_reclaim_keys' policy)
bool over_reclaim_threshold(const sa_engine *e, uint64_t n_keys);
// waits for the engine stream
int sync_stream(sa_engine *e);
// key-table slots (sa_stats.table_capacity without a device read)
uint64_t table_capacity(const sa_engine *e);
}  // namespace sa_grp
