// sa_results.h -- host-side result holders shared by the engine and the group
// (sa_red_result_free / sa_sketch_result_free delete these).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

#include "spanagg.h"

// Page-locked result blocks reused across flushes.  A flush at C4 scale hands
// back ~170 MB of columns; pageable std::vector columns cost a zero fill (and
// its page faults) plus a staged D2H copy, so a group flush DMAs into one of
// these blocks instead.  A result holds its block until sa_red_result_free,
// which returns it here; the pool is shared with the results, so a result
// may outlive the group that made it.
struct PinPool {
  std::mutex mu;
  std::vector<std::pair<void *, size_t>> blocks;  // free blocks
  static constexpr size_t kKeep = 2;              // free blocks kept for the next flushes
  ~PinPool() {
    for (auto &b : blocks) (void)hipHostFree(b.first);
  }
  // a free block of at least `bytes` (the smallest that fits), else a new one
  void *take(size_t bytes, size_t *got) {
    {
      std::lock_guard<std::mutex> l(mu);
      size_t best = blocks.size();
      for (size_t i = 0; i < blocks.size(); ++i)
        if (blocks[i].second >= bytes && (best == blocks.size() || blocks[i].second < blocks[best].second)) best = i;
      if (best < blocks.size()) {
        auto b = blocks[best];
        blocks.erase(blocks.begin() + (long)best);
        *got = b.second;
        return b.first;
      }
    }
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    *got = bytes;
    return p;
  }
  void give(void *p, size_t bytes) {
    void *drop = p;
    {
      std::lock_guard<std::mutex> l(mu);
      if (blocks.size() < kKeep) {
        blocks.emplace_back(p, bytes);
        drop = nullptr;
      } else {  // keep the larger blocks: a flush needs one at least as large as the last
        size_t small = 0;
        for (size_t i = 1; i < blocks.size(); ++i)
          if (blocks[i].second < blocks[small].second) small = i;
        if (blocks[small].second < bytes) {
          drop = blocks[small].first;
          blocks[small] = std::make_pair(p, bytes);
        }
      }
    }
    if (drop) (void)hipHostFree(drop);
  }
};

struct red_holder {
  sa_red_result r;
  std::vector<uint64_t> keys, counts, calls, sum_ns;
  std::vector<double> sum;
  // columns in a page-locked block of `pool` (group flush) instead of the vectors
  std::shared_ptr<PinPool> pool;
  void *pin = nullptr;
  size_t pin_bytes = 0;
  ~red_holder() {
    if (pin) pool->give(pin, pin_bytes);
  }
};

struct exp_holder {
  sa_exp_result r;
  std::vector<uint64_t> keys, count, zero, sum_ns, buckets;
  std::vector<double> sum, min, max;
  std::vector<int32_t> scale, offset;
  std::vector<uint32_t> nb;
};

struct sketch_holder {
  sa_sketch_result r;
  std::vector<uint8_t> hll;
  std::vector<uint32_t> cms;
};
