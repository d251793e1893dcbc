// sa_results.h -- host-side result holders shared by the engine and the group
// (sa_red_result_free / sa_sketch_result_free delete these).
#pragma once
#include <cstdint>
#include <vector>

#include "spanagg.h"

struct red_holder {
  sa_red_result r;
  std::vector<uint64_t> keys, counts, calls, sum_ns;
  std::vector<double> sum;
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
