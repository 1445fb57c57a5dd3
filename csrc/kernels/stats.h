// Device helper shared by the loss kernels (misc.hip, lenet_fc.hip).
#pragma once

#include "kernels.h"

namespace mcc {
namespace gpu {

// One workgroup's partial statistic into the fixed-point accumulator (the
// workgroup sum is formed in a fixed order, so the total is deterministic).
// A non-finite or oversized partial (a diverged run) is not converted -- the
// conversion is undefined there -- and an add that wraps the 64-bit sum is
// detected from the returned old value; both set the sticky flag
// stats[kStatNaN], which the readers report as NaN loss / MSE.
__device__ __forceinline__ void stat_add(unsigned long long* stats, int i, float t) {
  if (i == 2) {
    atomicAdd(stats + 2, (unsigned long long)(t + 0.5f));
    return;
  }
  const double d = (double)t * kStatScale;
  if (!(d >= 0.0 && d < 9.2e18)) {  // NaN, inf, negative or past 2^63
    atomicOr(stats + kStatNaN, 1ull);
    return;
  }
  const unsigned long long v = (unsigned long long)__double2ll_rn(d);
  const unsigned long long old = atomicAdd(stats + i, v);
  if (old + v < old) atomicOr(stats + kStatNaN, 1ull);
}

}  // namespace gpu
}  // namespace mcc
