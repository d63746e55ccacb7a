// mjh_rng.h — the env layer's device random stream (mjh_fuse.hip, mjh_mgr.hip).
//
// Counter-based: U[0, 1) element `idx` of the draw keyed (seed, call-site key,
// *step counter) is a splitmix64 finalizer chain over those values, so draws
// are stateless and a captured graph draws anew whenever the device step
// counter changes. 24 random bits per float.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mjh_abi.h"

namespace mjh {

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct Rng {
  unsigned long long base;
  __device__ Rng(unsigned long long seed, unsigned long long key, const mjh_i64* ctr) {
    const unsigned long long step = ctr ? (unsigned long long)*ctr : 0ull;
    base = mix64(seed ^ mix64(key ^ mix64(step + 0x9e3779b97f4a7c15ull)));
  }
  __device__ __forceinline__ float u01(unsigned long long idx) const {
    return (float)(mix64(base + (idx + 1ull) * 0x9e3779b97f4a7c15ull) >> 40) * (1.f / 16777216.f);
  }
};

}  // namespace mjh
