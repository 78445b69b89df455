// lds_table.hpp — open-addressing hash table in LDS keyed by the packed 128-bit
// word key (keys.hpp).  Used by the map kernel (per-block pre-aggregation) and
// the reduce kernel (per-bucket running table).
//
// Claim protocol (no spin inside a branch, so lanes of one wave can never
// dead-lock on each other): a slot's k1 goes EMPTY -> PENDING by 64-bit LDS CAS,
// the claimer writes k0, then publishes k1.  A prober that sees PENDING simply
// re-reads the same slot on its next loop iteration; the claimer finishes its
// publish inside the iteration in which it won the CAS.
#pragma once
#include <hip/hip_runtime.h>

#include "keys.hpp"

namespace wc {
namespace dev {

__device__ __forceinline__ uint64_t lds_load_u64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Returns the slot holding (k0,k1), claiming an empty one if the key is new
// (claimed = true).  Returns -1 after `max_probe` occupied mismatches.
__device__ __forceinline__ int lds_find_or_claim(uint64_t* k0s, uint64_t* k1s, uint32_t mask, uint64_t k0,
                                                 uint64_t k1, uint32_t slot, int max_probe, bool& claimed) {
  claimed = false;
  int probes = 0;
  for (;;) {
    uint64_t cur = lds_load_u64(&k1s[slot]);
    if (cur == K1_EMPTY) {
      const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&k1s[slot]), 0ull,
                                      (unsigned long long)K1_PENDING);
      if (prev == K1_EMPTY) {
        k0s[slot] = k0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __hip_atomic_store(&k1s[slot], k1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        claimed = true;
        return (int)slot;
      }
      cur = prev;
    }
    if (cur != K1_PENDING) {
      if (cur == k1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (k0s[slot] == k0) return (int)slot;
      }
      if (++probes >= max_probe) return -1;
      slot = (slot + 1) & mask;
    }
  }
}

// Wave-level helpers.
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

// Exclusive prefix count of set predicate among lower lanes + wave total.
__device__ __forceinline__ uint32_t wave_rank(bool pred, uint32_t& total) {
  const uint64_t b = __ballot(pred);
  total = (uint32_t)__popcll(b);
  const uint64_t lt = (lane_id() == 0) ? 0ull : (~0ull >> (64 - lane_id()));
  return (uint32_t)__popcll(b & lt);
}

}  // namespace dev
}  // namespace wc
