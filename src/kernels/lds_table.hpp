// lds_table.hpp — group-probed hash table in LDS keyed by the packed 128-bit
// word key (keys.hpp).  Used by the map kernel (per-block combiner) and the
// reduce kernel (per-bucket slice of the running table).
//
// Layout: slots are grouped by 4; a parallel array of 32-bit tags (derived
// from the placement hash) lets one ds_read_b128 test a whole group, so a
// lookup is ONE dependent LDS round trip in the common case even at 80-90%
// load, instead of a chain of single-slot probes (which made every wave wait
// for its unluckiest lane).  Groups fill left to right and slots are never
// freed until the table is cleared, so linear probing over groups is exact.
//
// Claim protocol (no spin inside a branch, so lanes of one wave can never
// dead-lock on each other): tag 0 -> PENDING by LDS CAS, the claimer writes
// k0/k1, then publishes the real tag (never 0 or PENDING).  A prober that sees
// PENDING in a group re-reads that group on its next loop iteration; the
// claimer always finishes its publish inside the iteration that won the CAS.
#pragma once
#include <hip/hip_runtime.h>

#include "keys.hpp"

namespace wc {
namespace dev {

constexpr uint32_t TAG_EMPTY = 0u;
constexpr uint32_t TAG_PENDING = 1u;

__device__ __forceinline__ uint32_t make_tag(uint64_t ph) { return ((uint32_t)ph & ~1u) | 2u; }
__device__ __forceinline__ uint32_t group_of(uint64_t ph, uint32_t ngroups) {
  return (uint32_t)(ph >> 32) & (ngroups - 1);
}

// Returns the slot holding (k0,k1) — claiming the first empty slot of the
// first non-full group if the key is new (claimed = true) — or -1 after
// `max_groups` full groups.
__device__ __forceinline__ int lds_find_or_claim(uint32_t* tags, uint64_t* k0s, uint64_t* k1s, uint32_t ngroups,
                                                 uint64_t ph, uint64_t k0, uint64_t k1, int max_groups,
                                                 bool& claimed) {
  const uint32_t tag = make_tag(ph);
  uint32_t g = group_of(ph, ngroups);
  int steps = 0;
  claimed = false;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  for (;;) {
    // Plain (non-volatile) load so it stays a ds_read_b128; the asm barrier
    // stops the compiler from reusing a previous iteration's value.
    asm volatile("" ::: "memory");
    const u32x4 q = *reinterpret_cast<const u32x4*>(&tags[4 * g]);
    const uint32_t m_match = (q.x == tag) | (q.y == tag) << 1 | (q.z == tag) << 2 | (q.w == tag) << 3;
    const uint32_t m_pend = (q.x == TAG_PENDING) | (q.y == TAG_PENDING) << 1 | (q.z == TAG_PENDING) << 2 |
                            (q.w == TAG_PENDING) << 3;
    const uint32_t m_empty = (q.x == TAG_EMPTY) | (q.y == TAG_EMPTY) << 1 | (q.z == TAG_EMPTY) << 2 |
                             (q.w == TAG_EMPTY) << 3;
    for (uint32_t mm = m_match; mm; mm &= mm - 1) {  // almost always 0 or 1 iteration
      const int s = 4 * g + (__ffs(mm) - 1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (k0s[s] == k0 && k1s[s] == k1) return s;
    }
    if (m_pend) continue;  // someone is publishing in this group: look again
    if (m_empty) {
      const int s = 4 * g + (__ffs(m_empty) - 1);
      if (atomicCAS(&tags[s], TAG_EMPTY, TAG_PENDING) == TAG_EMPTY) {
        k0s[s] = k0;
        k1s[s] = k1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __hip_atomic_store(&tags[s], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        claimed = true;
        return s;
      }
      continue;  // lost the race for that slot: re-read the group
    }
    if (++steps >= max_groups) return -1;
    g = (g + 1) & (ngroups - 1);
  }
}

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
