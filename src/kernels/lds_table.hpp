// lds_table.hpp — group-probed hash table in LDS keyed by the packed 128-bit
// word key (keys.hpp): the per-bucket slice of the running key table held by
// the reduce and table-split kernels (reduce.hip).
//
// Layout: slots come in groups of 4 stored together (SlotGroup, 80 B): four
// 32-bit tags derived from the placement hash, then the four k1 and four k0.
// A lookup reads the whole group with five ds_read_b128 issued back to back —
// ONE dependent LDS round trip — and compares in registers, so the common
// case (key present) needs no further LDS reads and no divergent branches.
// Groups fill left to right and slots are never freed until the table is
// cleared, so linear probing over groups is exact.
//
// Claim protocol (no spin inside a branch, so lanes of one wave can never
// dead-lock on each other): tag 0 -> PENDING by LDS CAS, the claimer writes
// k0/k1, then publishes the real tag (never 0 or PENDING).  The tag is the
// publish flag: a reader only trusts k0/k1 of a slot whose tag it saw
// published, and it reads the tags before the keys (LDS executes one wave's
// accesses in order).  A prober that sees PENDING in a group re-reads the
// group on its next loop iteration; the claimer always finishes its publish
// inside the iteration that won the CAS.
#pragma once
#include <hip/hip_runtime.h>

#include "keys.hpp"

// Diagnostic counts of the claim loop (`st`: RedLds counters in WC_RED_STAMPS builds, else null).
#define WC_LDS_STAT(counter) \
  do {                       \
    if (st) atomicAdd(&st[(counter)], 1ull); \
  } while (0)

namespace wc {
namespace dev {

constexpr uint32_t TAG_EMPTY = 0u;
constexpr uint32_t TAG_PENDING = 1u;

struct alignas(16) SlotGroup {
  uint32_t tag[4];
  uint64_t k1[4];
  uint64_t k0[4];
};
static_assert(sizeof(SlotGroup) == 80, "SlotGroup layout");

// The bucket bits of the placement hash are the low bits (constant inside a
// slice), so tags and groups are taken from a multiplied copy: its high bits
// depend on every bit of the hash.
__device__ __forceinline__ uint32_t slice_hash(uint32_t ph) { return ph * 0x9E3779B1u; }
__device__ __forceinline__ uint32_t make_tag(uint32_t ph) { return (slice_hash(ph) & ~1u) | 2u; }
__device__ __forceinline__ uint32_t group_of(uint32_t ph, uint32_t ngroups) {
  return (uint32_t)(((uint64_t)slice_hash(ph) * ngroups) >> 32);
}
// A key's probe sequence: its home group g1, a second group g2 != g1 from
// other hash bits, then g2 + 1, g2 + 2, ...  Overflow from a full home group
// lands in a random group instead of the neighbour (no clusters), and a lookup
// that reads the tags of g1 and g2 in one round trip finds almost every key.
__device__ __forceinline__ uint32_t group2_of(uint32_t ph, uint32_t ngroups) {
  const uint32_t d = (slice_hash(ph) >> 4) & (ngroups - 1);
  return group_of(ph, ngroups) ^ (d ? d : 1u);
}
__device__ __forceinline__ uint32_t probe_group(uint32_t g1, uint32_t g2, uint32_t step, uint32_t ngroups) {
  return step == 0 ? g1 : ((g2 + step - 1) & (ngroups - 1));
}

// Returns the slot (4 * group + lane-in-group) holding (k0,k1) — claiming the
// first empty slot of the first non-full group if the key is new
// (claimed = true) — or -1 after `max_groups` full groups.  find = false skips
// the lookup (the caller knows the key is not in the slice: table split).
__device__ __forceinline__ int lds_find_or_claim(SlotGroup* groups, uint32_t ngroups, uint32_t ph, uint64_t k0,
                                                 uint64_t k1, int max_groups, bool& claimed, bool find = true,
                                                 unsigned long long* st = nullptr) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  const uint32_t tag = make_tag(ph);
  const uint32_t g1 = group_of(ph, ngroups), g2 = group2_of(ph, ngroups);
  uint32_t g = g1;
  int steps = 0;
  claimed = false;
  for (;;) {
    // Plain loads stay ds_read_b128; the asm barrier stops reuse across iterations.
    asm volatile("" ::: "memory");
    SlotGroup& G = groups[g];
    const u32x4 t = *reinterpret_cast<const u32x4*>(G.tag);
    const u64x2 a1 = *reinterpret_cast<const u64x2*>(&G.k1[0]);
    const u64x2 b1 = *reinterpret_cast<const u64x2*>(&G.k1[2]);
    const u64x2 a0 = *reinterpret_cast<const u64x2*>(&G.k0[0]);
    const u64x2 b0 = *reinterpret_cast<const u64x2*>(&G.k0[2]);
    const bool h0 = find && t.x == tag && a1.x == k1 && a0.x == k0;
    const bool h1 = find && t.y == tag && a1.y == k1 && a0.y == k0;
    const bool h2 = find && t.z == tag && b1.x == k1 && b0.x == k0;
    const bool h3 = find && t.w == tag && b1.y == k1 && b0.y == k0;
    WC_LDS_STAT(RS_PROBE_ITERS);
    if (h0 | h1 | h2 | h3) return 4 * (int)g + (h0 ? 0 : (h1 ? 1 : (h2 ? 2 : 3)));
    if (t.x == TAG_PENDING || t.y == TAG_PENDING || t.z == TAG_PENDING || t.w == TAG_PENDING) {
      WC_LDS_STAT(RS_PENDING);
      continue;  // someone is publishing in this group: look again
    }
    const int e = t.x == TAG_EMPTY ? 0 : (t.y == TAG_EMPTY ? 1 : (t.z == TAG_EMPTY ? 2 : (t.w == TAG_EMPTY ? 3 : -1)));
    if (e >= 0) {
      if (atomicCAS(&G.tag[e], TAG_EMPTY, TAG_PENDING) == TAG_EMPTY) {
        G.k0[e] = k0;
        G.k1[e] = k1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __hip_atomic_store(&G.tag[e], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        claimed = true;
        WC_LDS_STAT(RS_CLAIMS);
        return 4 * (int)g + e;
      }
      WC_LDS_STAT(RS_CAS_FAIL);
      continue;  // lost the race for that slot: re-read the group
    }
    if (++steps >= max_groups) return -1;
    g = probe_group(g1, g2, (uint32_t)steps, ngroups);
  }
}

// Next slot of the probe sequence (cursor: -1 at the start, then kept by the
// caller) whose key is (k0, k1), or -1 at the first group with an empty slot.
// LONG keys may sit in several slots (colliding words, keys.hpp): the caller
// verifies bytes.  Read-only: the slice must not change concurrently.
__device__ __forceinline__ int lds_find_next(const SlotGroup* groups, uint32_t ngroups, uint32_t ph, uint64_t k0,
                                             uint64_t k1, int& cursor) {
  const uint32_t tag = make_tag(ph);
  const uint32_t g1 = group_of(ph, ngroups), g2 = group2_of(ph, ngroups);
  uint32_t step = cursor < 0 ? 0u : (uint32_t)cursor / 4;
  int i = cursor < 0 ? 0 : (cursor & 3) + 1;
  for (; step < ngroups; ++step, i = 0) {
    const uint32_t g = probe_group(g1, g2, step, ngroups);
    const SlotGroup& G = groups[g];
    bool empty = false;
    for (; i < 4; ++i) {
      if (G.tag[i] == TAG_EMPTY) {
        empty = true;
      } else if (G.tag[i] == tag && G.k1[i] == k1 && G.k0[i] == k0) {
        cursor = (int)(4 * step) + i;
        return 4 * (int)g + i;
      }
    }
    if (empty) return -1;
  }
  return -1;
}

__device__ __forceinline__ uint32_t slot_tag(const SlotGroup* groups, int s) { return groups[s >> 2].tag[s & 3]; }
__device__ __forceinline__ uint64_t slot_k0(const SlotGroup* groups, int s) { return groups[s >> 2].k0[s & 3]; }
__device__ __forceinline__ uint64_t slot_k1(const SlotGroup* groups, int s) { return groups[s >> 2].k1[s & 3]; }

}  // namespace dev
}  // namespace wc
