// rmc_fpset.h — the HBM fingerprint set (TLC's FPSet),
// shared by the BFS kernels (rmc_kernels.hip) and the insert microbenchmark
// (rmc_fpset_bench.hip).
//
// Two tiers:
//   main  M: the fingerprints of every COMPLETED level.  8 B keys, open
//            addressing, linear probing.  Read-only while a level is
//            expanded, so the 70% of successors that are duplicates of older
//            states cost one plain (non-atomic, never-dirtying) probe.
//   level L: the fingerprints first seen in the CURRENT level, 16 B entries
//            (fp, val) with val = parent global index << 26 | ordinal << 16 |
//            hidden.  atomicMin on val keeps the successor first in TLC order
//            (parent position in the level, then the action's ordinal in Next:
//            TLC -workers 1 first-wins under VIEW, SURVEY.md §7 hard part 1);
//            hidden = the variables VIEW drops (electionCtr, restartCtr, acked;
//            Pull: the counters), carried so losers can count same-level
//            hidden-variable collisions.
// At the end of a level k_merge moves L's keys into M and L is cleared.  Empty
// slots hold ~0 (a fingerprint of ~0 is mapped to ~0 - 1 by canon_from_sums).
#pragma once
#include <hip/hip_runtime.h>
#include "rmc_engine.h"

namespace rmc {

constexpr unsigned long long EMPTY = ~0ULL;
// candidate slot word: bit 63 = found in M (a state of an earlier level);
// else hidden << 47 | L slot
constexpr unsigned long long CAND_DUP = 1ULL << 63;
constexpr unsigned long long CAND_SLOT_MASK = (1ULL << 47) - 1;
constexpr int VAL_RANK_SHIFT = 16;  // val = rank << 16 | hidden; rank = pg << 10 | ordinal

__host__ __device__ __forceinline__ unsigned long long fp_slot(unsigned long long fp, unsigned long long mask) {
  return (fp ^ (fp >> 29)) & mask;
}

// Is fp in M?  M is never more than 0.9 full, so the probe meets an empty slot.
__device__ __forceinline__ bool main_contains(const unsigned long long* __restrict__ Mk, unsigned long long mask,
                                              unsigned long long fp) {
  unsigned long long slot = fp_slot(fp, mask);
  for (unsigned long long probe = 0; probe <= mask; probe++) {
    const unsigned long long k = Mk[slot];
    if (k == fp) return true;
    if (k == EMPTY) return false;
    slot = (slot + 1) & mask;
  }
  return false;
}

// Insert fp with value val into L; returns the slot (EMPTY if L is too full: the
// driver grows L and redoes the chunk, whose L inserts are idempotent).  One
// returning atomic per probe: the CAS doubles as the read.
__device__ __forceinline__ unsigned long long level_insert(unsigned long long* L, unsigned long long mask,
                                                           unsigned long long fp, unsigned long long val,
                                                           DevStatus* st) {
  unsigned long long slot = fp_slot(fp, mask);
  // a probe run this long means the level tier is (nearly) full: give up and
  // let the driver grow it rather than walk the whole table
  const unsigned long long limit = mask < 4096 ? mask : 4096;
  for (unsigned long long probe = 0; probe <= limit; probe++) {
    unsigned long long* e = L + 2 * slot;
    const unsigned long long prev = atomicCAS(e, EMPTY, fp);
    if (prev == EMPTY || prev == fp) {
      atomicMin(e + 1, val);
      return slot;
    }
    slot = (slot + 1) & mask;
  }
  atomicOr(&st->cap_flags, 1u << E_CAP_LEVEL);
  return EMPTY;
}

// Insert a key known to be absent (merge, rehash) into M.
__device__ __forceinline__ bool main_insert_new(unsigned long long* Mk, unsigned long long mask, unsigned long long fp) {
  unsigned long long slot = fp_slot(fp, mask);
  for (unsigned long long probe = 0; probe <= mask; probe++) {
    if (atomicCAS(Mk + slot, EMPTY, fp) == EMPTY) return true;
    slot = (slot + 1) & mask;
  }
  return false;
}

// The candidate's probe: CAND_DUP if an earlier level holds its fingerprint,
// else its L slot with its hidden variables (for the collision count).
__device__ __forceinline__ unsigned long long fpset_probe(const unsigned long long* __restrict__ Mk,
                                                          unsigned long long mmask, unsigned long long* L,
                                                          unsigned long long lmask, unsigned long long fp,
                                                          unsigned long long val, DevStatus* st) {
  if (main_contains(Mk, mmask, fp)) return CAND_DUP;
  const unsigned long long slot = level_insert(L, lmask, fp, val, st);
  return slot == EMPTY ? CAND_DUP : (((val & 0xFFFFULL) << 47) | slot);
}

}  // namespace rmc
