// rmc_fpset.h — the HBM fingerprint set's insert (TLC's FPSet, SURVEY.md §8a
// E1), shared by the BFS kernels (rmc_kernels.hip) and the insert
// microbenchmark (tools/fpset_bench.hip).
//
// Open addressing, linear probing, 16 B entries (fp u64, val u64); empty =
// both words ~0.  val = (level << 48) | (global parent index << 10) | ordinal,
// so atomicMin keeps the successor first in TLC order.
#pragma once
#include <hip/hip_runtime.h>
#include "rmc_engine.h"

namespace rmc {

constexpr unsigned long long EMPTY = ~0ULL;

// Insert fp with value val; returns the slot.  val = (level << 48) | rank.
// One returning atomic per probe: the CAS doubles as the read (measured
// faster than a 16 B load first: 976 vs 989 ms of k_expand on the bench cfg).
// An entry from an earlier level has a smaller val, so the atomicMin that
// claims first-in-TLC-order within the level never changes it.
__device__ __forceinline__ unsigned long long table_insert(unsigned long long* T, unsigned long long mask,
                                                           unsigned long long fp, unsigned long long val,
                                                           unsigned level, DevStatus* st) {
  (void)level;
  if (fp == EMPTY) fp = EMPTY - 1;
  unsigned long long slot = (fp ^ (fp >> 29)) & mask;
  for (unsigned long long probe = 0; probe <= mask; probe++) {
    unsigned long long* e = T + 2 * slot;
    unsigned long long prev = atomicCAS(e, EMPTY, fp);
    if (prev == EMPTY || prev == fp) {
      atomicMin(e + 1, val);
      return slot;
    }
    slot = (slot + 1) & mask;
  }
  atomicOr(&st->cap_flags, 1u << E_CAP_TABLE);
  return 0;
}

}  // namespace rmc
