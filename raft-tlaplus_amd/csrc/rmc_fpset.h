// rmc_fpset.h — the HBM fingerprint set (TLC's FPSet),
// shared by the BFS kernels (rmc_kernels.hip) and the insert microbenchmark
// (rmc_fpset_bench.hip).
//
// Open addressing, linear probing, 16 B entries (fp, val), empty = both ~0.
//   val = rank << 16 | hidden,  rank = (parent global index + 1) << 10 | ordinal
// rank orders successors as TLC -workers 1 generates them (parent position in
// BFS order, then the action's ordinal in Next); atomicMin on val keeps the
// first one (TLC's first-wins under VIEW, SURVEY.md §7 hard part 1).  hidden =
// the variables VIEW drops (electionCtr, restartCtr, acked; Pull: the
// counters), carried so that same-level losers can count hidden-variable
// collisions.  The initial state's val is 0, below every rank.
//
// No level field is needed: parents of level L+1's states are level L's, and
// global indices grow level by level, so an entry is from an EARLIER level iff
// its val < floor = (first global index of the parents' level + 1) << 26.  An
// insert that finds its fingerprint from an earlier level leaves the entry
// untouched (plain loads, no write); only new fingerprints and same-level
// duplicates pay the atomicMin.  On the bench workload nearly every duplicate
// is a same-level one (profiles/r04/fpstats_raft_n3v2e2.txt: 4.09e9 CAS, 1.89e9
// won; 5.21e9 atomicMin for 6.75e9 inserts).
#pragma once
#include <hip/hip_runtime.h>
#include "rmc_engine.h"

namespace rmc {

constexpr unsigned long long EMPTY = ~0ULL;
// candidate slot word: CAND_DUP = no entry (error / failed insert); else
// hidden << 47 | slot
constexpr unsigned long long CAND_DUP = 1ULL << 63;
constexpr unsigned long long CAND_SLOT_MASK = (1ULL << 47) - 1;
// k_expand's tile dedup: CAND_REF | hidden << 47 | the candidate index of the
// same tile round's representative, which inserted the fingerprint (slots
// are below 2^46, so bit 46 is free in a slot word)
constexpr unsigned long long CAND_REF = 1ULL << 46;
constexpr unsigned long long CAND_REF_MASK = CAND_REF - 1;
constexpr int VAL_RANK_SHIFT = 16;   // val = rank << 16 | hidden
constexpr int VAL_FLOOR_SHIFT = 26;  // floor = (global index + 1) << 26 (rank << 16 with ordinal 0)

// Home slot: the TOP bits of fp times an odd constant (a bijection, so as
// uniform as fp, and independent of fp_owner's raw high word).  With top bits
// a key's home slot in a table of 2^a slots is the prefix of its home slot in
// one of 2^b >= 2^a slots, so a rehash into a larger table walks the new table
// in address order.
//
// RMC_SLOT_ALIGN = 4: the home slot is rounded down to a multiple of 4 (a
// 64 B aligned group of 16 B entries), so the insert's first group load
// touches one aligned 64 B block instead of straddling two 3 times in 4.
#ifndef RMC_SLOT_ALIGN
#define RMC_SLOT_ALIGN 1
#endif
__host__ __device__ __forceinline__ unsigned long long fp_slot(unsigned long long fp, unsigned long long mask) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int sh = __clzll((long long)mask);
#else
  const int sh = __builtin_clzll(mask);
#endif
  return ((fp * 0x9E3779B97F4A7C15ULL) >> sh) & mask & ~(unsigned long long)(RMC_SLOT_ALIGN - 1);
}

// Owner of a fingerprint among W shards (sharded search): multiply-shift range
// reduction of the high word (independent of the slot, which is a hash of all of fp).
__host__ __device__ __forceinline__ int fp_owner(unsigned long long fp, int W) {
  return (int)(((fp >> 32) * (unsigned long long)W) >> 32);
}

// Diagnostic build only (-DRMC_FPSTATS): exact counts of what the inserts do
// (inserts, 4-entry group loads, CAS issued / won, atomicMin issued), read
// back with read_fpstats(); the product build compiles them away.
#ifdef RMC_FPSTATS
static __device__ unsigned long long g_fpstats[8];
#define FPSTAT(i) atomicAdd(&g_fpstats[i], 1ULL)
#else
#define FPSTAT(i) ((void)0)
#endif
enum { FPS_INSERT = 0, FPS_GROUP = 1, FPS_CAS = 2, FPS_CAS_WON = 3, FPS_MIN = 4 };

// Insert fp with value val; returns the slot, or EMPTY when the probe run is
// too long (the table is too full: the driver grows it and redoes the chunk,
// whose inserts are idempotent).
//
// Two protocols.  The default (below, after #else): the first four entries of
// the probe run are read with 16 B loads issued together; a hit decides
// without an atomic (earlier level) or with one atomicMin (same level); else a
// CAS per slot from the first EMPTY-or-other slot on.  The alternative
// (-DRMC_FP_READPROBE) reads the whole run in groups of four and takes at most
// one CAS per probe step.  Measured on the bench workload (r03, CLI, 8M
// parents per launch, interleaved runs): k_expand 918 ms per check with the
// default vs 1025 ms with the read probe, though the read probe writes less
// (WRITE_SIZE 1.43 vs 2.06 GB per launch): its loop of dependent 64 B group
// loads is longer than the default's single group + CAS.
//
// RMC_FP_READPROBE: the probe run is READ, four entries (64 B) per group of plain 16 B loads
// issued together, up to the first entry that is fp or EMPTY.  Keys are never
// removed or moved while a level is expanded, so a key read with a plain load
// is really there -- an earlier level's copy of fp is final (no atomic, no
// write), a same-level copy only needs its atomicMin, and another key means
// "go on".  A slot seen EMPTY may have been claimed since (the XCD's L2 is not
// coherent with the other XCDs' atomics), so it takes ONE CAS, whose returned
// key decides; a CAS lost to another key resumes the READ probe after it.  So
// a wave issues at most one CAS instruction per probe step.  (On gfx950 every
// device-scope atomic executes at the memory side, MI355X_MICROARCH.md
// 'Global float atomics': the r02 protocol's CAS per slot past the first
// four entries was a memory round trip and a WRITE_SIZE transaction per
// occupied slot passed.)
#ifdef RMC_FP_READPROBE
__device__ __forceinline__ unsigned long long fpset_insert(unsigned long long* T, unsigned long long mask,
                                                           unsigned long long fp, unsigned long long val,
                                                           unsigned long long floor, DevStatus* st) {
  FPSTAT(FPS_INSERT);
  unsigned long long slot = fp_slot(fp, mask);
  const unsigned long long limit = mask < 4096 ? mask : 4096;
  const ulonglong2* E = reinterpret_cast<const ulonglong2*>(T);
  for (unsigned long long probe = 0; probe <= limit;) {
    FPSTAT(FPS_GROUP);
    ulonglong2 e[4];
    if (slot + 3 <= mask) {
#pragma unroll
      for (int q = 0; q < 4; q++) e[q] = E[slot + q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) e[q] = E[(slot + q) & mask];
    }
    int k = 4;
    unsigned long long kv = 0;
    bool found = false;
#pragma unroll
    for (int q = 3; q >= 0; q--)
      if (e[q].x == fp || e[q].x == EMPTY) { k = q; kv = e[q].y; found = e[q].x == fp; }
    slot = (slot + (unsigned long long)k) & mask;
    probe += (unsigned long long)k;
    if (k == 4) continue;  // four other keys: read on
    if (found) {
      // same level (or its claimer's min in flight): values only decrease, so
      // a snapshot already below val means this successor lost -- no atomic
      if (kv >= floor && val < kv) { FPSTAT(FPS_MIN); atomicMin(T + 2 * slot + 1, val); }
      return slot;
    }
    FPSTAT(FPS_CAS);
    const unsigned long long prev = atomicCAS(T + 2 * slot, EMPTY, fp);
    if (prev == EMPTY) {
      FPSTAT(FPS_CAS_WON);
      FPSTAT(FPS_MIN);
      atomicMin(T + 2 * slot + 1, val);
      return slot;
    }
    if (prev == fp) {
      // claimed by another lane this level (a value of ~0: its claimer's
      // atomicMin is still in flight, >= floor, so this one takes part)
      const unsigned long long cur = __hip_atomic_load(T + 2 * slot + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur >= floor && val < cur) { FPSTAT(FPS_MIN); atomicMin(T + 2 * slot + 1, val); }
      return slot;
    }
    slot = (slot + 1) & mask;  // another key took it since the load
    probe++;
  }
  atomicOr(&st->cap_flags, 1u << E_CAP_TABLE);
  return EMPTY;
}
#else
// default protocol: four entries read, then a CAS per probe
__device__ __forceinline__ unsigned long long fpset_insert(unsigned long long* T, unsigned long long mask,
                                                           unsigned long long fp, unsigned long long val,
                                                           unsigned long long floor, DevStatus* st) {
  FPSTAT(FPS_INSERT);
  FPSTAT(FPS_GROUP);
  unsigned long long slot = fp_slot(fp, mask);
#ifndef RMC_FP_FAST
#define RMC_FP_FAST 4
#endif
  if (RMC_FP_FAST > 0 && slot + (RMC_FP_FAST - 1) <= mask) {
    const ulonglong2* E = reinterpret_cast<const ulonglong2*>(T) + slot;
    ulonglong2 e[RMC_FP_FAST > 0 ? RMC_FP_FAST : 1];
#ifdef RMC_FP_COHERENT
    // agent-scope loads: served coherently with the other XCDs' atomics
    // instead of from a possibly stale line in this XCD's L2 (a stale EMPTY
    // sends a same-level duplicate into a CAS that fails)
#pragma unroll
    for (int q = 0; q < RMC_FP_FAST; q++) {
      e[q].x = __hip_atomic_load(T + 2 * (slot + q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      e[q].y = __hip_atomic_load(T + 2 * (slot + q) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    (void)E;
#else
#pragma unroll
    for (int q = 0; q < RMC_FP_FAST; q++) e[q] = E[q];
#endif
    int k = RMC_FP_FAST;
    unsigned long long kv = 0;
    bool found = false;
#pragma unroll
    for (int q = RMC_FP_FAST - 1; q >= 0; q--)
      if (e[q].x == fp || e[q].x == EMPTY) { k = q; kv = e[q].y; found = e[q].x == fp; }
    slot = (slot + (unsigned long long)k) & mask;  // k == RMC_FP_FAST may step past the last slot: wrap
    if (found) {
      if (kv >= floor && val < kv) { FPSTAT(FPS_MIN); atomicMin(T + 2 * slot + 1, val); }
      return slot;
    }
  }
  const unsigned long long limit = mask < 4096 ? mask : 4096;
  for (unsigned long long probe = 0; probe <= limit; probe++) {
    unsigned long long* e = T + 2 * slot;
    FPSTAT(FPS_CAS);
    const unsigned long long prev = atomicCAS(e, EMPTY, fp);
    if (prev == EMPTY) {
      FPSTAT(FPS_CAS_WON);
      FPSTAT(FPS_MIN);
      atomicMin(e + 1, val);
      return slot;
    }
    if (prev == fp) {
      // claimed since the group load (a sibling's race: 2.2e9 of the bench
      // workload's 4.1e9 CAS): the atomicMin without reading the value first
      // -- no dependent round trip; an earlier level's value is below
      // floor <= val, so the min leaves it unchanged.  Measured (CLI, fresh
      // process, 3 interleaved runs): k_expand 827 vs 852 ms per check for
      // 1.5% more atomicMin (profiles/r04/ab_blindmin_r04r.txt).
      FPSTAT(FPS_MIN);
      atomicMin(e + 1, val);
      return slot;
    }
    slot = (slot + 1) & mask;
  }
  atomicOr(&st->cap_flags, 1u << E_CAP_TABLE);
  return EMPTY;
}
#endif

// The default protocol split in two for pure-insert kernels (k_insert_recv):
// the first four entries of SEVERAL keys' probe runs are loaded before any is
// decided, so their loads are in flight together; each key then continues
// from its loaded group exactly as fpset_insert does.
__device__ __forceinline__ bool fpset_group_load(const unsigned long long* T, unsigned long long mask,
                                                 unsigned long long fp, ulonglong2 (&e)[4]) {
  const unsigned long long slot = fp_slot(fp, mask);
  if (slot + 3 > mask) return false;
  const ulonglong2* E = reinterpret_cast<const ulonglong2*>(T) + slot;
#pragma unroll
  for (int q = 0; q < 4; q++) e[q] = E[q];
  return true;
}
__device__ __forceinline__ unsigned long long fpset_insert_loaded(unsigned long long* T, unsigned long long mask,
                                                                  unsigned long long fp, unsigned long long val,
                                                                  unsigned long long floor, DevStatus* st,
                                                                  const ulonglong2 (&e)[4], bool loaded) {
  unsigned long long slot = fp_slot(fp, mask);
  if (loaded) {
    int k = 4;
    unsigned long long kv = 0;
    bool found = false;
#pragma unroll
    for (int q = 3; q >= 0; q--)
      if (e[q].x == fp || e[q].x == EMPTY) { k = q; kv = e[q].y; found = e[q].x == fp; }
    slot = (slot + (unsigned long long)k) & mask;
    if (found) {
      if (kv >= floor && val < kv) atomicMin(T + 2 * slot + 1, val);
      return slot;
    }
  }
  const unsigned long long limit = mask < 4096 ? mask : 4096;
  for (unsigned long long probe = 0; probe <= limit; probe++) {
    unsigned long long* p = T + 2 * slot;
    const unsigned long long prev = atomicCAS(p, EMPTY, fp);
    if (prev == EMPTY) {
      atomicMin(p + 1, val);
      return slot;
    }
    if (prev == fp) {  // claimed since the load: the min without reading first (as fpset_insert)
      atomicMin(p + 1, val);
      return slot;
    }
    slot = (slot + 1) & mask;
  }
  atomicOr(&st->cap_flags, 1u << E_CAP_TABLE);
  return EMPTY;
}

// The value of fp's entry (~0 if absent): read-only probe.
__device__ __forceinline__ unsigned long long fpset_value(const unsigned long long* T, unsigned long long mask,
                                                          unsigned long long fp) {
  unsigned long long slot = fp_slot(fp, mask);
  for (unsigned long long probe = 0; probe <= mask; probe++) {
    const ulonglong2 e = reinterpret_cast<const ulonglong2*>(T)[slot];
    if (e.x == fp) return e.y;
    if (e.x == EMPTY) break;
    slot = (slot + 1) & mask;
  }
  return EMPTY;
}

// fp_bits = 128: 32 B entries (fp.a, fp.b, val, unused).  The slot is claimed
// by a CAS of the first word; the claimer then publishes the second.  A lane
// that finds the first word equal must compare the second; if its claimer (in
// another wave) has not published it after a bounded wait, the lane cannot
// decide -- E_RETRY, and the driver redoes the chunk (idempotent; every key of
// the chunk is complete by then).
__device__ __forceinline__ unsigned long long fpset_insert128(unsigned long long* T, unsigned long long mask, Fp128 fp,
                                                              unsigned long long val, unsigned long long floor,
                                                              DevStatus* st) {
  unsigned long long slot = fp_slot(fp.a, mask);
  if (slot + 1 <= mask) {  // fast path: the first two entries of the run, plain loads
    const ulonglong2* E = reinterpret_cast<const ulonglong2*>(T) + 2 * slot;
    const ulonglong2 k0 = E[0], v0 = E[1], k1 = E[2], v1 = E[3];
    int k = 2;
    unsigned long long kv = 0;
    bool found = false;
    if (k1.x == fp.a || k1.x == EMPTY) { k = 1; kv = v1.x; found = k1.x == fp.a && k1.y == fp.b; }
    if (k0.x == fp.a || k0.x == EMPTY) { k = 0; kv = v0.x; found = k0.x == fp.a && k0.y == fp.b; }
    slot = (slot + (unsigned long long)k) & mask;
    if (found) {
      if (kv >= floor && val < kv) atomicMin(T + 4 * slot + 2, val);
      return slot;
    }
  }
  const unsigned long long limit = mask < 4096 ? mask : 4096;
  for (unsigned long long probe = 0; probe <= limit; probe++) {
    unsigned long long* e = T + 4 * slot;
    const unsigned long long prev = atomicCAS(e, EMPTY, fp.a);
    const bool claimed = prev == EMPTY;
    // One instruction for the whole wave: the claimer publishes its second
    // word, every other lane reads it (CAS of EMPTY by EMPTY: no change).
    // Lanes of one atomic instruction are served in lane order, as in the
    // claiming CAS, so a same-wave duplicate reads the claimer's word;
    // correctness does not depend on it (E_RETRY below).
    unsigned long long lo = atomicCAS(e + 1, EMPTY, claimed ? fp.b : EMPTY);
    if (claimed) {
      atomicMin(e + 2, val);
      return slot;
    }
    if (prev == fp.a) {
      // claimed by another wave whose publish is one instruction behind its
      // claim: wait a bounded while for it (no wave waits on this one)
      for (int t = 0; lo == EMPTY && t < 64; t++) {
        __builtin_amdgcn_s_sleep(2);
        lo = __hip_atomic_load(e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lo == EMPTY) {
        atomicOr(&st->cap_flags, 1u << E_RETRY);
        return EMPTY;
      }
      if (lo == fp.b) {  // the min without reading first (as fpset_insert)
        atomicMin(e + 2, val);
        return slot;
      }
    }
    slot = (slot + 1) & mask;
  }
  atomicOr(&st->cap_flags, 1u << E_CAP_TABLE);
  return EMPTY;
}

// The candidate word: CAND_DUP, or hidden << 47 | slot.
__device__ __forceinline__ unsigned long long cand_word(unsigned long long slot, unsigned long long val) {
  return slot == EMPTY ? CAND_DUP : (((val & 0xFFFFULL) << 47) | slot);
}

// After every insert of the round: did the candidate (rank; its hidden
// variables in the low 16 bits of `hidden`) win the entry whose value is v?
// A same-level loser with other hidden variables is a hidden-variable collision.
__device__ __forceinline__ bool fpset_won(unsigned long long v, unsigned long long rank, unsigned long long floor,
                                          unsigned long long hidden, bool& collision) {
  const bool win = (v >> VAL_RANK_SHIFT) == rank;
  collision = !win && v >= floor && ((v ^ hidden) & 0xFFFFULL) != 0;
  return win;
}

}  // namespace rmc
