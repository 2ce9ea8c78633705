// rmc_kernels.hip — level-synchronous BFS kernels for gfx950 (MI355X).
//
// Per BFS level, per chunk of parents.  Parents are
// processed in tiles of PB consecutive states (Tile<N>), one 256-thread block
// per tile:
//   k_expand       stage the tile in LDS; H_pi(parent) for every server
//                  permutation; evaluate every Next binding lane-per-parent
//                  (one binding per wave step, so fixed actions are wave-
//                  uniform); then lane-per-successor: rebuild the delta,
//                  compute the canonical fingerprint incrementally from H_pi,
//                  insert it into the HBM fingerprint set with first-in-TLC-
//                  order-wins semantics (atomicMin on (parent, ordinal)),
//                  leaving entries of earlier levels unwritten (rmc_fpset.h).
//   k_mark         one thread per parent: which of its candidates won, and
//                  each winner's rank in TLC order; same-level hidden-variable
//                  collisions are counted here.
//   (scan)         exclusive scan of winners per parent -> output positions.
//   k_materialize  same tiling: compact the tile's winners in LDS, regenerate
//                  each lane-per-winner, write it to its TLC-order slot of the
//                  next frontier, write the trace record, check invariants.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include "rmc_spec.h"
#include "rmc_engine.h"
#include "rmc_fpset.h"

namespace rmc {

__constant__ Model cM;

constexpr int WAVE = 64;
constexpr int EXPAND_SEGS = 8;  // candidate-buffer segments of the single-shard k_expand (one per XCD)

// XCD-aware block -> tile map (MI355X_MICROARCH.md, workgroup dispatch: blocks
// b and b + 8 share an XCD and its L2).  RMC_XCD_REMAP = 1 gives each of the 8
// XCD labels one contiguous run of tiles, so neighbouring tiles -- whose
// successors are often the same states -- probe and re-read the same
// fingerprint-set lines through one L2.  A bijection on [0, n) for any n;
// placement is a speed choice only, the tile a block computes is all that
// changes.
#ifndef RMC_XCD_REMAP
#define RMC_XCD_REMAP 0
#endif
__device__ __forceinline__ unsigned long long xcd_tile(unsigned long long b, unsigned long long n) {
#if RMC_XCD_REMAP
  const unsigned long long q = n >> 3, r = n & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
#else
  (void)n;
  return b;
#endif
}
// cand_ob = ordinal << 16 | flags | binding (10 bits)
constexpr uint32_t OB_ERR = 0x8000u;    // evaluation error: no successor
constexpr uint32_t OB_LOCAL = 0x4000u;  // sharded search: this shard owns the fp and k_expand inserted it
constexpr uint32_t OB_TDUP = 0x2000u;   // sharded search: repeats an earlier-ranked candidate of its tile (k_tile_dedup)

__device__ __forceinline__ int lane_id() { return threadIdx.x & (WAVE - 1); }
// Orders one wave's LDS accesses across lanes: the LDS serves a wave's
// instructions in order, so it suffices that every earlier LDS write has
// completed and that the compiler moves no LDS access across this point.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ unsigned long long lanemask_lt() {
  int l = lane_id();
  return l ? (~0ULL >> (64 - l)) : 0ULL;
}

// first-in-TLC-order error / violation keys: (parent_global << 20) | (ordinal << 10) | binding
__device__ __forceinline__ unsigned long long order_key(unsigned long long pg, int ordinal, int b) {
  return (pg << 20) | ((unsigned long long)ordinal << 10) | (unsigned long long)b;
}

// Diagnostic build only (-DRMC_STAMPS): per-phase block time of k_expand,
// summed over blocks (thread 0's shader-clock deltas, with an extra barrier
// between phases A and B).  Read the shares, not the absolute time.
#ifdef RMC_STAMPS
__device__ unsigned long long g_stamps[32];
#define STAMP(i)                                                   \
  do {                                                             \
    __syncthreads();                                               \
    if (tid == 0) {                                                \
      unsigned long long t_ = clock64();                           \
      atomicAdd(&g_stamps[i], t_ - t_prev);                        \
      t_prev = t_;                                                 \
    }                                                              \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif
void read_stamps(unsigned long long* out) {
#ifdef RMC_STAMPS
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), 32 * sizeof(unsigned long long));
#else
  for (int i = 0; i < 32; i++) out[i] = 0;
#endif
}

bool diag_build() {
#ifdef RMC_DIAG
  return true;
#else
  return false;
#endif
}
void read_fpstats(unsigned long long* out) {
#ifdef RMC_FPSTATS
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fpstats), 8 * sizeof(unsigned long long));
#else
  for (int i = 0; i < 8; i++) out[i] = 0;
#endif
}

// Parents per expand/materialize tile: one per lane of a wave in phase B.
template <int N>
struct Tile {
  static constexpr int PB = 64;  // = one 64-bit parent mask per binding in k_expand
};

// Dynamic LDS layout of k_expand (bytes; the launch computes the same).
[[maybe_unused]] constexpr int LIVE_WORDS = 4;  // message bitmask words per parent (kmax <= 124)
// Phase C's tile-local dedup of the HBM inserts (single shard, 64-bit
// fingerprints; see k_expand).  Measured and not the default (r06, bench
// workload, CLI, three interleaved rounds, profiles/r06/ab_tile_dedup.txt):
// it cuts the inserts from 6.75e9 to 4.23e9 and the memory-side atomics from
// 9.30e9 to 5.05e9 per check (2.7 per new state; RMC_FPSTATS,
// profiles/r06/fpstats_tile_dedup.txt), yet k_expand takes 710 ms against
// 662 -- the atomics are not what bounds it; the round's barrier is.
#ifndef RMC_TILE_DEDUP
#define RMC_TILE_DEDUP 0
#endif
[[maybe_unused]] constexpr int DEDUP = 256;  // LDS slots of one 256-successor round's table (+ its 256 fingerprints)
// Persistent k_expand (-DRMC_EXPAND_PERSIST=1, measured and rejected in r05):
// a grid of resident blocks walks the tiles, and each block stages tile t+G's
// parent rows into a second LDS buffer by LDS-DMA while tile t runs phases
// B-C.  The second buffer costs 12.5 KB of LDS per block on the bench
// workload: 4 blocks per CU instead of 7, and the hidden staging does not buy
// back the lost occupancy -- k_expand 1,122 vs 729 ms per check, two
// interleaved runs each (profiles/r05/ab_persistent_expand.txt).  The default
// stages one tile per block synchronously.
#ifndef RMC_EXPAND_PERSIST
#define RMC_EXPAND_PERSIST 0
#endif
// Phase A (k_expand) and the tile staging of k_materialize issue all of a
// thread's loads before its first LDS write (stage_rows_batched); 0 = the
// r01-r06 loop form, kept for the A/B.
#ifndef RMC_STAGE_BATCH
#define RMC_STAGE_BATCH 1
#endif
// Single-shard k_expand: tile t's candidates start at t x PB x min(maxsucc,
// 256) instead of a reservation by a returning atomic (a memory round trip on
// every block's critical path); 0 = the r02-r06 per-XCD counters.
#ifndef RMC_TILE_SLOTS
#define RMC_TILE_SLOTS 1
#endif
// RMC_LDS_TRIM: the per-parent live-message mask holds (kmax + 31) / 32
// words instead of LIVE_WORDS, and the tile prefix sBase is 16-bit (a tile
// has at most 64 x 812 candidates): on the bench workload 20.4 KB per block
// instead of 21.1 KB, so eight blocks fit a CU's 160 KB of LDS, not seven.
#ifndef RMC_LDS_TRIM
#define RMC_LDS_TRIM 1
#endif
#if RMC_LDS_TRIM
typedef uint16_t base_t;
#else
typedef uint32_t base_t;
#endif
// RMC_ACT_MAJOR: phase C's lanes take the tile's successors grouped by
// action (action slot, then parent, then ordinal) instead of parent-major, so
// a wave runs one or two actions' code in eval_known instead of every action
// its 64 lanes happen to mix.  Each lane still stores its candidate at its
// TLC-order position in the tile's range, so the candidate layout and every
// later kernel are unchanged.  Phase B counts each (action slot, parent)
// pair's successors (16-bit halves of LDS words), and wave 1 turns the counts
// into a flattened prefix beside wave 0's reservation (no extra barrier).
// Measured and not the default (r06, bench workload, CLI, three interleaved
// rounds, profiles/r06/ab_act_major.txt): k_expand 685-686 ms against
// 661 parent-major -- the lookup (a search over nact x 64 prefixes, a rank
// below the action's first ordinal) and the scattered candidate stores cost
// more than the divergence they remove.
#ifndef RMC_ACT_MAJOR
#define RMC_ACT_MAJOR 0
#endif
#if RMC_ACT_MAJOR && (!RMC_STAGE_BATCH || RMC_EXPAND_PERSIST)
#error "RMC_ACT_MAJOR stages its tables in the batched one-tile phase A (RMC_STAGE_BATCH=1, RMC_EXPAND_PERSIST=0)"
#endif
struct ExpandLds {
  int Wp, lw, off_AP, off_Ms, off_Mask, off_Ord, off_Base, off_BOff, off_Live, off_Desc, off_O2b, off_MOff, off_Hash, off_S2, bytes;
};
__host__ __device__ inline ExpandLds expand_lds(int PB, int words, int ordw, int msbytes, int nfixed, int nord, int kmax,
                                                int nact) {
  ExpandLds L;
#if RMC_LDS_TRIM
  L.lw = (kmax + 31) >> 5;
  if (L.lw < 1) L.lw = 1;
#else
  (void)kmax;
  L.lw = LIVE_WORDS;
#endif
  L.Wp = words | 1;  // odd row stride: lane-per-parent LDS reads are bank-conflict free
  int o = (PB * L.Wp * 4 + 7) & ~7;
  L.off_Ms = o;  // per-parent message sums (MsgSums<N>, 8 B aligned)
  o += PB * msbytes;
  L.off_AP = o;  // RMC_ACT_MAJOR: per (action slot, parent) successor counts, then their prefix (u16)
#if RMC_ACT_MAJOR
  o += ((nact * PB + 2) * 2 + 7) & ~7;
#else
  (void)nact;
#endif
  L.off_Ord = o;  // per parent: bitmask over TLC ordinals of its enabled bindings
  o += PB * ordw * 4;
  L.off_Base = o;  // exclusive prefix over the tile's parents of their successor counts
  o += ((PB + 1) * (int)sizeof(base_t) + 3) & ~3;
  // the model's binding tables, staged once per block: a lane's own binding
  // then costs LDS reads instead of dependent vector loads of __constant__ data
  L.off_Desc = o;  // fixed binding -> descriptor (Model::fb_desc)
  o += nfixed * 4;
  L.off_O2b = o;  // TLC ordinal -> binding (Model::ord2b)
  o += ((nord + 1) & ~1) * 2;
  L.off_MOff = o;  // message action id -> its first ordinal
  o += ((A_NUM + 1) & ~1) * 2;
  o = (o + 7) & ~7;
  // phase B only (dead in phase C, where the dedup table reuses the bytes)
  L.off_Mask = o;  // per fixed binding: the tile's parents that pass may_enable (64-bit masks)
  L.off_Hash = o;  // phase C: DEDUP fingerprints (8 B) + DEDUP representatives (4 B)
  o += nfixed * 8;
  L.off_BOff = o;  // exclusive prefix over fixed bindings of the passing pairs
  o += (nfixed + 1) * 4;
  L.off_Live = o;  // per parent: bitmask over DOMAIN messages that can enable an action (msg_live)
  o += PB * L.lw * 4;
#if RMC_TILE_DEDUP
  const int hash_end = L.off_Hash + DEDUP * 12;  // DEDUP u32 slots + 256 u64 fingerprints
  o = o > hash_end ? o : hash_end;
#endif
  o = (o + 15) & ~15;
  L.off_S2 = o;  // persistent kernel: the second parent-row buffer (the next tile, in flight)
#if RMC_EXPAND_PERSIST
  o += PB * L.Wp * 4;
#endif
  L.bytes = o;
  return L;
}

// LDS-DMA: lane l of the wave loads the dword at gsrc into LDS byte address
// lds_dst + 4 l (lds_dst wave-uniform).  Written as asm so that hipcc neither
// counts it (it would drain it with vmcnt(0) at every barrier and before every
// LDS read it cannot prove disjoint) nor reorders LDS accesses across it; its
// completion is waited for explicitly (vmcnt(0) + a barrier) before the
// buffer is read.  M0 is saved and restored in the same statement.
__device__ __forceinline__ void lds_dma_dword(const uint32_t* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// Rows [p0, p0 + np) of the frontier -> LDS rows of stride Wp words at dst,
// by LDS-DMA: wave w takes rows w, w+4, ..., one instruction per 64 words of
// a row (lanes past the row's end masked off), so the padded stride is kept.
__device__ __forceinline__ void stage_rows_async(const uint32_t* __restrict__ frontier, unsigned long long p0, int np,
                                                 int words, int Wp, uint32_t* dst) {
  const int wv = threadIdx.x / WAVE, l = lane_id();
  for (int p = wv; p < np; p += 256 / WAVE) {
    const uint32_t* row = frontier + (p0 + p) * (unsigned long long)words;
    const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_addr(dst + p * Wp));
    for (int c = 0; c < words; c += WAVE)
      if (c + l < words) lds_dma_dword(row + c + l, base + 4u * (uint32_t)c);
  }
}
__device__ __forceinline__ void wait_lds_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// The same rows through registers (rows are a multiple of 4 words, 16 B
// aligned: 16 B loads, 4 LDS writes each).  (Staging only each row's used
// words -- headers first, then the 16 B units up to the last message -- was
// measured and rejected: k_expand 852 vs 829 ms, k_materialize 447 vs 432 per
// check; the dependent header load costs more than the bytes it saves.
// profiles/r04/ab_stage_trim_r04u.txt)
__device__ __forceinline__ void stage_rows_sync(const uint32_t* __restrict__ frontier, unsigned long long p0, int np,
                                                int words, int Wp, uint32_t* dst) {
  const uint4* src = reinterpret_cast<const uint4*>(frontier + p0 * (unsigned long long)words);
  for (int q = threadIdx.x; q < np * (words >> 2); q += 256) {
    const int w = q << 2, p = w / words;
    const uint4 v = src[q];
    uint32_t* d = dst + p * Wp + (w - p * words);
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
}

// The same copy with every load of a batch issued before the batch's first
// LDS write (NT threads, up to U 16 B loads per thread per batch).  Written as
// a plain loop, hipcc waits for each load (vmcnt(0)) before the next
// iteration issues its own: one dependent HBM round trip per 16 B step, i.e.
// three per 64-row tile of the bench workload in k_expand (256 threads) and
// six in k_materialize (128 threads), all on the block's critical path.
template <int NT, int U>
__device__ __forceinline__ void stage_rows_batched(const uint32_t* __restrict__ frontier, unsigned long long p0,
                                                   int np, int words, int Wp, uint32_t* dst) {
  const uint4* src = reinterpret_cast<const uint4*>(frontier + p0 * (unsigned long long)words);
  const int nq = np * (words >> 2);
  for (int q0 = (int)threadIdx.x; q0 < nq; q0 += NT * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (q0 + u * NT < nq) v[u] = src[q0 + u * NT];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int q = q0 + u * NT;
      if (q < nq) {
        const int w = q << 2, p = w / words;
        uint32_t* d = dst + p * Wp + (w - p * words);
        d[0] = v[u].x;
        d[1] = v[u].y;
        d[2] = v[u].z;
        d[3] = v[u].w;
      }
    }
  }
}

__device__ __forceinline__ int select_bit(const uint32_t* w, int j) {  // j-th set bit (0-based)
  for (int q = 0;; q++) {
    uint32_t x = w[q];
    int c = __popc(x);
    if (j < c) {
      for (int k = 0; k < j; k++) x &= x - 1u;
      return 32 * q + (__ffs(x) - 1);
    }
    j -= c;
  }
}
__device__ __forceinline__ int select_bit64(unsigned long long x, int r) {  // r-th set bit of x (0-based), in registers
  int pos = 0, c;
  c = __popc((uint32_t)x); if (r >= c) { r -= c; x >>= 32; pos += 32; }
  c = __popc((uint32_t)x & 0xFFFFu); if (r >= c) { r -= c; x >>= 16; pos += 16; }
  c = __popc((uint32_t)x & 0xFFu); if (r >= c) { r -= c; x >>= 8; pos += 8; }
  c = __popc((uint32_t)x & 0xFu); if (r >= c) { r -= c; x >>= 4; pos += 4; }
  c = __popc((uint32_t)x & 0x3u); if (r >= c) { r -= c; x >>= 2; pos += 2; }
  return pos + (r >= (int)(x & 1u) ? 1 : 0);
}
__device__ __forceinline__ int rank_below(const uint32_t* w, int bit) {  // set bits below `bit`
  int r = 0;
  for (int q = 0; q < (bit >> 5); q++) r += __popc(w[q]);
  uint32_t m = (bit & 31) ? ((1u << (bit & 31)) - 1u) : 0u;
  return r + __popc(w[bit >> 5] & m);
}

// One block = one tile of PB consecutive parents, 256 threads.
//   A: parents -> LDS (coalesced, odd row stride).
//   B: lane-per-parent binding evaluation.  Within a wave every lane runs the
//      SAME binding of a different parent, so the fixed-binding actions are
//      wave-uniform; enabled bindings and their TLC ordinals go to per-parent
//      LDS bitmasks.
//   C: lane-per-successor.  The tile's enabled (parent, binding) pairs are
//      enumerated densely; each lane rebuilds its successor delta, computes
//      the canonical fingerprint of parent+delta (delta_fp: signature-pruned
//      permutations, rmc_spec.h) and inserts it.  Candidates are laid out per
//      parent in TLC ordinal order.
// Occupancy target (waves per SIMD) for k_expand: 8 caps it at 64 VGPRs with
// no extra scratch for N <= 4, 4% faster than the compiler's 78-VGPR choice
// on the bench workload (1.289 s vs 1.340 s).
// The persistent form holds two parent-row buffers (about 31 KB of LDS per
// block on the bench workload): at most 5 blocks per CU fit, so it is
// compiled for 5 waves per SIMD (96 VGPRs; at 7 its tile loop spilled 49
// VGPRs to scratch).
#ifndef RMC_EXPAND_WAVES
#if RMC_EXPAND_PERSIST
#define RMC_EXPAND_WAVES 5
#else
#define RMC_EXPAND_WAVES 7
#endif
#endif
// FPW: fingerprint width in 64-bit words (1, or 2 for fp_bits = 128).
template <int N, int FPW>
struct SumsOf {
  using T = MsgSums<N>;
};
template <int N>
struct SumsOf<N, 2> {
  using T = MsgSums2<N>;
};
template <int N>
__device__ __forceinline__ MsgSums<N>& sums1(MsgSums<N>& m) { return m; }
template <int N>
__device__ __forceinline__ MsgSums<N>& sums1(MsgSums2<N>& m) { return m.m; }
template <int SPEC, int N, int FPW, bool G = false>
// waves per SIMD: as many as fit without scratch spills (N >= 4 and 128-bit
// fingerprints need more registers; a spill costs a scratch store per binding)
// G: the instantiation for models with compiled guards or actions (rmc_guard.cpp):
// 5 waves at N <= 3, so the guard/effect machine's registers do not spill
__global__ __launch_bounds__(256, (N >= 5 ? (FPW == 2 ? 2 : 3) : N == 4 ? (FPW == 2 ? 3 : 4) : FPW == 2 ? 4 : G ? 5 : RMC_EXPAND_WAVES)) void k_expand(const uint32_t* __restrict__ frontier, unsigned long long nparents,
                                                unsigned long long pbase, unsigned long long floor, int sharded,
                                                int shard_self,
                                                unsigned long long* __restrict__ table, unsigned long long mask,
                                                unsigned long long* __restrict__ cand_slot,
                                                uint32_t* __restrict__ cand_ob, uint32_t* __restrict__ par_off,
                                                uint32_t* __restrict__ par_n,
                                                unsigned long long* __restrict__ counters, unsigned long long cand_cap,
                                                DevStatus* st, unsigned long long* __restrict__ cand_val
#ifdef RMC_DIAG
                                                , int diag
#endif
                                                ) {
#ifndef RMC_DIAG
  constexpr int diag = 0;  // RMC_DIAG builds: stop after a phase (4: staging, 3: bindings, 2: + successor
                           // deltas, 1: + fingerprints and tile dedup, no global insert)
#endif
  constexpr int PB = Tile<N>::PB;
  extern __shared__ __align__(16) unsigned char lds[];
  __shared__ unsigned long long sG;
  __shared__ int sOver;
  __shared__ int sAFirst[MAXACT], sAEnd[MAXACT], sAChunk[MAXACT + 1];
#if RMC_ACT_MAJOR
  __shared__ uint16_t sAOff[MAXACT + 1];  // action slot -> its first ordinal (Model::act_off), + ordinal_limit
  __shared__ uint8_t sMSlot[A_NUM];       // message action id -> its action slot (Model::msg_act_slot)
#endif
  using MS = typename SumsOf<N, FPW>::T;
  // the tile's LDS arrays (the same layout in both kernel forms)
#define RMC_EXPAND_LDS_ARRAYS                                                                         \
  const int words = cM.words, ordw = cM.ord_words;                                                     \
  const ExpandLds L = expand_lds(PB, words, ordw, (int)sizeof(MS), cM.nfixed, cM.ordinal_limit, cM.kmax, cM.nact); \
  MS* sMS = (MS*)(lds + L.off_Ms);                                                                     \
  uint32_t* sOrd = (uint32_t*)(lds + L.off_Ord);                                                       \
  base_t* sBase = (base_t*)(lds + L.off_Base);                                                         \
  uint32_t* sLive = (uint32_t*)(lds + L.off_Live);                                                     \
  unsigned long long* sMask = (unsigned long long*)(lds + L.off_Mask);                                 \
  uint32_t* sBOff = (uint32_t*)(lds + L.off_BOff);                                                     \
  uint32_t* sDesc = (uint32_t*)(lds + L.off_Desc);                                                     \
  uint16_t* sO2b = (uint16_t*)(lds + L.off_O2b);                                                       \
  uint16_t* sMOff = (uint16_t*)(lds + L.off_MOff);                                                     \
  uint16_t* sAP = (uint16_t*)(lds + L.off_AP);                                                          \
  (void)sMS, (void)sOrd, (void)sBase, (void)sLive, (void)sMask, (void)sBOff, (void)sDesc, (void)sO2b, (void)sMOff, (void)sAP;
#ifdef RMC_STAMPS
  unsigned long long t_prev = clock64();
#endif
#if RMC_EXPAND_PERSIST
  // ---- A: the block's tiles are blockIdx.x, blockIdx.x + G, ...  Tile t's
  //      rows were put in flight (LDS-DMA) before tile t-G's phase B; the
  //      wait below retires them, and tile t+G's go in flight into the other
  //      buffer, whose last reader (tile t-G's phase C) is past the barrier.
  //      Every tile is walked even after a capacity flag: k_mark and the scan
  //      run before the host reads the flags, and they read every parent's
  //      par_off / par_n.  (An early exit on the flag left them stale -- a
  //      fault in k_mark on a fresh model's message-slot widening.)
  const unsigned long long ntiles = (nparents + PB - 1) / PB;
  {
    const int tid = threadIdx.x;
    RMC_EXPAND_LDS_ARRAYS
    // the model's binding tables: once per block
    for (int q = tid; q < cM.nfixed; q += 256) sDesc[q] = cM.fb_desc[q];
    for (int q = tid; q < cM.ordinal_limit; q += 256) sO2b[q] = cM.ord2b[q];
    for (int q = tid; q < A_NUM; q += 256) sMOff[q] = (uint16_t)cM.act_off[cM.msg_act_slot[q]];
    if (blockIdx.x < ntiles && lds_addr(lds) + (uint32_t)L.bytes <= 65536u)
      stage_rows_async(frontier, blockIdx.x * (unsigned long long)PB,
                       (int)min((unsigned long long)PB, nparents - blockIdx.x * (unsigned long long)PB), words, L.Wp,
                       (uint32_t*)lds);
  }
  unsigned long long tile = blockIdx.x;
  for (int buf = 0; tile < ntiles; tile += gridDim.x, buf ^= 1) {
    // Everything per lane or per model is re-derived here from values the
    // compiler cannot see are the same every tile (the thread id, the model's
    // address): otherwise it hoists the lane addresses, masks and model loads
    // of the whole body out of the walk and holds them live across it -- 76
    // VGPRs of scratch spills at the 7-wave register budget.
    int tid_ = threadIdx.x;
    asm volatile("" : "+v"(tid_));
    const int tid = tid_;
    const __attribute__((address_space(4))) Model* mp4 = (const __attribute__((address_space(4))) Model*)&cM;
    asm volatile("" : "+s"(mp4));
    const Model& tM = *(const Model*)mp4;
#define cM tM
    RMC_EXPAND_LDS_ARRAYS
    uint32_t* sS = (uint32_t*)(lds + (buf ? L.off_S2 : 0));
    const unsigned long long p0 = tile * PB;
    const int np = (int)((nparents - p0) < (unsigned long long)PB ? (nparents - p0) : PB);
    wait_lds_dma();
    __syncthreads();  // the tile's rows have landed; the previous tile's phase C is done with every LDS array
    // (LDS-DMA takes its destination from M0, of which only the low 16 bits
    // are trusted here: a layout past 64 KB -- rows widened near their cap on
    // N = 5 -- stages each tile synchronously instead)
    if (lds_addr(lds) + (uint32_t)L.bytes > 65536u) {
      stage_rows_sync(frontier, p0, np, words, L.Wp, sS);
    } else if (tile + gridDim.x < ntiles) {
      const unsigned long long q0 = (tile + gridDim.x) * PB;
      stage_rows_async(frontier, q0, (int)min((unsigned long long)PB, nparents - q0), words, L.Wp,
                       (uint32_t*)(lds + (buf ? 0 : L.off_S2)));
    }
    for (int q = tid; q < PB * ordw; q += 256) sOrd[q] = 0;
    for (int q = tid; q < PB * L.lw; q += 256) sLive[q] = 0;
    for (int q = tid; q < PB * (int)(sizeof(MS) / 4); q += 256) ((uint32_t*)sMS)[q] = 0;
    __syncthreads();
#else
  for (int once = 0; once < 1; once++) {  // one tile per block (`continue` ends it)
    const int tid = threadIdx.x;
    RMC_EXPAND_LDS_ARRAYS
    uint32_t* sS = (uint32_t*)lds;
    const unsigned long long p0 = xcd_tile(blockIdx.x, gridDim.x) * PB;
    const int np = (int)((nparents - p0) < (unsigned long long)PB ? (nparents - p0) : PB);
    // ---- A: stage the tile (contiguous in HBM) into padded LDS rows, and the
    //      model's binding tables.  Every load of a thread -- table entries
    //      first, then its rows' 16 B pieces -- is issued before its first
    //      LDS write: one memory round trip for the phase instead of one per
    //      16 B step and per table (RMC_STAGE_BATCH=0: the loop form).
#if RMC_STAGE_BATCH
    static_assert(MAXFIXED <= 256 && A_NUM <= 256, "one table entry per thread");
    const uint32_t vdesc = tid < cM.nfixed ? cM.fb_desc[tid] : 0u;
    const uint32_t vmoff = tid < A_NUM ? (uint32_t)cM.msg_off[tid] : 0u;
    uint32_t vo2b[4];  // ordinal_limit < 1024
    // each action slot's fixed bindings (phase B's chunk table, wave 0)
    const int vfirst = tid < cM.nact ? (int)cM.act_fb_first[tid] : 0, vend = tid < cM.nact ? (int)cM.act_fb_end[tid] : 0;
#if RMC_ACT_MAJOR
    const int vaoff = tid < cM.nact ? cM.act_off[tid] : cM.ordinal_limit;
    const int vmslot = tid < A_NUM ? cM.msg_act_slot[tid] : 0;
#endif
#pragma unroll
    for (int u = 0; u < 4; u++) vo2b[u] = tid + 256 * u < cM.ordinal_limit ? (uint32_t)cM.ord2b[tid + 256 * u] : 0u;
    stage_rows_batched<256, 4>(frontier, p0, np, words, L.Wp, sS);
    if (tid < cM.nfixed) sDesc[tid] = vdesc;
    if (tid < A_NUM) sMOff[tid] = (uint16_t)vmoff;
#if RMC_ACT_MAJOR
    if (tid <= cM.nact) sAOff[tid] = (uint16_t)vaoff;
    if (tid < A_NUM) sMSlot[tid] = (uint8_t)vmslot;
    for (int q = tid; q < (cM.nact * PB + 2) / 2; q += 256) ((uint32_t*)sAP)[q] = 0;
#endif
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (tid + 256 * u < cM.ordinal_limit) sO2b[tid + 256 * u] = (uint16_t)vo2b[u];
#else
    stage_rows_sync(frontier, p0, np, words, L.Wp, sS);
    for (int q = tid; q < cM.nfixed; q += 256) sDesc[q] = cM.fb_desc[q];
    for (int q = tid; q < cM.ordinal_limit; q += 256) sO2b[q] = cM.ord2b[q];
    for (int q = tid; q < A_NUM; q += 256) sMOff[q] = (uint16_t)cM.act_off[cM.msg_act_slot[q]];
#endif
    for (int q = tid; q < PB * ordw; q += 256) sOrd[q] = 0;
    for (int q = tid; q < PB * L.lw; q += 256) sLive[q] = 0;
    for (int q = tid; q < PB * (int)(sizeof(MS) / 4); q += 256) ((uint32_t*)sMS)[q] = 0;
    __syncthreads();
#endif
  STAMP(0);
  if (diag == 4) {  // staging only (a checksum keeps it live)
    uint32_t x = 0;
    for (int q = tid; q < np * words; q += 256) x ^= sS[(q / words) * L.Wp + q % words];
    if (tid < np) par_n[p0 + tid] = x;
    continue;
  }
  // ---- B: enabled bindings, lane per parent
  {
    const int p = tid % PB, bstride = 256 / PB;
    if (p < np) {
      PState<SPEC, N> s{sS + p * L.Wp};
      const int nm = s.nmsg();
      // the parent's message sums (MsgSums): each of its messages hashed once
      // here instead of once per successor in phase C; and which messages can
      // enable an action at all (84% of DOMAIN messages cannot on the bench
      // workload: delivered, and not newer than their receiver)
      // (Summing a lane's share in registers and publishing one LDS atomic
      // per nonzero word was measured and rejected: k_expand 839 vs 827 ms
      // per check, profiles/r04/ab_sums_reg_r04y.txt.)
      for (int k = tid / PB; k < nm; k += bstride) {
        int src, dst;
        const uint32_t w = s.msg(k);
        if (msg_live<SPEC, N>(s, w)) atomicOr(&sLive[p * L.lw + (k >> 5)], 1u << (k & 31));
        const uint64_t u = msg_u<SPEC>(w, src, dst);
        MsgSums<N>& m1 = sums1<N>(sMS[p]);
        atomicAdd(&m1.sig[src], (uint32_t)u);
        atomicAdd(&m1.sig[dst], (uint32_t)(u >> 32));
        if (src != dst) atomicAdd((unsigned long long*)&m1.S[MsgSums<N>::pair(src, dst)], (unsigned long long)u);
        if constexpr (FPW == 2) {
          if (src != dst)
            atomicAdd((unsigned long long*)&sMS[p].S2[MsgSums<N>::pair(src, dst)],
                      (unsigned long long)msg_u2<SPEC>(w));
        }
      }
    }
    STAMP(15);  // message sums done (diagnostic build: phase B split)
    // eval_one: one (parent pp, binding b) pair; enabled -> the ordinal bit,
    // errors and message-capacity overflow flagged
    auto record = [&](int pp, int b, const Delta& d, int slot) {
#if RMC_ACT_MAJOR
      atomicAdd((uint32_t*)sAP + ((slot * PB + pp) >> 1), 1u << (16 * (pp & 1)));
#else
      (void)slot;
#endif
      if (d.err) {
        if (d.err == E_DOMAIN) atomicMin(&st->err_key, order_key(pbase + p0 + pp, d.ordinal, b));
        else atomicOr(&st->cap_flags, 1u << d.err);
      } else {
        int adds = 0;
#pragma unroll
        for (int q = 0; q < MAXOPS; q++) adds += (q < d.nops && d.opk[q] < 0);
        const int nn = h_nmsg(sS[pp * L.Wp]) + adds;
        if (nn > cM.kmax) {  // the row needs more message slots: the driver widens the rows (rmc_engine.cpp)
          atomicOr(&st->cap_flags, 1u << E_CAP_MSG);
          atomicMax(&st->max_msgs, (unsigned)nn);
        }
      }
      atomicOr(&sOrd[pp * ordw + (d.ordinal >> 5)], 1u << (d.ordinal & 31));
    };
    // Fixed bindings.  (1) guard masks: wave w0 takes bindings w0, w0+4, ...,
    // its lanes the tile's parents; bit p of sMask[b] = may_enable(parent p,
    // b), the guard's leading conjuncts.  (2) The pairs that pass, grouped by
    // action and padded to whole waves: every wave step runs ONE action's code
    // (a scalar branch) on 64 (parent, binding) pairs, instead of one binding
    // for 64 parents of which most fail its guard.
    const int w0 = tid / PB;
    for (int b = w0; b < cM.nfixed; b += bstride) {
      bool g = false;
      if (p < np) {
        PState<SPEC, N> s{sS + p * L.Wp};
        g = may_enable_d<SPEC, N, G>(s, cM, sDesc[b]);  // the descriptor from LDS, not a vector load per binding
      }
      const unsigned long long m = __ballot(g);
      if (p == 0) sMask[b] = m;
    }
    __syncthreads();
    STAMP(16);  // guard masks done
    if (tid < WAVE) {  // sBOff = exclusive prefix over bindings of the pairs that pass
      unsigned carry = 0;
      for (int b0 = 0; b0 < cM.nfixed; b0 += WAVE) {
        const int b = b0 + tid;
        const unsigned c = b < cM.nfixed ? (unsigned)__popcll(sMask[b]) : 0u;
        unsigned incl = c;
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {
          unsigned y = __shfl_up(incl, o, WAVE);
          if (tid >= o) incl += y;
        }
        if (b < cM.nfixed) sBOff[b] = carry + incl - c;
        carry += __shfl(incl, WAVE - 1, WAVE);
      }
      if (tid == 0) sBOff[cM.nfixed] = carry;
    }
#if RMC_STAGE_BATCH
    // the chunk table below is wave 0's too: its sBOff reads need only this
    // wave's writes done (one block barrier fewer per tile: k_expand 657-658
    // vs 662-665 ms per check, profiles/r06/ab_phase_b_barriers.txt; building
    // the table in every wave to drop the next barrier too measured 662-664)
    if (tid < WAVE) wave_lds_sync();
#else
    __syncthreads();
#endif
    if (tid < WAVE) {  // per action slot (lane): its first wave-sized chunk of passing pairs
      const int a = tid;
      int c = 0;
      if (a < cM.nact) {
#if RMC_STAGE_BATCH
        const int f = vfirst, e = vend;  // loaded in phase A
#else
        const int f = cM.act_fb_first[a], e = cM.act_fb_end[a];
#endif
        sAFirst[a] = f;
        sAEnd[a] = e;
        c = ((int)(sBOff[e] - sBOff[f]) + WAVE - 1) / WAVE;
      }
      int incl = c;
#pragma unroll
      for (int o = 1; o < WAVE; o <<= 1) {
        int y = __shfl_up(incl, o, WAVE);
        if (tid >= o) incl += y;
      }
      if (a <= cM.nact) sAChunk[a] = incl - c;
    }
    __syncthreads();
    STAMP(17);  // pair prefix + action chunk table done
    {
      const int nchunks = sAChunk[cM.nact];
      for (int c = w0; c < nchunks; c += bstride) {
        int a = 0;
        while (sAChunk[a + 1] <= c) a++;
        a = __builtin_amdgcn_readfirstlane(a);  // wave-uniform: the action dispatch is a scalar branch
        const int g = (int)sBOff[sAFirst[a]] + (c - sAChunk[a]) * WAVE + p;
        if (g < (int)sBOff[sAEnd[a]]) {
          int lo = sAFirst[a], hi = sAEnd[a] - 1;  // binding: sBOff[lo] <= g < sBOff[lo + 1]
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((int)sBOff[mid] <= g) lo = mid; else hi = mid - 1;
          }
          const int pp = select_bit64(sMask[lo], g - (int)sBOff[lo]);
          PState<SPEC, N> s{sS + pp * L.Wp};
          Delta d;
          // (x from the LDS descriptor: a per-lane cM.fb_x load was a dependent round trip per chunk)
          if (eval_fixed<SPEC, N, G>(s, cM, a, (int)((sDesc[lo] >> 8) & 0xFFu), d)) record(pp, lo, d, a);
        }
      }
    }
    STAMP(1);  // fixed bindings done (diagnostic build: phase B split)
    if (p < np) {
      PState<SPEC, N> s{sS + p * L.Wp};
      const int nm = s.nmsg();
      (void)nm;
#ifdef RMC_STAMPS
      {  // binding statistics: message bindings, live ones (act_message's fast reject passes), wave steps
        const int B = cM.nfixed + nm;
        int live = 0;
        for (int k = 0; k < nm; k++) {
          const uint32_t w = s.msg(k);
          live += !(msg_count(w) == 0 && msg_term<SPEC>(w) <= a_term(s.A(msg_dst<SPEC>(w))));
        }
        int steps = (B - w0 + bstride - 1) / bstride, lsteps = (cM.nfixed + live - w0 + bstride - 1) / bstride;
        for (int o = 32; o > 0; o >>= 1) {
          steps = max(steps, __shfl_xor(steps, o, WAVE));
          lsteps = max(lsteps, __shfl_xor(lsteps, o, WAVE));
        }
        if (w0 == 0) {
          atomicAdd(&g_stamps[8], 1ULL);
          atomicAdd(&g_stamps[9], (unsigned long long)nm);
          atomicAdd(&g_stamps[10], (unsigned long long)live);
        }
        if ((tid & (WAVE - 1)) == 0) {
          atomicAdd(&g_stamps[11], (unsigned long long)steps);
          atomicAdd(&g_stamps[12], (unsigned long long)lsteps);
        }
        if (tid == 0) atomicAdd(&g_stamps[13], (unsigned long long)sBOff[cM.nfixed]);  // fixed pairs passing the guard
        if (tid == 0) atomicAdd(&g_stamps[14], (unsigned long long)sAChunk[cM.nact]);  // their wave chunks
      }
#endif
      // the parent's live messages, every 4th one per wave
      int t = 0;
      for (int q = 0; q < L.lw; q++) {
        uint32_t x = sLive[p * L.lw + q];
        while (x) {
          const int k = 32 * q + __ffs(x) - 1;
          x &= x - 1u;
          if ((t++ & (bstride - 1)) == w0) {
            Delta d;
            d.srv = -1; d.nops = 0; d.hdr = s.hdr(); d.err = 0; d.act = -1;
            if (act_message<SPEC, N>(s, cM, k, d)) {
              d.ordinal = sMOff[d.act] + k;
#if RMC_ACT_MAJOR
              record(p, cM.nfixed + k, d, sMSlot[d.act]);
#else
              record(p, cM.nfixed + k, d, 0);
#endif
            }
          }
        }
      }
      if constexpr (G) {
        // compiled message handlers (rmc_guard.cpp compile_handler): every DOMAIN
        // element, each handler on its own (no live-message prefilter: the
        // compiled guard alone decides)
        for (int c = 0; c < cM.nmsgc; c++) {
          const int q = cM.msgc_q[c];
          const int off = sMOff[A_C0 + q];
          for (int k = 0; k < nm; k++)
            if ((t++ & (bstride - 1)) == w0) {
              Delta d;
#if RMC_ACT_MAJOR
              if (eval_msgc<SPEC, N>(s, cM, q, k, off + k, d))
                record(p, cM.nfixed + MSGC_STRIDE * (1 + q) + k, d, sMSlot[A_C0 + q]);
#else
              if (eval_msgc<SPEC, N>(s, cM, q, k, off + k, d)) record(p, cM.nfixed + MSGC_STRIDE * (1 + q) + k, d, 0);
#endif
            }
        }
      }
    }
  }
  __syncthreads();
  STAMP(2);
  // ---- per-parent successor counts -> tile prefix (wave 0), one global reservation per tile
  if (tid < 64) {
    int c = 0;
    if (tid < np)
      for (int q = 0; q < ordw; q++) c += __popc(sOrd[tid * ordw + q]);  // one ordinal per enabled binding
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      int y = __shfl_up(incl, o, WAVE);
      if (tid >= o) incl += y;
    }
    if (tid < PB) sBase[tid + 1] = (base_t)incl;
    if (tid == 0) sBase[0] = 0;
    int total = __shfl(incl, 63, WAVE);
    // one reservation per tile.  The single-shard search spreads them over 8
    // counters (one per XCD, 128 B apart) and 8 segments of the candidate
    // buffer: one counter for the whole grid serialized ~3x10^4 returning
    // atomics per launch on one address.  The sharded search needs its
    // candidates dense, so it keeps one counter.
    if (tid == 0) {
#if RMC_EXPAND_PERSIST
      const int seg = sharded ? 0 : (int)((p0 / PB) & (EXPAND_SEGS - 1));
#else
      const int seg = sharded ? 0 : (int)(blockIdx.x & (EXPAND_SEGS - 1));  // the block's XCD label
#endif
#if RMC_TILE_SLOTS
      if (!sharded) {
        // a fixed slot range per tile (the buffer holds PB x min(maxsucc,
        // 256) candidates per tile: cand_cap's sizing), so the base needs no
        // returning atomic -- the tile's count is added for the host
        // (generated states) by an atomic whose result nobody waits for
        const unsigned long long tcap = (unsigned long long)PB * (unsigned long long)min(max_successors(cM), 256);
        const unsigned long long g0 = (p0 / PB) * tcap;
        if (total) atomicAdd(&counters[16 * seg], (unsigned long long)total);
        sG = g0;
        sOver = (unsigned long long)total > tcap || g0 + (unsigned long long)total > cand_cap;
      } else
#endif
      {
        const unsigned long long seg_cap = sharded ? cand_cap : cand_cap / EXPAND_SEGS;
        const unsigned long long c = total ? atomicAdd(&counters[16 * seg], (unsigned long long)total) : 0ULL;
        sG = seg * seg_cap + c;
        sOver = c + (unsigned long long)total > seg_cap;  // (c itself may be past the segment: no modulo test)
      }
    }
  }
#if RMC_ACT_MAJOR
  if (tid >= 64 && tid < 128) {  // wave 1, beside wave 0's reservation: the flattened
    // exclusive prefix over (action slot, parent) of phase B's counts, in place;
    // sAP[nact * PB] = the tile's total
    const int l = tid - 64;
    unsigned carry = 0;
    for (int a = 0; a < cM.nact; a++) {
      const unsigned c = sAP[a * PB + l];
      unsigned incl = c;
#pragma unroll
      for (int o = 1; o < WAVE; o <<= 1) {
        const unsigned y = __shfl_up(incl, o, WAVE);
        if (l >= o) incl += y;
      }
      sAP[a * PB + l] = (uint16_t)(carry + incl - c);
      carry += __shfl(incl, WAVE - 1, WAVE);
    }
    if (l == 0) sAP[cM.nact * PB] = (uint16_t)carry;
  }
#endif
#if RMC_TILE_DEDUP
  // phase C's dedup table for round 0 (its bytes are phase B's, dead now)
  if (FPW == 1 && !sharded) ((uint32_t*)(lds + L.off_Hash))[tid] = ~0u;
#endif
  __syncthreads();
  const int total = (int)sBase[np];
  const unsigned long long gbase = sG;
  if (tid < np) {
    par_off[p0 + tid] = (uint32_t)(gbase + sBase[tid]);
    par_n[p0 + tid] = sBase[tid + 1] - sBase[tid];
  }
  if (sOver) {
    if (tid == 0) atomicOr(&st->cap_flags, 1u << E_CAP_SUCC);
    continue;
  }
  if (diag == 3) continue;  // bindings only
#ifdef RMC_STAMPS
  // diagnostic: phase C without the fingerprint-set inserts (stamp 7), so the
  // inserts' share is the difference from the real phase C (stamp 3)
  {
    __shared__ unsigned long long sSink;
    unsigned long long acc = 0;
    for (int idx = tid; idx < total; idx += 256) {
      int lo = 0, hi = np - 1;
      while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if ((int)sBase[mid] <= idx) lo = mid; else hi = mid - 1;
      }
      const int p = lo;
      const int ord = select_bit(sOrd + p * ordw, idx - (int)sBase[p]);
      const int b = sO2b[ord];
      PState<SPEC, N> s{sS + p * L.Wp};
      Delta d;
      eval_known<SPEC, N, G>(s, cM, b, b < cM.nfixed ? sDesc[b] : 0u, ord, d);
      if constexpr (FPW == 2) {
        if (!d.err) acc ^= delta_fp_sums2<SPEC, N>(s, cM, d, sMS[p]).b;
      } else {
        if (!d.err) acc ^= delta_fp_sums<SPEC, N>(s, cM, d, sMS[p]);
      }
    }
    if (acc == 0x123456789ULL) sSink = acc;
    __syncthreads();
    if (tid == 0) {
      unsigned long long t_ = clock64();
      atomicAdd(&g_stamps[7], t_ - t_prev);
      t_prev = t_;
    }
  }
#endif
  // ---- C: fingerprints + inserts, lane per successor.  The tile's
  //      successors are enumerated parent-major in TLC ordinal order, which
  //      is exactly their order in the candidate buffer: lane idx writes
  //      candidate gbase + idx, so a wave's candidate stores are contiguous
  //      (binding-major enumeration scattered them: one 32 B write request per
  //      8 B store, ~0.7 GB of extra HBM writes per launch on the bench cfg).
#if RMC_TILE_DEDUP
  // Tile-local dedup of the inserts (single shard, 64-bit fingerprints).
  // Phase C's successors come in rounds of 256 (lane = tid).  Successors of
  // the same round with the same fingerprint (commuting actions of sibling
  // parents) send ONE insert to the HBM set: the lowest round index, which is
  // the lowest TLC rank, since candidates are numbered in TLC order.  The
  // others could never lower that entry's minimum.  They store CAND_REF |
  // hidden << 47 | the representative's candidate index, and k_mark_tiles
  // reads the entry through it (never a winner; hidden collisions are
  // counted as if they had inserted).  The LDS table: DEDUP u32 slots, each
  // holding the lowest round index of its key (~0 = empty), plus the round's
  // fingerprints by index for the key compare.  Unlike the r03 form (three
  // barriers per round; the others waited for their representative's insert
  // to learn its slot), one barrier per round, and no lane waits on another's
  // HBM insert.  Round 0's table is cleared before the reservation barrier.
  if constexpr (FPW == 1) {
    if (!sharded && !diag) {
      uint32_t* sDT = (uint32_t*)(lds + L.off_Hash);
      unsigned long long* sDF = (unsigned long long*)(lds + L.off_Hash + DEDUP * 4);
      for (int r0 = 0; r0 < total; r0 += 256) {
        if (r0) {  // the previous round is done with the table
          __syncthreads();
          sDT[tid] = ~0u;
          __syncthreads();
        }
        const int idx = r0 + tid;
        const bool act = idx < total;
        uint32_t obw = OB_ERR;
        unsigned long long fp = 0, val = 0;
        int h = 0;
        if (act) {
          int lo = 0, hi = np - 1;  // parent p: sBase[p] <= idx < sBase[p+1]
          while (lo < hi) {
            int mid = (lo + hi + 1) >> 1;
            if ((int)sBase[mid] <= idx) lo = mid; else hi = mid - 1;
          }
          const int p = lo;
          const int ord = select_bit(sOrd + p * ordw, idx - (int)sBase[p]);
          const int b = sO2b[ord];
          PState<SPEC, N> s{sS + p * L.Wp};
          Delta d;
          eval_known<SPEC, N, G>(s, cM, b, b < cM.nfixed ? sDesc[b] : 0u, ord, d);
          obw = ((uint32_t)d.ordinal << 16) | (uint32_t)b | (d.err ? OB_ERR : 0u);
          if (!d.err) {
            const unsigned long long pg = pbase + p0 + p;
            val = ((((pg + 1) << 10) | (unsigned long long)d.ordinal) << VAL_RANK_SHIFT) |
                  (unsigned long long)hidden_of<SPEC>(d.hdr);
            fp = delta_fp_sums<SPEC, N>(s, cM, d, sums1<N>(sMS[p]));
            sDF[tid] = fp;  // before the claim below: a lane that finds tid in a slot reads it
            asm volatile("" ::: "memory");
            h = (int)((fp ^ (fp >> 31)) & (DEDUP - 1));
            for (;;) {  // at most 256 keys in DEDUP slots: a slot is always found
              const uint32_t v = atomicCAS(&sDT[h], ~0u, (uint32_t)tid);
              if (v == ~0u) break;
              if (sDF[v] == fp) {
                atomicMin(&sDT[h], (uint32_t)tid);
                break;
              }
              h = (h + 1) & (DEDUP - 1);
            }
          }
        }
        __syncthreads();
        unsigned long long slot = CAND_DUP;
        if (act && !(obw & OB_ERR)) {
          const uint32_t rep = sDT[h];
          if (rep == (uint32_t)tid) slot = cand_word(fpset_insert(table, mask, fp, val, floor, st), val);
          else slot = CAND_REF | ((val & 0xFFFFULL) << 47) | (gbase + (unsigned long long)(r0 + (int)rep));
        }
        if (act) {
          const unsigned long long t = gbase + (unsigned long long)idx;
          cand_slot[t] = slot;
          cand_ob[t] = obw;
        }
      }
      STAMP(3);
      continue;
    }
  }
#endif
  // (A wave-level dedup of equal fingerprints before the HBM probe -- a
  // 64-slot LDS table per wave, only each key's first lane probing -- was
  // measured and rejected: it cut the global inserts from 6.75e9 to 4.84e9,
  // the CAS from 4.10e9 to 2.65e9 and the atomicMin from 5.29e9 to 3.37e9 per
  // check, yet k_expand took 1,019 ms instead of 824: the LDS table costs
  // more than the HBM operations it saves.  profiles/r04/ab_wave_dedup_r04w.txt)
  for (int idx = tid; idx < total; idx += 256) {
#if RMC_ACT_MAJOR
    // lane idx -> (action slot a, parent p, its j-th successor of that action):
    // the last flattened entry whose prefix is <= idx (it has a successor)
    int lo = 0, hi = cM.nact * PB - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((int)sAP[mid] <= idx) lo = mid; else hi = mid - 1;
    }
    const int p = lo & (PB - 1), a = lo / PB;
    const int r = rank_below(sOrd + p * ordw, sAOff[a]) + (idx - (int)sAP[lo]);  // its rank among p's successors
    const int ord = select_bit(sOrd + p * ordw, r);
    const int pos = (int)sBase[p] + r;  // its TLC-order position in the tile
#else
    int lo = 0, hi = np - 1;  // parent p: sBase[p] <= idx < sBase[p+1]
    while (lo < hi) {
      int mid = (lo + hi + 1) >> 1;
      if ((int)sBase[mid] <= idx) lo = mid; else hi = mid - 1;
    }
    const int p = lo;
    const int ord = select_bit(sOrd + p * ordw, idx - (int)sBase[p]);
    const int pos = idx;
#endif
    const int b = sO2b[ord];
    PState<SPEC, N> s{sS + p * L.Wp};
    Delta d;
    eval_known<SPEC, N, G>(s, cM, b, b < cM.nfixed ? sDesc[b] : 0u, ord, d);
    const unsigned long long t = gbase + (unsigned long long)pos;
    const unsigned long long pg = pbase + p0 + p;
    unsigned long long slot = CAND_DUP;
    uint32_t local = 0;
    if (!d.err) {
      // TLC-order rank (parent global index, Next ordinal) above the hidden variables
      unsigned long long val = ((((pg + 1) << 10) | (unsigned long long)d.ordinal) << VAL_RANK_SHIFT) |
                               (unsigned long long)hidden_of<SPEC>(d.hdr);
      if constexpr (FPW == 2) {
        const Fp128 fp = delta_fp_sums2<SPEC, N>(s, cM, d, sMS[p]);
        slot = cand_word(fpset_insert128(table, mask, fp, val, floor, st), val);
      } else {
        unsigned long long fp = diag == 2 ? (unsigned long long)d.hdr ^ d.w[0] ^ d.opc[0]
                                          : delta_fp_sums<SPEC, N>(s, cM, d, sMS[p]);
        if (diag) {
          slot = fp;
        } else if (sharded) {  // the fp's owner inserts it: here when that is this shard, else k_insert_recv
          if (fp_owner(fp, sharded) == shard_self) {
            // as the single-shard search (a full table flags E_CAP_TABLE: the
            // round is redone), plus the fp: the table may grow before k_mark_gen
            slot = cand_word(fpset_insert(table, mask, fp, val, floor, st), val);
            cand_val[t] = fp;
            local = OB_LOCAL;
          } else {
            slot = fp;
            cand_val[t] = val;
          }
        } else {
          slot = cand_word(fpset_insert(table, mask, fp, val, floor, st), val);
        }
      }
    }
    cand_slot[t] = slot;
    cand_ob[t] = ((uint32_t)d.ordinal << 16) | (uint32_t)b | (d.err ? OB_ERR : local);
  }
  STAMP(3);
  }  // tile loop
#if RMC_EXPAND_PERSIST
#undef cM
#endif
#undef RMC_EXPAND_LDS_ARRAYS
#if RMC_EXPAND_PERSIST
  wait_lds_dma();  // (the last tile issues no prefetch: a guard that nothing is in flight at exit)
#endif
}

// One thread per parent: which of its candidates won their fingerprint, and
// each winner's rank among the parent's winners (candidates are stored in TLC
// ordinal order, so the rank is the output order).  cand_win = 1 + rank, 0 =
// lost.  A same-level loser whose hidden variables differ from the winner's is
// a hidden-variable collision (SURVEY.md §7 hard part 1), counted as the
// oracles count them.
__global__ __launch_bounds__(256) void k_mark(unsigned long long nparents, unsigned long long pbase,
                                              unsigned long long floor, int ew,
                                              const unsigned long long* __restrict__ table,
                                              const unsigned long long* __restrict__ cand_slot,
                                              const uint32_t* __restrict__ cand_ob,
                                              const uint32_t* __restrict__ par_off, const uint32_t* __restrict__ par_n,
                                              uint16_t* __restrict__ cand_win, uint32_t* __restrict__ par_win,
                                              DevStatus* st) {
  unsigned long long p = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nparents) return;
  uint32_t off = par_off[p], n = par_n[p];
  uint32_t cnt = 0, coll = 0;
  const unsigned long long base = (pbase + p + 1) << 10;  // ranks count parents from 1 (Init's val is 0)
  // the candidates' table reads are independent: issue up to 8 before using any
  constexpr int U = 8;
  for (uint32_t t0 = off; t0 < off + n; t0 += U) {
    uint32_t ob[U];
    unsigned long long sl[U], v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t t = t0 + u;
      ob[u] = t < off + n ? cand_ob[t] : OB_ERR;
      sl[u] = (ob[u] & OB_ERR) ? CAND_DUP : cand_slot[t];
      unsigned long long w = sl[u];
      if (!(w & CAND_DUP) && (w & CAND_REF)) w = cand_slot[w & CAND_REF_MASK];  // tile-dedup reference
      if (w & CAND_DUP) sl[u] = CAND_DUP;
      // entry = ew words, value in the word after the key (ew 2: fp, val; ew 4: fp.a, fp.b, val, -)
      v[u] = (w & CAND_DUP) ? ~0ULL : table[ew * (w & CAND_SLOT_MASK) + (ew >> 1)];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t t = t0 + u;
      if (t >= off + n) break;
      bool c = false;
      const bool win = !(sl[u] & CAND_DUP) && fpset_won(v[u], base | (ob[u] >> 16), floor, sl[u] >> 47, c);
      coll += c ? 1u : 0u;
      cand_win[t] = win ? (uint16_t)(++cnt) : (uint16_t)0;
    }
  }
  par_win[p] = cnt;
  if (coll) atomicAdd(&st->hidden_coll, (unsigned long long)coll);
}

// The same marking, a wave per k_expand tile (64 parents): a tile's
// candidates are one contiguous range, so the wave reads them coalesced, 64
// at a time, and ranks the winners inside each parent's segment with ballots
// (the parents' running counts carried in LDS from one 64-candidate step to
// the next).  The table reads stay random (only candidates k_expand did not
// already find in an earlier level).
#ifndef RMC_MARK_WPB
#define RMC_MARK_WPB 4
#endif
constexpr int MARK_WPB = RMC_MARK_WPB;  // waves (tiles) per k_mark_tiles block
#ifndef RMC_MARK_U
#define RMC_MARK_U 4
#endif
constexpr int MARK_U = RMC_MARK_U;  // 64-candidate steps whose loads are issued together
__global__ __launch_bounds__(MARK_WPB * WAVE) void k_mark_tiles(unsigned long long nparents, unsigned long long pbase,
                                                    unsigned long long floor, int ew,
                                                    const unsigned long long* __restrict__ table,
                                                    const unsigned long long* __restrict__ cand_slot,
                                                    const uint32_t* __restrict__ cand_ob,
                                                    const uint32_t* __restrict__ par_off,
                                                    const uint32_t* __restrict__ par_n, uint16_t* __restrict__ cand_win,
                                                    uint32_t* __restrict__ par_win, DevStatus* st) {
  __shared__ uint32_t sOff[MARK_WPB][WAVE + 1], sCarry[MARK_WPB][WAVE];
  const int w = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
  const unsigned long long bx = xcd_tile(blockIdx.x, gridDim.x);
  const unsigned long long p0 = (bx * MARK_WPB + w) * WAVE;
  const bool active = p0 < nparents;
  const int np = active ? (int)((nparents - p0) < WAVE ? (nparents - p0) : WAVE) : 0;
#if RMC_STAGE_BATCH
  // Wave-local throughout: a wave's parents, carries and candidate range are
  // its own, so no block barrier (LDS ops of one wave complete in order; the
  // compiler barrier keeps them in program order).  Each lane loads its
  // parent's offset and count in one round trip; every step's candidate
  // words are loaded before the binary searches and the table reads.
  uint32_t my_off = 0u, my_n = 0u;
  if (lane < np) {
    my_off = par_off[p0 + lane];
    my_n = par_n[p0 + lane];
  }
  const uint32_t off0 = __shfl(my_off, 0, WAVE);
  if (lane < np) {
    sOff[w][lane] = my_off - off0;
    sCarry[w][lane] = 0;
    if (lane == np - 1) sOff[w][np] = my_off + my_n - off0;
  }
  wave_lds_sync();
  const int total = active ? (int)sOff[w][np] : 0;
  const int steps = total;
#else
  const uint32_t off0 = active ? par_off[p0] : 0u;
  if (lane < np) {
    sOff[w][lane] = par_off[p0 + lane] - off0;
    sCarry[w][lane] = 0;
    if (lane == np - 1) sOff[w][np] = par_off[p0 + lane] + par_n[p0 + lane] - off0;
  }
  __syncthreads();
  const int total = active ? (int)sOff[w][np] : 0;
  int steps = 0;  // block-uniform trip count (the loop holds a barrier)
  for (int q = 0; q < MARK_WPB; ++q) {
    const bool qa = (bx * MARK_WPB + q) * WAVE < nparents;
    if (qa) {
      const unsigned long long qp = (bx * MARK_WPB + q) * WAVE;
      const int qn = (int)((nparents - qp) < WAVE ? (nparents - qp) : WAVE);
      const int qt = (int)sOff[q][qn];
      steps = steps > qt ? steps : qt;
    }
  }
#endif
  uint32_t coll = 0;
  const unsigned long long base0 = pbase + p0 + 1;  // ranks count parents from 1
  // MARK_U steps per round: their candidate and table loads are all issued
  // before the first ballot (the kernel waits on those random reads)
  for (int i0 = 0; i0 < steps; i0 += MARK_U * WAVE) {
    uint32_t obv[MARK_U];
    unsigned long long slv[MARK_U], vv[MARK_U];
    int pv[MARK_U];
#if RMC_STAGE_BATCH
    // (the loads are unconditional -- lanes past the range re-read the
    // range's last candidate, a DUP reads slot 0 -- so no branch splits them
    // and the compiler issues them back to back)
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      const int idx = i0 + u * WAVE + lane;
      const unsigned long long t = (unsigned long long)off0 + (idx < total ? idx : total - 1);
      obv[u] = cand_ob[t];
      slv[u] = cand_slot[t];
    }
    // a tile-dedup reference (CAND_REF) reads the entry through its
    // representative's word (same tile: an L2 hit); its own rank and hidden
    // bits then make it a loser and count its collision (fpset_won)
    unsigned long long rw[MARK_U];
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      if (i0 + u * WAVE + lane >= total) obv[u] = OB_ERR;
      if (obv[u] & OB_ERR) slv[u] = CAND_DUP;  // (the slot word is used only without OB_ERR)
#if RMC_TILE_DEDUP
      const bool ref = !(slv[u] & CAND_DUP) && (slv[u] & CAND_REF);
      rw[u] = cand_slot[ref ? (slv[u] & CAND_REF_MASK) : (unsigned long long)off0];
      if (!ref) rw[u] = slv[u];
#else
      rw[u] = slv[u];  // (no references without the tile dedup: no extra load)
#endif
    }
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      const unsigned long long sl = (rw[u] & CAND_DUP) ? 0ULL : (rw[u] & CAND_SLOT_MASK);
      vv[u] = table[ew * sl + (ew >> 1)];
      if (rw[u] & CAND_DUP) {
        vv[u] = ~0ULL;
        slv[u] = CAND_DUP;  // (a representative whose insert failed: the chunk is redone)
      }
    }
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      const int idx = i0 + u * WAVE + lane;
      int lo = 0, hi = np - 1;  // parent p: sOff[p] <= idx < sOff[p+1]
      if (idx < total)
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if ((int)sOff[w][mid] <= idx) lo = mid; else hi = mid - 1;
        }
      pv[u] = lo;
    }
#else
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      const int idx = i0 + u * WAVE + lane;
      pv[u] = 0;
      obv[u] = OB_ERR;
      slv[u] = CAND_DUP;
      if (idx < total) {
        int lo = 0, hi = np - 1;  // parent p: sOff[p] <= idx < sOff[p+1]
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if ((int)sOff[w][mid] <= idx) lo = mid; else hi = mid - 1;
        }
        pv[u] = lo;
        const unsigned long long t = (unsigned long long)off0 + idx;
        obv[u] = cand_ob[t];
        const unsigned long long s0 = cand_slot[t];  // read beside ob, used only without OB_ERR
        slv[u] = (obv[u] & OB_ERR) ? CAND_DUP : s0;
      }
    }
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      unsigned long long w = slv[u];
      if (!(w & CAND_DUP) && (w & CAND_REF)) w = cand_slot[w & CAND_REF_MASK];  // tile-dedup reference
      if (w & CAND_DUP) slv[u] = CAND_DUP;
      vv[u] = (w & CAND_DUP) ? ~0ULL : table[ew * (w & CAND_SLOT_MASK) + (ew >> 1)];
    }
#endif
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      const int iu = i0 + u * WAVE, idx = iu + lane, p = pv[u];
      bool win = false;
      if (idx < total && !(slv[u] & CAND_DUP)) {
        bool c = false;
        win = fpset_won(vv[u], ((base0 + p) << 10) | (obv[u] >> 16), floor, slv[u] >> 47, c);
        coll += c ? 1u : 0u;
      }
      const unsigned long long m = __ballot(win);
      if (idx < total) {
        const int first = (int)sOff[w][p] - iu;  // parent p's first lane in this step (may be < 0)
        const int endl = (int)sOff[w][p + 1] - iu;  // one past its last lane (may be > 64)
        const unsigned long long from = first > 0 ? ~((1ULL << first) - 1ULL) : ~0ULL;
        const uint32_t r = sCarry[w][p] + (uint32_t)__popcll(m & lanemask_lt() & from);
        cand_win[(unsigned long long)off0 + idx] = win ? (uint16_t)(r + 1u) : (uint16_t)0;
        if (lane == (endl < WAVE ? endl : WAVE) - 1) {  // p's last lane in this step carries its count on
          const unsigned long long to = endl < WAVE ? ((1ULL << endl) - 1ULL) : ~0ULL;
          sCarry[w][p] += (uint32_t)__popcll(m & from & to);
        }
      }
#if RMC_STAGE_BATCH
      wave_lds_sync();  // the carries are read by other lanes of this wave in the next step
#else
      __syncthreads();  // the carries are read by other lanes in the next step
#endif
    }
  }
  if (lane < np) par_win[p0 + lane] = sCarry[w][lane];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) coll += __shfl_xor(coll, o, WAVE);
  if (lane == 0 && coll) atomicAdd(&st->hidden_coll, (unsigned long long)coll);
}

// Materialize the level's new states, tile by tile (same tiling as k_expand,
// so a tile's candidates are one contiguous range).  Winners are compacted
// into an LDS list and processed lane-per-winner: regenerate the successor
// from the LDS-staged parent and its binding, write it to its TLC-order slot
// of the next frontier, write the trace record, check the cfg's invariants.
#ifndef RMC_MAT_LIST
#define RMC_MAT_LIST 512
#endif
constexpr int MAT_LIST = RMC_MAT_LIST;
// Threads per k_materialize block.  A tile of PB = 64 parents yields about
// PB winners on average (every distinct state is a parent once), so 256
// threads left most lanes idle in the winner loop.  Measured on the bench
// workload (k_materialize ms per check): 256 thr/1024-entry list 585, 128/512
// 539, 128/256 544, 64/256 627 (LDS-limited blocks, slower tile staging).
#ifndef RMC_MAT_THREADS
#define RMC_MAT_THREADS 128
#endif
constexpr int MAT_T = RMC_MAT_THREADS;
static_assert(MAT_T % 64 == 0 && MAT_T >= 64, "one thread per tile parent");
// waves per SIMD the register allocation must allow (0: the compiler's choice)
#ifdef RMC_MAT_WAVES
#define RMC_MAT_BOUNDS __launch_bounds__(MAT_T, RMC_MAT_WAVES)
#elif RMC_STAGE_BATCH
// the batched staging's registers take the N <= 3 library instantiation from
// 95 to 97 VGPRs (4 waves per SIMD); bounded at 5 it allocates 96, no scratch
#define RMC_MAT_BOUNDS __launch_bounds__(MAT_T, (N <= 3 && !G) ? 5 : 1)
#else
#define RMC_MAT_BOUNDS __launch_bounds__(MAT_T)
#endif
template <int SPEC, int N, bool G = false>
__global__ RMC_MAT_BOUNDS void k_materialize(const uint32_t* __restrict__ frontier, unsigned long long nparents,
                                                     unsigned long long pbase, const uint32_t* __restrict__ cand_ob,
                                                     const uint16_t* __restrict__ cand_win,
                                                     const uint32_t* __restrict__ par_off,
                                                     const uint32_t* __restrict__ par_n,
                                                     const uint32_t* __restrict__ par_pos, uint32_t* __restrict__ out,
                                                     unsigned long long out_base_global,
                                                     unsigned long long* __restrict__ tr_parent,
                                                     uint16_t* __restrict__ tr_bind,
                                                     const MatPiece* __restrict__ pieces, int npieces,
                                                     DevStatus* st) {
  constexpr int PB = Tile<N>::PB;  // must be k_expand's tile: a tile's candidates are contiguous only within one expand tile
  extern __shared__ __align__(16) unsigned char lds[];
  // winner list: (rank << 16 | candidate index in the tile) and the candidate's ordinal/binding word,
  // both read coalesced in the compaction pass instead of per winner later
  __shared__ uint32_t sOff[PB + 1], sPos[PB], sList[MAT_LIST], sListOb[MAT_LIST];
  __shared__ uint32_t sDesc[MAXFIXED];  // Model::fb_desc (see k_expand)
  __shared__ int sCount;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1);
  const int words = cM.words, Wp = words | 1;
  uint32_t* sS = (uint32_t*)lds;
  const unsigned long long p0 = xcd_tile(blockIdx.x, gridDim.x) * PB;
  const int np = (int)((nparents - p0) < (unsigned long long)PB ? (nparents - p0) : PB);
  const uint32_t start = par_off[p0];
#if RMC_STAGE_BATCH
  // every load first (binding table, the tile's offsets and positions, its
  // rows), then the LDS writes: one round trip (stage_rows_batched)
  constexpr int DU = (MAXFIXED + MAT_T - 1) / MAT_T;
  uint32_t vdesc[DU];
#pragma unroll
  for (int u = 0; u < DU; u++) vdesc[u] = tid + MAT_T * u < cM.nfixed ? cM.fb_desc[tid + MAT_T * u] : 0u;
  uint32_t voff = 0, vpos = 0, vn = 0;
  if (tid < np) {
    voff = par_off[p0 + tid];
    vpos = par_pos[p0 + tid];
    vn = par_n[p0 + tid];
  }
  stage_rows_batched<MAT_T, 8>(frontier, p0, np, words, Wp, sS);
#pragma unroll
  for (int u = 0; u < DU; u++)
    if (tid + MAT_T * u < cM.nfixed) sDesc[tid + MAT_T * u] = vdesc[u];
  if (tid < np) {
    sOff[tid] = voff - start;
    sPos[tid] = vpos;
    if (tid == np - 1) sOff[np] = voff + vn - start;
  }
#else
  const uint4* src = reinterpret_cast<const uint4*>(frontier + p0 * (unsigned long long)words);
  for (int q = tid; q < np * (words >> 2); q += MAT_T) {
    const int w = q << 2, p = w / words;
    const uint4 v = src[q];
    uint32_t* d = sS + p * Wp + (w - p * words);
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
  for (int q = tid; q < cM.nfixed; q += MAT_T) sDesc[q] = cM.fb_desc[q];
  if (tid < np) {
    sOff[tid] = par_off[p0 + tid] - start;
    sPos[tid] = par_pos[p0 + tid];
    if (tid == np - 1) sOff[np] = par_off[p0 + tid] + par_n[p0 + tid] - start;
  }
#endif
  __syncthreads();
  const int total = (int)sOff[np];
  int my_max = 0;  // largest |DOMAIN messages| this thread wrote (reduced per block below)
#ifdef RMC_ROWSTATS
  unsigned long long my_words = 0;  // diagnostic: the words this thread's rows hold (16 B units)
#endif
  for (int r0 = 0; r0 < total; r0 += MAT_LIST) {
    if (tid == 0) sCount = 0;
    __syncthreads();
    const int rn = total - r0 < MAT_LIST ? total - r0 : MAT_LIST;
#if RMC_STAGE_BATCH
    // MU steps of MAT_T candidates per batch: their win words and ordinal
    // words are loaded together (the ordinal words of losers too -- the same
    // lines), then one LDS reservation per wave for the batch's winners
    constexpr int MU = 4;
    for (int b0 = 0; b0 < rn; b0 += MAT_T * MU) {  // block-uniform trip count (ballots)
      uint32_t cw[MU], cob[MU];
#pragma unroll
      for (int u = 0; u < MU; u++) {
        const int idx = b0 + u * MAT_T + tid;
        cw[u] = 0u;
        cob[u] = 0u;
        if (idx < rn) {
          cw[u] = (uint32_t)cand_win[start + r0 + idx];
          cob[u] = cand_ob[start + r0 + idx];
        }
      }
      unsigned long long m[MU];
      int cnt = 0;
#pragma unroll
      for (int u = 0; u < MU; u++) {
        m[u] = __ballot(cw[u] != 0u);
        cnt += __popcll(m[u]);
      }
      int base = 0;
      if (lane == 0 && cnt) base = atomicAdd(&sCount, cnt);
      base = __shfl(base, 0, WAVE);
#pragma unroll
      for (int u = 0; u < MU; u++) {
        if (cw[u]) {
          const int at = base + __popcll(m[u] & lanemask_lt());
          sList[at] = ((cw[u] - 1u) << 16) | (uint32_t)(r0 + b0 + u * MAT_T + tid);
          sListOb[at] = cob[u];
        }
        base += __popcll(m[u]);
      }
    }
#else
    for (int idx = tid; idx < ((rn + MAT_T - 1) / MAT_T) * MAT_T; idx += MAT_T) {
      const uint32_t cw = idx < rn ? (uint32_t)cand_win[start + r0 + idx] : 0u;
      const bool w = cw != 0;
      unsigned long long m = __ballot(w);
      int base = 0;
      if (lane == 0 && m) base = atomicAdd(&sCount, __popcll(m));
      base = __shfl(base, 0, WAVE);
      if (w) {
        const int at = base + __popcll(m & lanemask_lt());
        sList[at] = ((cw - 1u) << 16) | (uint32_t)(r0 + idx);
        sListOb[at] = cand_ob[start + r0 + idx];
      }
    }
#endif
    __syncthreads();
    const int nw = sCount;
    for (int e = tid; e < nw; e += MAT_T) {
      const int idx = (int)(sList[e] & 0xFFFFu);
      int lo = 0, hi = np - 1;  // parent p: sOff[p] <= idx < sOff[p+1]
      while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if ((int)sOff[mid] <= idx) lo = mid; else hi = mid - 1;
      }
      const int p = lo;
      const uint32_t ob = sListOb[e];
      const int b = (int)(ob & 0x3FFu);
      const int rank = (int)(sList[e] >> 16);
      PState<SPEC, N> s{sS + p * Wp};
      Delta d;
      eval_known<SPEC, N, G>(s, cM, b, b < cM.nfixed ? sDesc[b] : 0u, (int)(ob >> 16), d);
      const unsigned long long dst = (unsigned long long)sPos[p] + rank;
      uint32_t* o;
      unsigned long long* tp;
      uint16_t* tb;
      if (npieces) {  // logical shards: straight into the next-level owner's rows and trace records
        int k = 0;
        while (k + 1 < npieces && pieces[k + 1].first <= dst) k++;
        const unsigned long long r = dst - pieces[k].first;
        o = pieces[k].out + r * (unsigned long long)words;
        tp = pieces[k].trp + r;
        tb = pieces[k].trb + r;
      } else {
        o = out + dst * (unsigned long long)words;
        tp = tr_parent + out_base_global + dst;
        tb = tr_bind + out_base_global + dst;
      }
      // All three point into device memory; typed so, the stores are global_*
      // rather than flat_* (a pointer read from `pieces` is generic).  A flat
      // store counts in lgkmcnt too, so every LDS wait after one also waited
      // for the store to reach memory: the row's 16 B stores went out one
      // HBM write round trip apart.  (A generic -> global -> generic cast
      // round trip is folded away; the pointers must stay global-typed.)
      gu32* go = (gu32*)o;
      __attribute__((address_space(1))) unsigned long long* gtp = (__attribute__((address_space(1))) unsigned long long*)tp;
      __attribute__((address_space(1))) uint16_t* gtb = (__attribute__((address_space(1))) uint16_t*)tb;
      int nn = 0;
      int err = apply_delta<SPEC, N, gu32*>(s, cM, d, go, &nn);
      if (err) atomicOr(&st->cap_flags, 1u << err);
      my_max = nn > my_max ? nn : my_max;
#ifdef RMC_ROWSTATS
      my_words += (unsigned long long)((1 + 4 * N + nn + 3) & ~3);
#endif
      const unsigned long long pg = pbase + p0 + p;
      *gtp = pg;
      *gtb = (uint16_t)b;
      // invariants read only the header and the server words: check them on
      // the parent + delta in place (SuccView), not on the row written to HBM
      const SuccView<SPEC, N> ns(s, d);
      int ierr = 0;
      int bad = check_invariants<SPEC, N>(ns, cM, ierr);
      if (ierr) atomicMin(&st->inv_err_key, order_key(pg, (int)(ob >> 16), b));
      else if (bad >= 0) atomicMin(&st->viol_key, order_key(pg, (int)(ob >> 16), b));
    }
    __syncthreads();
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int y = __shfl_xor(my_max, o, WAVE);
    my_max = y > my_max ? y : my_max;
  }
  // one hot address for the whole grid: only a wave that raises the max pays an atomic
  if (lane == 0 && (unsigned)my_max > __hip_atomic_load(&st->max_msgs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMax(&st->max_msgs, (unsigned)my_max);
#ifdef RMC_ROWSTATS
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) my_words += __shfl_xor(my_words, o, WAVE);
  if (lane == 0 && my_words) atomicAdd(&st->row_words, my_words);
#endif
}

// ------------------------------------------------- sharded search
// Bucketing by owner (the remote candidates only: k_expand inserted the
// local-owner ones) without global atomics: per-block LDS histograms land in
// an owner-major [W][nblocks] array; its exclusive scan gives every (owner,
// block) pair its offset in the send buffer (= owner segment + earlier blocks).
constexpr int BUCKET_MAXW = 64;
__global__ __launch_bounds__(256) void k_owner_count(const unsigned long long* __restrict__ cand_fp,
                                                     const uint32_t* __restrict__ cand_ob, unsigned long long n, int W,
                                                     unsigned int* __restrict__ blk_counts) {
  __shared__ unsigned int h[BUCKET_MAXW];
  const unsigned nb = gridDim.x;
  if (threadIdx.x < W) h[threadIdx.x] = 0;
  __syncthreads();
  unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) {
    uint32_t ob = cand_ob[t];
    unsigned long long fp = cand_fp[t];  // loaded beside ob (used only for a remote candidate)
    asm volatile("" : "+v"(ob), "+v"(fp));  // both loads issued before the branch (hipcc would sink fp's past it)
    if (!(ob & (OB_ERR | OB_LOCAL | OB_TDUP))) atomicAdd(&h[fp_owner(fp, W)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < W) blk_counts[(size_t)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

// Generator-side dedup of the remote-owner candidates, one block per
// k_expand tile (its candidates are one contiguous range).  37 % of a tile's
// successors repeat a fingerprint another successor of the same tile produced
// (commuting actions of sibling parents).  Only the lowest-ranked of them (the
// first in TLC order) can win at the owner, so the others need not travel:
// one whose hidden variables equal that representative's is marked OB_TDUP
// and its cand_val becomes the representative's candidate index.  Its outcome
// is then known from the representative's flag: it loses, and it is a
// hidden-variable collision exactly when the representative lost with one
// (k_mark_recv's flag 2).  A repeat with other hidden variables is sent as
// before (the owner counts its collision against the real winner).  Windows
// of DEDUP_WIN candidates; repeats across windows are sent, as before.
constexpr int DEDUP_WIN = 512, DEDUP_SLOTS = 1024;
__global__ __launch_bounds__(256) void k_tile_dedup(unsigned long long nparents, const uint32_t* __restrict__ par_off,
                                                    const uint32_t* __restrict__ par_n,
                                                    const unsigned long long* __restrict__ cand_fp,
                                                    unsigned long long* __restrict__ cand_val,
                                                    uint32_t* __restrict__ cand_ob) {
  __shared__ unsigned long long sK[DEDUP_SLOTS], sV[DEDUP_SLOTS];
  __shared__ uint32_t sI[DEDUP_SLOTS];
  constexpr int PB = 64;  // = Tile<N>::PB, every N
  const unsigned long long p0 = (unsigned long long)blockIdx.x * PB;
  const unsigned long long pl = min(nparents, p0 + PB) - 1;
  const uint32_t t0 = par_off[p0], t1 = par_off[pl] + par_n[pl];
  for (uint32_t w0 = t0; w0 < t1; w0 += DEDUP_WIN) {
    const uint32_t w1 = min(t1, w0 + (uint32_t)DEDUP_WIN);
    for (int q = threadIdx.x; q < DEDUP_SLOTS; q += 256) {
      sK[q] = EMPTY;
      sV[q] = ~0ULL;
    }
    __syncthreads();
    constexpr int PER = DEDUP_WIN / 256;
    int h[PER];
    unsigned long long v[PER];
#pragma unroll
    for (int u = 0; u < PER; u++) {
      const uint32_t t = w0 + threadIdx.x + 256u * u;
      h[u] = -1;
      if (t < w1 && !(cand_ob[t] & (OB_ERR | OB_LOCAL))) {
        const unsigned long long fp = cand_fp[t];
        v[u] = cand_val[t];
        int k = (int)((fp * 0x9E3779B97F4A7C15ULL) >> 54);  // top 10 bits
        for (;;) {  // <= DEDUP_WIN keys in DEDUP_SLOTS slots: a slot is always found
          const unsigned long long prev = atomicCAS(&sK[k], EMPTY, fp);
          if (prev == EMPTY || prev == fp) break;
          k = (k + 1) & (DEDUP_SLOTS - 1);
        }
        atomicMin(&sV[k], v[u]);
        h[u] = k;
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; u++)
      if (h[u] >= 0 && sV[h[u]] == v[u]) sI[h[u]] = w0 + threadIdx.x + 256u * u;  // the representative
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; u++) {
      if (h[u] < 0) continue;
      const unsigned long long rv = sV[h[u]];
      if (rv != v[u] && ((rv ^ v[u]) & 0xFFFFULL) == 0) {
        const uint32_t t = w0 + threadIdx.x + 256u * u;
        cand_ob[t] |= OB_TDUP;
        cand_val[t] = sI[h[u]];
      }
    }
    __syncthreads();  // the next window resets the table
  }
}

// Scatter (fp, val) records into per-owner segments of the send buffer;
// perm[t] = the record's position (replies come back in send order).
__global__ __launch_bounds__(256) void k_bucket(const unsigned long long* __restrict__ cand_fp,
                                                const unsigned long long* __restrict__ cand_val,
                                                const uint32_t* __restrict__ cand_ob, unsigned long long n, int W,
                                                const unsigned int* __restrict__ blk_off,
                                                unsigned long long* __restrict__ send, uint32_t* __restrict__ perm,
                                                const unsigned long long* __restrict__ dbase) {
  __shared__ unsigned int h[BUCKET_MAXW];
  __shared__ unsigned long long db[BUCKET_MAXW];
  const unsigned nb = gridDim.x;
  if (threadIdx.x < W) {
    h[threadIdx.x] = blk_off[(size_t)threadIdx.x * nb + blockIdx.x];
    // dbase (shards sharing the device): record `pos` of owner o goes to the
    // byte address db[o] + 16 * pos -- straight into o's receive buffer
    db[threadIdx.x] = dbase ? dbase[threadIdx.x] : (unsigned long long)send;
  }
  __syncthreads();
  unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  // the candidate's three words loaded together (fp and val are used only
  // for a remote candidate; the lines are read anyway)
  uint32_t ob = cand_ob[t];
  unsigned long long fp = cand_fp[t], val = cand_val[t];
  asm volatile("" : "+v"(ob), "+v"(fp), "+v"(val));  // all three issued before the branch (hipcc would sink two)
  if (ob & (OB_ERR | OB_LOCAL | OB_TDUP)) {
    perm[t] = 0xFFFFFFFFu;
    return;
  }
  const int o = fp_owner(fp, W);
  unsigned pos = atomicAdd(&h[o], 1u);
  // a device address (another shard's receive buffer, or send): global stores
  __attribute__((address_space(1))) unsigned long long* dst =
      reinterpret_cast<__attribute__((address_space(1))) unsigned long long*>(db[o] + 16ULL * pos);
  dst[0] = fp;
  dst[1] = val;
  perm[t] = pos;
}

// Owner side: insert every received (fp, val); first in TLC order wins.
#ifndef RMC_RECV_U
#define RMC_RECV_U 4
#endif
constexpr int RECV_U = RMC_RECV_U;
__global__ __launch_bounds__(256) void k_insert_recv(const unsigned long long* __restrict__ recv, unsigned long long n,
                                                     unsigned long long* __restrict__ table, unsigned long long mask,
                                                     unsigned long long floor,
                                                     unsigned long long* __restrict__ recv_slot, DevStatus* st) {
  // RECV_U records per thread (consecutive records on consecutive threads of
  // each step, for the L2 locality of a parent's duplicates).  Three batched
  // memory steps: every record loaded (unconditionally: lanes past n re-read
  // the last record, so no branch splits the batch and hipcc issues the
  // loads back to back), every first probe group loaded, every CAS a group
  // left to do issued; only a CAS lost to another key (rare) falls back to
  // the probe loop.  (The r04 form loaded the records and ran the CAS of
  // each record after the previous one's had returned: eight dependent
  // round trips per thread.)
  constexpr int U = RECV_U;
  if (n == 0) return;
  const unsigned long long j0 = (unsigned long long)blockIdx.x * blockDim.x * U + threadIdx.x;
  unsigned long long fp[U], v[U], slot[U], prev[U];
  ulonglong2 e[U][4];
  bool ld[U], cas[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned long long j = j0 + (unsigned long long)u * blockDim.x;
    const unsigned long long jc = j < n ? j : n - 1;
    fp[u] = recv[2 * jc];
    v[u] = recv[2 * jc + 1];
  }
#pragma unroll
  for (int u = 0; u < U; u++) ld[u] = fpset_group_load(table, mask, fp[u], e[u]);
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned long long j = j0 + (unsigned long long)u * blockDim.x;
    slot[u] = EMPTY;
    cas[u] = false;
    if (j >= n) continue;
    unsigned long long s0 = fp_slot(fp[u], mask);
    if (ld[u]) {
      int k = 4;
      unsigned long long kv = 0;
      bool found = false;
#pragma unroll
      for (int q = 3; q >= 0; q--)
        if (e[u][q].x == fp[u] || e[u][q].x == EMPTY) { k = q; kv = e[u][q].y; found = e[u][q].x == fp[u]; }
      if (found) {  // decided by the group: an earlier level's copy needs nothing, a same-level one its min
        s0 = (s0 + (unsigned long long)k) & mask;
        if (kv >= floor && v[u] < kv) atomicMin(table + 2 * s0 + 1, v[u]);
        slot[u] = s0;
        continue;
      }
      if (k < 4) {  // the first EMPTY of the group: claim it
        slot[u] = (s0 + (unsigned long long)k) & mask;
        cas[u] = true;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++)
    if (cas[u]) prev[u] = atomicCAS(table + 2 * slot[u], EMPTY, fp[u]);
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned long long j = j0 + (unsigned long long)u * blockDim.x;
    if (j >= n) continue;
    if (cas[u] && (prev[u] == EMPTY || prev[u] == fp[u])) {
      atomicMin(table + 2 * slot[u] + 1, v[u]);  // claimed, or claimed since the load: the min (as fpset_insert)
    } else if (slot[u] == EMPTY || cas[u]) {
      // no group (table end), four other keys, or the slot went to another
      // key since the load: the probe loop from the group's start
      slot[u] = fpset_insert_loaded(table, mask, fp[u], v[u], floor, st, e[u], ld[u] && !cas[u]);
    }
    recv_slot[j] = cand_word(slot[u], v[u]);
  }
}

// Owner side, after all of the round's inserts: did the record win its fp?
// newcount += number of winners (= entries added to the table this round);
// same-level losers with other hidden variables are counted as in k_mark.
__global__ __launch_bounds__(256) void k_mark_recv(const unsigned long long* __restrict__ recv,
                                                   const unsigned long long* __restrict__ recv_slot,
                                                   unsigned long long n, const unsigned long long* __restrict__ table,
                                                   unsigned long long floor, uint8_t* __restrict__ flag,
                                                   unsigned long long* __restrict__ newcount, DevStatus* st,
                                                   const unsigned long long* __restrict__ fbase,
                                                   const unsigned long long* __restrict__ rseg, int W) {
  // RECV_U records per thread, their table reads issued together (as k_insert_recv)
  constexpr int U = RECV_U;
  // fbase (shards sharing the device): the flag of record j, received from
  // source q (rseg[q] <= j < rseg[q+1]), goes straight to the byte address
  // fbase[q] + j in q's flag buffer
  __shared__ unsigned long long sfb[BUCKET_MAXW], srs[BUCKET_MAXW + 1];
  if (fbase) {
    if (threadIdx.x < W) sfb[threadIdx.x] = fbase[threadIdx.x];
    if (threadIdx.x <= W) srs[threadIdx.x] = rseg[threadIdx.x];
    __syncthreads();
  }
  const unsigned long long j0 = (unsigned long long)blockIdx.x * blockDim.x * U + threadIdx.x;
  unsigned long long rs[U], tv[U], mv[U];
  // every record's slot word and value first (unconditional: lanes past n
  // re-read the last record), then every table read (a DUP reads slot 0)
  if (n == 0) return;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned long long j = j0 + (unsigned long long)u * blockDim.x;
    const unsigned long long jc = j < n ? j : n - 1;
    rs[u] = recv_slot[jc];
    mv[u] = recv[2 * jc + 1];
  }
#pragma unroll
  for (int u = 0; u < U; u++) tv[u] = table[2 * ((rs[u] & CAND_DUP) ? 0ULL : (rs[u] & CAND_SLOT_MASK)) + 1];
  unsigned int wins = 0, colls = 0;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned long long j = j0 + (unsigned long long)u * blockDim.x;
    if (j >= n) continue;
    bool w = false, c = false;
    if (!(rs[u] & CAND_DUP)) {
      const unsigned long long mine = mv[u];
      w = fpset_won(tv[u], mine >> VAL_RANK_SHIFT, floor, mine, c);
      colls += c;
    }
    // 1 won; 2 lost with a hidden-variable collision (the generator's OB_TDUP
    // repeats of this record collide too); 0 lost
    const uint8_t fl = w ? 1 : c ? 2 : 0;
    if (fbase) {
      int lo = 0, hi = W - 1;  // source q: srs[q] <= j < srs[q+1]
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (srs[mid] <= j) lo = mid; else hi = mid - 1;
      }
      *reinterpret_cast<__attribute__((address_space(1))) uint8_t*>(sfb[lo] + j) = fl;  // global, not flat (no lgkm wait)
    } else {
      flag[j] = fl;
    }
    wins += w;
  }
  if (colls) atomicAdd(&st->hidden_coll, (unsigned long long)colls);
  __shared__ unsigned int c;
  if (threadIdx.x == 0) c = 0;
  __syncthreads();
  for (int o = 32; o > 0; o >>= 1) wins += __shfl_xor(wins, o, WAVE);
  if (lane_id() == 0 && wins) atomicAdd(&c, wins);
  __syncthreads();
  if (threadIdx.x == 0 && c) atomicAdd(newcount, (unsigned long long)c);
}

// Generator side: per parent, winners ranked in TLC ordinal order, as k_mark
// does for the single-shard search.  A remote-owner candidate's outcome is the
// owner's flag (returned in send order); a local-owner one is read from this
// shard's table at the slot k_expand recorded -- or, when the table grew since
// (`moved`), found again by its fp -- with the same-level hidden-variable
// collisions counted as k_mark counts them.  newcount += local winners (=
// entries they added).
__global__ __launch_bounds__(256) void k_mark_gen(unsigned long long nparents, unsigned long long pbase,
                                                  const uint32_t* __restrict__ par_off,
                                                  const uint32_t* __restrict__ par_n,
                                                  const uint32_t* __restrict__ cand_ob,
                                                  const unsigned long long* __restrict__ cand_fp,
                                                  const unsigned long long* __restrict__ cand_val,
                                                  const uint32_t* __restrict__ perm,
                                                  const uint8_t* __restrict__ flag_back,
                                                  const unsigned long long* __restrict__ table, unsigned long long mask,
                                                  unsigned long long floor, int moved, uint16_t* __restrict__ cand_win,
                                                  uint32_t* __restrict__ par_win, unsigned long long* __restrict__ newcount,
                                                  DevStatus* st) {
  const unsigned long long p = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t nloc = 0, coll = 0;
  if (p < nparents) {
    const uint32_t off = par_off[p], n = par_n[p];
    uint32_t cnt = 0;
    const unsigned long long base = (pbase + p + 1) << 10;
    constexpr int U = 8;
    // A candidate's decision is a chain of up to four dependent reads (its
    // ob word; then its slot word, value or record position; then the table
    // entry, the owner's flag or a tile representative's position; then
    // that one's flag).  Each stage is read for all U candidates of a step
    // before the next stage starts, every load unconditional (an unused
    // stage reads index 0 / the step's first candidate), so a step costs four
    // round trips instead of up to four per candidate.
    for (uint32_t t0 = off; t0 < off + n; t0 += U) {
      uint32_t ob[U], pq[U], pt[U];
      uint8_t fb[U], fb2[U];
      bool w[U];
      unsigned long long v[U], mine[U], cv[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t t = t0 + u < off + n ? t0 + u : off + n - 1;
        ob[u] = cand_ob[t];
        mine[u] = cand_fp[t];
        cv[u] = cand_val[t];
        pq[u] = perm[t];
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        if (t0 + u >= off + n) ob[u] = OB_ERR;
        const bool local = (ob[u] & (OB_ERR | OB_LOCAL)) == OB_LOCAL;
        if (local && (mine[u] & CAND_DUP)) ob[u] |= OB_ERR;  // the insert failed: the round was redone
        const bool loc = (ob[u] & (OB_ERR | OB_LOCAL)) == OB_LOCAL, tdup = !(ob[u] & (OB_ERR | OB_LOCAL)) && (ob[u] & OB_TDUP);
        const bool remote = !(ob[u] & (OB_ERR | OB_LOCAL | OB_TDUP));
        v[u] = table[2 * (loc && !moved ? (mine[u] & CAND_SLOT_MASK) : 0ULL) + 1];
        fb[u] = flag_back[remote ? pq[u] : 0u];
        pt[u] = perm[tdup ? (uint32_t)cv[u] : 0u];
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const bool tdup = !(ob[u] & (OB_ERR | OB_LOCAL)) && (ob[u] & OB_TDUP);
        fb2[u] = flag_back[tdup ? pt[u] : 0u];
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        w[u] = false;
        if (ob[u] & OB_ERR) continue;
        if (ob[u] & OB_LOCAL) {
          if (moved) v[u] = fpset_value(table, mask, cv[u]);  // the set was rehashed since the insert
          mine[u] >>= 47;
        } else if (ob[u] & OB_TDUP) {  // loses to its tile's representative; collides when that did
          coll += fb2[u] == 2 ? 1u : 0u;
        } else {
          w[u] = fb[u] == 1;
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t t = t0 + u;
        if (t >= off + n) break;
        if ((ob[u] & (OB_ERR | OB_LOCAL)) == OB_LOCAL) {
          bool c = false;
          w[u] = fpset_won(v[u], base | (ob[u] >> 16), floor, mine[u], c);
          coll += c ? 1u : 0u;
          nloc += w[u] ? 1u : 0u;
        }
        cand_win[t] = w[u] ? (uint16_t)(++cnt) : (uint16_t)0;
      }
    }
    par_win[p] = cnt;
  }
  __shared__ unsigned int sn, sc;
  if (threadIdx.x == 0) sn = sc = 0;
  __syncthreads();
  if (nloc) atomicAdd(&sn, nloc);
  if (coll) atomicAdd(&sc, coll);
  __syncthreads();
  if (threadIdx.x == 0 && sn) atomicAdd(newcount, (unsigned long long)sn);
  if (threadIdx.x == 0 && sc) atomicAdd(&st->hidden_coll, (unsigned long long)sc);
}

unsigned long long bucket_blocks(unsigned long long n) { return n ? (n + 255) / 256 : 1; }
void launch_tile_dedup(const LevelArgs& a, unsigned long long* cand_fp, unsigned long long* cand_val,
                       uint32_t* cand_ob, hipStream_t s) {
  if (!a.nparents) return;
  hipLaunchKernelGGL(k_tile_dedup, dim3((unsigned)((a.nparents + 63) / 64)), dim3(256), 0, s, a.nparents, a.par_off,
                     a.par_n, cand_fp, cand_val, cand_ob);
}
void launch_owner_count(const unsigned long long* cand_fp, const uint32_t* cand_ob, unsigned long long n, int W,
                        unsigned int* blk_counts, hipStream_t s) {
  hipLaunchKernelGGL(k_owner_count, dim3((unsigned)bucket_blocks(n)), dim3(256), 0, s, cand_fp, cand_ob, n, W,
                     blk_counts);
}
void launch_bucket(const unsigned long long* cand_fp, const unsigned long long* cand_val, const uint32_t* cand_ob,
                   unsigned long long n, int W, const unsigned int* blk_off, unsigned long long* send, uint32_t* perm,
                   hipStream_t s, const unsigned long long* dbase) {
  if (!n) return;
  hipLaunchKernelGGL(k_bucket, dim3((unsigned)bucket_blocks(n)), dim3(256), 0, s, cand_fp, cand_val, cand_ob, n, W,
                     blk_off, send, perm, dbase);
}
void launch_insert_recv(const unsigned long long* recv, unsigned long long n, unsigned long long* table,
                        unsigned long long mask, unsigned long long floor, unsigned long long* recv_slot, DevStatus* st,
                        hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_insert_recv, dim3((unsigned)((n + 256 * RECV_U - 1) / (256 * RECV_U))), dim3(256), 0, s, recv, n,
                     table, mask, floor, recv_slot, st);
}
void launch_mark_recv(const unsigned long long* recv, const unsigned long long* recv_slot, unsigned long long n,
                      const unsigned long long* table, unsigned long long floor, uint8_t* flag,
                      unsigned long long* newcount, DevStatus* st, hipStream_t s, const unsigned long long* fbase,
                      const unsigned long long* rseg, int W) {
  if (!n) return;
  hipLaunchKernelGGL(k_mark_recv, dim3((unsigned)((n + 256 * RECV_U - 1) / (256 * RECV_U))), dim3(256), 0, s, recv,
                     recv_slot, n, table, floor, flag, newcount, st, fbase, rseg, W);
}
// k_mark_gen's work with k_mark_tiles's shape: a wave per k_expand tile (the
// tile's candidates are one contiguous range in the sharded layout too), its
// lanes over 64 candidates per step, four steps per round.  Each stage of a
// candidate's decision chain (ob / slot word / value / record position, then
// the table entry / the owner's flag / a tile representative's position,
// then that one's flag) is loaded for all four steps before the next stage,
// every load unconditional.  Ranks by ballot inside each parent's segment,
// as k_mark_tiles.  Measured and not the default (r06, 8 logical shards,
// kernel trace of one CLI check, profiles/r06/s3/kernels_logical8_gen_tiles.txt):
// 362 ms per check against 105 ms for the thread-per-parent k_mark_gen with
// its stages batched (kernels_logical8_cli.txt); the cause is not
// understood -- both read the same bytes, and this form is coalesced.
#ifndef RMC_MARK_GEN_TILES
#define RMC_MARK_GEN_TILES 0
#endif
__global__ __launch_bounds__(MARK_WPB * WAVE) void k_mark_gen_tiles(
    unsigned long long nparents, unsigned long long pbase, const uint32_t* __restrict__ par_off,
    const uint32_t* __restrict__ par_n, const uint32_t* __restrict__ cand_ob,
    const unsigned long long* __restrict__ cand_fp, const unsigned long long* __restrict__ cand_val,
    const uint32_t* __restrict__ perm, const uint8_t* __restrict__ flag_back,
    const unsigned long long* __restrict__ table, unsigned long long mask, unsigned long long floor, int moved,
    uint16_t* __restrict__ cand_win, uint32_t* __restrict__ par_win, unsigned long long* __restrict__ newcount,
    DevStatus* st) {
  __shared__ uint32_t sOff[MARK_WPB][WAVE + 1], sCarry[MARK_WPB][WAVE];
  const int w = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
  const unsigned long long p0 = ((unsigned long long)blockIdx.x * MARK_WPB + w) * WAVE;
  const bool active = p0 < nparents;
  const int np = active ? (int)((nparents - p0) < WAVE ? (nparents - p0) : WAVE) : 0;
  uint32_t my_off = 0u, my_n = 0u;
  if (lane < np) {
    my_off = par_off[p0 + lane];
    my_n = par_n[p0 + lane];
  }
  const uint32_t off0 = __shfl(my_off, 0, WAVE);
  if (lane < np) {
    sOff[w][lane] = my_off - off0;
    sCarry[w][lane] = 0;
    if (lane == np - 1) sOff[w][np] = my_off + my_n - off0;
  }
  wave_lds_sync();
  const int total = active ? (int)sOff[w][np] : 0;
  uint32_t coll = 0, nloc = 0;
  const unsigned long long base0 = pbase + p0 + 1;  // ranks count parents from 1
  for (int i0 = 0; i0 < total; i0 += MARK_U * WAVE) {
    uint32_t ob[MARK_U], pq[MARK_U], pt[MARK_U];
    unsigned long long mine[MARK_U], cv[MARK_U], v[MARK_U];
    uint8_t fb[MARK_U], fb2[MARK_U];
    int pv[MARK_U];
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      const int idx = i0 + u * WAVE + lane;
      const unsigned long long t = (unsigned long long)off0 + (idx < total ? idx : total - 1);
      ob[u] = cand_ob[t];
      mine[u] = cand_fp[t];
      cv[u] = cand_val[t];
      pq[u] = perm[t];
    }
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      if (i0 + u * WAVE + lane >= total) ob[u] = OB_ERR;
      if ((ob[u] & (OB_ERR | OB_LOCAL)) == OB_LOCAL && (mine[u] & CAND_DUP)) ob[u] |= OB_ERR;  // its round was redone
      const bool loc = (ob[u] & (OB_ERR | OB_LOCAL)) == OB_LOCAL;
      const bool tdup = !(ob[u] & (OB_ERR | OB_LOCAL)) && (ob[u] & OB_TDUP);
      const bool remote = !(ob[u] & (OB_ERR | OB_LOCAL | OB_TDUP));
      v[u] = table[2 * (loc && !moved ? (mine[u] & CAND_SLOT_MASK) : 0ULL) + 1];
      fb[u] = flag_back[remote ? pq[u] : 0u];
      pt[u] = perm[tdup ? (uint32_t)cv[u] : 0u];
    }
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      const bool tdup = !(ob[u] & (OB_ERR | OB_LOCAL)) && (ob[u] & OB_TDUP);
      fb2[u] = flag_back[tdup ? pt[u] : 0u];
    }
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      const int idx = i0 + u * WAVE + lane;
      int lo = 0, hi = np - 1;  // parent p: sOff[p] <= idx < sOff[p+1]
      if (idx < total)
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if ((int)sOff[w][mid] <= idx) lo = mid; else hi = mid - 1;
        }
      pv[u] = lo;
    }
#pragma unroll
    for (int u = 0; u < MARK_U; ++u) {
      const int iu = i0 + u * WAVE, idx = iu + lane, p = pv[u];
      bool win = false;
      if (!(ob[u] & OB_ERR)) {
        if (ob[u] & OB_LOCAL) {
          if (moved) v[u] = fpset_value(table, mask, cv[u]);  // the set was rehashed since the insert
          bool c = false;
          win = fpset_won(v[u], ((base0 + p) << 10) | (ob[u] >> 16), floor, mine[u] >> 47, c);
          coll += c ? 1u : 0u;
          nloc += win ? 1u : 0u;
        } else if (ob[u] & OB_TDUP) {  // loses to its tile's representative; collides when that did
          coll += fb2[u] == 2 ? 1u : 0u;
        } else {
          win = fb[u] == 1;
        }
      }
      const unsigned long long m = __ballot(win);
      if (idx < total) {
        const int first = (int)sOff[w][p] - iu;
        const int endl = (int)sOff[w][p + 1] - iu;
        const unsigned long long from = first > 0 ? ~((1ULL << first) - 1ULL) : ~0ULL;
        const uint32_t r = sCarry[w][p] + (uint32_t)__popcll(m & lanemask_lt() & from);
        cand_win[(unsigned long long)off0 + idx] = win ? (uint16_t)(r + 1u) : (uint16_t)0;
        if (lane == (endl < WAVE ? endl : WAVE) - 1) {
          const unsigned long long to = endl < WAVE ? ((1ULL << endl) - 1ULL) : ~0ULL;
          sCarry[w][p] += (uint32_t)__popcll(m & from & to);
        }
      }
      wave_lds_sync();  // the carries are read by other lanes of this wave in the next step
    }
  }
  if (lane < np) par_win[p0 + lane] = sCarry[w][lane];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    coll += __shfl_xor(coll, o, WAVE);
    nloc += __shfl_xor(nloc, o, WAVE);
  }
  if (lane == 0 && coll) atomicAdd(&st->hidden_coll, (unsigned long long)coll);
  if (lane == 0 && nloc) atomicAdd(newcount, (unsigned long long)nloc);
}
void launch_mark_gen(const LevelArgs& a, int moved, const uint32_t* perm, const uint8_t* flag_back,
                     unsigned long long* newcount, hipStream_t s) {
  if (!a.nparents) return;
#if RMC_MARK_GEN_TILES
  hipLaunchKernelGGL(k_mark_gen_tiles, dim3((unsigned)((a.nparents + MARK_WPB * WAVE - 1) / (MARK_WPB * WAVE))),
                     dim3(MARK_WPB * WAVE), 0, s, a.nparents, a.pbase, a.par_off, a.par_n, a.cand_ob, a.cand_slot,
                     a.cand_val, perm, flag_back, a.table, a.mask, a.floor, moved, a.cand_win, a.par_win, newcount, a.st);
#else
  hipLaunchKernelGGL(k_mark_gen, dim3((unsigned)((a.nparents + 255) / 256)), dim3(256), 0, s, a.nparents, a.pbase,
                     a.par_off, a.par_n, a.cand_ob, a.cand_slot, a.cand_val, perm, flag_back, a.table, a.mask, a.floor,
                     moved, a.cand_win, a.par_win, newcount, a.st);
#endif
}
int host_fp_owner(unsigned long long fp, int W) { return fp_owner(fp, W); }

// ------------------------------------------------------------ host driver
struct Launch {
  template <int SPEC, int N>
  static void expand(const LevelArgs& a, hipStream_t s) {
    if constexpr (SPEC != KRAFT) {
      if (a.model->gany) {  // compiled guards: 64-bit fingerprints only (rmc_engine.cpp checks)
        if (a.model->fpw == 2) throw std::runtime_error("compiled guards need 64-bit fingerprints");
        return expand_w<SPEC, N, 1, true>(a, s);
      }
    }
    if (a.model->fpw == 2) return expand_w<SPEC, N, 2>(a, s);
    return expand_w<SPEC, N, 1>(a, s);
  }
  template <int SPEC, int N, int FPW, bool G = false>
  static void expand_w(const LevelArgs& a, hipStream_t s) {
    constexpr int PB = Tile<N>::PB;
    unsigned long long blocks = (a.nparents + PB - 1) / PB;
    const Model& M = *a.model;
    ExpandLds L = expand_lds(PB, M.words, M.ord_words, (int)sizeof(typename SumsOf<N, FPW>::T), M.nfixed,
                             M.ordinal_limit, M.kmax, M.nact);
#if RMC_EXPAND_PERSIST
    {  // resident blocks only: as many as the CUs hold at this LDS size
      static int cached_bytes = -1, cached_grid = 0;
      if (cached_bytes != L.bytes) {
        int dev = 0, cus = 0, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_expand<SPEC, N, FPW, G>, 256,
                                                         L.bytes) != hipSuccess)
          throw std::runtime_error("k_expand: occupancy query failed");
        cached_grid = std::max(1, cus * std::max(1, per_cu));
        cached_bytes = L.bytes;
      }
      blocks = std::min<unsigned long long>(blocks, (unsigned long long)cached_grid);
    }
#endif
    hipLaunchKernelGGL((k_expand<SPEC, N, FPW, G>), dim3((unsigned)blocks), dim3(256), L.bytes, s, a.frontier, a.nparents, a.pbase,
                       a.floor, a.sharded, a.shard_self, a.table, a.mask, a.cand_slot, a.cand_ob, a.par_off, a.par_n, a.counters, a.cand_cap,
                       a.st, a.cand_val
#ifdef RMC_DIAG
                       , a.diag
#endif
                       );
  }
  template <int SPEC, int N>
  static void materialize(const LevelArgs& a, hipStream_t s) {
    constexpr int PB = Tile<N>::PB;  // must be k_expand's tile: a tile's candidates are contiguous only within one expand tile
    unsigned long long blocks = (a.nparents + PB - 1) / PB;
    size_t lds_bytes = (size_t)PB * (a.model->words | 1) * 4;
    if constexpr (SPEC != KRAFT) {
      if (a.model->gany) {
        hipLaunchKernelGGL((k_materialize<SPEC, N, true>), dim3((unsigned)blocks), dim3(MAT_T), lds_bytes, s, a.frontier,
                           a.nparents, a.pbase, a.cand_ob, a.cand_win, a.par_off, a.par_n, a.par_pos, a.out,
                           a.out_base_global, a.tr_parent, a.tr_bind, a.pieces, a.npieces, a.st);
        return;
      }
    }
    hipLaunchKernelGGL((k_materialize<SPEC, N>), dim3((unsigned)blocks), dim3(MAT_T), lds_bytes, s, a.frontier, a.nparents,
                       a.pbase, a.cand_ob, a.cand_win, a.par_off, a.par_n, a.par_pos, a.out, a.out_base_global,
                       a.tr_parent, a.tr_bind, a.pieces, a.npieces, a.st);
  }
};

template <int SPEC>
static void dispatch_n(int N, bool expand, const LevelArgs& a, hipStream_t s) {
  switch (N) {
    case 2: expand ? Launch::expand<SPEC, 2>(a, s) : Launch::materialize<SPEC, 2>(a, s); break;
    case 3: expand ? Launch::expand<SPEC, 3>(a, s) : Launch::materialize<SPEC, 3>(a, s); break;
    case 4: expand ? Launch::expand<SPEC, 4>(a, s) : Launch::materialize<SPEC, 4>(a, s); break;
    case 5: expand ? Launch::expand<SPEC, 5>(a, s) : Launch::materialize<SPEC, 5>(a, s); break;
  }
}
static void dispatch(int spec, int N, bool expand, const LevelArgs& a, hipStream_t s) {
#ifdef RMC_DEV_ONE  // development builds only: one instantiation (Raft, N = 3, 64-bit) compiles in seconds
  if (spec == RAFT && N == 3) expand ? Launch::expand_w<RAFT, 3, 1>(a, s) : Launch::materialize<RAFT, 3>(a, s);
#else
  switch (spec) {
    case RAFT: dispatch_n<RAFT>(N, expand, a, s); break;
    case FLEX: dispatch_n<FLEX>(N, expand, a, s); break;
    case FSYNC: dispatch_n<FSYNC>(N, expand, a, s); break;
    case PULL: dispatch_n<PULL>(N, expand, a, s); break;
    case PULL2: dispatch_n<PULL2>(N, expand, a, s); break;
    case KRAFT:  // the KRaft lowering is for N <= 3 (model load enforces it)
      if (N == 2) expand ? Launch::expand<KRAFT, 2>(a, s) : Launch::materialize<KRAFT, 2>(a, s);
      if (N == 3) expand ? Launch::expand<KRAFT, 3>(a, s) : Launch::materialize<KRAFT, 3>(a, s);
      break;
  }
#endif
}

void launch_expand(int spec, int N, const LevelArgs& a, hipStream_t s) { dispatch(spec, N, true, a, s); }
void launch_materialize(int spec, int N, const LevelArgs& a, hipStream_t s) { dispatch(spec, N, false, a, s); }
void launch_mark(const LevelArgs& a, hipStream_t s) {
#ifdef RMC_MARK_THREADS
  unsigned long long blocks = (a.nparents + 255) / 256;
  hipLaunchKernelGGL(k_mark, dim3((unsigned)blocks), dim3(256), 0, s, a.nparents, a.pbase, a.floor,
                     a.model->fpw == 2 ? 4 : 2, a.table,
                     a.cand_slot, a.cand_ob, a.par_off, a.par_n, a.cand_win, a.par_win, a.st);
#else
  unsigned long long blocks = (a.nparents + MARK_WPB * WAVE - 1) / (MARK_WPB * WAVE);
  hipLaunchKernelGGL(k_mark_tiles, dim3((unsigned)blocks), dim3(MARK_WPB * WAVE), 0, s, a.nparents, a.pbase, a.floor,
                     a.model->fpw == 2 ? 4 : 2, a.table,
                     a.cand_slot, a.cand_ob, a.par_off, a.par_n, a.cand_win, a.par_win, a.st);
#endif
}
// Move every entry of the fingerprint set into a larger one (values kept).
// Grid-stride: a table of 2^32 slots or more would need a grid of 2^32
// threads or more, past HIP's launch limit.
// ew = entry width in words (2: fp, val; 4: fp.a, fp.b, val, -); every word moves.
__global__ __launch_bounds__(256) void k_rehash(const unsigned long long* __restrict__ old, unsigned long long nold,
                                                unsigned long long* __restrict__ nt, unsigned long long mask, int ew,
                                                DevStatus* st) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long e = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; e < nold; e += stride) {
    unsigned long long k = old[ew * e];
    if (k == EMPTY) continue;
    unsigned long long slot = fp_slot(k, mask);
    unsigned long long probe = 0;
    // read the run, CAS only a slot seen empty (an atomic is a memory-side
    // round trip on gfx950; an occupied slot read with a plain load is final)
    for (; probe <= mask; probe++) {
      if (nt[ew * slot] == EMPTY) {
        unsigned long long prev = atomicCAS(nt + ew * slot, EMPTY, k);
        if (prev == EMPTY) {
          for (int w = 1; w < ew; w++) nt[ew * slot + w] = old[ew * e + w];
          break;
        }
      }
      slot = (slot + 1) & mask;
    }
    if (probe > mask) atomicOr(&st->cap_flags, 1u << E_CAP_TABLE);
  }
}
void launch_rehash(const unsigned long long* old, unsigned long long nold, unsigned long long* nt,
                   unsigned long long nmask, DevStatus* st, hipStream_t s, int ew) {
  unsigned long long blocks = (nold + 255) / 256;
  if (blocks > (1ULL << 22)) blocks = 1ULL << 22;  // 2^30 threads, each striding
  hipLaunchKernelGGL(k_rehash, dim3((unsigned)blocks), dim3(256), 0, s, old, nold, nt, nmask, ew, st);
}
size_t scan_temp_bytes(unsigned long long n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
  return bytes;
}
void launch_scan(void* temp, size_t temp_bytes, const uint32_t* in, uint32_t* out, unsigned long long n,
                 hipStream_t s) {
  (void)hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, (int)n, s);
}

// ------------------------------------------------ compact host rows
// Host-frontier levels are kept compact: each packed row trimmed after its
// last DOMAIN message (1 + 4N + nmsg words, nmsg from the header word), rows
// back to back.  Rows are packed on the device before they
// cross PCIe and unpacked into fixed-stride rows in the input window, so the
// kernels never see the compact form.  A wave per row: lane l moves word l
// (coalesced on both sides); rows in the same wave-step are consecutive.
// A row's length comes from its header word, so it is bounded here: a header
// whose message count would take the row past max_words (the row width) is a
// row that was never written -- k_materialize leaves a successor it could not
// fit unwritten and flags the capacity -- and is clamped instead of letting
// k_pack_rows read past the row and the copy-out past the pack buffer; the
// flag ends the check with status 3 (the caller reads it at the level end).
__global__ __launch_bounds__(256) void k_row_words(const uint32_t* __restrict__ rows, unsigned long long n, int W,
                                                   int hdr_words, int max_words, uint32_t* __restrict__ lens32,
                                                   uint8_t* __restrict__ lens8, unsigned* __restrict__ flag) {
  const unsigned long long r = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  uint32_t len = (uint32_t)hdr_words + (rows[r * (unsigned long long)W] & 0xFFu);
  if (len > (uint32_t)max_words) {
    len = (uint32_t)max_words;
    atomicOr(flag, 1u);
  }
  lens32[r] = len;
  lens8[r] = (uint8_t)len;
}
__global__ __launch_bounds__(256) void k_widen_lens(const uint8_t* __restrict__ lens8, unsigned long long n,
                                                    uint32_t* __restrict__ lens32) {
  const unsigned long long r = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n) lens32[r] = lens8[r];
}
__global__ __launch_bounds__(256) void k_pack_rows(const uint32_t* __restrict__ rows, unsigned long long n, int W,
                                                   const uint32_t* __restrict__ offs,
                                                   const uint32_t* __restrict__ lens32, uint32_t* __restrict__ out) {
  const unsigned long long waves = (unsigned long long)gridDim.x * (blockDim.x / WAVE);
  for (unsigned long long r = (unsigned long long)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE; r < n;
       r += waves) {
    const uint32_t len = lens32[r];
    const uint32_t* src = rows + r * (unsigned long long)W;
    uint32_t* dst = out + offs[r];
    for (uint32_t l = lane_id(); l < len; l += WAVE) dst[l] = src[l];
  }
}
__global__ __launch_bounds__(256) void k_unpack_rows(const uint32_t* __restrict__ in, unsigned long long n, int W,
                                                     const uint32_t* __restrict__ offs,
                                                     const uint32_t* __restrict__ lens32, uint32_t* __restrict__ rows) {
  const unsigned long long waves = (unsigned long long)gridDim.x * (blockDim.x / WAVE);
  for (unsigned long long r = (unsigned long long)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE; r < n;
       r += waves) {
    const uint32_t len = lens32[r] < (uint32_t)W ? lens32[r] : (uint32_t)W;  // host lens: never past the row
    const uint32_t* src = in + offs[r];
    uint32_t* dst = rows + r * (unsigned long long)W;
    for (uint32_t l = lane_id(); l < (uint32_t)W; l += WAVE) dst[l] = l < len ? src[l] : 0u;
  }
}
static unsigned grid_for(unsigned long long n, unsigned per) {
  unsigned long long g = (n + per - 1) / per;
  return (unsigned)(g < 1 ? 1 : g > (1u << 20) ? (1u << 20) : g);
}
void launch_row_words(const uint32_t* rows, unsigned long long n, int W, int hdr_words, int max_words,
                      uint32_t* lens32, uint8_t* lens8, unsigned* flag, hipStream_t s) {
  if (!n) return;
  k_row_words<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(rows, n, W, hdr_words, max_words, lens32, lens8, flag);
}
void launch_widen_lens(const uint8_t* lens8, unsigned long long n, uint32_t* lens32, hipStream_t s) {
  if (!n) return;
  k_widen_lens<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(lens8, n, lens32);
}
void launch_pack_rows(const uint32_t* rows, unsigned long long n, int W, const uint32_t* offs, const uint32_t* lens32,
                      uint32_t* out, hipStream_t s) {
  if (!n) return;
  k_pack_rows<<<grid_for(n, 4), 256, 0, s>>>(rows, n, W, offs, lens32, out);
}
void launch_unpack_rows(const uint32_t* in, unsigned long long n, int W, const uint32_t* offs, const uint32_t* lens32,
                        uint32_t* rows, hipStream_t s) {
  if (!n) return;
  k_unpack_rows<<<grid_for(n, 4), 256, 0, s>>>(in, n, W, offs, lens32, rows);
}

// ------------------------------------------------ widening the rows mid-check
// A successor that needs more message slots than the rows have (E_CAP_MSG in
// k_expand) widens every row of the current level and of the next level so
// far, and the chunk is redone (rmc_engine.cpp).  The TLC ordinals of the
// message bindings depend on the slot count, so the chunk's first attempt
// left ranks of the old numbering in the entries it claimed: every entry
// whose rank lies in the chunk's parents' range [lo, hi) goes back to the
// value of a freshly claimed entry (~0), and the redo's atomicMin sets it
// anew.  (Entries of earlier chunks hold other parents' ranks: TLC order
// between them is decided by the parent, not the ordinal.)
__global__ __launch_bounds__(256) void k_reset_ranks(unsigned long long* __restrict__ T, unsigned long long slots,
                                                     int ew, unsigned long long lo, unsigned long long hi) {
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < slots;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    unsigned long long* v = T + (unsigned long long)ew * i + (ew >> 1);
    const unsigned long long r = *v >> VAL_RANK_SHIFT;
    if (*v != EMPTY && r >= lo && r < hi) *v = EMPTY;
  }
}
// rows of Wo words (src, contiguous) -> rows of Wn >= Wo words at dst, zero-padded; a wave per row
__global__ __launch_bounds__(256) void k_restride(const uint32_t* __restrict__ src, unsigned long long n, int Wo, int Wn,
                                                  uint32_t* __restrict__ dst) {
  const unsigned long long waves = (unsigned long long)gridDim.x * (blockDim.x / WAVE);
  for (unsigned long long r = (unsigned long long)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE; r < n;
       r += waves) {
    const uint32_t* s = src + r * (unsigned long long)Wo;
    uint32_t* d = dst + r * (unsigned long long)Wn;
    for (int l = lane_id(); l < Wn; l += WAVE) d[l] = l < Wo ? s[l] : 0u;
  }
}
void launch_reset_ranks(unsigned long long* table, unsigned long long slots, int ew, unsigned long long lo,
                        unsigned long long hi, hipStream_t s) {
  unsigned long long blocks = (slots + 255) / 256;
  if (blocks > (1ULL << 20)) blocks = 1ULL << 20;
  k_reset_ranks<<<(unsigned)blocks, 256, 0, s>>>(table, slots, ew, lo, hi);
}
void launch_restride(const uint32_t* src, unsigned long long n, int Wo, int Wn, uint32_t* dst, hipStream_t s) {
  if (!n) return;
  k_restride<<<grid_for(n, 4), 256, 0, s>>>(src, n, Wo, Wn, dst);
}

// ------------------------------------------------ batched device copies
// The logical-shard transport (rmc_sharded.cpp LocalComm): every transfer of
// one exchange step in ONE launch (blockIdx.y = transfer, blockIdx.x = 64 KiB
// piece) instead of a hipMemcpyAsync per (source, destination, buffer).
// Each piece is copied in the widest unit both ends share: when src and dst
// agree mod 16 (8, 4, 2) a byte head brings both to that alignment, the body
// moves 16 (8, 4, 2) B per lane with four loads in flight before the stores,
// and a byte tail ends it.  (The trace records -- 8 B parent indices, 2 B
// bindings -- and the 1 B win flags land at arbitrary element offsets: a byte
// loop for anything not 16 B aligned cost them ~1 B per lane per step.)
template <class T>
__device__ __forceinline__ void copy_units(const char* src, char* dst, unsigned long long n) {
  constexpr int U = 4;
  const unsigned long long head = (sizeof(T) - ((unsigned long long)src & (sizeof(T) - 1))) & (sizeof(T) - 1);
  const unsigned long long h = head < n ? head : n;
  if (threadIdx.x < h) dst[threadIdx.x] = src[threadIdx.x];
  const unsigned long long nv = (n - h) / sizeof(T);
  const T* s = reinterpret_cast<const T*>(src + h);
  T* d = reinterpret_cast<T*>(dst + h);
  for (unsigned long long i0 = threadIdx.x; i0 < nv; i0 += (unsigned long long)blockDim.x * U) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const unsigned long long i = i0 + (unsigned long long)u * blockDim.x;
      if (i < nv) v[u] = s[i];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const unsigned long long i = i0 + (unsigned long long)u * blockDim.x;
      if (i < nv) d[i] = v[u];
    }
  }
  for (unsigned long long i = h + nv * sizeof(T) + threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}
__global__ __launch_bounds__(256) void k_multi_copy(const CopyDesc* __restrict__ d, int n) {
  constexpr unsigned long long PIECE = 64 << 10;
  for (int q = blockIdx.y; q < n; q += gridDim.y) {
    const CopyDesc c = d[q];
    for (unsigned long long b0 = (unsigned long long)blockIdx.x * PIECE; b0 < c.bytes;
         b0 += (unsigned long long)gridDim.x * PIECE) {
      const unsigned long long m = (c.bytes < b0 + PIECE ? c.bytes : b0 + PIECE) - b0;
      const char* src = (const char*)c.src + b0;
      char* dst = (char*)c.dst + b0;
      const unsigned long long x = (unsigned long long)src ^ (unsigned long long)dst;
      if (!(x & 15)) copy_units<uint4>(src, dst, m);
      else if (!(x & 7)) copy_units<uint2>(src, dst, m);
      else if (!(x & 3)) copy_units<uint32_t>(src, dst, m);
      else if (!(x & 1)) copy_units<uint16_t>(src, dst, m);
      else copy_units<uint8_t>(src, dst, m);
    }
  }
}
void launch_multi_copy(const CopyDesc* d, int n, unsigned long long max_bytes, hipStream_t s) {
  if (n <= 0) return;
  const unsigned long long pieces = (max_bytes + (64 << 10) - 1) / (64 << 10);
  dim3 grid((unsigned)(pieces < 1 ? 1 : pieces > 2048 ? 2048 : pieces), (unsigned)(n > 65535 ? 65535 : n));
  k_multi_copy<<<grid, 256, 0, s>>>(d, n);
}

// ------------------------------------------------ simulation (TLC -simulate)
// One lane per walker: a random behaviour from Init, up to `depth` steps.  Each
// step evaluates every Next binding of the current state (all lanes of a wave
// on the same binding, as in k_expand phase B), picks one enabled successor
// uniformly at random, writes it, and checks the cfg's invariants on it.  A
// state with no successor ends the behaviour (-deadlock).  The chosen bindings
// are recorded so the host can replay a violating behaviour into a trace.
__device__ __forceinline__ unsigned long long splitmix(unsigned long long& x) {
  unsigned long long z = (x += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
constexpr int SIM_BLOCK = 64;
template <int SPEC, int N>
__global__ __launch_bounds__(SIM_BLOCK) void k_simulate(const uint32_t* __restrict__ init, unsigned long long walkers,
                                                        unsigned depth, unsigned long long seed, uint16_t* __restrict__ binds,
                                                        unsigned long long* __restrict__ counters, SimStatus* ss,
                                                        DevStatus* st) {
  extern __shared__ __align__(16) unsigned char lds[];
  const int words = cM.words, Wp = words | 1;
  const int tid = threadIdx.x;
  uint32_t* cur = (uint32_t*)lds + tid * Wp;                             // odd stride: conflict-free
  uint32_t* nxt = (uint32_t*)lds + SIM_BLOCK * Wp + tid * words;         // 16 B aligned rows for apply_delta
  const unsigned long long w = (unsigned long long)blockIdx.x * SIM_BLOCK + tid;
  if (w >= walkers) return;
  for (int q = 0; q < words; q++) cur[q] = init[q];
  unsigned long long rng = seed ^ (w * 0xD1B54A32D192ED03ULL);
  unsigned steps = 0;
  // every behaviour runs to its end (no early stop when another one fails):
  // the round's counts and its reported failure are then a function of the seed
  for (; steps < depth; steps++) {
    PState<SPEC, N> s{cur};
    const int nm = s.nmsg(), B = nbindings(cM, nm);
    int cnt = 0;
    for (int x = 0; x < B; x++) {
      Delta d;
      if (eval_binding<SPEC, N, SPEC != KRAFT>(s, cM, binding_at(cM, x, nm), d)) cnt++;
    }
    if (!cnt) break;  // no successor: the behaviour ends (-deadlock)
    int r = (int)(splitmix(rng) % (unsigned long long)cnt);
    Delta d;
    int b = 0;
    for (int x = 0; x < B; x++) {
      b = binding_at(cM, x, nm);
      if (eval_binding<SPEC, N, SPEC != KRAFT>(s, cM, b, d) && r-- == 0) break;
    }
    binds[w * depth + steps] = (uint16_t)b;
    if (d.err) {  // an evaluation error in Next (TLC stops with an error)
      atomicMin(&ss->key, (w << 20) | ((unsigned long long)(steps + 1) << 2) | 2ULL);
      steps++;
      break;
    }
    int e = apply_delta<SPEC, N>(s, cM, d, nxt);
    if (e) { atomicOr(&st->cap_flags, 1u << e); break; }
    for (int q = 0; q < words; q++) cur[q] = nxt[q];
    int ierr = 0;
    PState<SPEC, N> ns{cur};
    int bad = check_invariants<SPEC, N>(ns, cM, ierr);
    if (ierr || bad >= 0) {
      atomicMin(&ss->key, (w << 20) | ((unsigned long long)(steps + 1) << 2) | (ierr ? 3ULL : 1ULL));
      steps++;
      break;
    }
  }
  atomicAdd(&counters[0], (unsigned long long)steps);  // states generated by this behaviour (after Init)
  atomicMax(&counters[1], (unsigned long long)steps);
}
template <int SPEC, int N>
static void launch_sim_t(const uint32_t* init, unsigned long long walkers, unsigned depth, unsigned long long seed,
                         uint16_t* binds, unsigned long long* counters, SimStatus* ss, DevStatus* st, int words,
                         hipStream_t s) {
  size_t lds = (size_t)SIM_BLOCK * ((words | 1) + words) * 4;
  hipLaunchKernelGGL((k_simulate<SPEC, N>), dim3((unsigned)((walkers + SIM_BLOCK - 1) / SIM_BLOCK)), dim3(SIM_BLOCK),
                     lds, s, init, walkers, depth, seed, binds, counters, ss, st);
}
void launch_simulate(int spec, int N, const uint32_t* init, unsigned long long walkers, unsigned depth,
                     unsigned long long seed, uint16_t* binds, unsigned long long* counters, SimStatus* ss,
                     DevStatus* st, int words, hipStream_t s) {
#define RMC_SIM(SP, NN) \
  if (spec == SP && N == NN) return launch_sim_t<SP, NN>(init, walkers, depth, seed, binds, counters, ss, st, words, s);
  RMC_SIM(RAFT, 3)
#ifndef RMC_DEV_ONE
  RMC_SIM(RAFT, 2) RMC_SIM(RAFT, 4) RMC_SIM(RAFT, 5)
  RMC_SIM(FLEX, 2) RMC_SIM(FLEX, 3) RMC_SIM(FLEX, 4) RMC_SIM(FLEX, 5)
  RMC_SIM(FSYNC, 2) RMC_SIM(FSYNC, 3) RMC_SIM(FSYNC, 4) RMC_SIM(FSYNC, 5)
  RMC_SIM(PULL, 2) RMC_SIM(PULL, 3) RMC_SIM(PULL, 4) RMC_SIM(PULL, 5)
  RMC_SIM(PULL2, 2) RMC_SIM(PULL2, 3) RMC_SIM(PULL2, 4) RMC_SIM(PULL2, 5)
  RMC_SIM(KRAFT, 2) RMC_SIM(KRAFT, 3)
#endif
#undef RMC_SIM
}

hipError_t upload_model(const Model& m) { return hipMemcpyToSymbol(HIP_SYMBOL(cM), &m, sizeof(Model)); }

}  // namespace rmc
