// rmc_engine.h — interface between the host driver (rmc_engine.cpp) and the
// HIP kernels (rmc_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include "rmc_spec.h"

namespace rmc {

struct DevStatus {
  unsigned long long err_key;      // first (TLC order) evaluation error in Next
  unsigned long long inv_err_key;  // first evaluation error inside an invariant
  unsigned long long viol_key;     // first new state violating an invariant
  unsigned cap_flags;              // bit e set: capacity overflow ErrCode e
  unsigned max_msgs;               // largest |DOMAIN messages| of a materialized state
  unsigned long long hidden_coll;  // same-level duplicates whose hidden variables differ from the winner's
  unsigned long long row_words;    // -DRMC_ROWSTATS builds: words of the materialized rows up to their last message
};

// simulation mode: the first behaviour to stop the run (violation / error)
struct SimStatus {
  // the failing behaviour with the lowest walker index (atomicMin, so the
  // report does not depend on wave scheduling): walker << 20 | steps << 2 |
  // kind (1 invariant violated, 2 evaluation error in Next, 3 in an
  // invariant); ~0 = none.  Decoded by the host into the fields below.
  unsigned long long key;
  unsigned stop;   // kind, 0 = none
  unsigned steps;  // steps of the failing behaviour (its last binding is the failing one)
  unsigned long long walker;
};

// Where a generator's winners go when the next-level owners share its device
// (logical shards): winners [first, next piece's first) in the generator's
// TLC order are rows out[0..], trace records trp[0..] / trb[0..].
struct MatPiece {
  unsigned long long first;
  uint32_t* out;
  unsigned long long* trp;
  uint16_t* trb;
};
struct LevelArgs {
  const Model* model;
  const uint32_t* frontier;
  unsigned long long nparents, pbase;
  unsigned level;  // level of the successors (parents are level-1)
  unsigned long long floor;  // (first global index of the parents' level) << 26: entries below are older
  int sharded;               // W > 0 shards: k_expand inserts only the fps this shard owns, the owners the rest
  int shard_self;            // this shard's id (sharded search)
  unsigned long long* table;  // fingerprint set: (fp, val) entries
  unsigned long long mask;
  unsigned long long* cand_slot;  // CAND_DUP or hidden << 47 | slot; sharded, remote owner: the candidate's fp
  unsigned long long* cand_val;   // sharded: remote owner: rank << 16 | hidden (rmc_fpset.h); local: the fp
  uint32_t* cand_ob;
  uint16_t* cand_win;
  uint32_t *par_off, *par_n, *par_win, *par_pos;
  unsigned long long* counters;
  unsigned long long cand_cap;
  uint32_t* out;
  unsigned long long out_base_global;
  unsigned long long* tr_parent;
  uint16_t* tr_bind;
  const MatPiece* pieces;  // k_materialize: npieces > 0 replaces out / tr_* (pieces[0].first == 0)
  int npieces;
  DevStatus* st;
  int diag;  // RMC_DIAG builds: k_expand stops after a phase (rmc_selftest_profile_expand); 0 = the real kernel
};

void launch_expand(int spec, int N, const LevelArgs& a, hipStream_t s);
void launch_mark(const LevelArgs& a, hipStream_t s);
void launch_materialize(int spec, int N, const LevelArgs& a, hipStream_t s);
// ew: entry width in 64-bit words (2: 64-bit fingerprints, 4: 128-bit)
void launch_rehash(const unsigned long long* old, unsigned long long nold, unsigned long long* nt,
                   unsigned long long nmask, DevStatus* st, hipStream_t s, int ew = 2);

// compact host-frontier rows (rmc_kernels.hip): words per row (1 + 4N + nmsg), pack / unpack
// (a header whose length would pass max_words is clamped to it and sets *flag: a row never written)
void launch_row_words(const uint32_t* rows, unsigned long long n, int W, int hdr_words, int max_words,
                      uint32_t* lens32, uint8_t* lens8, unsigned* flag, hipStream_t s);
void launch_widen_lens(const uint8_t* lens8, unsigned long long n, uint32_t* lens32, hipStream_t s);
void launch_pack_rows(const uint32_t* rows, unsigned long long n, int W, const uint32_t* offs, const uint32_t* lens32,
                      uint32_t* out, hipStream_t s);
void launch_unpack_rows(const uint32_t* in, unsigned long long n, int W, const uint32_t* offs, const uint32_t* lens32,
                        uint32_t* rows, hipStream_t s);
// widening the rows mid-check (rmc_kernels.hip): reset the chunk's claimed ranks, restride rows
void launch_reset_ranks(unsigned long long* table, unsigned long long slots, int ew, unsigned long long lo,
                        unsigned long long hi, hipStream_t s);
void launch_restride(const uint32_t* src, unsigned long long n, int Wo, int Wn, uint32_t* dst, hipStream_t s);
// batched device-to-device copies (one launch for a whole exchange step)
struct CopyDesc {
  const void* src;
  void* dst;
  unsigned long long bytes;
};
void launch_multi_copy(const CopyDesc* d, int n, unsigned long long max_bytes, hipStream_t s);
size_t scan_temp_bytes(unsigned long long n);
void launch_scan(void* temp, size_t temp_bytes, const uint32_t* in, uint32_t* out, unsigned long long n,
                 hipStream_t s);
hipError_t upload_model(const Model& m);

// sharded search (rmc_sharded.cpp)
unsigned long long bucket_blocks(unsigned long long n);
// blk_counts / blk_off: owner-major [W][bucket_blocks(n)]
// sharded search: generator-side dedup of a tile's remote-owner candidates (OB_TDUP)
void launch_tile_dedup(const LevelArgs& a, unsigned long long* cand_fp, unsigned long long* cand_val,
                       uint32_t* cand_ob, hipStream_t s);
void launch_owner_count(const unsigned long long* cand_fp, const uint32_t* cand_ob, unsigned long long n, int W,
                        unsigned int* blk_counts, hipStream_t s);
void launch_bucket(const unsigned long long* cand_fp, const unsigned long long* cand_val, const uint32_t* cand_ob,
                   unsigned long long n, int W, const unsigned int* blk_off, unsigned long long* send, uint32_t* perm,
                   hipStream_t s, const unsigned long long* dbase = nullptr);
void launch_insert_recv(const unsigned long long* recv, unsigned long long n, unsigned long long* table,
                        unsigned long long mask, unsigned long long floor, unsigned long long* recv_slot, DevStatus* st,
                        hipStream_t s);
void launch_mark_recv(const unsigned long long* recv, const unsigned long long* recv_slot, unsigned long long n,
                      const unsigned long long* table, unsigned long long floor, uint8_t* flag,
                      unsigned long long* newcount, DevStatus* st, hipStream_t s,
                      const unsigned long long* fbase = nullptr, const unsigned long long* rseg = nullptr, int W = 0);
// k_mark for the sharded search: a (cand_ob, cand_slot, cand_val,
// par_off/par_n -> cand_win/par_win, table/mask/floor, pbase, st); moved = the
// table grew since k_expand (local-owner candidates are found by fp)
void launch_mark_gen(const LevelArgs& a, int moved, const uint32_t* perm, const uint8_t* flag_back,
                     unsigned long long* newcount, hipStream_t s);
int host_fp_owner(unsigned long long fp, int W);
void read_stamps(unsigned long long* out);  // -DRMC_STAMPS diagnostic builds
void read_fpstats(unsigned long long* out);
bool diag_build();  // compiled with -DRMC_DIAG (k_expand phase cutoffs)  // -DRMC_FPSTATS diagnostic builds (8 counters, rmc_fpset.h)
void launch_simulate(int spec, int N, const uint32_t* init, unsigned long long walkers, unsigned depth,
                     unsigned long long seed, uint16_t* binds, unsigned long long* counters, SimStatus* ss,
                     DevStatus* st, int words, hipStream_t s);

// host-side (rmc_host.cpp): replay + formatting use the same action code
int host_eval_apply(const Model& M, const uint32_t* parent, int binding, uint32_t* out, int* ordinal, int* act,
                    int* err);
unsigned long long host_fingerprint(const Model& M, const uint32_t* S);
void host_fingerprint2(const Model& M, const uint32_t* S, unsigned long long* ab);  // 128-bit (fp_bits 128)
int host_check_invariants(const Model& M, const uint32_t* S, int* err);
int host_fp_check(const Model& M, const uint32_t* parent, int binding, const uint32_t* row);

}  // namespace rmc
