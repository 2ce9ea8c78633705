// rmc_spec.h — packed state layout and the four Raft specs' Next actions as
// __host__ __device__ functions over it.  Shared by the HIP kernels and the
// host-side trace replay of librmc.  (The CPU oracle in oracle/ is a separate,
// independent restatement and does not include this file.)
//
// Packed state (u32 words; all specs):
//   S[0]            header: nmsg 0-7 | electionCtr 8-11 | restartCtr 12-15 |
//                   acked[v] 16+2v (0 Nil, 1 FALSE, 2 TRUE)
//   S[1+4i+0] (A)   server i: currentTerm 0-3 | state 4-5 | votedFor/leader 6-8
//                   (7 = Nil) | Len(log) 9-11 | commitIndex 12-14 |
//                   fsyncIndex 15-17 | votesGranted 18-24 | pendingResponse 25-31
//   S[1+4i+1] (B)   log: entry x (0-based) at 6x: term 0-3 | value 4-5
//   S[1+4i+2] (C)   nextIndex[i][j] at 3j (PullRaft: unused; PullRaftVariant2:
//                   votesLastEntry[i][j] for j != i at 7*slot(i, j), slot =
//                   j - (j > i): index+1 0-2 (0 = Nil) | term 3-6)
//   S[1+4i+3] (D)   matchIndex[i][j] at 3j
//   PullRaft: bits 6-8 of A hold leader[i]; PullRaftVariant2: leader[i] in
//   6-8 and votedFor[i] in 15-17 (the fsyncIndex bits of RaftFsync).
//   S[1+4N+k]       DOMAIN messages, ascending = TLC's value order; record in
//                   bits 3-31 (layouts below), count (messages[m]) in bits 0-2.
//
// Message records are laid out MSB-first in exactly the order TLC compares
// them (RecordValue.compareTo: field count, then sorted field names with
// their values), so unsigned comparison of two words IS TLC's order and a
// sorted word array IS TLC's DOMAIN enumeration order (SURVEY.md §7 hard part
// 3, Appendix A.4).  Field-name orders:
//   Raft.tla:251-256 RVReq  {mdest, mlastLogIndex, mlastLogTerm, msource, mterm, mtype}
//   Raft.tla:374-378 RVResp {mdest, msource, mterm, mtype, mvoteGranted}
//   Raft.tla:277-284 AEReq  {mcommitIndex, mdest, mentries, mprevLogIndex, mprevLogTerm, msource, mterm, mtype}
//   Raft.tla:422-427 AEResp {mdest, mmatchIndex, msource, msuccess, mterm, mtype}
//   PullRaft.tla:361-364 LeaderNotify {mdest, msource, mterm, mtype}
//   PullRaft.tla:405-410 PullReq {same names as RVReq}
//   PullRaft.tla:426-433 PullResp fail {mdest, mlastCommonEntry, msource, msuccess, mterm, mtype}
//   PullRaft.tla:480-486 PullResp ok   {mcommitIndex, mdest, mentries, msource, msuccess, mterm, mtype}
//   PullRaftVariant2.tla:317-323 RVResp {mdest, mlastLogIndex, mlastLogTerm, msource, mterm, mtype, mvoteGranted}
//   PullRaftVariant2.tla:369-377 LeaderNotify {mdest, mlastCommonEntry, msource, mterm, mtype}, where
//                       mlastCommonEntry is Nil (below every record) or [index, term]
#pragma once
#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RMC_HD __host__ __device__ __forceinline__
#else
#define RMC_HD static inline
#endif
// Compiled guards (guard_vm) are evaluated only in code instantiated for them:
// the device kernels take them as a template flag, launched with it only for a
// model that has one (inlining the machine into every kernel costs the library
// actions registers and spills); host code always has it.
#if defined(__HIP_DEVICE_COMPILE__)
#define RMC_G_DEFAULT false
#else
#define RMC_G_DEFAULT true
#endif

namespace rmc {

enum SpecKind { RAFT = 0, FLEX = 1, FSYNC = 2, PULL = 3, PULL2 = 4, KRAFT = 5 };
// the pull family (PullRaft, PullRaftVariant2): no nextIndex, LeaderNotify, pull replication
constexpr bool pullish(int spec) { return spec == PULL || spec == PULL2; }
enum SrvState { FOLLOWER = 0, CANDIDATE = 1, LEADER = 2 };
enum MType { RVREQ = 0, RVRESP = 1, AEREQ = 2, AERESP = 3, LNREQ = 4, PEREQ = 5, PERESP = 6,
             KBQREQ = 7, KBQRESP = 8, KFREQ = 9, KFRESP = 10 };  // KRaft's BeginQuorum*, Fetch*
enum ActId {
  A_RESTART = 0, A_REQUESTVOTE, A_TIMEOUT, A_RVIJ, A_BECOMELEADER, A_CLIENT, A_ADVCOMMIT,
  A_APPENDENTRIES, A_ADVFSYNC, A_UPDATETERM, A_HRVREQ, A_HRVRESP, A_REJAE, A_ACCAE, A_HAERESP,
  A_REJPULL, A_ACCPULL, A_LEARN, A_SENDPULL, A_HSUCC, A_HFAIL,
  // KRaft (pull-raft/KRaft.tla:823-840)
  A_KREJFETCH, A_KDIVFETCH, A_KACCFETCH, A_KHBQ, A_KSENDFETCH, A_KHSUCC, A_KHDIV, A_KHERR,
  // the network actions every module defines but leaves out of Next (Raft.tla:509-522, :540-541):
  // DuplicateMessage(m) / DropMessage(m), bound by \E m \in DOMAIN messages (the TLA+ front end
  // lowers them when a module's Next re-enables them; rmc_tla.cpp)
  A_DUP, A_DROP,
  // actions the TLA+ front end compiles whole (guard and effect, rmc_guard.cpp
  // compile_effect): Model::gstart / estart hold their programs
  A_C0, A_C1, A_C2, A_C3, A_NUM
};
constexpr int MAXCOMPILED = 4;
// binding forms: \E i \in Server (K_I), i \in Server, v \in Value (K_IV), i, j \in Server (K_IJ), a message
// handler ranging over DOMAIN messages with one enabled action per element (K_MSG), and an action bound
// by \E m \in DOMAIN messages that is NOT exclusive with the handlers (K_M: its bindings are fixed
// bindings, one per message slot k = x, encoded in a fixed binding's (i, jv) as k & 15, k >> 4)
// bindings, one per message slot k = x, encoded in a fixed binding's (i, jv) as k & 15, k >> 4), and a
// message handler the front end compiles whole (K_MSGC, rmc_guard.cpp compile_handler): evaluated on every
// DOMAIN element on its own (not assumed exclusive with the library's handlers), its binding for slot k is
// nfixed + MSGC_STRIDE * (1 + q) + k for compiled action A_C0 + q -- independent of the slot count, so trace
// records written before a widening keep their meaning
enum ActKind { K_I = 0, K_IV = 1, K_IJ = 2, K_MSG = 3, K_M = 4, K_MSGC = 5 };
constexpr int MSGC_STRIDE = 128;
enum ErrCode {
  E_NONE = 0,
  E_DOMAIN = 1,     // TLC evaluation error: sequence applied outside its domain
  E_CAP_LOG = 2,    // log longer than the packed layout holds
  E_CAP_MSG = 3,    // more messages than msg_cap_K
  E_CAP_COUNT = 4,  // message multiplicity > 7
  E_CAP_TERM = 5,   // term > 15
  E_CAP_FIELD = 6,  // an index field > 7
  E_CAP_SUCC = 7,   // more successors for one state than the candidate buffer holds
  E_CAP_TABLE = 8,  // fingerprint set full
  E_CAP_FRONTIER = 9,
  E_RETRY = 10  // fp_bits 128: a key's second word was read before its claimer stored it (the chunk is redone)
};
constexpr int NILS = 7;
constexpr int MAXN = 7, MAXV = 4, MAXLOG = 5, MAXOPS = 7, MAXPERM = 120, MAXACT = 16, MAXFIXED = 192;
constexpr int MAXGCODE = 512;
// apply_delta on the device: the merge stops at the wave's largest message
// count and reads the parent's messages four per LDS round trip.  Measured
// and not the default (r06, bench workload, CLI, three interleaved rounds,
// profiles/r06/ab_merge_batch.txt): k_materialize 242-244 ms against 240-241
// for the loop form (M.kmax steps, one dependent read per step) -- the
// merge's LDS chain is not what bounds k_materialize.
#ifndef RMC_MERGE_BATCH
#define RMC_MERGE_BATCH 0
#endif  // words of compiled guard code (Model::gcode)

struct Model {
  int spec, N, V, E, R, EQ, RQ, lfae, lfiq, ffbr;
  int kmax, words;  // words = 1 + 4N + kmax
  int nperm;
  uint32_t perm[MAXPERM];  // permutation p maps server j -> (perm[p] >> 3j) & 7
  // invariant ids in cfg order: 0 LHAAV, 1 NLD, 2 CERM, 3 NTLISE, 4 NIS (KRaft); the classic Raft
  // properties, opt-in (not defined by the reference specs): 5 ElectionSafety, 6 LogMatching,
  // 7 LeaderCompleteness, 8 StateMachineSafety
  int ninv, inv[9];
  int nact, act_id[MAXACT], act_kind[MAXACT], act_off[MAXACT];
  int nfixed;
  uint8_t fb_act[MAXFIXED], fb_x[MAXFIXED];  // fixed binding -> (action slot, binding index)
  // fixed binding -> slot | x << 8 | act_id << 16 | i << 24 | j-or-v << 28 (one load instead of a chain)
  uint32_t fb_desc[MAXFIXED];
  uint8_t act_fb_first[MAXACT], act_fb_end[MAXACT];  // action slot -> its fixed bindings [first, end)
  int msg_act_slot[A_NUM];                   // action slot of each message action
  uint16_t msg_off[A_NUM];                   // = act_off[msg_act_slot[a]]: its first ordinal (one load, not a chain)
  unsigned long long msg_act_mask;           // bit a: message action a is a disjunct of this model's Next
  int ordinal_limit;
  int fpw;                    // fingerprint width in 64-bit words (1: 64-bit, 2: 128-bit)
  int bind_words, ord_words;  // u32 words of a per-parent bitmask over bindings / over ordinals
  uint16_t ord2b[1024];       // TLC ordinal -> binding (fixed bindings; message actions: nfixed + DOMAIN index)
  // Compiled guards (the TLA+ front end, rmc_tla.cpp compile_guard): an action
  // whose module text keeps the library action's effect but states its own
  // guard runs the library effect unguarded, behind this program.  gstart[a]
  // = first word of action id a's program in gcode, -1 = the library guard.
  int16_t gstart[A_NUM];
  // Compiled effects (rmc_guard.cpp compile_effect): estart[k] = first word of
  // action A_C0 + k's effect program in gcode (its guard is at gstart[A_C0 + k])
  int16_t estart[MAXCOMPILED];
  int gany;  // some action has a compiled guard (or is compiled whole)
  // compiled message handlers (K_MSGC): how many, and each one's compiled-action index q (A_C0 + q)
  int nmsgc;
  int8_t msgc_q[MAXCOMPILED];
  uint32_t gcode[MAXGCODE];
};
// Bindings a parent with nm DOMAIN elements has, and the idx-th of them: the
// fixed bindings, one per DOMAIN element for the library's handlers, then one
// per element for each compiled handler (host loops; the order is immaterial,
// successors are ordered by their TLC ordinal).
RMC_HD int nbindings(const Model& M, int nm) { return M.nfixed + nm * (1 + M.nmsgc); }
RMC_HD int binding_at(const Model& M, int idx, int nm) {
  if (idx < M.nfixed + nm) return idx;
  const int r = idx - M.nfixed - nm;
  return M.nfixed + MSGC_STRIDE * (1 + M.msgc_q[r / nm]) + r % nm;
}
// Successors one parent can have at most (the candidate buffers' bound).
RMC_HD int max_successors(const Model& M) { return M.nfixed + M.kmax * (1 + M.nmsgc); }

// ------------------------------------------------------------- bit helpers
RMC_HD uint32_t getb(uint32_t w, int pos, int width) { return (w >> pos) & ((1u << width) - 1u); }
RMC_HD uint32_t setb(uint32_t w, int pos, int width, uint32_t v) {
  uint32_t m = ((1u << width) - 1u) << pos;
  return (w & ~m) | ((v << pos) & m);
}
// header
RMC_HD int h_nmsg(uint32_t h) { return (int)(h & 0xFF); }
RMC_HD int h_ectr(uint32_t h) { return (int)getb(h, 8, 4); }
RMC_HD int h_rctr(uint32_t h) { return (int)getb(h, 12, 4); }
RMC_HD int h_acked(uint32_t h, int v) { return (int)getb(h, 16 + 2 * v, 2); }
// server word A
RMC_HD int a_term(uint32_t a) { return (int)getb(a, 0, 4); }
RMC_HD int a_st(uint32_t a) { return (int)getb(a, 4, 2); }
RMC_HD int a_voted(uint32_t a) { return (int)getb(a, 6, 3); }
RMC_HD int a_len(uint32_t a) { return (int)getb(a, 9, 3); }
RMC_HD int a_commit(uint32_t a) { return (int)getb(a, 12, 3); }
RMC_HD int a_fsync(uint32_t a) { return (int)getb(a, 15, 3); }
RMC_HD int a_votes(uint32_t a) { return (int)getb(a, 18, 7); }
RMC_HD int a_pending(uint32_t a) { return (int)getb(a, 25, 7); }
// The variables VIEW drops, from a header word (16 bits): electionCtr,
// restartCtr and acked (Raft.tla:115, FlexibleRaft.tla:117, RaftFsync.tla:117,
// PullRaftVariant2.tla:114); PullRaft's view keeps acked, so only the counters
// (PullRaft.tla:123).
template <int SPEC>
RMC_HD uint32_t hidden_of(uint32_t h) {
  return (SPEC == 3 /* PULL */ || SPEC == 5 /* KRAFT, KRaft.tla:154 */) ? (h >> 8) & 0xFFu : (h >> 8) & 0xFFFFu;
}
// PullRaftVariant2: votedFor[i] (bits 15-17 of A) and votesLastEntry row (C)
RMC_HD int a_votedfor2(uint32_t a) { return (int)getb(a, 15, 3); }
RMC_HD int vle_slot(int i, int j) { return j - (j > i ? 1 : 0); }
RMC_HD uint32_t vle_get(uint32_t c, int i, int j) { return (c >> (7 * vle_slot(i, j))) & 0x7Fu; }  // 0 = Nil
RMC_HD uint32_t vle_set(uint32_t c, int i, int j, int index, int term) {
  return setb(c, 7 * vle_slot(i, j), 7, (uint32_t)((index + 1) | (term << 3)));
}
// log word B
RMC_HD int e_term(uint32_t b, int x) { return (int)getb(b, 6 * x, 4); }
RMC_HD int e_value(uint32_t b, int x) { return (int)getb(b, 6 * x + 4, 2); }
RMC_HD uint32_t e_pack(int term, int value) { return (uint32_t)(term | (value << 4)); }
// C/D rows
RMC_HD int row_get(uint32_t w, int j) { return (int)getb(w, 3 * j, 3); }
RMC_HD uint32_t row_set(uint32_t w, int j, int v) { return setb(w, 3 * j, 3, (uint32_t)v); }

// ------------------------------------------------------------ messages
struct MsgF {
  int type, term, src, dst;
  int lli, llt;               // mlastLogIndex, mlastLogTerm
  int granted;                // mvoteGranted
  int pli, plt;               // mprevLogIndex, mprevLogTerm
  int nent, eterm, evalue;    // mentries
  int commit;                 // mcommitIndex
  int success, midx;          // msuccess, mmatchIndex
  int lci, lct;               // mlastCommonEntry.index/.term
  int lcenil;                 // PullRaftVariant2 LeaderNotify: mlastCommonEntry = Nil
  int count;
};
RMC_HD MsgF msg_zero() {
  MsgF f;
  f.type = f.term = f.src = f.dst = f.lli = f.llt = f.granted = f.pli = f.plt = 0;
  f.nent = f.eterm = f.evalue = f.commit = f.success = f.midx = f.lci = f.lct = f.lcenil = f.count = 0;
  return f;
}
struct Bits {
  uint32_t v;
  int pos;
  RMC_HD void put(int x, int w) { pos -= w; v |= ((uint32_t)x & ((1u << w) - 1u)) << pos; }
};
struct Rd {
  uint32_t v;
  int pos;
  RMC_HD int get(int w) { pos -= w; return (int)((v >> pos) & ((1u << w) - 1u)); }
};
// PullRaftVariant2's record classes, in TLC order (field count, then names):
//   cls0 LeaderNotify (5 fields): dst | lce Nil 0 / record 1 | lce.index 3 | lce.term 4 | src | term
//   cls1 6 fields, mdest first: dst | 0 = PullResp fail (mlastCommonEntry < mlastLogIndex) | 1 = request
//   cls2 PullResp ok (7 fields, mcommitIndex first), as PullRaft's cls3
//   cls3 RVResp (7 fields, mdest first): dst | lli | llt | src | term | granted
template <int SPEC>
RMC_HD uint32_t msg_encode(const MsgF& f) {
  Bits b{0u, 32};
  if (SPEC == PULL2) {
    switch (f.type) {
      case LNREQ:
        b.put(0, 2); b.put(f.dst, 3); b.put(f.lcenil ? 0 : 1, 1); b.put(f.lcenil ? 0 : f.lci, 3);
        b.put(f.lcenil ? 0 : f.lct, 4); b.put(f.src, 3); b.put(f.term, 4); break;
      case RVRESP:
        b.put(3, 2); b.put(f.dst, 3); b.put(f.lli, 3); b.put(f.llt, 4); b.put(f.src, 3); b.put(f.term, 4);
        b.put(f.granted, 1); break;
      case RVREQ: case PEREQ:
        b.put(1, 2); b.put(f.dst, 3); b.put(1, 1); b.put(f.lli, 3); b.put(f.llt, 4); b.put(f.src, 3); b.put(f.term, 4);
        b.put(f.type == RVREQ ? 1 : 0, 1); break;
      default: /* PERESP */
        if (!f.success) {
          b.put(1, 2); b.put(f.dst, 3); b.put(0, 1); b.put(f.lci, 3); b.put(f.lct, 4); b.put(f.src, 3); b.put(0, 1); b.put(f.term, 4);
        } else {
          b.put(2, 2); b.put(f.commit, 3); b.put(f.dst, 3); b.put(f.nent, 1); b.put(f.eterm, 4); b.put(f.evalue, 2);
          b.put(f.src, 3); b.put(1, 1); b.put(f.term, 4);
        }
        break;
    }
  } else if (SPEC != PULL) {
    switch (f.type) {
      case RVRESP: b.put(0, 2); b.put(f.dst, 3); b.put(f.src, 3); b.put(f.term, 4); b.put(f.granted, 1); break;
      case RVREQ: b.put(1, 2); b.put(f.dst, 3); b.put(0, 1); b.put(f.lli, 3); b.put(f.llt, 4); b.put(f.src, 3); b.put(f.term, 4); break;
      case AERESP: b.put(1, 2); b.put(f.dst, 3); b.put(1, 1); b.put(f.midx, 3); b.put(f.src, 3); b.put(f.success, 1); b.put(f.term, 4); break;
      default: /* AEREQ */
        b.put(2, 2); b.put(f.commit, 3); b.put(f.dst, 3); b.put(f.nent, 1); b.put(f.eterm, 4); b.put(f.evalue, 2);
        b.put(f.pli, 3); b.put(f.plt, 4); b.put(f.src, 3); b.put(f.term, 4); break;
    }
  } else {
    switch (f.type) {
      case LNREQ: b.put(0, 2); b.put(f.dst, 3); b.put(f.src, 3); b.put(f.term, 4); break;
      case RVRESP: b.put(1, 2); b.put(f.dst, 3); b.put(f.src, 3); b.put(f.term, 4); b.put(f.granted, 1); break;
      case RVREQ: case PEREQ:
        b.put(2, 2); b.put(f.dst, 3); b.put(1, 1); b.put(f.lli, 3); b.put(f.llt, 4); b.put(f.src, 3); b.put(f.term, 4);
        b.put(f.type == RVREQ ? 1 : 0, 1); break;
      default: /* PERESP */
        if (!f.success) {
          b.put(2, 2); b.put(f.dst, 3); b.put(0, 1); b.put(f.lci, 3); b.put(f.lct, 4); b.put(f.src, 3); b.put(0, 1); b.put(f.term, 4);
        } else {
          b.put(3, 2); b.put(f.commit, 3); b.put(f.dst, 3); b.put(f.nent, 1); b.put(f.eterm, 4); b.put(f.evalue, 2);
          b.put(f.src, 3); b.put(1, 1); b.put(f.term, 4);
        }
        break;
    }
  }
  return b.v | ((uint32_t)f.count & 7u);
}
template <int SPEC>
RMC_HD MsgF msg_decode(uint32_t w) {
  MsgF f = msg_zero();
  Rd r{w, 32};
  f.count = (int)(w & 7u);
  int cls = r.get(2);
  if (SPEC == PULL2) {
    if (cls == 0) {
      f.type = LNREQ; f.dst = r.get(3); f.lcenil = r.get(1) ? 0 : 1; f.lci = r.get(3); f.lct = r.get(4);
      f.src = r.get(3); f.term = r.get(4);
    } else if (cls == 1) {
      f.dst = r.get(3);
      if (r.get(1) == 0) { f.type = PERESP; f.success = 0; f.lci = r.get(3); f.lct = r.get(4); f.src = r.get(3); r.get(1); f.term = r.get(4); }
      else { f.lli = r.get(3); f.llt = r.get(4); f.src = r.get(3); f.term = r.get(4); f.type = r.get(1) ? RVREQ : PEREQ; }
    } else if (cls == 2) {
      f.type = PERESP; f.success = 1; f.commit = r.get(3); f.dst = r.get(3); f.nent = r.get(1); f.eterm = r.get(4);
      f.evalue = r.get(2); f.src = r.get(3); r.get(1); f.term = r.get(4);
    } else {
      f.type = RVRESP; f.dst = r.get(3); f.lli = r.get(3); f.llt = r.get(4); f.src = r.get(3); f.term = r.get(4);
      f.granted = r.get(1);
    }
  } else if (SPEC != PULL) {
    if (cls == 0) { f.type = RVRESP; f.dst = r.get(3); f.src = r.get(3); f.term = r.get(4); f.granted = r.get(1); }
    else if (cls == 1) {
      f.dst = r.get(3);
      if (r.get(1) == 0) { f.type = RVREQ; f.lli = r.get(3); f.llt = r.get(4); f.src = r.get(3); f.term = r.get(4); }
      else { f.type = AERESP; f.midx = r.get(3); f.src = r.get(3); f.success = r.get(1); f.term = r.get(4); }
    } else {
      f.type = AEREQ; f.commit = r.get(3); f.dst = r.get(3); f.nent = r.get(1); f.eterm = r.get(4); f.evalue = r.get(2);
      f.pli = r.get(3); f.plt = r.get(4); f.src = r.get(3); f.term = r.get(4);
    }
  } else {
    if (cls == 0) { f.type = LNREQ; f.dst = r.get(3); f.src = r.get(3); f.term = r.get(4); }
    else if (cls == 1) { f.type = RVRESP; f.dst = r.get(3); f.src = r.get(3); f.term = r.get(4); f.granted = r.get(1); }
    else if (cls == 2) {
      f.dst = r.get(3);
      if (r.get(1) == 0) { f.type = PERESP; f.success = 0; f.lci = r.get(3); f.lct = r.get(4); f.src = r.get(3); r.get(1); f.term = r.get(4); }
      else { f.lli = r.get(3); f.llt = r.get(4); f.src = r.get(3); f.term = r.get(4); f.type = r.get(1) ? RVREQ : PEREQ; }
    } else {
      f.type = PERESP; f.success = 1; f.commit = r.get(3); f.dst = r.get(3); f.nent = r.get(1); f.eterm = r.get(4);
      f.evalue = r.get(2); f.src = r.get(3); r.get(1); f.term = r.get(4);
    }
  }
  return f;
}
// Bit positions (LSB index) of msource / mdest / mterm within a message word,
// from the MSB-first layouts of msg_encode (checked against msg_decode by the
// CPU test tests/test_layout.py):
//   Raft  cls0 RVResp  dst27 src24 term20 | cls1 RVReq dst27 src16 term12 |
//         cls1 AEResp  dst27 src20 term15 | cls2 AEReq dst24 src7  term3
//   Pull  cls0 LN      dst27 src24 term20 | cls1 RVResp dst27 src24 term20 |
//         cls2 fail    dst27 src16 term11 | cls2 req   dst27 src16 term12 (isRV at 11) |
//         cls3 ok      dst24 src14 term9
//   Pull2 cls0 LN      dst27 src16 term12 | cls1 fail   dst27 src16 term11 |
//         cls1 req     dst27 src16 term12 (isRV at 11) | cls2 ok dst24 src14 term9 |
//         cls3 RVResp  dst27 src17 term13
template <int SPEC>
RMC_HD void msg_srcdst_pos(uint32_t w, int& sp, int& dp) {
  int cls = (int)(w >> 30);
  if (SPEC == KRAFT) {  // 3-bit classes (kr_encode): the FetchResponses' servers are their correlation's
    const int c3 = (int)(w >> 29);
    dp = c3 >= 4 ? 17 : 26;
    sp = c3 >= 4 ? 26 : c3 == 0 ? 21 : c3 == 1 ? 19 : 16;
    return;
  }
  if (SPEC == PULL2) {
    if (cls == 0 || cls == 1) { dp = 27; sp = 16; }
    else if (cls == 2) { dp = 24; sp = 14; }
    else { dp = 27; sp = 17; }
  } else if (SPEC != PULL) {
    if (cls == 0) { dp = 27; sp = 24; }
    else if (cls == 1) { dp = 27; sp = ((w >> 26) & 1u) ? 20 : 16; }
    else { dp = 24; sp = 7; }
  } else {
    if (cls <= 1) { dp = 27; sp = 24; }
    else if (cls == 2) { dp = 27; sp = 16; }
    else { dp = 24; sp = 14; }
  }
}
template <int SPEC>
RMC_HD int msg_type(uint32_t w) {
  int cls = (int)(w >> 30);
  if (SPEC == KRAFT) {
    const int c3 = (int)(w >> 29);
    return c3 == 0 ? KBQREQ : c3 == 1 ? KBQRESP : c3 == 2 ? (((w >> 23) & 1u) ? RVREQ : KFREQ) : c3 == 3 ? RVRESP : KFRESP;
  }
  if (SPEC == PULL2) {
    if (cls == 0) return LNREQ;
    if (cls == 1) return ((w >> 26) & 1u) ? (((w >> 11) & 1u) ? RVREQ : PEREQ) : PERESP;
    if (cls == 2) return PERESP;
    return RVRESP;
  }
  if (SPEC != PULL) {
    if (cls == 0) return RVRESP;
    if (cls == 1) return ((w >> 26) & 1u) ? AERESP : RVREQ;
    return AEREQ;
  }
  if (cls == 0) return LNREQ;
  if (cls == 1) return RVRESP;
  if (cls == 2) return ((w >> 26) & 1u) ? (((w >> 11) & 1u) ? RVREQ : PEREQ) : PERESP;
  return PERESP;
}
template <int SPEC>
RMC_HD int msg_term(uint32_t w) {
  int cls = (int)(w >> 30);
  int pos;
  if (SPEC == KRAFT) {  // mepoch, 2 bits
    const int c3 = (int)(w >> 29);
    return (int)((w >> (c3 <= 3 ? 24 : c3 == 4 ? 15 : c3 == 5 ? 10 : 11)) & 3u);
  }
  if (SPEC == PULL2) {
    if (cls == 0) pos = 12;
    else if (cls == 1) pos = ((w >> 26) & 1u) ? 12 : 11;
    else if (cls == 2) pos = 9;
    else pos = 13;
  } else if (SPEC != PULL) {
    if (cls == 0) pos = 20;
    else if (cls == 1) pos = ((w >> 26) & 1u) ? 15 : 12;
    else pos = 3;
  } else {
    if (cls <= 1) pos = 20;
    else if (cls == 2) pos = ((w >> 26) & 1u) ? 12 : 11;
    else pos = 9;
  }
  return (int)((w >> pos) & 15u);
}
template <int SPEC>
RMC_HD int msg_dst(uint32_t w) {
  int sp, dp;
  msg_srcdst_pos<SPEC>(w, sp, dp);
  return (int)((w >> dp) & 7u);
}
RMC_HD uint32_t msg_rec(uint32_t w) { return w >> 3; }
RMC_HD int msg_count(uint32_t w) { return (int)(w & 7u); }

// ------------------------------------------------------------ KRaft messages
// KRaft (pull-raft/KRaft.tla) records, MSB-first in TLC's order (field count,
// then sorted field names with their values), class in bits 29-31:
//   c0 BeginQuorumRequest  (4 fields) mdest 26 | mepoch 24 | msource 21
//   c1 BeginQuorumResponse (5)        mdest 26 | mepoch 24 | merror 22 | msource 19
//   c2 6 fields: mdest 26 | mepoch 24 | then the third name: mfetchOffset (0,
//      FetchRequest: mfetchOffset 21 | mlastFetchedEpoch 19) < mlastLogEpoch (1,
//      RequestVoteRequest: mlastLogEpoch 21 | mlastLogOffset 19) at bit 23 | msource 16
//   c3 RequestVoteResponse (7)        mdest 26 | mepoch 24 | merror 22 | mleader 19 | msource 16 | mvoteGranted 15
//   c4 FetchResponse NotOk (9)  correlation | mepoch 15 | merror 13 | mhwm 11 | mleader 8
//   c5 FetchResponse Ok (10)    correlation | mentries (length 16, epoch 14, value 12) | mepoch 10 | mhwm 8 | mleader 5
//   c6 FetchResponse Diverging (11) correlation | mdivergingEndOffset 15 | mdivergingEpoch 13 | mepoch 11 | mhwm 9 | mleader 6
// correlation (the FetchRequest answered; its name sorts first) = mdest 26 |
// mepoch 24 | mfetchOffset 22 | mlastFetchedEpoch 20 | msource 17; the
// response's own mdest / msource are its correlation's msource / mdest, and
// its constant fields (mresult per class; merror = Nil for Ok / Diverging,
// KRaft.tla:670, :729) are not stored.  Value codes keep TLC's order: servers
// by name, mleader Nil 0 < servers 1.., merror FencedLeaderEpoch 0 < Nil 1 <
// NotLeader 2 < UnknownLeader 3 (model values by name); epochs and offsets 2
// bits (the model loader requires MaxElections <= 2, |Value| <= 3, N <= 3).
enum KErr { KE_FENCED = 0, KE_NIL = 1, KE_NOTLEADER = 2, KE_UNKNOWN = 3 };
enum KRes { KR_NOTOK = 4, KR_OK = 5, KR_DIV = 6 };  // = the FetchResponse's class
struct KMsg {
  int cls, dst, src, epoch, err, leader;  // leader: -1 = Nil
  int granted, f1, f2;                    // RVReq: lastLogEpoch, lastLogOffset; FetchReq: fetchOffset, lastFetchedEpoch
  int cepoch, cfo, clfe;                  // FetchResponse: correlation's mepoch, mfetchOffset, mlastFetchedEpoch
  int elen, eepoch, evalue, hwm, divend, divepoch;
  int count;
};
RMC_HD KMsg kmsg_zero() {
  KMsg m;
  m.cls = m.dst = m.src = m.epoch = m.err = m.granted = m.f1 = m.f2 = 0;
  m.cepoch = m.cfo = m.clfe = m.elen = m.eepoch = m.evalue = m.hwm = m.divend = m.divepoch = m.count = 0;
  m.leader = -1;
  m.err = KE_NIL;
  return m;
}
RMC_HD uint32_t kbits(int v, int pos, int w) { return ((uint32_t)v & ((1u << w) - 1u)) << pos; }
RMC_HD uint32_t kr_encode(const KMsg& m) {
  uint32_t w = (uint32_t)m.cls << 29;
  const int ld = m.leader < 0 ? 0 : m.leader + 1;
  switch (m.cls) {
    case 0: w |= kbits(m.dst, 26, 3) | kbits(m.epoch, 24, 2) | kbits(m.src, 21, 3); break;
    case 1: w |= kbits(m.dst, 26, 3) | kbits(m.epoch, 24, 2) | kbits(m.err, 22, 2) | kbits(m.src, 19, 3); break;
    case 2:
      w |= kbits(m.dst, 26, 3) | kbits(m.epoch, 24, 2) | kbits(m.granted, 23, 1) | kbits(m.f1, 21, 2) |
           kbits(m.f2, 19, 2) | kbits(m.src, 16, 3);
      break;
    case 3:
      w |= kbits(m.dst, 26, 3) | kbits(m.epoch, 24, 2) | kbits(m.err, 22, 2) | kbits(ld, 19, 3) | kbits(m.src, 16, 3) |
           kbits(m.granted, 15, 1);
      break;
    default:  // FetchResponse: correlation (a request from dst to src)
      w |= kbits(m.src, 26, 3) | kbits(m.cepoch, 24, 2) | kbits(m.cfo, 22, 2) | kbits(m.clfe, 20, 2) | kbits(m.dst, 17, 3);
      if (m.cls == KR_NOTOK) w |= kbits(m.epoch, 15, 2) | kbits(m.err, 13, 2) | kbits(m.hwm, 11, 2) | kbits(ld, 8, 3);
      else if (m.cls == KR_OK)
        w |= kbits(m.elen, 16, 1) | kbits(m.eepoch, 14, 2) | kbits(m.evalue, 12, 2) | kbits(m.epoch, 10, 2) |
             kbits(m.hwm, 8, 2) | kbits(ld, 5, 3);
      else
        w |= kbits(m.divend, 15, 2) | kbits(m.divepoch, 13, 2) | kbits(m.epoch, 11, 2) | kbits(m.hwm, 9, 2) |
             kbits(ld, 6, 3);
      break;
  }
  return w | ((uint32_t)m.count & 7u);
}
RMC_HD int kget(uint32_t w, int pos, int wd) { return (int)((w >> pos) & ((1u << wd) - 1u)); }
RMC_HD KMsg kr_decode(uint32_t w) {
  KMsg m = kmsg_zero();
  m.count = (int)(w & 7u);
  m.cls = (int)(w >> 29);
  int ld = 0;
  switch (m.cls) {
    case 0: m.dst = kget(w, 26, 3); m.epoch = kget(w, 24, 2); m.src = kget(w, 21, 3); break;
    case 1: m.dst = kget(w, 26, 3); m.epoch = kget(w, 24, 2); m.err = kget(w, 22, 2); m.src = kget(w, 19, 3); break;
    case 2:
      m.dst = kget(w, 26, 3); m.epoch = kget(w, 24, 2); m.granted = kget(w, 23, 1); m.f1 = kget(w, 21, 2);
      m.f2 = kget(w, 19, 2); m.src = kget(w, 16, 3);
      break;
    case 3:
      m.dst = kget(w, 26, 3); m.epoch = kget(w, 24, 2); m.err = kget(w, 22, 2); ld = kget(w, 19, 3);
      m.src = kget(w, 16, 3); m.granted = kget(w, 15, 1);
      break;
    default:
      m.src = kget(w, 26, 3); m.cepoch = kget(w, 24, 2); m.cfo = kget(w, 22, 2); m.clfe = kget(w, 20, 2);
      m.dst = kget(w, 17, 3);
      if (m.cls == KR_NOTOK) { m.epoch = kget(w, 15, 2); m.err = kget(w, 13, 2); m.hwm = kget(w, 11, 2); ld = kget(w, 8, 3); }
      else if (m.cls == KR_OK) {
        m.elen = kget(w, 16, 1); m.eepoch = kget(w, 14, 2); m.evalue = kget(w, 12, 2); m.epoch = kget(w, 10, 2);
        m.hwm = kget(w, 8, 2); ld = kget(w, 5, 3);
      } else {
        m.divend = kget(w, 15, 2); m.divepoch = kget(w, 13, 2); m.epoch = kget(w, 11, 2); m.hwm = kget(w, 9, 2);
        ld = kget(w, 6, 3);
      }
      break;
  }
  m.leader = ld - 1;
  return m;
}
// The fingerprint's view of a KRaft message body: msource / mdest masked (the
// pair sums key them) and mleader as its relation to them (Nil, = source, =
// destination, the third server): a function of the relabelled message that
// is injective for N <= 3.
RMC_HD uint32_t kr_body(uint32_t w, int sp, int dp) {
  uint32_t r = w & ~((7u << sp) | (7u << dp));
  const int c3 = (int)(w >> 29);
  if (c3 < 3) return r;
  const int lp = c3 == 3 ? 19 : c3 == 4 ? 8 : c3 == 5 ? 5 : 6;
  const int ld = (int)((w >> lp) & 7u), src = (int)((w >> sp) & 7u), dst = (int)((w >> dp) & 7u);
  const uint32_t rel = ld == 0 ? 0u : ld - 1 == src ? 1u : ld - 1 == dst ? 2u : 3u;
  return (r & ~(7u << lp)) | (rel << lp);
}

// ------------------------------------------------------------------ delta
// A successor = parent + (one server's words replaced) + (message ops) +
// (new header).  Every Next disjunct of the four specs changes at most one
// server's variables, so this is exact.
struct Delta {
  int srv;
  uint32_t w[4];
  int nops;
  int opk[MAXOPS];       // parent DOMAIN index modified in place, or -1 = insert
  uint32_t opc[MAXOPS];  // resulting message word (record | count)
  uint32_t hdr;
  int ordinal;
  int act;
  int err;
};

template <int SPEC, int N>
struct PState {
  const uint32_t* S;
  RMC_HD uint32_t hdr() const { return S[0]; }
  RMC_HD uint32_t A(int i) const { return S[1 + 4 * i]; }
  RMC_HD uint32_t B(int i) const { return S[2 + 4 * i]; }
  RMC_HD uint32_t Cw(int i) const { return S[3 + 4 * i]; }
  RMC_HD uint32_t Dw(int i) const { return S[4 + 4 * i]; }
  RMC_HD int nmsg() const { return h_nmsg(S[0]); }
  RMC_HD uint32_t msg(int k) const { return S[1 + 4 * N + k]; }
  RMC_HD int term(int i) const { return a_term(A(i)); }
  RMC_HD int st(int i) const { return a_st(A(i)); }
  RMC_HD int len(int i) const { return a_len(A(i)); }
  // index of the message with the same record as w, or -1 (binary search:
  // DOMAIN is sorted by record)
  RMC_HD int find(uint32_t w) const {
    int lo = 0, hi = nmsg() - 1;
    uint32_t r = msg_rec(w);
    while (lo <= hi) {
      int mid = (lo + hi) >> 1;
      uint32_t x = msg_rec(msg(mid));
      if (x == r) return mid;
      if (x < r) lo = mid + 1; else hi = mid - 1;
    }
    return -1;
  }
};

// log helpers (1-based TLA+ indices; out of domain -> E_DOMAIN)
RMC_HD int log_term_at(uint32_t a, uint32_t b, int idx, int& err) {
  if (idx < 1 || idx > a_len(a)) { err = E_DOMAIN; return 0; }
  return e_term(b, idx - 1);
}
RMC_HD int log_value_at(uint32_t a, uint32_t b, int idx, int& err) {
  if (idx < 1 || idx > a_len(a)) { err = E_DOMAIN; return 0; }
  return e_value(b, idx - 1);
}
RMC_HD int last_term(uint32_t a, uint32_t b) { int L = a_len(a); return L ? e_term(b, L - 1) : 0; }
RMC_HD void log_append(uint32_t& a, uint32_t& b, int term, int value, int& err) {
  int L = a_len(a);
  if (L >= MAXLOG) { err = E_CAP_LOG; return; }
  b = setb(b, 6 * L, 6, e_pack(term, value));
  a = setb(a, 9, 3, (uint32_t)(L + 1));
}
RMC_HD void log_truncate(uint32_t& a, uint32_t& b, int n) {  // keep entries 1..n (n <= Len)
  a = setb(a, 9, 3, (uint32_t)n);
  b &= (n >= 5) ? 0x3FFFFFFFu : ((1u << (6 * n)) - 1u);
}
RMC_HD int popc7(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popc(x);
#else
  return __builtin_popcount(x);
#endif
}

// Emitting message ops into the delta.  Written with compile-time indices so
// the Delta stays in registers (a runtime-indexed array would go to scratch).
RMC_HD void push_op(Delta& d, int k, uint32_t c) {
#pragma unroll
  for (int q = 0; q < MAXOPS; q++)
    if (q == d.nops) { d.opk[q] = k; d.opc[q] = c; }
  d.nops++;
}
RMC_HD bool ops_have_rec(const Delta& d, uint32_t w) {
  bool hit = false;
#pragma unroll
  for (int q = 0; q < MAXOPS; q++)
    if (q < d.nops && msg_rec(d.opc[q]) == msg_rec(w)) hit = true;
  return hit;
}
template <int SPEC, int N>
RMC_HD bool op_send_once(const PState<SPEC, N>& s, Delta& d, uint32_t rec1) {
  // rec1 = record with count 1; disabled if the record is already in DOMAIN
  if (s.find(rec1) >= 0) return false;
  if (ops_have_rec(d, rec1)) return false;
  push_op(d, -1, rec1);
  return true;
}
template <int SPEC, int N>
RMC_HD void op_send_any(const PState<SPEC, N>& s, Delta& d, uint32_t rec1) {  // _SendNoRestriction
  int k = s.find(rec1);
  if (k < 0) { push_op(d, -1, rec1); return; }
  uint32_t w = s.msg(k);
  if (msg_count(w) >= 7) { d.err = E_CAP_COUNT; return; }
  push_op(d, k, w + 1u);
}
template <int SPEC, int N>
RMC_HD bool op_reply(const PState<SPEC, N>& s, Delta& d, uint32_t resp1, int req_k) {
  // Raft.tla:170-176 (Raft increments an existing response);
  // FlexibleRaft.tla:148-151, RaftFsync.tla:149-152, PullRaft.tla:158-161 (response must be new)
  uint32_t req = s.msg(req_k);
  if (!(msg_count(req) > 0)) return false;
  int k = s.find(resp1);
  if (k >= 0 && SPEC != RAFT) return false;
  push_op(d, req_k, req - 1u);
  if (k >= 0) {
    uint32_t w = s.msg(k);
    if (msg_count(w) >= 7) { d.err = E_CAP_COUNT; return true; }
    push_op(d, k, w + 1u);
  } else {
    push_op(d, -1, resp1);
  }
  return true;
}
template <int SPEC, int N>
RMC_HD void op_discard(const PState<SPEC, N>& s, Delta& d, int k) {  // Raft.tla:164-167 (count > 0 checked by caller)
  push_op(d, k, s.msg(k) - 1u);
}

template <int SPEC, int N>
RMC_HD void begin_srv(const PState<SPEC, N>& s, Delta& d, int i) {
  d.srv = i; d.w[0] = s.A(i); d.w[1] = s.B(i); d.w[2] = s.Cw(i); d.w[3] = s.Dw(i);
}

RMC_HD uint32_t all_rows(int N, int v) {
  uint32_t w = 0;
  for (int j = 0; j < N; j++) w |= (uint32_t)v << (3 * j);
  return w;
}

// LastCommonEntry(i, lastIndex, lastTerm) (PullRaft.tla:211-226,
// PullRaftVariant2.tla:202-217): the highest index of log[i] whose entry
// compares <= (lastIndex, lastTerm) (term first), with its term; [0, 0] if none.
RMC_HD int last_common_entry(uint32_t a, uint32_t b, int lastIndex, int lastTerm, int& term) {
  int idx = 0;
  for (int x = 1; x <= a_len(a); x++) {
    int t = e_term(b, x - 1);
    int cmp = t > lastTerm ? 1 : (t == lastTerm && x > lastIndex) ? 1 : (t == lastTerm && x == lastIndex) ? 0 : -1;
    if (cmp <= 0) idx = x;
  }
  term = idx ? e_term(b, idx - 1) : 0;
  return idx;
}

// ------------------------------------------------------------------ KRaft
// pull-raft/KRaft.tla.  Server words: A = currentEpoch 0-3 | state 4-5 (+ bit
// 25) | leader 6-8 | Len(log) 9-11 | highWatermark 12-14 | votedFor 15-17 |
// votesGranted 18-24; B = log ([epoch, value] entries, as Raft's [term, value]);
// C = pendingFetch (valid 0 | mepoch 1-2 | mfetchOffset 3-4 |
// mlastFetchedEpoch 5-6 | mdest 7-9; msource is the server itself);
// D = endOffset row.  States: Follower 0, Candidate 1, Leader 2, Unattached 3,
// Voted 4, IllegalState 5 (only Leader has low bits 2, so a_st() == LEADER
// stays exact for the shared invariants).
enum KState { KS_FOLLOWER = 0, KS_CANDIDATE = 1, KS_LEADER = 2, KS_UNATTACHED = 3, KS_VOTED = 4, KS_ILLEGAL = 5 };
RMC_HD int kr_st(uint32_t a) { return (int)(getb(a, 4, 2) | (getb(a, 25, 1) << 2)); }
RMC_HD uint32_t kr_set_st(uint32_t a, int st) { return setb(setb(a, 4, 2, (uint32_t)st & 3u), 25, 1, (uint32_t)st >> 2); }
RMC_HD int kr_leader(uint32_t a) { int l = a_voted(a); return l == NILS ? -1 : l; }  // -1 = Nil
RMC_HD uint32_t kr_set_leader(uint32_t a, int l) { return setb(a, 6, 3, l < 0 ? (uint32_t)NILS : (uint32_t)l); }
RMC_HD int kr_last_epoch(uint32_t a, uint32_t b) { int L = a_len(a); return L ? e_term(b, L - 1) : 0; }
RMC_HD uint32_t kr_pf(int epoch, int fo, int lfe, int dest) {
  return 1u | ((uint32_t)epoch << 1) | ((uint32_t)fo << 3) | ((uint32_t)lfe << 5) | ((uint32_t)dest << 7);
}
// CompareEntries (KRaft.tla:247-251)
RMC_HD int kr_cmp(int o1, int e1, int o2, int e2) {
  if (e1 > e2) return 1;
  if (e1 == e2 && o1 > o2) return 1;
  if (e1 == e2 && o1 == o2) return 0;
  return -1;
}
// a transition record [state, epoch, leader] (KRaft.tla:329-349)
struct KTr { int st, epoch, leader; };
RMC_HD KTr kr_illegal() { return KTr{KS_ILLEGAL, 0, -1}; }  // SetIllegalState (:329-330)
template <int SPEC, int N>
RMC_HD KTr kr_maybe_transition(const PState<SPEC, N>& s, int i, int leaderId, int epoch) {  // :351-367
  const uint32_t a = s.A(i);
  const int st = kr_st(a), cur = a_term(a), ld = kr_leader(a);
  // HasConsistentLeader (:316-327)
  const bool consistent = leaderId == i ? st == KS_LEADER : (epoch != cur || leaderId < 0 || ld < 0 || ld == leaderId);
  if (!consistent) return kr_illegal();
  // TransitionToFollower (:344-349)
  auto to_follower = [&]() {
    if (cur == epoch && (st == KS_FOLLOWER || st == KS_LEADER)) return kr_illegal();
    return KTr{KS_FOLLOWER, epoch, leaderId};
  };
  if (epoch > cur) return leaderId < 0 ? KTr{KS_UNATTACHED, epoch, -1} : to_follower();
  if (leaderId >= 0 && ld < 0) return to_follower();
  return KTr{st, cur, ld};
}
// MaybeHandleCommonResponse (:369-392)
template <int SPEC, int N>
RMC_HD KTr kr_common_response(const PState<SPEC, N>& s, int i, int leaderId, int epoch, int err, bool& handled) {
  const uint32_t a = s.A(i);
  const int cur = a_term(a);
  handled = true;
  if (epoch < cur) return KTr{kr_st(a), cur, kr_leader(a)};
  if (epoch > cur || err != KE_NIL) return kr_maybe_transition(s, i, leaderId, epoch);
  if (leaderId >= 0 && kr_leader(a) < 0) return KTr{KS_FOLLOWER, cur, leaderId};
  handled = false;
  return KTr{kr_st(a), cur, kr_leader(a)};
}
RMC_HD uint32_t kr_apply(uint32_t a, const KTr& t) {
  return kr_set_leader(setb(kr_set_st(a, t.st), 0, 4, (uint32_t)t.epoch), t.leader);
}
// Reply (:220-227): a FetchResponse must be new; other responses increment
template <int SPEC, int N>
RMC_HD bool kr_reply(const PState<SPEC, N>& s, Delta& d, const KMsg& resp, int req_k) {
  const uint32_t r1 = kr_encode(resp) | 1u;
  const uint32_t req = s.msg(req_k);
  if (!(msg_count(req) > 0)) return false;
  const int k = s.find(r1);
  if (k >= 0 && resp.cls >= KR_NOTOK) return false;
  push_op(d, req_k, req - 1u);
  if (k >= 0) {
    const uint32_t w = s.msg(k);
    if (msg_count(w) >= 7) { d.err = E_CAP_COUNT; return true; }
    push_op(d, k, w + 1u);
  } else {
    push_op(d, -1, r1);
  }
  return true;
}
// EndOffsetForEpoch (:285-301) -> offset, epoch
RMC_HD int kr_end_offset_for_epoch(uint32_t a, uint32_t b, int lfe, int& ep) {
  int off = 0;
  for (int x = 1; x <= a_len(a); x++)
    if (e_term(b, x - 1) <= lfe) off = x;
  ep = off ? e_term(b, off - 1) : 0;
  return off;
}

template <int SPEC, int N>
RMC_HD bool kr_fixed(const PState<SPEC, N>& s, const Model& M, int act, int i, int jv, Delta& d) {
  const uint32_t a = s.A(i), b = s.B(i);
  const int st = kr_st(a);
  switch (act) {
    case A_RESTART: {  // KRaft.tla:423-432
      if (!(h_rctr(s.hdr()) < M.R)) return false;
      begin_srv(s, d, i);
      uint32_t x = kr_set_leader(kr_set_st(a, KS_FOLLOWER), -1);
      x = setb(x, 18, 7, 0);   // votesGranted = {}
      x = setb(x, 12, 3, 0);   // highWatermark = 0
      d.w[0] = x;
      d.w[2] = 0;              // pendingFetch = Nil
      d.w[3] = 0;              // endOffset[i] = [j |-> 0]
      d.hdr = setb(s.hdr(), 12, 4, (uint32_t)(h_rctr(s.hdr()) + 1));
      return true;
    }
    case A_REQUESTVOTE: {  // :439-456
      const int ec = h_ectr(s.hdr());
      if (!(ec < M.E)) return false;
      if (!(st == KS_FOLLOWER || st == KS_CANDIDATE || st == KS_UNATTACHED)) return false;
      const int e1 = a_term(a) + 1;
      if (e1 > 3) { d.err = E_CAP_TERM; return true; }
      KMsg m = kmsg_zero();
      m.cls = 2; m.granted = 1; m.epoch = e1; m.f1 = kr_last_epoch(a, b); m.f2 = a_len(a); m.src = i; m.count = 1;
      for (int j = 0; j < N; j++) {
        if (j == i) continue;
        m.dst = j;
        if (!op_send_once(s, d, kr_encode(m))) return false;  // SendMultipleOnce
      }
      begin_srv(s, d, i);
      uint32_t x = kr_set_leader(kr_set_st(a, KS_CANDIDATE), -1);
      x = setb(x, 0, 4, (uint32_t)e1);
      x = setb(x, 15, 3, (uint32_t)i);     // votedFor = i
      x = setb(x, 18, 7, 1u << i);         // votesGranted = {i}
      d.w[0] = x;
      d.w[2] = 0;                          // pendingFetch = Nil
      d.hdr = setb(s.hdr(), 8, 4, (uint32_t)(ec + 1));
      return true;
    }
    case A_BECOMELEADER: {  // :546-558
      if (st != KS_CANDIDATE) return false;
      if (!(popc7((uint32_t)a_votes(a)) * 2 > N)) return false;
      KMsg m = kmsg_zero();
      m.cls = 0; m.epoch = a_term(a); m.src = i; m.count = 1;
      for (int j = 0; j < N; j++) {
        if (j == i) continue;
        m.dst = j;
        if (!op_send_once(s, d, kr_encode(m))) return false;
      }
      begin_srv(s, d, i);
      d.w[0] = kr_set_leader(kr_set_st(a, KS_LEADER), i);
      d.w[3] = 0;  // endOffset[i] = [j |-> 0]
      return true;
    }
    case A_CLIENT: {  // :594-603
      if (st != KS_LEADER || h_acked(s.hdr(), jv) != 0) return false;
      begin_srv(s, d, i);
      log_append(d.w[0], d.w[1], a_term(a), jv, d.err);
      d.hdr = setb(s.hdr(), 16 + 2 * jv, 2, 1);  // acked[v] = FALSE
      return true;
    }
    case A_KSENDFETCH: {  // :607-624
      if (i == jv || st != KS_FOLLOWER || kr_leader(a) != jv || (s.Cw(i) & 1u)) return false;
      KMsg m = kmsg_zero();
      m.cls = 2; m.granted = 0; m.epoch = a_term(a); m.f1 = a_len(a); m.f2 = kr_last_epoch(a, b);
      m.src = i; m.dst = jv; m.count = 1;
      op_send_any(s, d, kr_encode(m));  // Send: _SendNoRestriction for a FetchRequest
      begin_srv(s, d, i);
      d.w[2] = kr_pf(m.epoch, m.f1, m.f2, jv);
      return true;
    }
  }
  return false;
}

template <int SPEC, int N>
RMC_HD bool kr_message(const PState<SPEC, N>& s, const Model& M, int k, Delta& d) {
  const uint32_t w = s.msg(k);
  if (!(msg_count(w) > 0)) return false;  // ReceivableMessage (:230-235): messages[m] > 0
  const KMsg m = kr_decode(w);
  const int i = m.dst, j = m.src;
  const uint32_t a = s.A(i), b = s.B(i);
  const int cur = a_term(a), st = kr_st(a);
  switch (m.cls) {
    case 2: {
      if (m.granted) {  // HandleRequestVoteRequest (:464-513)
        d.act = A_HRVREQ;
        KMsg r = kmsg_zero();
        r.cls = 3; r.src = i; r.dst = j; r.count = 1;
        if (m.epoch < cur) {  // error = FencedLeaderEpoch: reply, no state change
          r.epoch = cur; r.leader = kr_leader(a); r.granted = 0; r.err = KE_FENCED;
          return kr_reply(s, d, r, k);
        }
        const KTr s0 = m.epoch > cur ? KTr{KS_UNATTACHED, m.epoch, -1} : KTr{st, cur, kr_leader(a)};
        const bool logOk = kr_cmp(m.f2, m.f1, a_len(a), kr_last_epoch(a, b)) >= 0;
        const int vf = a_votedfor2(a);
        const bool grant = (s0.st == KS_UNATTACHED || (s0.st == KS_VOTED && vf == j)) && logOk;
        // TransitionToVoted (:335-339): state0 is Unattached here
        const KTr fin = (grant && s0.st == KS_UNATTACHED) ? KTr{KS_VOTED, m.epoch, -1} : s0;
        r.epoch = m.epoch; r.leader = fin.leader; r.granted = grant; r.err = KE_NIL;
        if (!kr_reply(s, d, r, k)) return false;
        begin_srv(s, d, i);
        uint32_t x = kr_apply(a, fin);
        if (grant) x = setb(x, 15, 3, (uint32_t)j);
        d.w[0] = x;
        if (fin.st != st) d.w[2] = 0;  // IF state # state' THEN pendingFetch' = Nil
        return true;
      }
      // a FetchRequest: RejectFetchRequest (:631-651) / DivergingFetchRequest
      // (:658-679) / AcceptFetchRequest (:703-736) -- exclusive per message
      KMsg r = kmsg_zero();
      r.src = i; r.dst = j; r.count = 1; r.cepoch = m.epoch; r.cfo = m.f1; r.clfe = m.f2;
      r.leader = kr_leader(a); r.epoch = cur; r.hwm = a_commit(a);
      int err = st != KS_LEADER ? KE_NOTLEADER : m.epoch < cur ? KE_FENCED : m.epoch > cur ? KE_UNKNOWN : KE_NIL;
      if (err != KE_NIL) {
        d.act = A_KREJFETCH;
        r.cls = KR_NOTOK; r.err = err;
        return kr_reply(s, d, r, k);
      }
      int ep = 0;
      const int off = kr_end_offset_for_epoch(a, b, m.f2, ep);
      const bool valid = (m.f1 == 0 && m.f2 == 0) || (m.f1 <= off && m.f2 == ep);  // ValidFetchPosition (:305-310)
      if (!valid) {
        d.act = A_KDIVFETCH;
        r.cls = KR_DIV; r.divepoch = ep; r.divend = off;
        return kr_reply(s, d, r, k);
      }
      d.act = A_KACCFETCH;
      const int offset = m.f1 + 1;
      const uint32_t ne = row_set(s.Dw(i), j, m.f1);  // newEndOffset
      // NewHighwaterMark (:689-701)
      int best = 0;
      for (int o = 1; o <= a_len(a); o++) {
        uint32_t set = 1u << i;
        for (int q = 0; q < N; q++)
          if (row_get(ne, q) >= o) set |= 1u << q;
        if (popc7(set) * 2 > N) best = o;
      }
      const int hwm = a_commit(a);
      const int nh = (best > 0 && e_term(b, best - 1) == cur) ? best : hwm;
      uint32_t hdr = s.hdr();
      for (int v = 0; v < M.V; v++) {
        if (h_acked(hdr, v) != 1) continue;
        bool in = false;
        for (int x = hwm + 1; x <= nh; x++)
          if (e_value(b, x - 1) == v) in = true;
        hdr = setb(hdr, 16 + 2 * v, 2, in ? 2u : 1u);
      }
      r.cls = KR_OK;
      if (offset <= a_len(a)) { r.elen = 1; r.eepoch = e_term(b, offset - 1); r.evalue = e_value(b, offset - 1); }
      r.hwm = nh < offset ? nh : offset;
      if (!kr_reply(s, d, r, k)) return false;
      d.hdr = hdr;
      begin_srv(s, d, i);
      d.w[0] = setb(a, 12, 3, (uint32_t)nh);
      d.w[3] = ne;
      return true;
    }
    case 3: {  // HandleRequestVoteResponse (:519-541)
      bool handled;
      const KTr ns = kr_common_response(s, i, m.leader, m.epoch, m.err, handled);
      d.act = A_HRVRESP;
      if (handled) {
        begin_srv(s, d, i);
        d.w[0] = kr_apply(a, ns);
      } else {
        if (st != KS_CANDIDATE) return false;
        if (m.granted) {
          begin_srv(s, d, i);
          d.w[0] = setb(a, 18 + j, 1, 1);
        }
      }
      op_discard(s, d, k);
      return true;
    }
    case 0: {  // HandleBeginQuorumRequest (:563-590)
      d.act = A_KHBQ;
      KMsg r = kmsg_zero();
      r.cls = 1; r.src = i; r.dst = j; r.count = 1;
      if (m.epoch < cur) {
        r.epoch = cur; r.err = KE_FENCED;
        return kr_reply(s, d, r, k);
      }
      const KTr ns = kr_maybe_transition(s, i, j, m.epoch);
      r.epoch = m.epoch; r.err = KE_NIL;
      if (!kr_reply(s, d, r, k)) return false;
      begin_srv(s, d, i);
      d.w[0] = kr_apply(a, ns);
      d.w[2] = 0;  // pendingFetch = Nil
      return true;
    }
    case 1: return false;  // BeginQuorumResponse: no action receives it
    default: {  // a FetchResponse: HandleSuccess / HandleDiverging / HandleError (:742-801)
      bool handled;
      const KTr ns = kr_common_response(s, i, m.leader, m.epoch, m.err, handled);
      if (s.Cw(i) != kr_pf(m.cepoch, m.cfo, m.clfe, j)) return false;  // pendingFetch[i] = m.correlation
      begin_srv(s, d, i);
      d.w[2] = 0;  // pendingFetch = Nil
      if (handled) {
        d.act = A_KHERR;
        d.w[0] = kr_apply(a, ns);
      } else if (m.cls == KR_OK) {
        d.act = A_KHSUCC;
        d.w[0] = setb(a, 12, 3, (uint32_t)m.hwm);
        if (m.elen) log_append(d.w[0], d.w[1], m.eepoch, m.evalue, d.err);
      } else if (m.cls == KR_DIV) {
        d.act = A_KHDIV;
        // TruncateLog / HighestCommonOffset (:255-282)
        int o = 0;
        for (int x = 1; x <= a_len(a); x++)
          if (kr_cmp(x, e_term(b, x - 1), m.divend, m.divepoch) <= 0) o = x;
        log_truncate(d.w[0], d.w[1], o);
      } else {
        return false;  // NotOk is always handled (merror # Nil)
      }
      op_discard(s, d, k);
      return true;
    }
  }
  return false;
}

// ---------------------------------------------------------------- actions
// Each returns true iff the action is enabled for the binding; d receives the
// successor.  Citations are to /root/reference/specifications/.

// ------------------------------------------------------- compiled guards
// A stack machine over the packed state for the guards the TLA+ front end
// compiles (rmc_tla.cpp compile_guard): one 32-bit word per instruction, op in
// the low 8 bits, a signed 24-bit operand above.  Values are ints: booleans
// 0/1, sets of servers / values / states as bitmasks, Nil and the record
// values in the packed state's own codes (the compiler types every operand).
// Jumps are relative to the next instruction (short-circuit /\ and \/, IF).
// Returns 1 (enabled), 0, or -1: a TLC evaluation error (a sequence indexed
// outside its domain).  Only models with a compiled guard reach it.
enum GOp : uint32_t {
  G_END = 0,   // return the top of the stack
  G_CONST,     // push imm
  G_ARG,       // push bound variable imm (0: i, 1: j or v)
  G_ST,        // x -> state[x]
  G_TERM,      // x -> currentTerm[x]
  G_VOTED,     // x -> votedFor[x] (Pull: leader[x]); Nil = 7
  G_VOTED2,    // x -> PullRaftVariant2 votedFor[x]
  G_LEN,       // x -> Len(log[x])
  G_COMMIT,    // x -> commitIndex[x]
  G_FSYNC,     // x -> fsyncIndex[x]
  G_VOTES,     // x -> votesGranted[x] (server bitmask)
  G_NEXT,      // x y -> nextIndex[x][y]
  G_MATCH,     // x y -> matchIndex[x][y]
  G_PEND,      // x y -> pendingResponse[x][y]
  G_LOGTERM,   // x k -> log[x][k].term   (error outside 1..Len)
  G_LOGVAL,    // x k -> log[x][k].value  (error outside 1..Len)
  G_ECTR,      // -> electionCtr
  G_RCTR,      // -> restartCtr
  G_ACKED,     // v -> acked[v] (0 Nil, 1 FALSE, 2 TRUE)
  G_ADD, G_SUB, G_MUL, G_NEG,
  G_EQ, G_NE, G_LT, G_LE, G_NOT,
  G_BIT,       // x S -> (S >> x) & 1   (x \in S)
  G_SETADD,    // S x -> S | 1 << x
  G_POPC,      // S -> Cardinality(S)
  G_SUBSETEQ,  // A B -> (A & ~B) == 0
  G_BOR, G_BAND, G_BDIFF,  // A B -> A | B, A & B, A & ~B (set union, intersection, difference)
  G_JZ,        // pop; jump imm if 0
  G_JNZ,       // pop; jump imm if not 0
  G_JMP,       // jump imm
  G_POP,
  G_ERR,       // evaluation error
  G_MF,        // -> field imm of the bound message (compiled message handlers; MF_* below)
  // effect programs only (effect_vm): store the top of the stack into the
  // successor -- server i's (the action's first bound variable) fields, the
  // header's counters and acked, a log entry appended to log[i], a
  // RequestVoteRequest sent as SendMultipleOnce sends each of its messages
  E_ST,        // x ->   state[i]' = x
  E_TERM,      // x ->   currentTerm[i]' = x            (> 15: capacity)
  E_VOTED,     // x ->   votedFor[i]' = x               (Nil = 7)
  E_VOTES,     // S ->   votesGranted[i]' = S
  E_COMMIT,    // x ->   commitIndex[i]' = x            (> 7: capacity)
  E_ECTR,      // x ->   electionCtr' = x
  E_RCTR,      // x ->   restartCtr' = x
  E_ACKED,     // v c -> acked[v]' = c                  (0 Nil, 1 FALSE, 2 TRUE)
  E_APPEND,    // t v -> log[i]' = Append(log[i], [term |-> t, value |-> v])
  E_NEXT,      // j x -> nextIndex[i][j]' = x           (> 7: capacity)
  E_MATCH,     // j x -> matchIndex[i][j]' = x          (> 7: capacity)
  E_PEND,      // j b -> pendingResponse[i][j]' = b
  E_RVREQ,     // term llt lli src dst -> the RequestVoteRequest record, sent new (imm 0: disabled if in
               // DOMAIN) or counted (imm 1: _SendNoRestriction)
  E_DISCARD,   // Discard(m): the bound message's count - 1 (Raft.tla:164-167; its count > 0 is the guard's)
  E_REPLY,     // Reply(response, m) (Raft.tla:170-176), imm = response type: RequestVoteResponse
               // (term granted src dst) or AppendEntriesResponse (term success matchIndex src dst)
  E_END,       // the successor is complete
  G_NUM
};
RMC_HD uint32_t g_ins(uint32_t op, int imm = 0) { return op | ((uint32_t)imm << 8); }
// G_MF fields of a Raft-family record (rmc_spec.h MsgF; the compiler's types in rmc_guard.cpp)
enum MsgField { MF_TYPE = 0, MF_TERM, MF_SRC, MF_DST, MF_COUNT, MF_GRANTED, MF_LLI, MF_LLT, MF_PLI, MF_PLT, MF_NENT,
                MF_ETERM, MF_EVALUE, MF_COMMIT, MF_SUCCESS, MF_MIDX, MF_NUM };
RMC_HD int msg_field(const MsgF& m, int f) {
  switch (f) {
    case MF_TYPE: return m.type;
    case MF_TERM: return m.term;
    case MF_SRC: return m.src;
    case MF_DST: return m.dst;
    case MF_COUNT: return m.count;
    case MF_GRANTED: return m.granted;
    case MF_LLI: return m.lli;
    case MF_LLT: return m.llt;
    case MF_PLI: return m.pli;
    case MF_PLT: return m.plt;
    case MF_NENT: return m.nent;
    case MF_ETERM: return m.eterm;
    case MF_EVALUE: return m.evalue;
    case MF_COMMIT: return m.commit;
    case MF_SUCCESS: return m.success;
    case MF_MIDX: return m.midx;
  }
  return 0;
}
// The stack lives in eight registers, shifted on push and pop (a dynamically
// indexed array would put it in scratch memory, and a real call would make
// every kernel that can reach it save its live registers around it: the
// kernels' register budgets are set for the library actions).  The compiler
// refuses a guard deeper than that (rmc_guard.cpp).
// EFF: an effect program (effect_vm): the same expression machine, reading the
// parent state, plus the E_* stores into the successor d (server i's words,
// the header, the message ops).  Returns 1 (enabled; d complete at E_END),
// 0 (disabled: a SendMultipleOnce message already in DOMAIN) or -1 (a TLC
// evaluation error); a value past the packed layout's field sets d.err.
// mk: the DOMAIN slot of the bound message of a compiled message handler
// (G_MF, E_DISCARD, E_REPLY), -1 otherwise.
template <int SPEC, int N, bool EFF>
RMC_HD int vm_run(const uint32_t* S, const Model& M, int pc, int i, int jv, Delta& d, int mk = -1) {
  int t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0, t6 = 0, t7 = 0;
  const PState<SPEC, N> s{S};
  uint32_t ea = 0, eb = 0, eh = 0;  // effects: server i's words A and B, the header
  if constexpr (EFF) {
    begin_srv(s, d, i);
    ea = d.w[0];
    eb = d.w[1];
    eh = s.hdr();
  }
#define GPUSH(x) do { const int x_ = (x); t7 = t6; t6 = t5; t5 = t4; t4 = t3; t3 = t2; t2 = t1; t1 = t0; t0 = x_; } while (0)
#define GPOP() do { t0 = t1; t1 = t2; t2 = t3; t3 = t4; t4 = t5; t5 = t6; t6 = t7; } while (0)
#define GBIN(e) do { const int a_ = t1, b_ = t0; GPOP(); t0 = (e); } while (0)
  for (int steps = 0; steps < MAXGCODE; steps++) {
    const uint32_t w = M.gcode[pc++];
    const int op = (int)(w & 0xFFu), imm = (int)w >> 8;
    switch (op) {
      case G_END: return t0 ? 1 : 0;
      case G_CONST: GPUSH(imm); break;
      case G_ARG: GPUSH(imm ? jv : i); break;
      case G_ST: t0 = s.st(t0 & 7); break;
      case G_TERM: t0 = s.term(t0 & 7); break;
      case G_VOTED: t0 = a_voted(s.A(t0 & 7)); break;
      case G_VOTED2: t0 = a_votedfor2(s.A(t0 & 7)); break;
      case G_LEN: t0 = s.len(t0 & 7); break;
      case G_COMMIT: t0 = a_commit(s.A(t0 & 7)); break;
      case G_FSYNC: t0 = a_fsync(s.A(t0 & 7)); break;
      case G_VOTES: t0 = a_votes(s.A(t0 & 7)); break;
      case G_NEXT: GBIN(row_get(s.Cw(a_ & 7), b_ & 7)); break;
      case G_MATCH: GBIN(row_get(s.Dw(a_ & 7), b_ & 7)); break;
      case G_PEND: GBIN((a_pending(s.A(a_ & 7)) >> (b_ & 7)) & 1); break;
      case G_LOGTERM:
      case G_LOGVAL: {
        const int x = t1 & 7, k = t0;
        const uint32_t a = s.A(x), b = s.B(x);
        if (k < 1 || k > a_len(a)) return -1;
        GPOP();
        t0 = op == G_LOGTERM ? e_term(b, k - 1) : e_value(b, k - 1);
        break;
      }
      case G_ECTR: GPUSH(h_ectr(s.hdr())); break;
      case G_RCTR: GPUSH(h_rctr(s.hdr())); break;
      case G_ACKED: t0 = h_acked(s.hdr(), t0 & 3); break;
      case G_ADD: GBIN(a_ + b_); break;
      case G_SUB: GBIN(a_ - b_); break;
      case G_MUL: GBIN(a_ * b_); break;
      case G_NEG: t0 = -t0; break;
      case G_EQ: GBIN(a_ == b_); break;
      case G_NE: GBIN(a_ != b_); break;
      case G_LT: GBIN(a_ < b_); break;
      case G_LE: GBIN(a_ <= b_); break;
      case G_NOT: t0 = !t0; break;
      case G_BIT: GBIN((b_ >> (a_ & 31)) & 1); break;
      case G_SETADD: GBIN(a_ | (1 << (b_ & 31))); break;
      case G_POPC: t0 = popc7((uint32_t)t0); break;
      case G_SUBSETEQ: GBIN((a_ & ~b_) == 0); break;
      case G_BOR: GBIN(a_ | b_); break;
      case G_BAND: GBIN(a_ & b_); break;
      case G_BDIFF: GBIN(a_ & ~b_); break;
      case G_JZ: { const int c_ = t0; GPOP(); if (!c_) pc += imm; break; }
      case G_JNZ: { const int c_ = t0; GPOP(); if (c_) pc += imm; break; }
      case G_JMP: pc += imm; break;
      case G_POP: GPOP(); break;
      case G_MF:  // decoded at each use: no record held in registers across the program
        if (mk < 0) return -1;
        GPUSH(msg_field(msg_decode<SPEC>(s.msg(mk)), imm));
        break;
      default:
        if constexpr (EFF) {
          switch (op) {
            case E_ST: ea = setb(ea, 4, 2, (uint32_t)t0); GPOP(); break;
            case E_TERM:
              if (t0 < 0 || t0 > 15) { d.err = E_CAP_TERM; return 1; }
              ea = setb(ea, 0, 4, (uint32_t)t0);
              GPOP();
              break;
            case E_VOTED: ea = setb(ea, 6, 3, (uint32_t)t0 & 7u); GPOP(); break;
            case E_VOTES: ea = setb(ea, 18, 7, (uint32_t)t0); GPOP(); break;
            case E_COMMIT:
              if (t0 < 0 || t0 > 7) { d.err = E_CAP_FIELD; return 1; }
              ea = setb(ea, 12, 3, (uint32_t)t0);
              GPOP();
              break;
            case E_ECTR:
            case E_RCTR:
              if (t0 < 0 || t0 > 15) { d.err = E_CAP_FIELD; return 1; }
              eh = setb(eh, op == E_ECTR ? 8 : 12, 4, (uint32_t)t0);
              GPOP();
              break;
            case E_ACKED: eh = setb(eh, 16 + 2 * (t1 & 3), 2, (uint32_t)t0 & 3u); GPOP(); GPOP(); break;
            case E_NEXT:
            case E_MATCH:
              if (t0 < 0 || t0 > 7) { d.err = E_CAP_FIELD; return 1; }
              if (op == E_NEXT) d.w[2] = row_set(d.w[2], t1 & 7, t0);
              else d.w[3] = row_set(d.w[3], t1 & 7, t0);
              GPOP();
              GPOP();
              break;
            case E_PEND: ea = setb(ea, 25 + (t1 & 7), 1, (uint32_t)t0 & 1u); GPOP(); GPOP(); break;
            case E_APPEND: {
              if (t1 < 0 || t1 > 15) { d.err = E_CAP_TERM; return 1; }
              int err = 0;
              log_append(ea, eb, t1, t0 & 3, err);
              if (err) { d.err = err; return 1; }
              GPOP();
              GPOP();
              break;
            }
            case E_RVREQ: {  // stack: term llt lli src dst (dst on top)
              MsgF m = msg_zero();
              m.type = RVREQ; m.term = t4; m.llt = t3; m.lli = t2; m.src = t1 & 7; m.dst = t0 & 7; m.count = 1;
              if (t4 < 0 || t4 > 15) { d.err = E_CAP_TERM; return 1; }
              if (t3 < 0 || t3 > 15 || t2 < 0 || t2 > 7) { d.err = E_CAP_FIELD; return 1; }
              GPOP(); GPOP(); GPOP(); GPOP(); GPOP();
              if (imm) {
                op_send_any(s, d, msg_encode<SPEC>(m));
                if (d.err) return 1;
              } else if (!op_send_once(s, d, msg_encode<SPEC>(m))) {
                return 0;  // already in DOMAIN: the action is disabled
              }
              break;
            }
            case E_DISCARD:
              if (mk < 0 || !(msg_count(s.msg(mk)) > 0)) return 0;
              op_discard(s, d, mk);
              break;
            case E_REPLY: {  // stack: term flag [matchIndex] src dst (dst on top)
              MsgF r = msg_zero();
              r.type = imm;
              r.count = 1;
              r.src = t1 & 7;
              r.dst = t0 & 7;
              GPOP();
              GPOP();
              if (imm == AERESP) {
                r.midx = t0;
                r.success = t1 & 1;
                r.term = t2;
                GPOP(); GPOP(); GPOP();
              } else {
                r.granted = t0 & 1;
                r.term = t1;
                GPOP(); GPOP();
              }
              if (r.term < 0 || r.term > 15) { d.err = E_CAP_TERM; return 1; }
              if (r.midx < 0 || r.midx > 7) { d.err = E_CAP_FIELD; return 1; }
              if (mk < 0 || !op_reply(s, d, msg_encode<SPEC>(r), mk)) return 0;
              if (d.err) return 1;
              break;
            }
            case E_END:
              d.w[0] = ea;
              d.w[1] = eb;
              d.hdr = eh;
              return 1;
            default: return -1;
          }
          break;
        } else {
          return -1;  // G_ERR
        }
    }
  }
#undef GPUSH
#undef GPOP
#undef GBIN
  return -1;
}
template <int SPEC, int N>
RMC_HD int guard_vm(const uint32_t* S, const Model& M, int pc, int i, int jv) {
  Delta unused;
  return vm_run<SPEC, N, false>(S, M, pc, i, jv, unused);
}
template <int SPEC, int N>
RMC_HD int effect_vm(const PState<SPEC, N>& s, const Model& M, int pc, int i, int jv, Delta& d, int mk = -1) {
  return vm_run<SPEC, N, true>(s.S, M, pc, i, jv, d, mk);
}

template <int SPEC, int N>
RMC_HD bool act_restart(const PState<SPEC, N>& s, const Model& M, int i, Delta& d, bool ug = false) {
  // Raft.tla:226-235; FlexibleRaft.tla:200-208; RaftFsync.tla:203-218; PullRaft.tla:258-265
  // (ug: a compiled guard stands in for the reference's, guard_vm)
  if (!ug && !(h_rctr(s.hdr()) < M.R)) return false;
  begin_srv(s, d, i);
  uint32_t a = d.w[0];
  a = setb(a, 4, 2, FOLLOWER);
  a = setb(a, 18, 7, 0);   // votesGranted[i] = {}
  a = setb(a, 25, 7, 0);   // pendingResponse[i] = [j |-> FALSE]
  a = setb(a, 12, 3, 0);   // commitIndex[i] = 0
  if (!pullish(SPEC)) d.w[2] = all_rows(N, 1);
  if (SPEC == PULL2) {  // PullRaftVariant2.tla:254-256: leader Nil, votesLastEntry[i] Nil (votedFor kept)
    a = setb(a, 6, 3, NILS);
    d.w[2] = 0;
  }
  d.w[3] = 0;
  if (SPEC == FSYNC) {
    int f = a_fsync(a), L = a_len(a);
    if (f == 0) log_truncate(a, d.w[1], 0);
    else if (L > 0 && L > f) log_truncate(a, d.w[1], f);
  }
  d.w[0] = a;
  int r = h_rctr(s.hdr()) + 1;
  if (r > 15) { d.err = E_CAP_FIELD; }
  d.hdr = setb(s.hdr(), 12, 4, (uint32_t)r);
  return true;
}

template <int SPEC, int N>
RMC_HD bool act_requestvote(const PState<SPEC, N>& s, const Model& M, int i, Delta& d, bool ug = false) {
  // Raft.tla:242-257 (FlexibleRaft.tla:215-230; PullRaft.tla:283-298 sets leader[i])
  int ec = h_ectr(s.hdr());
  int st = s.st(i);
  if (!ug && !(ec < M.E && (st == FOLLOWER || st == CANDIDATE))) return false;
  if (ec + 1 > 15) { d.err = E_CAP_FIELD; return true; }
  int t1 = s.term(i) + 1;
  if (t1 > 15) { d.err = E_CAP_TERM; return true; }
  uint32_t a = s.A(i), b = s.B(i);
  MsgF m = msg_zero();
  m.type = RVREQ; m.term = t1; m.llt = last_term(a, b); m.lli = a_len(a); m.src = i; m.count = 1;
  for (int j = 0; j < N; j++) {
    if (j == i) continue;
    m.dst = j;
    if (!op_send_once(s, d, msg_encode<SPEC>(m))) return false;  // SendMultipleOnce / SendMultiple
  }
  begin_srv(s, d, i);
  a = setb(a, 4, 2, CANDIDATE);
  a = setb(a, 0, 4, (uint32_t)t1);
  if (SPEC == PULL2) {  // PullRaftVariant2.tla:284-286: votedFor = i, leader = Nil
    a = setb(a, 15, 3, (uint32_t)i);
    a = setb(a, 6, 3, NILS);
  } else {
    a = setb(a, 6, 3, (uint32_t)i);
  }
  a = setb(a, 18, 7, 1u << i);
  d.w[0] = a;
  d.hdr = setb(s.hdr(), 8, 4, (uint32_t)(ec + 1));
  return true;
}

template <int SPEC, int N>
RMC_HD bool act_timeout(const PState<SPEC, N>& s, const Model& M, int i, Delta& d, bool ug = false) {  // RaftFsync.tla:222-230
  int ec = h_ectr(s.hdr());
  int st = s.st(i);
  if (!ug && !(ec < M.E && (st == FOLLOWER || st == CANDIDATE))) return false;
  if (ec + 1 > 15) { d.err = E_CAP_FIELD; return true; }
  int t1 = s.term(i) + 1;
  if (t1 > 15) { d.err = E_CAP_TERM; return true; }
  begin_srv(s, d, i);
  uint32_t a = d.w[0];
  a = setb(a, 4, 2, CANDIDATE);
  a = setb(a, 0, 4, (uint32_t)t1);
  a = setb(a, 6, 3, (uint32_t)i);
  a = setb(a, 18, 7, 1u << i);
  d.w[0] = a;
  d.hdr = setb(s.hdr(), 8, 4, (uint32_t)(ec + 1));
  return true;
}

template <int SPEC, int N>
RMC_HD bool act_rvij(const PState<SPEC, N>& s, const Model& M, int i, int j, Delta& d, bool ug = false) {  // RaftFsync.tla:234-243
  if (!ug && (s.st(i) != CANDIDATE || i == j)) return false;
  uint32_t a = s.A(i), b = s.B(i);
  MsgF m = msg_zero();
  m.type = RVREQ; m.term = a_term(a); m.llt = last_term(a, b); m.lli = a_len(a); m.src = i; m.dst = j; m.count = 1;
  return op_send_once(s, d, msg_encode<SPEC>(m));
}

template <int SPEC, int N>
RMC_HD bool act_appendentries(const PState<SPEC, N>& s, const Model& M, int i, int j, Delta& d) {
  // Raft.tla:263-285; FlexibleRaft.tla:236-256; RaftFsync.tla:249-272
  if (i == j || s.st(i) != LEADER) return false;
  uint32_t a = s.A(i), b = s.B(i);
  if (SPEC == RAFT && ((a_pending(a) >> j) & 1)) return false;
  int nxt = row_get(s.Cw(i), j);
  int prevLogIndex = nxt - 1;
  int prevLogTerm = prevLogIndex > 0 ? log_term_at(a, b, prevLogIndex, d.err) : 0;
  if (d.err) return true;
  int L = a_len(a);
  int lastEntry = L < nxt ? L : nxt;  // Min({Len(log[i]), nextIndex[i][j]})
  if (SPEC == FSYNC && M.lfae && !(a_fsync(a) >= lastEntry)) return false;
  int nent = lastEntry - nxt + 1;   // SubSeq(log[i], nextIndex[i][j], lastEntry)
  if (nent < 0) nent = 0;
  MsgF m = msg_zero();
  m.type = AEREQ; m.term = a_term(a); m.pli = prevLogIndex; m.plt = prevLogTerm; m.nent = nent;
  if (nent) { m.eterm = log_term_at(a, b, nxt, d.err); m.evalue = log_value_at(a, b, nxt, d.err); }
  int ci = a_commit(a);
  m.commit = ci < lastEntry ? ci : lastEntry;
  m.src = i; m.dst = j; m.count = 1;
  if (prevLogIndex > 7) { d.err = E_CAP_FIELD; return true; }
  uint32_t w = msg_encode<SPEC>(m);
  if (SPEC == RAFT) {
    if (nent == 0) { if (!op_send_once(s, d, w)) return false; }  // _SendOnce (Raft.tla:146-148)
    else op_send_any(s, d, w);                                     // _SendNoRestriction
    begin_srv(s, d, i);
    d.w[0] = setb(d.w[0], 25 + j, 1, 1);  // pendingResponse[i][j] = TRUE
  } else {
    if (!op_send_once(s, d, w)) return false;
  }
  return true;
}

template <int SPEC, int N>
RMC_HD bool act_becomeleader(const PState<SPEC, N>& s, const Model& M, int i, Delta& d, bool ug = false) {
  // Raft.tla:289-300; FlexibleRaft.tla:260-269; RaftFsync.tla:276-285; PullRaft.tla:354-366
  if (!ug && s.st(i) != CANDIDATE) return false;
  uint32_t a = s.A(i);
  int vg = a_votes(a);
  bool q = SPEC == FLEX ? popc7((uint32_t)vg) >= M.EQ : popc7((uint32_t)vg) * 2 > N;
  if (!ug && !q) return false;
  if (SPEC == PULL) {
    MsgF m = msg_zero();
    m.type = LNREQ; m.term = a_term(a); m.src = i; m.count = 1;
    for (int j = 0; j < N; j++) {
      if ((vg >> j) & 1) continue;
      m.dst = j;
      if (!op_send_once(s, d, msg_encode<SPEC>(m))) return false;
    }
  }
  if (SPEC == PULL2) {
    // PullRaftVariant2.tla:368-377: every other server; the last common entry
    // for those whose last entry the votes reported, else Nil
    MsgF m = msg_zero();
    m.type = LNREQ; m.term = a_term(a); m.src = i; m.count = 1;
    const uint32_t b = s.B(i), c = s.Cw(i);
    for (int j = 0; j < N; j++) {
      if (j == i) continue;
      m.dst = j;
      const uint32_t v = vle_get(c, i, j);
      m.lcenil = v == 0;
      m.lci = m.lct = 0;
      if (v) m.lci = last_common_entry(a, b, (int)(v & 7u) - 1, (int)(v >> 3), m.lct);
      if (!op_send_once(s, d, msg_encode<SPEC>(m))) return false;
    }
  }
  begin_srv(s, d, i);
  d.w[0] = setb(d.w[0], 4, 2, LEADER);
  if (SPEC == PULL2) d.w[0] = setb(d.w[0], 6, 3, (uint32_t)i);  // leader' = i
  if (SPEC == RAFT) d.w[0] = setb(d.w[0], 25, 7, 0);
  if (!pullish(SPEC)) {
    int nx = a_len(a) + 1;
    if (nx > 7) { d.err = E_CAP_FIELD; return true; }
    d.w[2] = all_rows(N, nx);
  }
  d.w[3] = 0;
  return true;
}

template <int SPEC, int N>
RMC_HD bool act_client(const PState<SPEC, N>& s, const Model& M, int i, int v, Delta& d, bool ug = false) {  // Raft.tla:304-313
  if (!ug && (s.st(i) != LEADER || h_acked(s.hdr(), v) != 0)) return false;
  begin_srv(s, d, i);
  log_append(d.w[0], d.w[1], s.term(i), v, d.err);
  d.hdr = setb(s.hdr(), 16 + 2 * v, 2, 1);  // acked[v] = FALSE
  return true;
}

template <int SPEC, int N>
RMC_HD int new_commit_index(const PState<SPEC, N>& s, const Model& M, int i, uint32_t matchrow, int& err) {
  // Raft.tla:322-335 / RaftFsync.tla:313-327 / FlexibleRaft.tla:296 / PullRaft.tla:446-458
  uint32_t a = s.A(i), b = s.B(i);
  int best = 0;
  for (int index = 1; index <= a_len(a); index++) {
    uint32_t set = 0;
    for (int k = 0; k < N; k++)
      if (row_get(matchrow, k) >= index) set |= 1u << k;
    if (!(SPEC == FSYNC && M.lfiq && index > a_fsync(a))) set |= 1u << i;
    int c = popc7(set);
    bool q = SPEC == FLEX ? c >= M.RQ : c * 2 > N;
    if (q) best = index;
  }
  if (best > 0 && log_term_at(a, b, best, err) == a_term(a)) return best;
  return a_commit(a);
}

template <int SPEC, int N>
RMC_HD uint32_t acked_after_commit(const PState<SPEC, N>& s, const Model& M, int i, int newCommit, int& err) {
  // acked' = [v |-> IF acked[v] = FALSE THEN v \in {log[i][k].value : k \in commitIndex[i]+1..new} ELSE acked[v]]
  uint32_t h = s.hdr();
  uint32_t a = s.A(i), b = s.B(i);
  for (int v = 0; v < M.V; v++) {
    if (h_acked(s.hdr(), v) != 1) continue;
    bool in = false;
    for (int k = a_commit(a) + 1; k <= newCommit; k++)
      if (log_value_at(a, b, k, err) == v) in = true;
    h = setb(h, 16 + 2 * v, 2, in ? 2u : 1u);
  }
  return h;
}

template <int SPEC, int N>
RMC_HD bool act_advcommit(const PState<SPEC, N>& s, const Model& M, int i, Delta& d) {  // Raft.tla:320-344
  if (s.st(i) != LEADER) return false;
  int nc = new_commit_index(s, M, i, s.Dw(i), d.err);
  if (d.err) return true;
  if (!(a_commit(s.A(i)) < nc)) return false;
  d.hdr = acked_after_commit(s, M, i, nc, d.err);
  begin_srv(s, d, i);
  d.w[0] = setb(d.w[0], 12, 3, (uint32_t)nc);
  return true;
}

template <int SPEC, int N>
RMC_HD bool act_advfsync(const PState<SPEC, N>& s, const Model& M, int i, Delta& d) {  // RaftFsync.tla:339-343
  uint32_t a = s.A(i);
  if (!(a_fsync(a) < a_len(a))) return false;
  begin_srv(s, d, i);
  d.w[0] = setb(a, 15, 3, (uint32_t)(a_fsync(a) + 1));
  return true;
}

template <int SPEC, int N>
RMC_HD bool act_sendpull(const PState<SPEC, N>& s, const Model& M, int i, int j, Delta& d) {  // PullRaft.tla:396-411
  uint32_t a = s.A(i), b = s.B(i);
  if (i == j || a_st(a) != FOLLOWER || a_voted(a) != j) return false;
  int lli = a_len(a);
  int llt = lli > 0 ? log_term_at(a, b, lli, d.err) : 0;
  MsgF m = msg_zero();
  m.type = PEREQ; m.term = a_term(a); m.lli = lli; m.llt = llt; m.src = i; m.dst = j; m.count = 1;
  return op_send_once(s, d, msg_encode<SPEC>(m));
}

// Can DOMAIN element w enable any action?  A delivered message (count 0)
// enables nothing unless its term is newer than its receiver's (UpdateTerm
// ranges over all of DOMAIN messages, Raft.tla:349-350).
template <int SPEC, int N>
RMC_HD bool msg_live(const PState<SPEC, N>& s, uint32_t w) {
  if (SPEC == KRAFT) return msg_count(w) > 0;  // every KRaft message action needs messages[m] > 0
  return !(msg_count(w) == 0 && msg_term<SPEC>(w) <= a_term(s.A(msg_dst<SPEC>(w))));
}

// ---- message-bound actions: exactly one can be enabled per DOMAIN element
template <int SPEC, int N>
RMC_HD bool act_message_any(const PState<SPEC, N>& s, const Model& M, int k, Delta& d) {
  if (SPEC == KRAFT) return kr_message(s, M, k, d);
  uint32_t w = s.msg(k);
  if (!msg_live<SPEC, N>(s, w)) return false;  // fast reject before the full decode
  MsgF m = msg_decode<SPEC>(w);
  int i = m.dst, j = m.src;
  uint32_t a = s.A(i), b = s.B(i);
  int cur = a_term(a);
  if (m.term > cur) {
    // UpdateTerm: Raft.tla:348-355 / PullRaft.tla:269-276 (count not required)
    d.act = A_UPDATETERM;
    begin_srv(s, d, i);
    uint32_t x = setb(a, 0, 4, (uint32_t)m.term);
    x = setb(x, 4, 2, FOLLOWER);
    x = setb(x, 6, 3, NILS);
    if (SPEC == PULL2) x = setb(x, 15, 3, NILS);  // PullRaftVariant2.tla:269-270: votedFor and leader
    d.w[0] = x;
    return true;
  }
  if (!(m.count > 0)) return false;  // ReceivableMessage: messages[m] > 0 (Raft.tla:182)
  int st = a_st(a);
  switch (m.type) {
    case RVREQ: {
      // HandleRequestVoteRequest: Raft.tla:360-381; PullRaft.tla:306-330 (mterm <= currentTerm)
      d.act = A_HRVREQ;
      int lt = last_term(a, b);
      bool logOk = m.llt > lt || (m.llt == lt && m.lli >= a_len(a));
      // PullRaftVariant2.tla:303-326: votedFor decides, the response carries the last entry
      int vf = SPEC == PULL2 ? a_votedfor2(a) : a_voted(a);
      bool grant = m.term == cur && logOk && (vf == NILS || vf == j);
      MsgF r = msg_zero();
      r.type = RVRESP; r.term = cur; r.granted = grant; r.src = i; r.dst = j; r.count = 1;
      if (SPEC == PULL2) { r.lli = a_len(a); r.llt = lt; }
      if (!op_reply(s, d, msg_encode<SPEC>(r), k)) return false;
      if (grant) { begin_srv(s, d, i); d.w[0] = setb(a, SPEC == PULL2 ? 15 : 6, 3, (uint32_t)j); }
      return true;
    }
    case RVRESP: {
      // HandleRequestVoteResponse: Raft.tla:386-401 (EqualTerm)
      if (m.term != cur) return false;
      d.act = A_HRVRESP;
      if (m.granted) {
        begin_srv(s, d, i);
        d.w[0] = setb(a, 18 + j, 1, 1);
        if (SPEC == PULL2) d.w[2] = vle_set(d.w[2], i, j, m.lli, m.llt);  // PullRaftVariant2.tla:342-344
      }
      op_discard(s, d, k);
      return true;
    }
    case AEREQ: {
      // LogOk: Raft.tla:406-410
      bool logOk;
      if (m.pli == 0) logOk = true;
      else logOk = m.pli > 0 && m.pli <= a_len(a) && m.plt == e_term(b, m.pli - 1);
      if (m.term < cur || (m.term == cur && st == FOLLOWER && !logOk)) {
        // RejectAppendEntriesRequest: Raft.tla:412-430
        d.act = A_REJAE;
        MsgF r = msg_zero();
        r.type = AERESP; r.term = cur; r.success = 0; r.midx = 0; r.src = i; r.dst = j; r.count = 1;
        return op_reply(s, d, msg_encode<SPEC>(r), k);
      }
      if (m.term != cur || !(st == FOLLOWER || st == CANDIDATE) || !logOk) return false;
      // AcceptAppendEntriesRequest: Raft.tla:454-485; FlexibleRaft.tla:421-450; RaftFsync.tla:449-481
      d.act = A_ACCAE;
      int L = a_len(a);
      int index = m.pli + 1;
      bool canAppend = m.nent != 0 && L == m.pli;
      uint32_t na = a, nb = b;
      if (SPEC == RAFT) {
        bool needs = (m.nent != 0 && L >= index) || (m.nent == 0 && L > m.pli);
        if (canAppend) log_append(na, nb, m.eterm, m.evalue, d.err);
        else if (needs && m.nent != 0) { log_truncate(na, nb, m.pli); log_append(na, nb, m.eterm, m.evalue, d.err); }
        else if (needs && m.nent == 0) log_truncate(na, nb, m.pli);
      } else {
        bool needs = m.nent != 0 && L >= index && e_term(b, index - 1) != m.eterm;
        if (canAppend) log_append(na, nb, m.eterm, m.evalue, d.err);
        else if (needs) { log_truncate(na, nb, m.pli); log_append(na, nb, m.eterm, m.evalue, d.err); }
      }
      na = setb(na, 4, 2, FOLLOWER);
      na = setb(na, 12, 3, (uint32_t)m.commit);
      if (SPEC == FSYNC && M.ffbr) na = setb(na, 15, 3, (uint32_t)a_len(na));
      MsgF r = msg_zero();
      r.type = AERESP; r.term = cur; r.success = 1; r.midx = m.pli + m.nent; r.src = i; r.dst = j; r.count = 1;
      if (r.midx > 7) { d.err = E_CAP_FIELD; return true; }
      if (!op_reply(s, d, msg_encode<SPEC>(r), k)) return false;
      d.srv = i; d.w[0] = na; d.w[1] = nb; d.w[2] = s.Cw(i); d.w[3] = s.Dw(i);
      return true;
    }
    case AERESP: {
      // HandleAppendEntriesResponse: Raft.tla:490-505 (EqualTerm)
      if (m.term != cur) return false;
      d.act = A_HAERESP;
      begin_srv(s, d, i);
      if (m.success) {
        if (m.midx + 1 > 7) { d.err = E_CAP_FIELD; return true; }
        d.w[2] = row_set(d.w[2], j, m.midx + 1);
        d.w[3] = row_set(d.w[3], j, m.midx);
      } else {
        int nx = row_get(d.w[2], j) - 1;
        d.w[2] = row_set(d.w[2], j, nx > 1 ? nx : 1);
      }
      if (SPEC == RAFT) d.w[0] = setb(d.w[0], 25 + j, 1, 0);
      op_discard(s, d, k);
      return true;
    }
    case LNREQ: {
      // LearnOfLeader: PullRaft.tla:383-391 (EqualTerm)
      if (m.term != cur) return false;
      d.act = A_LEARN;
      begin_srv(s, d, i);
      d.w[0] = setb(a, 6, 3, (uint32_t)j);
      // PullRaftVariant2.tla:404-406: NeedsTruncation (:171-173) -> TruncateLog (:176-179)
      if (SPEC == PULL2 && !m.lcenil && a_len(a) >= m.lci) log_truncate(d.w[0], d.w[1], m.lci);
      op_discard(s, d, k);
      return true;
    }
    case PEREQ: {
      if (m.term != cur || st != LEADER) return false;
      // ValidPullPosition: PullRaft.tla:192-196
      bool valid;
      if (m.lli == 0) valid = true;
      else valid = m.lli > 0 && m.lli <= a_len(a) && m.llt == e_term(b, m.lli - 1);
      if (!valid) {
        // RejectPullEntriesRequest: PullRaft.tla:418-436, LastCommonEntry :211-226
        d.act = A_REJPULL;
        MsgF r = msg_zero();
        r.type = PERESP; r.term = cur; r.success = 0; r.lci = last_common_entry(a, b, m.lli, m.llt, r.lct);
        r.src = i; r.dst = j; r.count = 1;
        return op_reply(s, d, msg_encode<SPEC>(r), k);
      }
      int index = m.lli + 1;
      if (!(index <= a_len(a))) return false;
      // AcceptPullEntriesRequest: PullRaft.tla:460-488
      d.act = A_ACCPULL;
      uint32_t nm = row_set(s.Dw(i), j, m.lli);
      int nc = new_commit_index(s, M, i, nm, d.err);
      uint32_t hdr = acked_after_commit(s, M, i, nc, d.err);
      MsgF r = msg_zero();
      r.type = PERESP; r.term = cur; r.success = 1; r.nent = 1;
      r.eterm = e_term(b, index - 1); r.evalue = e_value(b, index - 1);
      r.commit = nc < index ? nc : index;
      r.src = i; r.dst = j; r.count = 1;
      if (!op_reply(s, d, msg_encode<SPEC>(r), k)) return false;
      d.hdr = hdr;
      begin_srv(s, d, i);
      d.w[3] = nm;
      d.w[0] = setb(d.w[0], 12, 3, (uint32_t)nc);
      return true;
    }
    case PERESP: {
      if (m.term != cur) return false;
      begin_srv(s, d, i);
      if (m.success) {
        // HandleSuccessPullEntriesResponse: PullRaft.tla:493-503
        d.act = A_HSUCC;
        d.w[0] = setb(d.w[0], 12, 3, (uint32_t)m.commit);
        log_append(d.w[0], d.w[1], m.eterm, m.evalue, d.err);
      } else {
        // HandleFailPullEntriesResponse: PullRaft.tla:510-520, TruncateLog :185-188
        d.act = A_HFAIL;
        if (m.lci > a_len(a)) { d.err = E_DOMAIN; return true; }
        log_truncate(d.w[0], d.w[1], m.lci);
      }
      op_discard(s, d, k);
      return true;
    }
  }
  return false;
}

// ... of those in this model's Next (a module may drop handlers from Next:
// the handlers' guards are mutually exclusive, so a dropped one leaves its
// messages with no enabled action rather than passing them to another)
template <int SPEC, int N>
RMC_HD bool act_message(const PState<SPEC, N>& s, const Model& M, int k, Delta& d) {
  return act_message_any<SPEC, N>(s, M, k, d) && ((M.msg_act_mask >> d.act) & 1ULL);
}

// A compiled message handler (K_MSGC, rmc_guard.cpp compile_handler) on
// DOMAIN element k: one program -- its guard conjuncts and its effects, in the
// text's order -- run with i = the message's mdest and jv = its msource (what
// the reference handlers' LET i == m.mdest, j == m.msource name).
template <int SPEC, int N>
RMC_HD bool eval_msgc(const PState<SPEC, N>& s, const Model& M, int q, int k, int ordinal, Delta& d) {
  d.srv = -1; d.nops = 0; d.hdr = s.hdr(); d.err = 0;
  d.act = A_C0 + q;
  d.ordinal = ordinal;
  if (k >= s.nmsg()) return false;
  uint32_t w = s.msg(k);
  int sp, dp;
  msg_srcdst_pos<SPEC>(w, sp, dp);
  const int e = effect_vm<SPEC, N>(s, M, M.estart[q], (int)((w >> dp) & 7u), (int)((w >> sp) & 7u), d, k);
  if (e < 0) { d.err = E_DOMAIN; return true; }
  return e != 0;
}

// A fixed binding given as (action id, its bound server i, its second bound
// variable jv) with its TLC ordinal already known: no table lookups, so a lane
// with its own binding issues no dependent loads before the action's guard.
template <int SPEC, int N, bool G = RMC_G_DEFAULT>
RMC_HD bool eval_fixed_id(const PState<SPEC, N>& s, const Model& M, int act, int i, int jv, int ordinal, Delta& d) {
  d.srv = -1; d.nops = 0; d.hdr = s.hdr(); d.err = 0;
  d.act = act;
  d.ordinal = ordinal;
  if (act == A_DUP || act == A_DROP) {
    // DuplicateMessage(m): Duplicate(m) -- m \in DOMAIN messages, messages[m] + 1 (Raft.tla:157-160, :512-514);
    // DropMessage(m): Discard(m) -- messages[m] > 0, messages[m] - 1 (Raft.tla:164-167, :519-521)
    const int k = i | (jv << 4);
    if (k >= s.nmsg()) return false;
    const uint32_t w = s.msg(k);
    if (act == A_DROP) {
      if (!(msg_count(w) > 0)) return false;
      push_op(d, k, w - 1u);
      return true;
    }
    if (msg_count(w) >= 7) { d.err = E_CAP_COUNT; return true; }
    push_op(d, k, w + 1u);
    return true;
  }
  if constexpr (G) {
    if (act >= A_C0) {  // compiled whole by the front end (rmc_guard.cpp): its guard, then its effect
      const int g = guard_vm<SPEC, N>(s.S, M, M.gstart[act], i, jv);
      if (g < 0) { d.err = E_DOMAIN; return true; }
      if (!g) return false;
      const int e = effect_vm<SPEC, N>(s, M, M.estart[act - A_C0], i, jv, d);
      if (e < 0) { d.err = E_DOMAIN; return true; }
      return e != 0;
    }
  }
  if (act >= A_C0) return false;  // (never: a model with compiled actions runs the G instantiation)
  if (SPEC == KRAFT) return kr_fixed(s, M, act, i, jv, d);
  bool ug = false;
  if constexpr (G) {
    if (M.gstart[act] >= 0) {  // a compiled guard (rmc_guard.cpp) instead of the library's
      const int g = guard_vm<SPEC, N>(s.S, M, M.gstart[act], i, jv);
      if (g < 0) { d.err = E_DOMAIN; return true; }
      if (!g) return false;
      ug = true;
    }
  }
  switch (act) {
    case A_RESTART: return act_restart(s, M, i, d, ug);
    case A_REQUESTVOTE: return act_requestvote(s, M, i, d, ug);
    case A_TIMEOUT: return act_timeout(s, M, i, d, ug);
    case A_RVIJ: return act_rvij(s, M, i, jv, d, ug);
    case A_BECOMELEADER: return act_becomeleader(s, M, i, d, ug);
    case A_CLIENT: return act_client(s, M, i, jv, d, ug);
    case A_ADVCOMMIT: return act_advcommit(s, M, i, d);
    case A_APPENDENTRIES: return act_appendentries(s, M, i, jv, d);
    case A_ADVFSYNC: return act_advfsync(s, M, i, d);
    case A_SENDPULL: return act_sendpull(s, M, i, jv, d);
  }
  return false;
}
// A fixed binding: action slot `slot` (a K_I / K_IV / K_IJ action of Next)
// with bound-variable index x (first bound variable fastest).
template <int SPEC, int N, bool G = RMC_G_DEFAULT>
RMC_HD bool eval_fixed(const PState<SPEC, N>& s, const Model& M, int slot, int x, Delta& d) {
  if (M.act_kind[slot] == K_M) return eval_fixed_id<SPEC, N, G>(s, M, M.act_id[slot], x & 15, x >> 4, M.act_off[slot] + x, d);
  return eval_fixed_id<SPEC, N, G>(s, M, M.act_id[slot], x % N, x / N, M.act_off[slot] + x, d);
}
// Binding b whose TLC ordinal is known (k_expand phase C, k_materialize):
// desc = M.fb_desc[b] for a fixed binding (staged in LDS by the kernels).
template <int SPEC, int N, bool G = RMC_G_DEFAULT>
RMC_HD bool eval_known(const PState<SPEC, N>& s, const Model& M, int b, uint32_t desc, int ordinal, Delta& d) {
  if (b < M.nfixed)
    return eval_fixed_id<SPEC, N, G>(s, M, (int)((desc >> 16) & 0xFFu), (int)((desc >> 24) & 15u), (int)(desc >> 28),
                                     ordinal, d);
  if constexpr (G) {
    if (b >= M.nfixed + MSGC_STRIDE) {
      const int r = b - M.nfixed - MSGC_STRIDE;
      return eval_msgc<SPEC, N>(s, M, r / MSGC_STRIDE, r % MSGC_STRIDE, ordinal, d);
    }
  }
  d.srv = -1; d.nops = 0; d.hdr = s.hdr(); d.err = 0;
  d.act = -1;
  const bool en = act_message(s, M, b - M.nfixed, d);
  d.ordinal = ordinal;
  return en;
}

// Evaluate binding b (fixed bindings first, then one per DOMAIN element).
template <int SPEC, int N, bool G = RMC_G_DEFAULT>
RMC_HD bool eval_binding(const PState<SPEC, N>& s, const Model& M, int b, Delta& d) {
  if (b < M.nfixed) return eval_fixed<SPEC, N, G>(s, M, M.fb_act[b], M.fb_x[b], d);
  if constexpr (G) {
    if (b >= M.nfixed + MSGC_STRIDE) {
      const int r = b - M.nfixed - MSGC_STRIDE, q = r / MSGC_STRIDE, k = r % MSGC_STRIDE;
      return eval_msgc<SPEC, N>(s, M, q, k, M.act_off[M.msg_act_slot[A_C0 + q]] + k, d);
    }
  }
  d.srv = -1; d.nops = 0; d.hdr = s.hdr(); d.err = 0;
  int k = b - M.nfixed;
  d.act = -1;
  bool en = act_message(s, M, k, d);
  if (en) d.ordinal = M.act_off[M.msg_act_slot[d.act]] + k;
  return en;
}

// A necessary condition for fixed binding b to be enabled (or to raise an
// evaluation error): the leading conjuncts of each action's guard, which read
// one header field or one server's state word.  may_enable false implies
// eval_binding returns false without an error, so k_expand evaluates only the
// (parent, binding) pairs that pass it.
template <int SPEC, int N, bool G = RMC_G_DEFAULT>
RMC_HD bool may_enable_d(const PState<SPEC, N>& s, const Model& M, uint32_t desc) {  // desc = M.fb_desc[b]
  const int i = (int)((desc >> 24) & 15u), jv = (int)(desc >> 28);
  {
    const int act = (int)((desc >> 16) & 0xFFu);
    if (act == A_DUP || act == A_DROP) {
      const int k = i | (jv << 4);
      return k < s.nmsg() && (act == A_DUP || msg_count(s.msg(k)) > 0);
    }
  }
  if constexpr (G) {
    if (M.gstart[(desc >> 16) & 0xFFu] >= 0) return true;  // a compiled guard: no prefilter
  }
  const uint32_t a = s.A(i);
  const int st = a_st(a);
  if (SPEC == KRAFT) {
    const int ks = kr_st(a);
    switch ((int)((desc >> 16) & 0xFFu)) {
      case A_RESTART: return h_rctr(s.hdr()) < M.R;
      case A_REQUESTVOTE:
        return h_ectr(s.hdr()) < M.E && (ks == KS_FOLLOWER || ks == KS_CANDIDATE || ks == KS_UNATTACHED);
      case A_BECOMELEADER: return ks == KS_CANDIDATE;
      case A_CLIENT: return ks == KS_LEADER && h_acked(s.hdr(), jv) == 0;
      case A_KSENDFETCH: return ks == KS_FOLLOWER && i != jv && kr_leader(a) == jv && !(s.Cw(i) & 1u);
    }
    return true;
  }
  switch ((int)((desc >> 16) & 0xFFu)) {
    case A_RESTART: return h_rctr(s.hdr()) < M.R;
    case A_REQUESTVOTE:
    case A_TIMEOUT: return h_ectr(s.hdr()) < M.E && (st == FOLLOWER || st == CANDIDATE);
    case A_RVIJ: return st == CANDIDATE && i != jv;
    case A_BECOMELEADER: return st == CANDIDATE;
    case A_CLIENT: return st == LEADER && h_acked(s.hdr(), jv) == 0;
    case A_ADVCOMMIT: return st == LEADER;
    case A_APPENDENTRIES: return st == LEADER && i != jv && !(SPEC == RAFT && ((a_pending(a) >> jv) & 1));
    case A_ADVFSYNC: return a_fsync(a) < a_len(a);
    case A_SENDPULL: return st == FOLLOWER && i != jv && a_voted(a) == jv;
  }
  return true;
}
template <int SPEC, int N, bool G = RMC_G_DEFAULT>
RMC_HD bool may_enable(const PState<SPEC, N>& s, const Model& M, int b) {
  return may_enable_d<SPEC, N, G>(s, M, M.fb_desc[b]);
}

// Write parent + delta as a packed row of M.words words (a multiple of 4),
// in order and without reading the output back: the inserted messages (at
// most MAXOPS) are sorted in registers and merged into the parent's message
// list (with its in-place count changes); the row leaves through a 4-word
// register window, 16 B per store on the device.  Rows are 16 B aligned.
// The 16 B row stores of apply_delta: through a generic pointer (host rows,
// k_simulate's LDS rows) or a global one (k_materialize: global_store, not
// flat_store -- a flat store counts in lgkmcnt too, so each later LDS wait
// would also wait for the store to reach HBM).
RMC_HD void row_store4(uint32_t* o, uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) {
#if defined(__HIP_DEVICE_COMPILE__)
  *reinterpret_cast<uint4*>(o) = make_uint4(b0, b1, b2, b3);
#else
  o[0] = b0; o[1] = b1; o[2] = b2; o[3] = b3;
#endif
}
#if defined(__HIPCC__)
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));  // a builtin vector: assignable in any address space
__device__ inline void row_store4(gu32* o, uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) {
  *reinterpret_cast<__attribute__((address_space(1))) u32x4_t*>(o) = u32x4_t{b0, b1, b2, b3};
}
#endif
template <int SPEC, int N, class OutP = uint32_t*>
RMC_HD int apply_delta(const PState<SPEC, N>& s, const Model& M, const Delta& d, OutP out, int* nmsg_out = nullptr) {
  constexpr uint32_t NONE = 0xFFFFFFFFu;  // never a message word (mdest would be 7)
  uint32_t ins[MAXOPS];
#pragma unroll
  for (int q = 0; q < MAXOPS; q++) ins[q] = NONE;
  int ni = 0;
#pragma unroll
  for (int q = 0; q < MAXOPS; q++) {
    if (q < d.nops && d.opk[q] < 0) {
      uint32_t w = d.opc[q];
#pragma unroll
      for (int r = 0; r < MAXOPS; r++) {  // insert into the sorted ins[] (NONE-padded)
        uint32_t lo = ins[r] < w ? ins[r] : w, hi = ins[r] < w ? w : ins[r];
        ins[r] = lo;
        w = hi;
      }
      ni++;
    }
  }
  const int n = s.nmsg(), nn = n + ni;
  if (nmsg_out) *nmsg_out = nn;
  if (nn > M.kmax) return E_CAP_MSG;
  uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0;
  int cnt = 0;
  OutP o = out;
#if defined(__HIP_DEVICE_COMPILE__)
  // device rows end after their last message: the 16 B stores past it (the
  // zero padding up to M.kmax slots) are masked off -- every reader stops at
  // the header's message count, so those words may hold anything.  Measured
  // (CLI, fresh process, 3 interleaved runs): k_materialize 431 vs 448 ms per
  // check, the GPU parity suites green (profiles/r04/ab_row_trim_r04t.txt).
  const int used = (1 + 4 * N + nn + 3) & ~3;
#endif
  auto emit = [&](uint32_t w) {
    b0 = b1;
    b1 = b2;
    b2 = b3;
    b3 = w;
    if (++cnt == 4) {
#if defined(__HIP_DEVICE_COMPILE__)
      if ((int)(o - out) < used) row_store4(o, b0, b1, b2, b3);
#else
      row_store4(o, b0, b1, b2, b3);
#endif
      o += 4;
      cnt = 0;
    }
  };
  auto pop_ins = [&]() {
    uint32_t w = ins[0];
#pragma unroll
    for (int r = 0; r + 1 < MAXOPS; r++) ins[r] = ins[r + 1];
    ins[MAXOPS - 1] = NONE;
    return w;
  };
  emit((d.hdr & ~0xFFu) | (uint32_t)nn);
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int t = 0; t < 4; t++) emit(i == d.srv ? d.w[t] : s.S[1 + 4 * i + t]);
  // The message slots, in lockstep: every lane runs the same M.kmax steps and
  // makes the same emits, so a wave's 16 B stores are whole-wave instructions
  // (a data-dependent merge loop made each lane store at its own iterations:
  // partial-wave store instructions).  Step j outputs the smaller of the next
  // parent message (in-place ops applied) and the next insert; past both, 0.
  int k = 0;
  auto pmsg = [&](int kk) {
    uint32_t w = kk < n ? s.msg(kk) : NONE;
#pragma unroll
    for (int q = 0; q < MAXOPS; q++)
      if (q < d.nops && d.opk[q] == kk) w = d.opc[q];
    return w;
  };
#if defined(__HIP_DEVICE_COMPILE__) && RMC_MERGE_BATCH
  // Device rows: the merge runs to the wave's largest message count, not to
  // M.kmax (the steps past a lane's own count emit zeros its masked stores
  // drop; the emitted word count is rounded up to whole 16 B stores, and
  // M.words is a multiple of 4, so it stays <= M.kmax), and it reads the
  // parent's messages four at a time: each block of four steps consumes at
  // most four of them, so their LDS loads are issued together at the
  // block's start instead of one dependent load per step.  (The wave-wide
  // max may read an inactive lane's stale count: it is clamped to M.kmax,
  // and every lane of the wave computes the same value.)
  int jmax = nn;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int y = __shfl_xor(jmax, o, 64);
    jmax = y > jmax ? y : jmax;
  }
  jmax = jmax < M.kmax ? jmax : M.kmax;
  const int head = 1 + 4 * N, steps = ((head + jmax + 3) & ~3) - head;
#pragma unroll 1
  for (int j0 = 0; j0 < steps; j0 += 4) {
    uint32_t m[4];
#pragma unroll
    for (int u = 0; u < 4; u++) m[u] = pmsg(k + u);
    int kk = 0;  // messages of m[] consumed so far (<= u at step u)
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (j0 + u >= steps) break;
      const uint32_t wp = kk == 0 ? m[0] : kk == 1 ? m[1] : kk == 2 ? m[2] : m[3];
      const bool take_ins = ins[0] < wp;
      const uint32_t w = take_ins ? ins[0] : wp;
      emit(w == NONE ? 0u : w);
      if (take_ins) (void)pop_ins();
      else kk++;
    }
    k += kk;
  }
#else
  uint32_t wp = pmsg(0);
#pragma unroll 1
  for (int j = 0; j < M.kmax; j++) {
    const bool take_ins = ins[0] < wp;
    const uint32_t w = take_ins ? ins[0] : wp;
    emit(w == NONE ? 0u : w);
    if (take_ins) {
      (void)pop_ins();
    } else {
      k++;
      wp = pmsg(k);
    }
  }
#endif
  return E_NONE;
}

// ------------------------------------------------------------- invariants
// The successor's header and server words, read in place from the parent and
// the Delta (k_materialize checks the invariants through it: no copy).  It
// holds values, not references: a reference to the Delta stored in an
// aggregate makes the compiler keep the Delta in scratch.
template <int SPEC, int N>
struct SuccView {
  const uint32_t* S;  // the parent's row
  uint32_t h, w0, w1, w2, w3;
  int srv;
  RMC_HD SuccView(const PState<SPEC, N>& p, const Delta& d)
      : S(p.S), h(d.hdr), w0(d.w[0]), w1(d.w[1]), w2(d.w[2]), w3(d.w[3]), srv(d.srv) {}
  RMC_HD uint32_t hdr() const { return h; }
  RMC_HD uint32_t A(int i) const { return i == srv ? w0 : S[1 + 4 * i]; }
  RMC_HD uint32_t B(int i) const { return i == srv ? w1 : S[2 + 4 * i]; }
  RMC_HD uint32_t Cw(int i) const { return i == srv ? w2 : S[3 + 4 * i]; }
  RMC_HD uint32_t Dw(int i) const { return i == srv ? w3 : S[4 + 4 * i]; }
  RMC_HD int term(int i) const { return a_term(A(i)); }
  RMC_HD int st(int i) const { return a_st(A(i)); }
  RMC_HD int len(int i) const { return a_len(A(i)); }
};

template <int SPEC, int N, class St>
RMC_HD bool inv_no_log_divergence(const St& s, int& err) {  // Raft.tla:588-596
  for (int s2 = 0; s2 < N; s2++)
    for (int s1 = 0; s1 < N; s1++) {
      if (s1 == s2) continue;
      uint32_t a1 = s.A(s1), a2 = s.A(s2);
      int c = a_commit(a1) < a_commit(a2) ? a_commit(a1) : a_commit(a2);
      for (int idx = 1; idx <= c; idx++) {
        if (idx > a_len(a1) || idx > a_len(a2)) { err = E_DOMAIN; return true; }
        if (((s.B(s1) >> (6 * (idx - 1))) & 63u) != ((s.B(s2) >> (6 * (idx - 1))) & 63u)) return false;
      }
    }
  return true;
}
template <int SPEC, int N, class St>
RMC_HD bool inv_leader_has_all_acked(const St& s, const Model& M) {  // Raft.tla:604-620
  for (int v = 0; v < M.V; v++) {
    if (h_acked(s.hdr(), v) != 2) continue;
    for (int i = 0; i < N; i++) {
      uint32_t a = s.A(i);
      if (a_st(a) != LEADER) continue;
      bool newer = false;
      for (int l = 0; l < N; l++)
        if (l != i && s.term(l) > a_term(a)) newer = true;
      if (newer) continue;
      bool has = false;
      for (int x = 0; x < a_len(a); x++)
        if (e_value(s.B(i), x) == v) has = true;
      if (!has) return false;
    }
  }
  return true;
}
template <int SPEC, int N, class St>
RMC_HD bool inv_committed_majority(const St& s, int& err) {  // Raft.tla:625-636
  bool any = false;
  for (int i = 0; i < N; i++) if (s.st(i) == LEADER && a_commit(s.A(i)) > 0) any = true;
  if (!any) return true;
  int size = N / 2 + 1;
  for (int i = 0; i < N; i++) {
    uint32_t ai = s.A(i);
    if (!(a_st(ai) == LEADER && a_commit(ai) > 0)) continue;
    int ci = a_commit(ai);
    for (uint32_t q = 0; q < (1u << N); q++) {
      if (popc7(q) != size || !((q >> i) & 1u)) continue;
      bool ok = true;
      for (int j = 0; j < N && ok; j++) {
        if (!((q >> j) & 1u)) continue;
        if (!(a_len(s.A(j)) >= ci)) { ok = false; break; }
        if (ci > a_len(ai)) { err = E_DOMAIN; return true; }
        if (((s.B(j) >> (6 * (ci - 1))) & 63u) != ((s.B(i) >> (6 * (ci - 1))) & 63u)) ok = false;
      }
      if (ok) return true;
    }
  }
  return false;
}
template <int SPEC, int N, class St>
RMC_HD bool inv_never_two_leaders(const St& s) {  // KRaft.tla:916-921
  for (int i = 0; i < N; i++)
    for (int j = 0; j < N; j++) {
      const int li = a_voted(s.A(i)), lj = a_voted(s.A(j));
      if (li != NILS && lj != NILS && li != lj && a_term(s.A(i)) == a_term(s.A(j))) return false;
    }
  return true;
}
template <int SPEC, int N, class St>
RMC_HD bool inv_no_illegal_state(const St& s) {  // KRaft.tla:887-889
  for (int i = 0; i < N; i++)
    if (kr_st(s.A(i)) == KS_ILLEGAL) return false;
  return true;
}
// The classic Raft safety properties (Ongaro's dissertation, Fig. 3.2), offered
// as opt-in invariants for the Raft-family modules (the reference's cfgs check
// only LeaderHasAllAckedValues and NoLogDivergence).  Their
// TLA+ text, which a user adds to a spec to have TLC check the same thing, is
// in INTEGRATION.md; sequence indices are bounded by Len, so none can raise an
// evaluation error.
//   ElectionSafety == \A s1, s2 \in Server : (s1 # s2 /\ state[s1] = Leader /\ state[s2] = Leader)
//                       => currentTerm[s1] # currentTerm[s2]
template <int SPEC, int N, class St>
RMC_HD bool inv_election_safety(const St& s) {
  for (int i = 0; i < N; i++)
    for (int j = i + 1; j < N; j++)
      if (a_st(s.A(i)) == LEADER && a_st(s.A(j)) == LEADER && a_term(s.A(i)) == a_term(s.A(j))) return false;
  return true;
}
//   LogMatching == \A s1, s2 \in Server : \A i \in 1..Min({Len(log[s1]), Len(log[s2])}) :
//                    log[s1][i].term = log[s2][i].term => SubSeq(log[s1], 1, i) = SubSeq(log[s2], 1, i)
template <int SPEC, int N, class St>
RMC_HD bool inv_log_matching(const St& s) {
  for (int i = 0; i < N; i++)
    for (int j = i + 1; j < N; j++) {
      const int L = a_len(s.A(i)) < a_len(s.A(j)) ? a_len(s.A(i)) : a_len(s.A(j));
      const uint32_t bi = s.B(i), bj = s.B(j);
      for (int x = L - 1; x >= 0; x--)  // the longest prefix whose last terms agree
        if (e_term(bi, x) == e_term(bj, x)) {
          const uint32_t m = x >= 4 ? 0x3FFFFFFFu : ((1u << (6 * (x + 1))) - 1u);
          if ((bi & m) != (bj & m)) return false;
          break;
        }
    }
  return true;
}
//   LeaderCompleteness == \A l \in Server :
//       (state[l] = Leader /\ \A s \in Server : currentTerm[s] <= currentTerm[l]) =>
//         \A s \in Server : \A i \in 1..Min({commitIndex[s], Len(log[s])}) :
//           i <= Len(log[l]) /\ log[l][i] = log[s][i]
// (a leader of the newest term holds every entry any server has committed)
template <int SPEC, int N, class St>
RMC_HD bool inv_leader_completeness(const St& s) {
  for (int l = 0; l < N; l++) {
    const uint32_t al = s.A(l);
    if (a_st(al) != LEADER) continue;
    bool newest = true;
    for (int k = 0; k < N; k++)
      if (a_term(s.A(k)) > a_term(al)) newest = false;
    if (!newest) continue;
    for (int k = 0; k < N; k++) {
      const uint32_t ak = s.A(k);
      const int c = a_commit(ak) < a_len(ak) ? a_commit(ak) : a_len(ak);
      if (c > a_len(al)) return false;
      for (int x = 0; x < c; x++)
        if (((s.B(l) >> (6 * x)) & 63u) != ((s.B(k) >> (6 * x)) & 63u)) return false;
    }
  }
  return true;
}
//   StateMachineSafety == \A s1, s2 \in Server :
//       \A i \in 1..Min({commitIndex[s1], commitIndex[s2], Len(log[s1]), Len(log[s2])}) : log[s1][i] = log[s2][i]
template <int SPEC, int N, class St>
RMC_HD bool inv_state_machine_safety(const St& s) {
  for (int i = 0; i < N; i++)
    for (int j = i + 1; j < N; j++) {
      const uint32_t ai = s.A(i), aj = s.A(j);
      int c = a_commit(ai) < a_commit(aj) ? a_commit(ai) : a_commit(aj);
      c = c < a_len(ai) ? c : a_len(ai);
      c = c < a_len(aj) ? c : a_len(aj);
      for (int x = 0; x < c; x++)
        if (((s.B(i) >> (6 * x)) & 63u) != ((s.B(j) >> (6 * x)) & 63u)) return false;
    }
  return true;
}
// returns -1 if all hold, else the position (in cfg order) of the violated one
template <int SPEC, int N, class St>
RMC_HD int check_invariants(const St& s, const Model& M, int& err) {
  for (int q = 0; q < M.ninv; q++) {
    bool ok = true;
    switch (M.inv[q]) {
      case 0: ok = inv_leader_has_all_acked<SPEC, N>(s, M); break;
      case 1: ok = inv_no_log_divergence<SPEC, N>(s, err); break;
      case 2: ok = inv_committed_majority<SPEC, N>(s, err); break;
      case 3: ok = inv_never_two_leaders<SPEC, N>(s); break;
      case 4: ok = inv_no_illegal_state<SPEC, N>(s); break;
      case 5: ok = inv_election_safety<SPEC, N>(s); break;
      case 6: ok = inv_log_matching<SPEC, N>(s); break;
      case 7: ok = inv_leader_completeness<SPEC, N>(s); break;
      case 8: ok = inv_state_machine_safety<SPEC, N>(s); break;
    }
    if (err) return -2;
    if (!ok) return q;
  }
  return -1;
}

// ---------------------------------------------------------------- hashing
// fp(s) = min over server permutations pi of mix(H_pi(s)), where H_pi is a sum
// of per-server and per-message 64-bit hashes of pi(s)'s view.  H_pi is an
// additive (multiset) hash, so a successor's H_pi is the parent's plus the
// delta's contribution; min over all of S_N makes fp a function of the view
// orbit (VIEW + SYMMETRY, Raft.tla:115-116).
RMC_HD uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
RMC_HD int perm_of(uint32_t P, int j) { return (int)((P >> (3 * j)) & 7u); }

template <int N>
RMC_HD uint32_t relabel_set(uint32_t set, uint32_t P) {
  uint32_t o = 0;
#pragma unroll
  for (int j = 0; j < N; j++)
    if ((set >> j) & 1u) o |= 1u << perm_of(P, j);
  return o;
}
template <int N>
RMC_HD uint32_t relabel_row(uint32_t row, uint32_t P) {
  uint32_t o = 0;
#pragma unroll
  for (int j = 0; j < N; j++) o |= ((row >> (3 * j)) & 7u) << (3 * perm_of(P, j));
  return o;
}
// PullRaftVariant2's votesLastEntry row of server i, relabelled by P
template <int N>
RMC_HD uint32_t relabel_vle(uint32_t c, int i, uint32_t P) {
  uint32_t o = 0;
  const int pi = perm_of(P, i);
#pragma unroll
  for (int j = 0; j < N; j++)
    if (j != i) o |= vle_get(c, i, j) << (7 * vle_slot(pi, perm_of(P, j)));
  return o;
}
// server i's words with every server-valued field relabelled by P
template <int SPEC, int N>
RMC_HD void relabel_server(uint32_t P, int i, uint32_t a, uint32_t c, uint32_t dd, uint32_t& a2, uint32_t& c2,
                           uint32_t& d2) {
  int v = a_voted(a);
  a2 = setb(a, 6, 3, v == NILS ? (uint32_t)NILS : (uint32_t)perm_of(P, v));
  if (SPEC == PULL2 || SPEC == KRAFT) {
    int v2 = a_votedfor2(a);
    a2 = setb(a2, 15, 3, v2 == NILS ? (uint32_t)NILS : (uint32_t)perm_of(P, v2));
  }
  a2 = setb(a2, 18, 7, relabel_set<N>(a_votes(a), P));
  if (SPEC != KRAFT) a2 = setb(a2, 25, 7, relabel_set<N>(a_pending(a), P));  // KRaft: bit 25 is state
  // KRaft's C word is pendingFetch[i]: its mdest relabelled
  c2 = SPEC == PULL2 ? relabel_vle<N>(c, i, P)
       : SPEC == KRAFT ? ((c & 1u) ? setb(c, 7, 3, (uint32_t)perm_of(P, (int)getb(c, 7, 3))) : c)
                       : relabel_row<N>(c, P);
  d2 = relabel_row<N>(dd, P);
}
template <int SPEC, int N>
RMC_HD uint64_t h_server(uint32_t P, int i, uint32_t a, uint32_t b, uint32_t c, uint32_t dd) {
  uint32_t a2, c2, d2;
  relabel_server<SPEC, N>(P, i, a, c, dd, a2, c2, d2);
  uint64_t lo = (uint64_t)a2 | ((uint64_t)b << 32);
  uint64_t hi = (uint64_t)c2 | ((uint64_t)d2 << 32);
  int pos = perm_of(P, i);
  return mix64(mix64(lo + 0x9E3779B97F4A7C15ULL * (uint64_t)(pos + 1)) ^ hi);
}
template <int SPEC>
RMC_HD uint64_t h_msg(uint32_t P, uint32_t w) {
  int sp, dp;
  msg_srcdst_pos<SPEC>(w, sp, dp);
  uint32_t s = (w >> sp) & 7u, d = (w >> dp) & 7u;
  uint32_t w2 = (SPEC == KRAFT ? kr_body(w, sp, dp) : (w & ~((7u << sp) | (7u << dp)))) |
                ((uint32_t)perm_of(P, (int)s) << sp) | ((uint32_t)perm_of(P, (int)d) << dp);
  return mix64((uint64_t)w2 * 0xD6E8FEB86659FD93ULL + 0xA0761D6478BD642FULL);
}
RMC_HD uint64_t h_acked_view(uint32_t hdr) {  // PullRaft's view includes acked (PullRaft.tla:123)
  return mix64(((uint64_t)(hdr >> 16) & 0xFFu) + 0xE7037ED1A0B428DBULL);
}

// ------------------------------------------------- canonical fingerprint
// VIEW + SYMMETRY (Raft.tla:115-116): fp(s) must be a function of the orbit
// of view(s) under server permutations.  Each server gets a signature that is
// permutation-EQUIVARIANT (sig of server i in s == sig of server pi(i) in
// pi(s)): its own scalar fields, its relational fields reduced to invariants
// (votedFor is Nil / self / other; |votesGranted|, self in votesGranted; the
// multisets of its nextIndex/matchIndex row entries for j != i, plus its own
// entry), and the multisets of the messages it sent and received with the
// server fields masked out.  Let Pi(s) = the permutations that put the
// servers in signature order (ties: every order within a tie).  Then
//     fp(s) = min over pi in Pi(s) of mix(H_pi(s))
// is orbit-invariant (Pi(sigma(s)) = Pi(s) o sigma^-1, so both minimise over
// the same set of relabelled states), and usually |Pi(s)| = 1 instead of N!.
// Signatures only prune; a tie just costs more permutations.
RMC_HD uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
RMC_HD uint32_t row_multiset(uint32_t row, int N, int i) {  // count of each value (0..7) in 4-bit fields, j != i
  uint32_t m = 0;
  for (int j = 0; j < N; j++)
    if (j != i) m += 1u << (4 * ((row >> (3 * j)) & 7u));
  return m;
}
template <int SPEC>
RMC_HD uint32_t msg_rest(uint32_t w) {  // the message with msource/mdest masked out
  int sp, dp;
  msg_srcdst_pos<SPEC>(w, sp, dp);
  return SPEC == KRAFT ? kr_body(w, sp, dp) : w & ~((7u << sp) | (7u << dp));
}
template <int SPEC, int N>
RMC_HD uint32_t server_sig_own(int i, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  int v = a_voted(a);
  uint32_t vcls = v == NILS ? 0u : (v == i ? 1u : 2u);
  uint32_t votes = (uint32_t)a_votes(a), pend = (uint32_t)a_pending(a);
  uint32_t x = (a & 0x0003FE3Fu);  // term | state | Len | commitIndex | fsyncIndex
  x ^= vcls << 6;
  if (SPEC == KRAFT) {  // votedFor (bits 15-17) by class; state bit 25; pendingFetch's mdest by class
    const int v2 = a_votedfor2(a);
    x = (x & ~(7u << 15)) | ((v2 == NILS ? 0u : (v2 == i ? 1u : 2u)) << 15);
    x ^= ((a >> 25) & 1u) << 26;
    if (c & 1u) c = setb(c, 7, 3, getb(c, 7, 3) == (uint32_t)a_voted(a) ? 1u : 2u);
    votes = 0;
    pend = 0;
    x ^= ((uint32_t)popc7((uint32_t)a_votes(a)) << 18) | (((uint32_t)(a_votes(a) >> i) & 1u) << 21);
  }
  if (SPEC == PULL2) {  // bits 15-17 are votedFor: its class, not its value
    const int v2 = a_votedfor2(a);
    x = (x & ~(7u << 15)) | ((v2 == NILS ? 0u : (v2 == i ? 1u : 2u)) << 15);
    // votesLastEntry row: the multiset of its entries (j != i)
    uint32_t ms = 0;
#pragma unroll
    for (int j = 0; j < N; j++)
      if (j != i) ms += mix32(vle_get(c, i, j) + 0x3C6EF372u);
    c = ms;
  }
  x ^= ((uint32_t)popc7(votes) << 18) | (((votes >> i) & 1u) << 21) | ((uint32_t)popc7(pend) << 22) |
       (((pend >> i) & 1u) << 25);
  uint32_t h = mix32(x + 0x9E3779B9u);
  h = mix32(h ^ b);
  h = mix32(h ^ ((SPEC == PULL2 || SPEC == KRAFT) ? c : row_multiset(c, N, i) + 0x85EBCA6Bu * (((c >> (3 * i)) & 7u) + 1u)));
  h = mix32(h ^ (row_multiset(d, N, i) + 0xC2B2AE35u * (((d >> (3 * i)) & 7u) + 1u)));
  return h;
}
// per-message contributions to the sender's / receiver's signature
template <int SPEC>
RMC_HD void msg_sig(uint32_t w, int& src, int& dst, uint32_t& hs, uint32_t& hd) {
  int sp, dp;
  msg_srcdst_pos<SPEC>(w, sp, dp);
  src = (int)((w >> sp) & 7u);
  dst = (int)((w >> dp) & 7u);
  uint32_t r = SPEC == KRAFT ? kr_body(w, sp, dp) : w & ~((7u << sp) | (7u << dp));
  hs = mix32(r ^ 0x27d4eb2fU);
  hd = mix32(r ^ 0x165667b1U);
}

// The successor parent + delta as seen by the fingerprint, without
// materializing it (a full state is the view with an empty delta).
template <int SPEC, int N>
struct DeltaView {
  const PState<SPEC, N>& s;
  const Delta& d;
  RMC_HD uint32_t sw(int i, int t) const { return i == d.srv ? d.w[t] : s.S[1 + 4 * i + t]; }
  RMC_HD uint32_t pmsg(int k) const {  // parent message k after in-place ops
    uint32_t w = s.msg(k);
#pragma unroll
    for (int q = 0; q < MAXOPS; q++)
      if (q < d.nops && d.opk[q] == k) w = d.opc[q];
    return w;
  }
};

// One pass over the view's messages: each message's server-free part
// (msource/mdest masked, count kept) is hashed once, u = mix64(rest); its low
// half joins the sender's signature, its high half the receiver's, and u
// joins the multiset sum S[src][dst] of its (source, destination) pair.  A
// permutation P then hashes the messages as
//     sum over ordered pairs (s, d) of mix64(S[s][d] + key(P(s), P(d)))
// -- a hash of the function "relabelled pair -> multiset of message bodies",
// i.e. of the relabelled message bag -- costing N(N-1) mixes, not |messages|.
// One message's contribution to the signatures and pair sums (subtracted when
// `neg`: the sums are additive mod 2^64 / 2^32, so a successor's sums are the
// parent's with its changed messages swapped out -- see delta_fp_sums).
template <int SPEC>
RMC_HD uint64_t msg_u(uint32_t w, int& src, int& dst) {
  int sp, dp;
  msg_srcdst_pos<SPEC>(w, sp, dp);
  src = (int)((w >> sp) & 7u);
  dst = (int)((w >> dp) & 7u);
  const uint32_t body = SPEC == KRAFT ? kr_body(w, sp, dp) : w & ~((7u << sp) | (7u << dp));
  return mix64((uint64_t)body * 0xD6E8FEB86659FD93ULL + 0xA0761D6478BD642FULL);
}
template <int SPEC, int N>
RMC_HD void msg_contrib(uint32_t w, bool neg, uint32_t (&sig)[N], uint64_t (&S)[N][N]) {
  int src, dst;
  uint64_t u = msg_u<SPEC>(w, src, dst);
  uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
  if (neg) {
    u = 0ULL - u;
    lo = 0u - lo;
    hi = 0u - hi;
  }
#pragma unroll
  for (int i = 0; i < N; i++) {
    sig[i] += (i == src ? lo : 0u) + (i == dst ? hi : 0u);
#pragma unroll
    for (int j = 0; j < N; j++)
      if (i != j) S[i][j] += (i == src && j == dst) ? u : 0ULL;
  }
}

template <int SPEC, int N>
RMC_HD void view_scan(const DeltaView<SPEC, N>& V, uint32_t (&sig)[N], uint64_t (&S)[N][N]) {
  const Delta& d = V.d;
  const int nm = V.s.nmsg();
#pragma unroll
  for (int i = 0; i < N; i++) {
    sig[i] = server_sig_own<SPEC, N>(i, V.sw(i, 0), V.sw(i, 1), V.sw(i, 2), V.sw(i, 3));
#pragma unroll
    for (int j = 0; j < N; j++) S[i][j] = 0;
  }
  auto add = [&](uint32_t w) { msg_contrib<SPEC, N>(w, false, sig, S); };
#pragma unroll 1
  for (int k = 0; k < nm; k++) add(V.pmsg(k));
#pragma unroll
  for (int q = 0; q < MAXOPS; q++)  // compile-time q: the Delta arrays stay in registers
    if (q < d.nops && d.opk[q] < 0) add(d.opc[q]);
}
// The permutation putting servers in signature order (server j -> its rank);
// ties = some signatures are equal.
template <int N>
RMC_HD uint32_t sig_perm(const uint32_t (&sig)[N], bool& ties) {
  uint32_t P0 = 0;
  ties = false;
#pragma unroll
  for (int j = 0; j < N; j++) {
    int r = 0;
#pragma unroll
    for (int k = 0; k < N; k++) {
      r += sig[k] < sig[j];
      ties |= (k != j && sig[k] == sig[j]);
    }
    P0 |= (uint32_t)r << (3 * j);
  }
  return P0;
}

template <int SPEC, int N>
RMC_HD uint64_t canon_from_sums(const Model& M, const DeltaView<SPEC, N>& V, const uint32_t (&sig)[N],
                                const uint64_t (&S)[N][N], uint32_t* P0_out = nullptr) {
  bool ties;
  const uint32_t P0 = sig_perm<N>(sig, ties);
  if (P0_out) *P0_out = ties ? 0xFFFFFFFFu : P0;
  const uint64_t aux = (SPEC == PULL || SPEC == KRAFT) ? h_acked_view(V.d.hdr) : 0ULL;  // KRaft.tla:154
  uint64_t best = ~0ULL;
  const int np = ties ? M.nperm : 1;
#if defined(RMC_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
  extern __device__ unsigned long long g_stamps[32];
  atomicAdd(&g_stamps[4], 1ULL);
  if (ties) atomicAdd(&g_stamps[5], 1ULL);
#endif
#pragma unroll 1
  for (int p = 0; p < np; p++) {
    uint32_t P = P0;
    if (ties) {
      P = M.perm[p];
      bool ok = true;
#pragma unroll
      for (int j = 0; j < N; j++)
#pragma unroll
        for (int k = 0; k < N; k++)
          if (sig[j] < sig[k] && perm_of(P, j) > perm_of(P, k)) ok = false;
      if (!ok) continue;
#if defined(RMC_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
      atomicAdd(&g_stamps[6], 1ULL);
#endif
    }
    uint64_t h = aux;
#pragma unroll 1
    for (int i = 0; i < N; i++) h += h_server<SPEC, N>(P, i, V.sw(i, 0), V.sw(i, 1), V.sw(i, 2), V.sw(i, 3));
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
      for (int j = 0; j < N; j++)
        if (i != j)
          h += mix64(S[i][j] + 0x9E3779B97F4A7C15ULL * (uint64_t)(8 * perm_of(P, i) + perm_of(P, j) + 1));
    uint64_t f = mix64(h);
    best = f < best ? f : best;
  }
  return best == ~0ULL ? best - 1 : best;  // ~0 marks an empty fingerprint-set slot
}
template <int SPEC, int N>
RMC_HD uint64_t canon_fp(const Model& M, const DeltaView<SPEC, N>& V, uint32_t* P0_out = nullptr) {
  uint32_t sig[N];
  uint64_t S[N][N];
  view_scan<SPEC, N>(V, sig, S);
  return canon_from_sums<SPEC, N>(M, V, sig, S, P0_out);
}

// The parent's message sums (what view_scan accumulates over the parent's
// messages alone): sig_m[i] = message part of server i's signature, S[i][j].
// k_expand computes them once per parent (LDS); each successor then costs
// O(|delta ops|) message hashes instead of O(|DOMAIN messages|).
template <int N>
struct MsgSums {
  uint64_t S[N * (N - 1)];  // ordered pairs i != j, row-major without the diagonal
  uint32_t sig[N];
  RMC_HD static int pair(int i, int j) { return i * (N - 1) + (j < i ? j : j - 1); }
};
// Canonical fp of parent + delta from the parent's message sums.  Equal to
// delta_fp bit for bit: the in-place ops swap a parent message's contribution
// for the new word's (the last op on a slot wins, as in DeltaView::pmsg), the
// inserts add theirs.
template <int SPEC, int N>
RMC_HD uint64_t delta_fp_sums(const PState<SPEC, N>& s, const Model& M, const Delta& d, const MsgSums<N>& ms) {
  const DeltaView<SPEC, N> V{s, d};
  uint32_t sig[N];
  uint64_t S[N][N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    sig[i] = server_sig_own<SPEC, N>(i, V.sw(i, 0), V.sw(i, 1), V.sw(i, 2), V.sw(i, 3)) + ms.sig[i];
#pragma unroll
    for (int j = 0; j < N; j++) S[i][j] = i == j ? 0ULL : ms.S[MsgSums<N>::pair(i, j)];
  }
#pragma unroll
  for (int q = 0; q < MAXOPS; q++) {
    if (q >= d.nops) continue;
    const int k = d.opk[q];
    if (k >= 0) {
      bool last = true;
#pragma unroll
      for (int r = q + 1; r < MAXOPS; r++)
        if (r < d.nops && d.opk[r] == k) last = false;
      if (!last) continue;
      msg_contrib<SPEC, N>(s.msg(k), true, sig, S);
    }
    msg_contrib<SPEC, N>(d.opc[q], false, sig, S);
  }
  return canon_from_sums<SPEC, N>(M, V, sig, S);
}

// ------------------------------------------------ 128-bit fingerprints
// fp_bits = 128 (SURVEY.md §7 hard part 2: min-of-hashes over permutations
// raises the collision rate, so a wider mode is offered).  The first word is
// the 64-bit fingerprint above, unchanged; the second is an independent
// 64-bit hash of the same relabelled view (other finalizer, other constants,
// its own message multiset sums S2), taken at the same permutation -- the
// one minimising (first word, second word).  Orbit invariance holds for the
// pair exactly as for the first word.
struct Fp128 {
  uint64_t a, b;
};
RMC_HD bool fp128_less(const Fp128& x, const Fp128& y) { return x.a < y.a || (x.a == y.a && x.b < y.b); }
RMC_HD uint64_t mix64b(uint64_t z) {  // MurmurHash3 fmix64
  z ^= z >> 33;
  z *= 0xff51afd7ed558ccdULL;
  z ^= z >> 33;
  z *= 0xc4ceb9fe1a85ec53ULL;
  return z ^ (z >> 33);
}
template <int SPEC>
RMC_HD uint64_t msg_u2(uint32_t w) {  // the second word's hash of a message body (servers masked)
  int sp, dp;
  msg_srcdst_pos<SPEC>(w, sp, dp);
  const uint32_t body = SPEC == KRAFT ? kr_body(w, sp, dp) : w & ~((7u << sp) | (7u << dp));
  return mix64b((uint64_t)body * 0x9FB21C651E98DF25ULL + 0x2545F4914F6CDD1DULL);
}
template <int SPEC, int N>
RMC_HD uint64_t h_server2(uint32_t P, int i, uint32_t a, uint32_t b, uint32_t c, uint32_t dd) {
  uint32_t a2, c2, d2;
  relabel_server<SPEC, N>(P, i, a, c, dd, a2, c2, d2);
  uint64_t lo = (uint64_t)a2 | ((uint64_t)b << 32);
  uint64_t hi = (uint64_t)c2 | ((uint64_t)d2 << 32);
  int pos = perm_of(P, i);
  return mix64b(mix64b(lo ^ (0xD1B54A32D192ED03ULL * (uint64_t)(pos + 1))) + hi);
}
// The parent's message sums for both words.
template <int N>
struct MsgSums2 {
  MsgSums<N> m;              // first word's sums and the signatures (as MsgSums)
  uint64_t S2[N * (N - 1)];  // second word's pair sums
};
template <int SPEC, int N>
RMC_HD void msg_contrib2(uint32_t w, bool neg, uint64_t (&S2)[N][N]) {
  int sp, dp;
  msg_srcdst_pos<SPEC>(w, sp, dp);
  const int src = (int)((w >> sp) & 7u), dst = (int)((w >> dp) & 7u);
  uint64_t u = msg_u2<SPEC>(w);
  if (neg) u = 0ULL - u;
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int j = 0; j < N; j++)
      if (i != j) S2[i][j] += (i == src && j == dst) ? u : 0ULL;
}
template <int SPEC, int N>
RMC_HD Fp128 canon_from_sums2(const Model& M, const DeltaView<SPEC, N>& V, const uint32_t (&sig)[N],
                              const uint64_t (&S)[N][N], const uint64_t (&S2)[N][N]) {
  bool ties;
  const uint32_t P0 = sig_perm<N>(sig, ties);
  const uint64_t aux = (SPEC == PULL || SPEC == KRAFT) ? h_acked_view(V.d.hdr) : 0ULL;
  const uint64_t aux2 =
      (SPEC == PULL || SPEC == KRAFT) ? mix64b(((uint64_t)(V.d.hdr >> 16) & 0xFFu) + 0x8CB92BA72F3D8DD7ULL) : 0ULL;
  Fp128 best{~0ULL, ~0ULL};
  const int np = ties ? M.nperm : 1;
#pragma unroll 1
  for (int p = 0; p < np; p++) {
    uint32_t P = P0;
    if (ties) {
      P = M.perm[p];
      bool ok = true;
#pragma unroll
      for (int j = 0; j < N; j++)
#pragma unroll
        for (int k = 0; k < N; k++)
          if (sig[j] < sig[k] && perm_of(P, j) > perm_of(P, k)) ok = false;
      if (!ok) continue;
    }
    uint64_t h = aux, h2 = aux2;
#pragma unroll 1
    for (int i = 0; i < N; i++) {
      h += h_server<SPEC, N>(P, i, V.sw(i, 0), V.sw(i, 1), V.sw(i, 2), V.sw(i, 3));
      h2 += h_server2<SPEC, N>(P, i, V.sw(i, 0), V.sw(i, 1), V.sw(i, 2), V.sw(i, 3));
    }
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
      for (int j = 0; j < N; j++)
        if (i != j) {
          const uint64_t key = (uint64_t)(8 * perm_of(P, i) + perm_of(P, j) + 1);
          h += mix64(S[i][j] + 0x9E3779B97F4A7C15ULL * key);
          h2 += mix64b(S2[i][j] + 0xC2B2AE3D27D4EB4FULL * key);
        }
    const Fp128 f{mix64(h), mix64b(h2)};
    if (fp128_less(f, best)) best = f;
  }
  if (best.a == ~0ULL) best.a--;  // ~0 marks an empty slot (first word) / a claim in flight (second word)
  if (best.b == ~0ULL) best.b--;
  return best;
}
// delta_fp_sums for both words (the first equals delta_fp_sums bit for bit).
template <int SPEC, int N>
RMC_HD Fp128 delta_fp_sums2(const PState<SPEC, N>& s, const Model& M, const Delta& d, const MsgSums2<N>& ms) {
  const DeltaView<SPEC, N> V{s, d};
  uint32_t sig[N];
  uint64_t S[N][N], S2[N][N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    sig[i] = server_sig_own<SPEC, N>(i, V.sw(i, 0), V.sw(i, 1), V.sw(i, 2), V.sw(i, 3)) + ms.m.sig[i];
#pragma unroll
    for (int j = 0; j < N; j++) {
      S[i][j] = i == j ? 0ULL : ms.m.S[MsgSums<N>::pair(i, j)];
      S2[i][j] = i == j ? 0ULL : ms.S2[MsgSums<N>::pair(i, j)];
    }
  }
#pragma unroll
  for (int q = 0; q < MAXOPS; q++) {
    if (q >= d.nops) continue;
    const int k = d.opk[q];
    if (k >= 0) {
      bool last = true;
#pragma unroll
      for (int r = q + 1; r < MAXOPS; r++)
        if (r < d.nops && d.opk[r] == k) last = false;
      if (!last) continue;
      msg_contrib<SPEC, N>(s.msg(k), true, sig, S);
      msg_contrib2<SPEC, N>(s.msg(k), true, S2);
    }
    msg_contrib<SPEC, N>(d.opc[q], false, sig, S);
    msg_contrib2<SPEC, N>(d.opc[q], false, S2);
  }
  return canon_from_sums2<SPEC, N>(M, V, sig, S, S2);
}
// The parent's message sums for both words (k_expand builds the same in LDS).
template <int SPEC, int N>
RMC_HD void msg_sums2(const PState<SPEC, N>& s, MsgSums2<N>& ms) {
  for (int k = 0; k < s.nmsg(); k++) {
    int src, dst;
    const uint64_t u = msg_u<SPEC>(s.msg(k), src, dst);
    ms.m.sig[src] += (uint32_t)u;
    ms.m.sig[dst] += (uint32_t)(u >> 32);
    if (src != dst) {
      ms.m.S[MsgSums<N>::pair(src, dst)] += u;
      ms.S2[MsgSums<N>::pair(src, dst)] += msg_u2<SPEC>(s.msg(k));
    }
  }
}
// 128-bit canonical fp of a full packed state.
template <int SPEC, int N>
RMC_HD Fp128 state_fp2(const PState<SPEC, N>& s, const Model& M) {
  Delta d;
  d.srv = -1;
  d.nops = 0;
  d.hdr = s.hdr();
  MsgSums2<N> ms{};
  msg_sums2<SPEC, N>(s, ms);
  return delta_fp_sums2<SPEC, N>(s, M, d, ms);
}

// Canonical fp of the successor parent + delta.
template <int SPEC, int N>
RMC_HD uint64_t delta_fp(const PState<SPEC, N>& s, const Model& M, const Delta& d) {
  return canon_fp<SPEC, N>(M, DeltaView<SPEC, N>{s, d});
}

// Canonical fp of a full packed state (the view with an empty delta).
template <int SPEC, int N>
RMC_HD uint64_t state_fp(const PState<SPEC, N>& s, const Model& M) {
  Delta d;
  d.srv = -1;
  d.nops = 0;
  d.hdr = s.hdr();
  return canon_fp<SPEC, N>(M, DeltaView<SPEC, N>{s, d});
}

}  // namespace rmc
