// rmc_host.cpp — host instantiations of the shared action code (rmc_spec.h):
// initial-state fingerprint, trace replay and invariant re-checks.  Compiled
// by hipcc as host code; no device work happens here.
#include "rmc_engine.h"

namespace rmc {

template <int SPEC, int N>
static int eval_apply_t(const Model& M, const uint32_t* parent, int b, uint32_t* out, int* ordinal, int* act,
                        int* err) {
  PState<SPEC, N> s{parent};
  Delta d;
  bool en = eval_binding<SPEC, N>(s, M, b, d);
  if (!en) return 0;
  if (ordinal) *ordinal = d.ordinal;
  if (act) *act = d.act;
  if (err) *err = d.err;
  if (d.err) return 1;
  int e = apply_delta<SPEC, N>(s, M, d, out);
  if (e && err) *err = e;
  return 1;
}

template <int SPEC, int N>
static unsigned long long fp_t(const Model& M, const uint32_t* S) {
  PState<SPEC, N> s{S};
  return state_fp<SPEC, N>(s, M);
}
template <int SPEC, int N>
static int fp2_t(const Model& M, const uint32_t* S, unsigned long long* ab) {
  PState<SPEC, N> s{S};
  const Fp128 f = state_fp2<SPEC, N>(s, M);
  ab[0] = f.a;
  ab[1] = f.b;
  return 0;
}

// Test hook: the three ways the fingerprint of a successor is computed agree
// (delta_fp from parent + delta, delta_fp_sums from the parent's message sums
// as k_expand does, state_fp of the materialized row).  0 = agree; 2 = the
// guard prefilter may_enable rejects an enabled binding.
template <int SPEC, int N>
static int fp_check_t(const Model& M, const uint32_t* parent, int b, const uint32_t* row) {
  PState<SPEC, N> s{parent};
  Delta d;
  if (!eval_binding<SPEC, N>(s, M, b, d)) return 0;
  // k_expand evaluates a fixed binding only if may_enable passes: it must hold
  // for every enabled binding (and every one that raises an error)
  if (b < M.nfixed && !may_enable<SPEC, N>(s, M, b)) return 2;
  if (d.err) return 0;
  MsgSums<N> ms{};
  for (int k = 0; k < s.nmsg(); k++) {
    int src, dst;
    const uint64_t u = msg_u<SPEC>(s.msg(k), src, dst);
    ms.sig[src] += (uint32_t)u;
    ms.sig[dst] += (uint32_t)(u >> 32);
    if (src != dst) ms.S[MsgSums<N>::pair(src, dst)] += u;
  }
  const unsigned long long a = delta_fp<SPEC, N>(s, M, d), c = delta_fp_sums<SPEC, N>(s, M, d, ms);
  PState<SPEC, N> t{row};
  const unsigned long long f = state_fp<SPEC, N>(t, M);
  // the 128-bit fingerprint: incremental (as k_expand<.., 2> computes it) == full, first word == the 64-bit one
  MsgSums2<N> ms2{};
  msg_sums2<SPEC, N>(s, ms2);
  const Fp128 g = delta_fp_sums2<SPEC, N>(s, M, d, ms2), h = state_fp2<SPEC, N>(t, M);
  return (a == f && c == f && g.a == h.a && g.b == h.b && g.a == f) ? 0 : 1;
}

template <int SPEC, int N>
static int inv_t(const Model& M, const uint32_t* S, int* err) {
  PState<SPEC, N> s{S};
  int e = 0;
  int r = check_invariants<SPEC, N>(s, M, e);
  if (err) *err = e;
  return r;
}

#define RMC_DISPATCH(FN, ...)                                    \
  switch (M.spec * 8 + M.N) {                                    \
    case RAFT * 8 + 2: return FN<RAFT, 2>(__VA_ARGS__);          \
    case RAFT * 8 + 3: return FN<RAFT, 3>(__VA_ARGS__);          \
    case RAFT * 8 + 4: return FN<RAFT, 4>(__VA_ARGS__);          \
    case RAFT * 8 + 5: return FN<RAFT, 5>(__VA_ARGS__);          \
    case FLEX * 8 + 2: return FN<FLEX, 2>(__VA_ARGS__);          \
    case FLEX * 8 + 3: return FN<FLEX, 3>(__VA_ARGS__);          \
    case FLEX * 8 + 4: return FN<FLEX, 4>(__VA_ARGS__);          \
    case FLEX * 8 + 5: return FN<FLEX, 5>(__VA_ARGS__);          \
    case FSYNC * 8 + 2: return FN<FSYNC, 2>(__VA_ARGS__);        \
    case FSYNC * 8 + 3: return FN<FSYNC, 3>(__VA_ARGS__);        \
    case FSYNC * 8 + 4: return FN<FSYNC, 4>(__VA_ARGS__);        \
    case FSYNC * 8 + 5: return FN<FSYNC, 5>(__VA_ARGS__);        \
    case PULL * 8 + 2: return FN<PULL, 2>(__VA_ARGS__);          \
    case PULL * 8 + 3: return FN<PULL, 3>(__VA_ARGS__);          \
    case PULL * 8 + 4: return FN<PULL, 4>(__VA_ARGS__);          \
    case PULL * 8 + 5: return FN<PULL, 5>(__VA_ARGS__);          \
    case PULL2 * 8 + 2: return FN<PULL2, 2>(__VA_ARGS__);        \
    case PULL2 * 8 + 3: return FN<PULL2, 3>(__VA_ARGS__);        \
    case PULL2 * 8 + 4: return FN<PULL2, 4>(__VA_ARGS__);        \
    case PULL2 * 8 + 5: return FN<PULL2, 5>(__VA_ARGS__);        \
    case KRAFT * 8 + 2: return FN<KRAFT, 2>(__VA_ARGS__);        \
    case KRAFT * 8 + 3: return FN<KRAFT, 3>(__VA_ARGS__);        \
  }

int host_eval_apply(const Model& M, const uint32_t* parent, int binding, uint32_t* out, int* ordinal, int* act,
                    int* err) {
  RMC_DISPATCH(eval_apply_t, M, parent, binding, out, ordinal, act, err);
  return -1;
}
unsigned long long host_fingerprint(const Model& M, const uint32_t* S) {
  RMC_DISPATCH(fp_t, M, S);
  return 0;
}
void host_fingerprint2(const Model& M, const uint32_t* S, unsigned long long* ab) {
  [&]() -> int { RMC_DISPATCH(fp2_t, M, S, ab); return -1; }();
}
int host_fp_check(const Model& M, const uint32_t* parent, int binding, const uint32_t* row) {
  RMC_DISPATCH(fp_check_t, M, parent, binding, row);
  return -1;
}
int host_check_invariants(const Model& M, const uint32_t* S, int* err) {
  RMC_DISPATCH(inv_t, M, S, err);
  return -1;
}

}  // namespace rmc

// ---------------------------------------------------------------------------
// Test hooks (never reached from rmc_check / raftmc): a sequential host BFS
// over the SAME lowered action code and fingerprint as the kernels, so the
// CPU test suite can check the lowering against the oracle without a GPU,
// and message-codec probes for the layout tests.
#include <unordered_map>
#include <vector>
#include <string>
#include <cstring>
#include "../../include/rmc.h"

namespace rmc {
std::vector<uint32_t> selftest_init_state(const Model& M) {
  std::vector<uint32_t> S(M.words, 0u);
  for (int i = 0; i < M.N; i++) {
    S[1 + 4 * i] = 1u | ((uint32_t)NILS << 6) | ((M.spec == PULL2 || M.spec == KRAFT) ? (uint32_t)NILS << 15 : 0u);
    if (M.spec == KRAFT) S[1 + 4 * i] = kr_set_st(S[1 + 4 * i], KS_UNATTACHED);
    S[3 + 4 * i] = (pullish(M.spec) || M.spec == KRAFT) ? 0u : all_rows(M.N, 1);
  }
  return S;
}
}  // namespace rmc

extern "C" int rmc_selftest_encode_msg(int spec, const int* f, uint32_t* out) {
  using namespace rmc;
  MsgF m = msg_zero();
  m.type = f[0]; m.term = f[1]; m.src = f[2]; m.dst = f[3]; m.lli = f[4]; m.llt = f[5]; m.granted = f[6];
  m.pli = f[7]; m.plt = f[8]; m.nent = f[9]; m.eterm = f[10]; m.evalue = f[11]; m.commit = f[12];
  m.success = f[13]; m.midx = f[14]; m.lci = f[15]; m.lct = f[16]; m.count = f[17];
  if (spec == PULL2) m.lcenil = f[18];  // the PullRaftVariant2 probe passes 19 fields
  MsgF d;
  int sp, dp, term, type;
  if (spec == PULL2) {
    *out = msg_encode<PULL2>(m); d = msg_decode<PULL2>(*out); msg_srcdst_pos<PULL2>(*out, sp, dp);
    term = msg_term<PULL2>(*out); type = msg_type<PULL2>(*out);
  } else if (spec == PULL) {
    *out = msg_encode<PULL>(m); d = msg_decode<PULL>(*out); msg_srcdst_pos<PULL>(*out, sp, dp);
    term = msg_term<PULL>(*out); type = msg_type<PULL>(*out);
  } else {
    *out = msg_encode<RAFT>(m); d = msg_decode<RAFT>(*out); msg_srcdst_pos<RAFT>(*out, sp, dp);
    term = msg_term<RAFT>(*out); type = msg_type<RAFT>(*out);
  }
  int ok = d.type == m.type && d.term == m.term && d.src == m.src && d.dst == m.dst && d.lli == m.lli &&
           d.llt == m.llt && d.granted == m.granted && d.pli == m.pli && d.plt == m.plt && d.nent == m.nent &&
           d.eterm == m.eterm && d.evalue == m.evalue && d.commit == m.commit && d.success == m.success &&
           d.midx == m.midx && d.lci == m.lci && d.lct == m.lct && d.lcenil == m.lcenil && d.count == m.count &&
           (int)((*out >> sp) & 7u) == m.src && (int)((*out >> dp) & 7u) == m.dst && term == m.term &&
           type == m.type;
  return ok ? 0 : 1;
}

// KRaft record probe (tests/test_kraft.py): f = cls, dst, src, epoch, err,
// leader (-1 Nil), granted, f1, f2, cepoch, cfo, clfe, elen, eepoch, evalue,
// hwm, divend, divepoch, count.  Packs with kr_encode and checks that
// kr_decode, the source/destination positions and the epoch read it back.
extern "C" int rmc_selftest_encode_kmsg(const int* f, uint32_t* out) {
  using namespace rmc;
  KMsg m = kmsg_zero();
  m.cls = f[0]; m.dst = f[1]; m.src = f[2]; m.epoch = f[3]; m.err = f[4]; m.leader = f[5]; m.granted = f[6];
  m.f1 = f[7]; m.f2 = f[8]; m.cepoch = f[9]; m.cfo = f[10]; m.clfe = f[11]; m.elen = f[12]; m.eepoch = f[13];
  m.evalue = f[14]; m.hwm = f[15]; m.divend = f[16]; m.divepoch = f[17]; m.count = f[18];
  *out = kr_encode(m);
  const KMsg d = kr_decode(*out);
  int sp, dp;
  msg_srcdst_pos<KRAFT>(*out, sp, dp);
  const int ok = d.cls == m.cls && d.dst == m.dst && d.src == m.src && d.epoch == m.epoch && d.err == m.err &&
                 d.leader == m.leader && d.granted == m.granted && d.f1 == m.f1 && d.f2 == m.f2 &&
                 d.cepoch == m.cepoch && d.cfo == m.cfo && d.clfe == m.clfe && d.elen == m.elen &&
                 d.eepoch == m.eepoch && d.evalue == m.evalue && d.hwm == m.hwm && d.divend == m.divend &&
                 d.divepoch == m.divepoch && d.count == m.count && (int)((*out >> sp) & 7u) == m.src &&
                 (int)((*out >> dp) & 7u) == m.dst && msg_term<KRAFT>(*out) == m.epoch;
  return ok ? 0 : 1;
}
