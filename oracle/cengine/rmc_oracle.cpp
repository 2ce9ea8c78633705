// rmc_oracle — CPU restatement of the four Raft specs under TLC -workers 1
// semantics.  TEST INFRASTRUCTURE ONLY: this is the checker the HIP path is
// compared against (and the CPU baseline bench.py times); it shares no code
// with raft-tlaplus_amd/.
//
// Restated from /root/reference/specifications/:
//   standard-raft/Raft.tla        (Next :527-539, invariants :588-620)
//   flexible-raft/FlexibleRaft.tla (Next :488-500)
//   raft-and-fsync/RaftFsync.tla  (Next :522-536)
//   pull-raft/PullRaft.tla        (Next :542-558)
//   pull-raft/PullRaftVariant2.tla (Next :560-576)
// TLC semantics: actions split per constant binding
// (first bound variable fastest), DOMAIN messages enumerated in TLC value
// order, FIFO BFS, first successor per fingerprint wins, invariants checked on
// new states, VIEW hides the aux variables, SYMMETRY = all server permutations.
//
// Fingerprints here are EXACT canonical forms (lexicographic minimum of a
// complete serialisation of the view over every server permutation that can
// attain it) hashed to 128 bits; the GPU path uses a different construction
// (min over permutations of a 64-bit additive hash), so agreement between the
// two is evidence for both.
//
// Parity unpinned against TLC: the reference ships no counts or traces and TLC
// (Java) is absent here and on the GPU box; this restatement is
// pinned by SURVEY.md Appendix B and by agreement with oracle/pyoracle.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>
#include <thread>
#include <atomic>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

namespace {

enum SpecKind { RAFT = 0, FLEX = 1, FSYNC = 2, PULL = 3, PULL2 = 4 };
enum MType : int8_t { RVREQ = 0, RVRESP, AEREQ, AERESP, LNREQ, PEREQ, PERESP };
enum SState : int8_t { FOLLOWER = 0, CANDIDATE = 1, LEADER = 2 };
constexpr int NIL = -1;
constexpr int MAXN = 8, MAXV = 4, MAXL = 8, MAXMSG = 192;

struct EvalError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// A message record.  Unused fields are 0 so memcmp over the record part is
// record equality.  `count` is the bag multiplicity (messages[m]).
struct Msg {
  int8_t type, term, src, dst;
  int8_t lastLogTerm, lastLogIndex;  // RequestVoteRequest, PullEntriesRequest
  int8_t voteGranted;                // RequestVoteResponse
  int8_t prevLogIndex, prevLogTerm;  // AppendEntriesRequest
  int8_t nent, eterm, evalue;        // mentries (0 or 1 entry)
  int8_t commit;                     // mcommitIndex
  int8_t success, matchIndex;        // AppendEntriesResponse, PullEntriesResponse
  int8_t lciIndex, lciTerm;          // mlastCommonEntry
  int8_t lceNil;                     // Variant2 LeaderNotifyRequest: mlastCommonEntry = Nil
  uint8_t count;
};
constexpr size_t REC_BYTES = offsetof(Msg, count);
inline bool rec_eq(const Msg& a, const Msg& b) { return memcmp(&a, &b, REC_BYTES) == 0; }

struct Entry { int8_t term, value; };

struct State {
  int16_t nmsg;
  int8_t electionCtr, restartCtr;
  int8_t acked[MAXV];  // -1 Nil, 0 FALSE, 1 TRUE
  int8_t term[MAXN], st[MAXN], voted[MAXN];  // voted = votedFor (Pull, Variant2: leader)
  int8_t voted2[MAXN];                        // Variant2: votedFor
  int8_t vleI[MAXN][MAXN], vleT[MAXN][MAXN];  // Variant2: votesLastEntry (index -1 = Nil)
  int8_t loglen[MAXN], commit[MAXN], fsync[MAXN];
  uint8_t votes[MAXN], pending[MAXN];  // bitsets over servers
  Entry log[MAXN][MAXL];
  int8_t next[MAXN][MAXN], match[MAXN][MAXN];
  Msg msgs[MAXMSG];  // DOMAIN messages, sorted in TLC order
};
constexpr size_t FIXED_BYTES = offsetof(State, msgs);

struct Config {
  SpecKind spec = RAFT;
  bool pull() const { return spec == PULL || spec == PULL2; }
  int N = 3, V = 1, E = 2, R = 0;
  int EQ = 0, RQ = 0;                       // FlexibleRaft quorum sizes
  bool lfae = false, lfiq = true, ffbr = true;  // RaftFsync policy flags
  bool inv_lhaav = true, inv_nld = true, inv_cerm = false;
  std::vector<std::string> inv_order;
};
Config C;

// ------------------------------------------------------------- TLC ordering
// TLC compares records by field count, then (sorted) field name and value in
// turn; sequences by length then elements; model values by name; FALSE<TRUE.
// We build a byte key with exactly that lexicographic order.
const char* type_name(int t) {
  static const char* n[] = {"RequestVoteRequest", "RequestVoteResponse", "AppendEntriesRequest",
                            "AppendEntriesResponse", "LeaderNotifyRequest", "PullEntriesRequest",
                            "PullEntriesResponse"};
  return n[t];
}
struct Key {
  uint8_t b[160];
  int n = 0;
  void byte(int v) { b[n++] = (uint8_t)v; }
  void str(const char* s) { while (*s) b[n++] = (uint8_t)*s++; b[n++] = 0; }
};
struct Field { const char* name; int kind; int v0, v1, v2; };
// kinds: 0 int/bool/server, 1 type name, 2 mentries seq, 3 lastCommonEntry record,
// 4 lastCommonEntry Nil-or-record (Variant2: the untyped model value Nil
// compares below any record)
void msg_key(const Msg& m, Key& k) {
  Field f[8];
  int nf = 0;
  auto add = [&](const char* nm, int kind, int a = 0, int b = 0, int c = 0) { f[nf++] = {nm, kind, a, b, c}; };
  add("mtype", 1, m.type);
  add("mterm", 0, m.term);
  add("msource", 0, m.src);
  add("mdest", 0, m.dst);
  switch (m.type) {
    case RVREQ: case PEREQ:
      add("mlastLogTerm", 0, m.lastLogTerm); add("mlastLogIndex", 0, m.lastLogIndex); break;
    case RVRESP:
      add("mvoteGranted", 0, m.voteGranted);
      if (C.spec == PULL2) { add("mlastLogIndex", 0, m.lastLogIndex); add("mlastLogTerm", 0, m.lastLogTerm); }
      break;
    case AEREQ:
      add("mprevLogIndex", 0, m.prevLogIndex); add("mprevLogTerm", 0, m.prevLogTerm);
      add("mentries", 2, m.nent, m.eterm, m.evalue); add("mcommitIndex", 0, m.commit); break;
    case AERESP: add("msuccess", 0, m.success); add("mmatchIndex", 0, m.matchIndex); break;
    case LNREQ:
      if (C.spec == PULL2) add("mlastCommonEntry", 4, m.lceNil, m.lciIndex, m.lciTerm);
      break;
    case PERESP:
      add("msuccess", 0, m.success);
      if (m.success) { add("mentries", 2, m.nent, m.eterm, m.evalue); add("mcommitIndex", 0, m.commit); }
      else add("mlastCommonEntry", 3, m.lciIndex, m.lciTerm);
      break;
  }
  std::sort(f, f + nf, [](const Field& a, const Field& b) { return strcmp(a.name, b.name) < 0; });
  k.n = 0;
  k.byte(nf);
  for (int i = 0; i < nf; i++) {
    k.str(f[i].name);
    switch (f[i].kind) {
      case 0: k.byte(f[i].v0); break;
      case 1: k.str(type_name(f[i].v0)); break;
      case 2:  // <<>> or << [term |-> t, value |-> v] >>
        k.byte(f[i].v0);
        if (f[i].v0) { k.byte(2); k.str("term"); k.byte(f[i].v1); k.str("value"); k.byte(f[i].v2); }
        break;
      case 3: k.byte(2); k.str("index"); k.byte(f[i].v0); k.str("term"); k.byte(f[i].v1); break;
      case 4:
        if (f[i].v0) k.byte(0);
        else { k.byte(1); k.byte(2); k.str("index"); k.byte(f[i].v1); k.str("term"); k.byte(f[i].v2); }
        break;
    }
  }
}
int tlc_cmp(const Msg& a, const Msg& b) {
  Key ka, kb;
  msg_key(a, ka);
  msg_key(b, kb);
  int n = std::min(ka.n, kb.n);
  int c = memcmp(ka.b, kb.b, n);
  if (c) return c;
  return ka.n - kb.n;
}

// ------------------------------------------------------------- bag helpers
int find_msg(const State& s, const Msg& m) {
  for (int k = 0; k < s.nmsg; k++)
    if (rec_eq(s.msgs[k], m)) return k;
  return -1;
}
void insert_msg(State& s, Msg m, int count) {  // m not in DOMAIN
  if (s.nmsg >= MAXMSG) throw EvalError("message capacity exceeded (oracle MAXMSG)");
  m.count = (uint8_t)count;
  int pos = s.nmsg;
  while (pos > 0 && tlc_cmp(s.msgs[pos - 1], m) > 0) {
    s.msgs[pos] = s.msgs[pos - 1];
    pos--;
  }
  s.msgs[pos] = m;
  s.nmsg++;
}
Msg mk(int type, int term, int src, int dst) {
  Msg m;
  memset(&m, 0, sizeof m);
  m.type = (int8_t)type; m.term = (int8_t)term; m.src = (int8_t)src; m.dst = (int8_t)dst;
  return m;
}

// Send variants (Raft.tla:129-155; FlexibleRaft.tla:127-133; RaftFsync.tla:132-134; PullRaft.tla:137-143)
bool send_once(State& t, const Msg& m) {
  if (find_msg(t, m) >= 0) return false;
  insert_msg(t, m, 1);
  return true;
}
void send_norestrict(State& t, const Msg& m) {
  int k = find_msg(t, m);
  if (k >= 0) t.msgs[k].count++;
  else insert_msg(t, m, 1);
}
// Reply (Raft.tla:170-176 increments an existing response; the other specs
// require the response to be absent: FlexibleRaft.tla:148-151 etc.)
bool reply(State& t, const Msg& response, int req_idx) {
  if (!(t.msgs[req_idx].count > 0)) return false;
  int k = find_msg(t, response);
  if (k >= 0) {
    if (C.spec != RAFT) return false;
    t.msgs[req_idx].count--;
    t.msgs[k].count++;
    return true;
  }
  t.msgs[req_idx].count--;
  insert_msg(t, response, 1);
  return true;
}

// --------------------------------------------------------------- helpers
inline int Len(const State& s, int i) { return s.loglen[i]; }
inline const Entry& log_at(const State& s, int i, int idx) {
  if (idx < 1 || idx > s.loglen[i]) throw EvalError("log[" + std::to_string(i) + "] applied to " + std::to_string(idx));
  return s.log[i][idx - 1];
}
inline int LastTerm(const State& s, int i) { return s.loglen[i] == 0 ? 0 : log_at(s, i, s.loglen[i]).term; }
inline int popc(unsigned x) { return __builtin_popcount(x); }
inline bool is_quorum(unsigned set) { return popc(set) * 2 > C.N; }  // Raft.tla:123
void append(State& t, int i, Entry e) {
  if (t.loglen[i] >= MAXL) throw EvalError("log capacity exceeded (oracle MAXL)");
  t.log[i][t.loglen[i]++] = e;
}
bool receivable(const State& s, int k, int type, bool equal) {  // Raft.tla:181-187
  const Msg& m = s.msgs[k];
  if (!(m.count > 0) || m.type != type) return false;
  return equal ? m.term == s.term[m.dst] : m.term <= s.term[m.dst];
}

// Successors are reported with their action id (for labels / stats).
enum Act {
  A_RESTART, A_REQUESTVOTE, A_TIMEOUT, A_REQUESTVOTE_IJ, A_BECOMELEADER, A_CLIENTREQUEST,
  A_ADVANCECOMMIT, A_APPENDENTRIES, A_ADVANCEFSYNC, A_UPDATETERM, A_HRVREQ, A_HRVRESP,
  A_REJECTAE, A_ACCEPTAE, A_HAERESP, A_REJECTPULL, A_ACCEPTPULL, A_LEARNOFLEADER,
  A_SENDPULL, A_HSUCCESSPULL, A_HFAILPULL, A_COUNT
};
const char* act_name(int a) {
  static const char* n[] = {"Restart", "RequestVote", "Timeout", "RequestVote", "BecomeLeader",
                            "ClientRequest", "AdvanceCommitIndex", "AppendEntries", "AdvanceFsyncIndex",
                            "UpdateTerm", "HandleRequestVoteRequest", "HandleRequestVoteResponse",
                            "RejectAppendEntriesRequest", "AcceptAppendEntriesRequest",
                            "HandleAppendEntriesResponse", "RejectPullEntriesRequest",
                            "AcceptPullEntriesRequest", "LearnOfLeader", "SendPullEntriesRequest",
                            "HandleSuccessPullEntriesResponse", "HandleFailPullEntriesResponse"};
  return n[a];
}

struct Emitter {
  virtual void emit(const State& t, int act) = 0;
  virtual ~Emitter() {}
};

// ----------------------------------------------------------------- actions
void Restart(const State& s, int i, Emitter& E) {
  // Raft.tla:226-235, FlexibleRaft.tla:200-208, RaftFsync.tla:203-218, PullRaft.tla:258-265
  if (!(s.restartCtr < C.R)) return;
  State t = s;
  t.st[i] = FOLLOWER;
  t.votes[i] = 0;
  for (int j = 0; j < C.N; j++) { t.next[i][j] = 1; t.match[i][j] = 0; }
  t.pending[i] = 0;
  t.commit[i] = 0;
  t.restartCtr++;
  if (C.spec == PULL2) {  // PullRaftVariant2.tla:251-260: leader and votesLastEntry reset too
    t.voted[i] = NIL;
    for (int j = 0; j < C.N; j++) { t.vleI[i][j] = -1; t.vleT[i][j] = 0; }
  }
  if (C.spec == FSYNC) {
    int f = s.fsync[i], L = s.loglen[i];
    if (f == 0) t.loglen[i] = 0;
    else if (L > 0 && L > f) t.loglen[i] = (int8_t)f;  // SubSeq(@, 1, fsyncIndex[i])
  }
  E.emit(t, A_RESTART);
}

void RequestVote(const State& s, int i, Emitter& E) {
  // Raft.tla:242-257 (= FlexibleRaft.tla:215-230; PullRaft.tla:283-298 sets leader[i])
  if (!(s.electionCtr < C.E)) return;
  if (!(s.st[i] == FOLLOWER || s.st[i] == CANDIDATE)) return;
  State t = s;
  for (int j = 0; j < C.N; j++) {
    if (j == i) continue;
    Msg m = mk(RVREQ, s.term[i] + 1, i, j);
    m.lastLogTerm = (int8_t)LastTerm(s, i);
    m.lastLogIndex = (int8_t)Len(s, i);
    if (find_msg(s, m) >= 0) return;  // SendMultipleOnce: all must be new
    insert_msg(t, m, 1);
  }
  t.st[i] = CANDIDATE;
  t.term[i] = (int8_t)(s.term[i] + 1);
  t.voted[i] = (int8_t)i;
  if (C.spec == PULL2) {  // PullRaftVariant2.tla:284-286: votedFor = i, leader = Nil
    t.voted2[i] = (int8_t)i;
    t.voted[i] = NIL;
  }
  t.votes[i] = (uint8_t)(1u << i);
  t.electionCtr++;
  E.emit(t, A_REQUESTVOTE);
}

void Timeout(const State& s, int i, Emitter& E) {  // RaftFsync.tla:222-230
  if (!(s.electionCtr < C.E)) return;
  if (!(s.st[i] == FOLLOWER || s.st[i] == CANDIDATE)) return;
  State t = s;
  t.st[i] = CANDIDATE;
  t.term[i] = (int8_t)(s.term[i] + 1);
  t.voted[i] = (int8_t)i;
  t.votes[i] = (uint8_t)(1u << i);
  t.electionCtr++;
  E.emit(t, A_TIMEOUT);
}

void RequestVoteIJ(const State& s, int i, int j, Emitter& E) {  // RaftFsync.tla:234-243
  if (s.st[i] != CANDIDATE || i == j) return;
  Msg m = mk(RVREQ, s.term[i], i, j);
  m.lastLogTerm = (int8_t)LastTerm(s, i);
  m.lastLogIndex = (int8_t)Len(s, i);
  State t = s;
  if (!send_once(t, m)) return;
  E.emit(t, A_REQUESTVOTE_IJ);
}

void AppendEntries(const State& s, int i, int j, Emitter& E) {
  // Raft.tla:263-285; FlexibleRaft.tla:236-256; RaftFsync.tla:249-272
  if (i == j || s.st[i] != LEADER) return;
  if (C.spec == RAFT && (s.pending[i] >> j & 1)) return;
  int nxt = s.next[i][j];
  int prevLogIndex = nxt - 1;
  int prevLogTerm = prevLogIndex > 0 ? log_at(s, i, prevLogIndex).term : 0;
  int lastEntry = std::min(Len(s, i), nxt);
  if (C.spec == FSYNC && C.lfae && !(s.fsync[i] >= lastEntry)) return;
  Msg m = mk(AEREQ, s.term[i], i, j);
  m.prevLogIndex = (int8_t)prevLogIndex;
  m.prevLogTerm = (int8_t)prevLogTerm;
  // SubSeq(log[i], nextIndex[i][j], lastEntry): at most one entry
  int nent = lastEntry - nxt + 1;
  if (nent < 0) nent = 0;
  if (nent > 1) throw EvalError("AppendEntries: more than one entry");
  m.nent = (int8_t)nent;
  if (nent) { const Entry& e = log_at(s, i, nxt); m.eterm = e.term; m.evalue = e.value; }
  m.commit = (int8_t)std::min((int)s.commit[i], lastEntry);
  State t = s;
  if (C.spec == RAFT) {
    t.pending[i] |= (uint8_t)(1u << j);
    if (nent == 0) { if (!send_once(t, m)) return; }  // _SendOnce for empty AE
    else send_norestrict(t, m);
  } else {
    if (!send_once(t, m)) return;
  }
  E.emit(t, A_APPENDENTRIES);
}

void LastCommonEntry(const State& s, int i, int lastIndex, int lastTerm, int& idx, int& term);
void BecomeLeader(const State& s, int i, Emitter& E) {
  // Raft.tla:289-300; FlexibleRaft.tla:260-269; RaftFsync.tla:276-285; PullRaft.tla:354-366
  if (s.st[i] != CANDIDATE) return;
  bool q = C.spec == FLEX ? popc(s.votes[i]) >= C.EQ : is_quorum(s.votes[i]);
  if (!q) return;
  State t = s;
  if (C.spec == PULL) {
    for (int j = 0; j < C.N; j++) {
      if (s.votes[i] >> j & 1) continue;
      Msg m = mk(LNREQ, s.term[i], i, j);
      if (find_msg(s, m) >= 0) return;
      insert_msg(t, m, 1);
    }
  }
  if (C.spec == PULL2) {  // PullRaftVariant2.tla:361-379: every other server, with the last common entry
    for (int j = 0; j < C.N; j++) {
      if (j == i) continue;
      Msg m = mk(LNREQ, s.term[i], i, j);
      if (s.vleI[i][j] < 0) m.lceNil = 1;
      else {
        int a, b;
        LastCommonEntry(s, i, s.vleI[i][j], s.vleT[i][j], a, b);
        m.lciIndex = (int8_t)a;
        m.lciTerm = (int8_t)b;
      }
      if (find_msg(s, m) >= 0) return;
      insert_msg(t, m, 1);
    }
    t.voted[i] = (int8_t)i;  // leader' = i
  }
  t.st[i] = LEADER;
  for (int j = 0; j < C.N; j++) {
    if (!C.pull()) t.next[i][j] = (int8_t)(Len(s, i) + 1);
    t.match[i][j] = 0;
  }
  if (C.spec == RAFT) t.pending[i] = 0;
  E.emit(t, A_BECOMELEADER);
}

void ClientRequest(const State& s, int i, int v, Emitter& E) {  // Raft.tla:304-313
  if (s.st[i] != LEADER || s.acked[v] != NIL) return;
  State t = s;
  append(t, i, Entry{s.term[i], (int8_t)v});
  t.acked[v] = 0;
  E.emit(t, A_CLIENTREQUEST);
}

unsigned agree_set(const State& s, int i, int index, const int8_t* matchrow) {
  // Raft.tla:323-324; RaftFsync.tla:313-315
  unsigned ks = 0;
  for (int k = 0; k < C.N; k++)
    if (matchrow[k] >= index) ks |= 1u << k;
  if (C.spec == FSYNC && C.lfiq && index > s.fsync[i]) return ks;
  return ks | (1u << i);
}
bool agree_ok(unsigned set) {
  return C.spec == FLEX ? popc(set) >= C.RQ : is_quorum(set);  // FlexibleRaft.tla:296
}
int new_commit_index(const State& s, int i, const int8_t* matchrow) {
  int best = 0;
  for (int index = 1; index <= Len(s, i); index++)
    if (agree_ok(agree_set(s, i, index, matchrow))) best = index;  // Max(agreeIndexes)
  if (best > 0 && log_at(s, i, best).term == s.term[i]) return best;
  return s.commit[i];
}
void update_acked(const State& s, State& t, int i, int newCommit) {  // Raft.tla:339-342
  for (int v = 0; v < C.V; v++) {
    if (s.acked[v] != 0) continue;
    bool in = false;
    for (int idx = s.commit[i] + 1; idx <= newCommit; idx++)
      if (log_at(s, i, idx).value == v) in = true;
    t.acked[v] = in ? 1 : 0;
  }
}

void AdvanceCommitIndex(const State& s, int i, Emitter& E) {  // Raft.tla:320-344
  if (s.st[i] != LEADER) return;
  int nc = new_commit_index(s, i, s.match[i]);
  if (!(s.commit[i] < nc)) return;
  State t = s;
  t.commit[i] = (int8_t)nc;
  update_acked(s, t, i, nc);
  E.emit(t, A_ADVANCECOMMIT);
}

void AdvanceFsyncIndex(const State& s, int i, Emitter& E) {  // RaftFsync.tla:339-343
  if (!(s.fsync[i] < Len(s, i))) return;
  State t = s;
  t.fsync[i]++;
  E.emit(t, A_ADVANCEFSYNC);
}

void UpdateTerm(const State& s, Emitter& E) {  // Raft.tla:348-355; PullRaft.tla:269-276
  for (int k = 0; k < s.nmsg; k++) {
    const Msg& m = s.msgs[k];
    if (!(m.term > s.term[m.dst])) continue;
    State t = s;
    t.term[m.dst] = m.term;
    t.st[m.dst] = FOLLOWER;
    t.voted[m.dst] = NIL;
    if (C.spec == PULL2) t.voted2[m.dst] = NIL;  // PullRaftVariant2.tla:269-270
    E.emit(t, A_UPDATETERM);
  }
}

void HandleRequestVoteRequest(const State& s, Emitter& E) {  // Raft.tla:360-381; PullRaft.tla:306-330
  for (int k = 0; k < s.nmsg; k++) {
    if (!receivable(s, k, RVREQ, false)) continue;
    const Msg& m = s.msgs[k];
    int i = m.dst, j = m.src;
    int lt = LastTerm(s, i);
    bool logOk = m.lastLogTerm > lt || (m.lastLogTerm == lt && m.lastLogIndex >= Len(s, i));
    // PullRaftVariant2.tla:303-326: the vote is votedFor's; the response carries the last entry
    const int8_t* vf = C.spec == PULL2 ? s.voted2 : s.voted;
    bool grant = m.term == s.term[i] && logOk && (vf[i] == NIL || vf[i] == j);
    Msg r = mk(RVRESP, s.term[i], i, j);
    r.voteGranted = grant;
    if (C.spec == PULL2) { r.lastLogIndex = (int8_t)Len(s, i); r.lastLogTerm = (int8_t)lt; }
    State t = s;
    if (!reply(t, r, k)) continue;
    if (grant) (C.spec == PULL2 ? t.voted2 : t.voted)[i] = (int8_t)j;
    E.emit(t, A_HRVREQ);
  }
}

void HandleRequestVoteResponse(const State& s, Emitter& E) {  // Raft.tla:386-401
  for (int k = 0; k < s.nmsg; k++) {
    if (!receivable(s, k, RVRESP, true)) continue;
    const Msg& m = s.msgs[k];
    State t = s;
    if (m.voteGranted) t.votes[m.dst] |= (uint8_t)(1u << m.src);
    if (m.voteGranted && C.spec == PULL2) {  // PullRaftVariant2.tla:342-344
      t.vleI[m.dst][m.src] = m.lastLogIndex;
      t.vleT[m.dst][m.src] = m.lastLogTerm;
    }
    t.msgs[k].count--;  // Discard
    E.emit(t, A_HRVRESP);
  }
}

bool LogOk(const State& s, int i, const Msg& m) {  // Raft.tla:406-410
  if (m.prevLogIndex == 0) return true;
  return m.prevLogIndex > 0 && m.prevLogIndex <= Len(s, i) &&
         m.prevLogTerm == log_at(s, i, m.prevLogIndex).term;
}

void RejectAppendEntriesRequest(const State& s, Emitter& E) {  // Raft.tla:412-430
  for (int k = 0; k < s.nmsg; k++) {
    if (!receivable(s, k, AEREQ, false)) continue;
    const Msg& m = s.msgs[k];
    int i = m.dst, j = m.src;
    if (!(m.term < s.term[i] || (m.term == s.term[i] && s.st[i] == FOLLOWER && !LogOk(s, i, m)))) continue;
    Msg r = mk(AERESP, s.term[i], i, j);
    r.success = 0;
    r.matchIndex = 0;
    State t = s;
    if (!reply(t, r, k)) continue;
    E.emit(t, A_REJECTAE);
  }
}

void AcceptAppendEntriesRequest(const State& s, Emitter& E) {
  // Raft.tla:454-485; FlexibleRaft.tla:421-450; RaftFsync.tla:449-481
  for (int k = 0; k < s.nmsg; k++) {
    if (!receivable(s, k, AEREQ, true)) continue;
    const Msg& m = s.msgs[k];
    int i = m.dst, j = m.src;
    int index = m.prevLogIndex + 1;
    if (!(s.st[i] == FOLLOWER || s.st[i] == CANDIDATE)) continue;
    if (!LogOk(s, i, m)) continue;
    int L = Len(s, i);
    bool canAppend = m.nent != 0 && L == m.prevLogIndex;  // Raft.tla:438-440
    State t = s;
    if (C.spec == RAFT) {
      // NeedsTruncation, Raft.tla:445-449; CASE arms :464-470
      bool needs = (m.nent != 0 && L >= index) || (m.nent == 0 && L > m.prevLogIndex);
      if (canAppend) append(t, i, Entry{m.eterm, m.evalue});
      else if (needs && m.nent != 0) { t.loglen[i] = m.prevLogIndex; append(t, i, Entry{m.eterm, m.evalue}); }
      else if (needs && m.nent == 0) t.loglen[i] = m.prevLogIndex;
    } else {
      // NeedsTruncation, FlexibleRaft.tla:413-416: also needs a term mismatch
      bool needs = m.nent != 0 && L >= index && log_at(s, i, index).term != m.eterm;
      if (canAppend) append(t, i, Entry{m.eterm, m.evalue});
      else if (needs) { t.loglen[i] = m.prevLogIndex; append(t, i, Entry{m.eterm, m.evalue}); }
    }
    // TruncateLog reads log[i][1..prevLogIndex]; LogOk guarantees prevLogIndex <= Len
    t.st[i] = FOLLOWER;
    t.commit[i] = m.commit;
    if (C.spec == FSYNC && C.ffbr) t.fsync[i] = t.loglen[i];  // RaftFsync.tla:468-470
    Msg r = mk(AERESP, s.term[i], i, j);
    r.success = 1;
    r.matchIndex = (int8_t)(m.prevLogIndex + m.nent);
    if (!reply(t, r, k)) continue;
    E.emit(t, A_ACCEPTAE);
  }
}

void HandleAppendEntriesResponse(const State& s, Emitter& E) {  // Raft.tla:490-505
  for (int k = 0; k < s.nmsg; k++) {
    if (!receivable(s, k, AERESP, true)) continue;
    const Msg& m = s.msgs[k];
    int i = m.dst, j = m.src;
    State t = s;
    if (m.success) {
      t.next[i][j] = (int8_t)(m.matchIndex + 1);
      t.match[i][j] = m.matchIndex;
    } else {
      t.next[i][j] = (int8_t)std::max(s.next[i][j] - 1, 1);
    }
    if (C.spec == RAFT) t.pending[i] &= (uint8_t)~(1u << j);
    t.msgs[k].count--;
    E.emit(t, A_HAERESP);
  }
}

// ---- PullRaft only
bool ValidPullPosition(const State& s, int i, const Msg& m) {  // PullRaft.tla:192-196
  if (m.lastLogIndex == 0) return true;
  return m.lastLogIndex > 0 && m.lastLogIndex <= Len(s, i) &&
         m.lastLogTerm == log_at(s, i, m.lastLogIndex).term;
}
int CompareEntries(int i1, int t1, int i2, int t2) {  // PullRaft.tla:203-207
  if (t1 > t2) return 1;
  if (t1 == t2 && i1 > i2) return 1;
  if (t1 == t2 && i1 == i2) return 0;
  return -1;
}
void LastCommonEntry(const State& s, int i, int lastIndex, int lastTerm, int& idx, int& term) {
  // PullRaft.tla:211-226
  idx = 0; term = 0;
  for (int x = 1; x <= Len(s, i); x++)
    if (CompareEntries(x, log_at(s, i, x).term, lastIndex, lastTerm) <= 0) idx = x;
  if (idx) term = log_at(s, i, idx).term;
}

void LearnOfLeader(const State& s, Emitter& E) {  // PullRaft.tla:383-391
  for (int k = 0; k < s.nmsg; k++) {
    if (!receivable(s, k, LNREQ, true)) continue;
    State t = s;
    const Msg& m = s.msgs[k];
    // PullRaftVariant2.tla:404-406: NeedsTruncation / TruncateLog (:171-179)
    if (C.spec == PULL2 && !m.lceNil && Len(s, m.dst) >= m.lciIndex) t.loglen[m.dst] = m.lciIndex;
    t.voted[s.msgs[k].dst] = s.msgs[k].src;
    t.msgs[k].count--;
    E.emit(t, A_LEARNOFLEADER);
  }
}

void SendPullEntriesRequest(const State& s, int i, int j, Emitter& E) {  // PullRaft.tla:396-411
  if (i == j || s.st[i] != FOLLOWER || s.voted[i] != j) return;
  int lli = Len(s, i);
  int llt = lli > 0 ? log_at(s, i, lli).term : 0;
  Msg m = mk(PEREQ, s.term[i], i, j);
  m.lastLogIndex = (int8_t)lli;
  m.lastLogTerm = (int8_t)llt;
  State t = s;
  if (!send_once(t, m)) return;
  E.emit(t, A_SENDPULL);
}

void RejectPullEntriesRequest(const State& s, Emitter& E) {  // PullRaft.tla:418-436
  for (int k = 0; k < s.nmsg; k++) {
    if (!receivable(s, k, PEREQ, true)) continue;
    const Msg& m = s.msgs[k];
    int i = m.dst, j = m.src;
    if (s.st[i] != LEADER) continue;
    if (ValidPullPosition(s, i, m)) continue;
    Msg r = mk(PERESP, s.term[i], i, j);
    r.success = 0;
    int a, b;
    LastCommonEntry(s, i, m.lastLogIndex, m.lastLogTerm, a, b);
    r.lciIndex = (int8_t)a;
    r.lciTerm = (int8_t)b;
    State t = s;
    if (!reply(t, r, k)) continue;
    E.emit(t, A_REJECTPULL);
  }
}

void AcceptPullEntriesRequest(const State& s, Emitter& E) {  // PullRaft.tla:460-488
  for (int k = 0; k < s.nmsg; k++) {
    if (!receivable(s, k, PEREQ, true)) continue;
    const Msg& m = s.msgs[k];
    int i = m.dst, j = m.src;
    int index = m.lastLogIndex + 1;
    if (s.st[i] != LEADER) continue;
    if (!ValidPullPosition(s, i, m)) continue;
    if (!(index <= Len(s, i))) continue;
    int8_t nm[MAXN];
    memcpy(nm, s.match[i], MAXN);
    nm[j] = m.lastLogIndex;
    int nc = new_commit_index(s, i, nm);  // NewCommitIndex, PullRaft.tla:446-458
    State t = s;
    memcpy(t.match[i], nm, MAXN);
    t.commit[i] = (int8_t)nc;
    update_acked(s, t, i, nc);
    Msg r = mk(PERESP, s.term[i], i, j);
    r.success = 1;
    r.nent = 1;
    const Entry& e = log_at(s, i, index);
    r.eterm = e.term;
    r.evalue = e.value;
    r.commit = (int8_t)std::min(nc, index);
    if (!reply(t, r, k)) continue;
    E.emit(t, A_ACCEPTPULL);
  }
}

void HandleSuccessPullEntriesResponse(const State& s, Emitter& E) {  // PullRaft.tla:493-503
  for (int k = 0; k < s.nmsg; k++) {
    if (!receivable(s, k, PERESP, true)) continue;
    const Msg& m = s.msgs[k];
    if (!m.success) continue;
    int i = m.dst;
    State t = s;
    t.commit[i] = m.commit;
    append(t, i, Entry{m.eterm, m.evalue});
    t.msgs[k].count--;
    E.emit(t, A_HSUCCESSPULL);
  }
}

void HandleFailPullEntriesResponse(const State& s, Emitter& E) {  // PullRaft.tla:510-520
  for (int k = 0; k < s.nmsg; k++) {
    if (!receivable(s, k, PERESP, true)) continue;
    const Msg& m = s.msgs[k];
    if (m.success) continue;
    int i = m.dst;
    State t = s;
    if (m.lciIndex > 0) {  // TruncateLog, PullRaft.tla:185-188
      for (int x = 1; x <= m.lciIndex; x++) log_at(s, i, x);  // domain check
      t.loglen[i] = m.lciIndex;
    } else {
      t.loglen[i] = 0;
    }
    t.msgs[k].count--;
    E.emit(t, A_HFAILPULL);
  }
}

// Next, split into TLC actions in TLC order.  Pairs enumerate with the first
// bound variable fastest: (n1,n1),(n2,n1),(n3,n1),(n1,n2),...
void Next(const State& s, Emitter& E) {
  const int N = C.N;
  auto pairs = [&](auto f) { for (int j = 0; j < N; j++) for (int i = 0; i < N; i++) f(i, j); };
  auto clients = [&]() { for (int v = 0; v < C.V; v++) for (int i = 0; i < N; i++) ClientRequest(s, i, v, E); };
  switch (C.spec) {
    case RAFT: case FLEX:  // Raft.tla:527-539, FlexibleRaft.tla:488-500
      for (int i = 0; i < N; i++) Restart(s, i, E);
      for (int i = 0; i < N; i++) RequestVote(s, i, E);
      for (int i = 0; i < N; i++) BecomeLeader(s, i, E);
      clients();
      for (int i = 0; i < N; i++) AdvanceCommitIndex(s, i, E);
      pairs([&](int i, int j) { AppendEntries(s, i, j, E); });
      UpdateTerm(s, E);
      HandleRequestVoteRequest(s, E);
      HandleRequestVoteResponse(s, E);
      RejectAppendEntriesRequest(s, E);
      AcceptAppendEntriesRequest(s, E);
      HandleAppendEntriesResponse(s, E);
      break;
    case FSYNC:  // RaftFsync.tla:522-536
      for (int i = 0; i < N; i++) Restart(s, i, E);
      for (int i = 0; i < N; i++) Timeout(s, i, E);
      pairs([&](int i, int j) { RequestVoteIJ(s, i, j, E); });
      for (int i = 0; i < N; i++) BecomeLeader(s, i, E);
      clients();
      for (int i = 0; i < N; i++) AdvanceCommitIndex(s, i, E);
      pairs([&](int i, int j) { AppendEntries(s, i, j, E); });
      for (int i = 0; i < N; i++) AdvanceFsyncIndex(s, i, E);
      UpdateTerm(s, E);
      HandleRequestVoteRequest(s, E);
      HandleRequestVoteResponse(s, E);
      RejectAppendEntriesRequest(s, E);
      AcceptAppendEntriesRequest(s, E);
      HandleAppendEntriesResponse(s, E);
      break;
    case PULL: case PULL2:  // PullRaft.tla:542-558; PullRaftVariant2.tla:560-576 (same disjuncts)
      for (int i = 0; i < N; i++) Restart(s, i, E);
      UpdateTerm(s, E);
      for (int i = 0; i < N; i++) RequestVote(s, i, E);
      HandleRequestVoteRequest(s, E);
      HandleRequestVoteResponse(s, E);
      for (int i = 0; i < N; i++) BecomeLeader(s, i, E);
      clients();
      RejectPullEntriesRequest(s, E);
      AcceptPullEntriesRequest(s, E);
      LearnOfLeader(s, E);
      pairs([&](int i, int j) { SendPullEntriesRequest(s, i, j, E); });
      HandleSuccessPullEntriesResponse(s, E);
      HandleFailPullEntriesResponse(s, E);
      break;
  }
}

State Init() {  // Raft.tla:197-218 (and the variants' Init)
  State s;
  memset(&s, 0, sizeof s);
  for (int v = 0; v < C.V; v++) s.acked[v] = NIL;
  for (int i = 0; i < C.N; i++) {
    s.term[i] = 1;
    s.st[i] = FOLLOWER;
    s.voted[i] = NIL;
    s.voted2[i] = NIL;
    for (int j = 0; j < C.N; j++) { s.next[i][j] = 1; s.match[i][j] = 0; s.vleI[i][j] = -1; }
  }
  return s;
}

// -------------------------------------------------------------- invariants
bool entry_eq(const Entry& a, const Entry& b) { return a.term == b.term && a.value == b.value; }
bool NoLogDivergence(const State& s) {  // Raft.tla:588-596
  for (int s2 = 0; s2 < C.N; s2++)
    for (int s1 = 0; s1 < C.N; s1++) {
      if (s1 == s2) continue;
      int c = std::min(s.commit[s1], s.commit[s2]);
      for (int idx = 1; idx <= c; idx++)
        if (!entry_eq(log_at(s, s1, idx), log_at(s, s2, idx))) return false;
    }
  return true;
}
bool LeaderHasAllAckedValues(const State& s) {  // Raft.tla:604-620
  for (int v = 0; v < C.V; v++) {
    if (s.acked[v] != 1) continue;
    for (int i = 0; i < C.N; i++) {
      if (s.st[i] != LEADER) continue;
      bool newer = false;
      for (int l = 0; l < C.N; l++)
        if (l != i && s.term[l] > s.term[i]) newer = true;
      if (newer) continue;
      bool has = false;
      for (int x = 0; x < s.loglen[i]; x++)
        if (s.log[i][x].value == v) has = true;
      if (!has) return false;
    }
  }
  return true;
}
bool CommittedEntriesReachMajority(const State& s) {  // Raft.tla:625-636
  bool any = false;
  for (int i = 0; i < C.N; i++) if (s.st[i] == LEADER && s.commit[i] > 0) any = true;
  if (!any) return true;
  int size = C.N / 2 + 1;
  for (int i = 0; i < C.N; i++) {
    if (!(s.st[i] == LEADER && s.commit[i] > 0)) continue;
    int ci = s.commit[i];
    for (unsigned q = 0; q < (1u << C.N); q++) {
      if (popc(q) != size || !(q >> i & 1)) continue;
      bool ok = true;
      for (int j = 0; j < C.N && ok; j++) {
        if (!(q >> j & 1)) continue;
        if (!(s.loglen[j] >= ci)) { ok = false; break; }
        if (!entry_eq(log_at(s, j, ci), log_at(s, i, ci))) ok = false;
      }
      if (ok) return true;
    }
  }
  return false;
}
// The classic Raft properties, opt-in (not defined by the reference's specs);
// restated from their TLA+ text in INTEGRATION.md.
bool ElectionSafety(const State& s) {
  for (int a = 0; a < C.N; a++)
    for (int b = 0; b < C.N; b++)
      if (a != b && s.st[a] == LEADER && s.st[b] == LEADER && s.term[a] == s.term[b]) return false;
  return true;
}
bool LogMatching(const State& s) {
  for (int a = 0; a < C.N; a++)
    for (int b = 0; b < C.N; b++)
      for (int i = 1; i <= std::min(s.loglen[a], s.loglen[b]); i++)
        if (log_at(s, a, i).term == log_at(s, b, i).term)
          for (int k = 1; k <= i; k++)
            if (!entry_eq(log_at(s, a, k), log_at(s, b, k))) return false;
  return true;
}
bool LeaderCompleteness(const State& s) {
  for (int l = 0; l < C.N; l++) {
    if (s.st[l] != LEADER) continue;
    bool newest = true;
    for (int k = 0; k < C.N; k++) if (s.term[k] > s.term[l]) newest = false;
    if (!newest) continue;
    for (int k = 0; k < C.N; k++)
      for (int i = 1; i <= std::min(s.commit[k], s.loglen[k]); i++)
        if (!(i <= s.loglen[l] && entry_eq(log_at(s, l, i), log_at(s, k, i)))) return false;
  }
  return true;
}
bool StateMachineSafety(const State& s) {
  for (int a = 0; a < C.N; a++)
    for (int b = 0; b < C.N; b++) {
      const int c = std::min(std::min(s.commit[a], s.commit[b]), std::min(s.loglen[a], s.loglen[b]));
      for (int i = 1; i <= c; i++)
        if (!entry_eq(log_at(s, a, i), log_at(s, b, i))) return false;
    }
  return true;
}
const char* check_invariants(const State& s) {
  for (auto& n : C.inv_order) {
    if (n == "ElectionSafety" && !ElectionSafety(s)) return "ElectionSafety";
    if (n == "LogMatching" && !LogMatching(s)) return "LogMatching";
    if (n == "LeaderCompleteness" && !LeaderCompleteness(s)) return "LeaderCompleteness";
    if (n == "StateMachineSafety" && !StateMachineSafety(s)) return "StateMachineSafety";
    if (n == "LeaderHasAllAckedValues" && !LeaderHasAllAckedValues(s)) return "LeaderHasAllAckedValues";
    if (n == "NoLogDivergence" && !NoLogDivergence(s)) return "NoLogDivergence";
    if (n == "CommittedEntriesReachMajority" && !CommittedEntriesReachMajority(s)) return "CommittedEntriesReachMajority";
  }
  return nullptr;
}

// ------------------------------------------------------- exact canonical form
// serialisation(pi) = [inv(server at pos 0..N-1)] ++ [relabelled server-valued
// fields at pos 0..N-1] ++ sorted(relabelled messages) (++ acked for Pull).
// inv() is permutation-invariant, so a minimal serialisation must sort the
// servers by inv(); only those permutations are tried.
struct Ser {
  uint8_t b[4096];
  int n = 0;
  void put(int v) { b[n++] = (uint8_t)v; }
};
void server_inv(const State& s, int i, Ser& o) {
  o.put(s.term[i]); o.put(s.st[i]); o.put(s.loglen[i]);
  for (int x = 0; x < s.loglen[i]; x++) { o.put(s.log[i][x].term); o.put(s.log[i][x].value); }
  o.put(s.commit[i]);
  if (C.spec == FSYNC) o.put(s.fsync[i]);
}
void canonical(const State& s, Ser& best) {
  const int N = C.N;
  // group servers by invariant bytes
  Ser inv[MAXN];
  for (int i = 0; i < N; i++) server_inv(s, i, inv[i]);
  int order[MAXN];
  for (int i = 0; i < N; i++) order[i] = i;
  auto less = [&](int a, int b) {
    int n = std::min(inv[a].n, inv[b].n);
    int c = memcmp(inv[a].b, inv[b].b, n);
    return c ? c < 0 : inv[a].n < inv[b].n;
  };
  auto same = [&](int a, int b) { return inv[a].n == inv[b].n && memcmp(inv[a].b, inv[b].b, inv[a].n) == 0; };
  std::stable_sort(order, order + N, less);
  // enumerate permutations within tie classes: iterate all permutations of
  // `order` that keep the inv-sorted property.
  int cur[MAXN];
  memcpy(cur, order, sizeof(int) * N);
  // class boundaries
  int cls[MAXN];
  for (int k = 0, c = 0; k < N; k++) { if (k > 0 && !same(order[k - 1], order[k])) c++; cls[k] = c; }
  bool have = false;
  uint32_t msgbuf[MAXMSG];
  while (true) {
    // cur[pos] = original server placed at position pos; p = inverse map
    int p[MAXN];
    for (int pos = 0; pos < N; pos++) p[cur[pos]] = pos;
    Ser o;
    for (int pos = 0; pos < N; pos++) { const Ser& v = inv[cur[pos]]; memcpy(o.b + o.n, v.b, v.n); o.n += v.n; }
    for (int pos = 0; pos < N; pos++) {
      int i = cur[pos];
      o.put(s.voted[i] == NIL ? 255 : p[s.voted[i]]);
      if (C.spec == PULL2) o.put(s.voted2[i] == NIL ? 255 : p[s.voted2[i]]);
      unsigned vg = 0, pd = 0;
      for (int j = 0; j < N; j++) {
        if (s.votes[i] >> j & 1) vg |= 1u << p[j];
        if (s.pending[i] >> j & 1) pd |= 1u << p[j];
      }
      o.put(vg);
      if (C.spec == RAFT) o.put(pd);
      for (int q = 0; q < N; q++) {
        int j = cur[q];
        if (!C.pull()) o.put(s.next[i][j]);
        o.put(s.match[i][j]);
        if (C.spec == PULL2) { o.put(s.vleI[i][j] + 1); o.put(s.vleT[i][j]); }
      }
    }
    if (C.spec == PULL) for (int v = 0; v < C.V; v++) o.put(s.acked[v] + 1);
    // messages: relabel, pack into sortable u64-ish byte strings
    int nm = s.nmsg;
    struct MB { uint8_t b[REC_BYTES + 1]; };
    static thread_local MB mb[MAXMSG];
    static thread_local int idx[MAXMSG];
    for (int k = 0; k < nm; k++) {
      Msg m = s.msgs[k];
      m.src = (int8_t)p[m.src];
      m.dst = (int8_t)p[m.dst];
      memcpy(mb[k].b, &m, REC_BYTES + 1);
      idx[k] = k;
    }
    std::sort(idx, idx + nm, [&](int a, int b) { return memcmp(mb[a].b, mb[b].b, REC_BYTES + 1) < 0; });
    o.put(nm);
    for (int k = 0; k < nm; k++) { memcpy(o.b + o.n, mb[idx[k]].b, REC_BYTES + 1); o.n += REC_BYTES + 1; }
    (void)msgbuf;
    if (!have || (o.n != best.n ? o.n < best.n : memcmp(o.b, best.b, o.n) < 0)) {
      best = o;
      have = true;
    }
    // next permutation within classes (lexicographic over positions)
    bool advanced = false;
    for (int start = N - 1; start >= 0 && !advanced; ) {
      int c = cls[start];
      int lo = start;
      while (lo > 0 && cls[lo - 1] == c) lo--;
      if (std::next_permutation(cur + lo, cur + start + 1)) advanced = true;
      else start = lo - 1;  // this class wrapped around (next_permutation reset it); carry
    }
    if (!advanced) break;
  }
}

struct Key128 { uint64_t a, b; };
inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
Key128 hash_ser(const Ser& o) {
  uint64_t h1 = 0x9E3779B97F4A7C15ULL ^ (uint64_t)o.n, h2 = 0xC2B2AE3D27D4EB4FULL + (uint64_t)o.n * 31;
  int k = 0;
  for (; k + 8 <= o.n; k += 8) {
    uint64_t w;
    memcpy(&w, o.b + k, 8);
    h1 = mix64(h1 ^ w) + 0x632BE59BD9B4E019ULL;
    h2 = mix64(h2 + w * 0xFF51AFD7ED558CCDULL) ^ (h2 >> 17);
  }
  uint64_t w = 0;
  memcpy(&w, o.b + k, o.n - k);
  h1 = mix64(h1 ^ w ^ 0xA5);
  h2 = mix64(h2 + w + 0x5A);
  return {h1, h2 | 1};  // b != 0 marks an occupied slot
}

// Fingerprint set: T shards (one per thread, chosen by the key's high bits),
// open addressing with linear probing over a table of any size (home slot =
// mulhi(a, size)).  A slot holds 96 bits of the 128-bit canonical-form hash
// (a + the high half of b; collision odds for 2e9 states ~ n^2 / 2^97 ~ 3e-11)
// plus the level that inserted it and the hidden (VIEW-dropped) variables: 16 B,
// so the 1.9e9-state rungs fit this container's memory.  level 0 = empty.
struct Slot { uint64_t a; uint32_t b; uint16_t level; uint16_t hidden; };
struct FPShard {
  std::vector<Slot> t;
  uint64_t count = 0;
  double max_load = 0.5;
  void init(uint64_t slots, double ml) {
    max_load = ml;
    t.assign(std::max<uint64_t>(slots, 1024), Slot{0, 0, 0, 0});
  }
  // the shard is chosen by a's high bits, so the home slot must not be: mix first
  inline uint64_t home(uint64_t a, uint64_t n) const {
    return (uint64_t)(((unsigned __int128)(a * 0x9E3779B97F4A7C15ULL) * n) >> 64);
  }
  void grow() {
    std::vector<Slot> old;
    old.swap(t);
    const uint64_t n = old.size() * 2;
    t.assign(n, Slot{0, 0, 0, 0});
    for (auto& s : old)
      if (s.level) {
        uint64_t h = home(s.a, n);
        while (t[h].level) h = (h + 1 == n) ? 0 : h + 1;
        t[h] = s;
      }
  }
  // returns nullptr if inserted, else the existing slot
  Slot* insert(Key128 k, uint16_t level, uint16_t hidden) {
    if ((double)(count + 1) > max_load * (double)t.size()) grow();
    const uint64_t n = t.size();
    const uint32_t b = (uint32_t)(k.b >> 32);
    uint64_t h = home(k.a, n);
    while (t[h].level) {
      if (t[h].a == k.a && t[h].b == b) return &t[h];
      h = (h + 1 == n) ? 0 : h + 1;
    }
    t[h] = Slot{k.a, b, level, hidden};
    count++;
    return nullptr;
  }
};

// electionCtr | restartCtr | acked[v]: the variables VIEW drops (Raft.tla:115-116;
// PullRaft keeps acked in its view).  16 bits: E, R <= 15 and V <= 4 are checked.
uint16_t hidden_of(const State& s) {
  uint32_t h = (uint32_t)s.electionCtr | ((uint32_t)s.restartCtr << 4);
  if (C.spec != PULL)
    for (int v = 0; v < C.V; v++) h |= (uint32_t)(s.acked[v] + 1) << (8 + 2 * v);
  return (uint16_t)h;
}

// ------------------------------------------------------- compact frontier rows
// A state is stored as its used fields only (N servers, V values, Len(log)
// entries, |DOMAIN messages| records), each field one nibble when it lies in
// [-1, 13] (value + 1), else an escape nibble 15 and the raw byte in two
// nibbles; rows are prefixed with their u16 byte length.  Unused State bytes
// decode to 0, as Init() leaves them; stale log entries past Len(log) are
// dropped (nothing reads them: log_at bounds-checks).
struct NibW {
  uint8_t* p; size_t n = 0;  // n = nibbles written
  inline void nib(unsigned v) { if (n & 1) p[n >> 1] |= (uint8_t)(v << 4); else p[n >> 1] = (uint8_t)v; n++; }
  inline void put(int v) {
    if (v >= -1 && v <= 13) nib((unsigned)(v + 1));
    else { nib(15); nib((uint8_t)v & 15); nib((uint8_t)v >> 4); }
  }
};
struct NibR {
  const uint8_t* p; size_t n = 0;
  inline unsigned nib() { unsigned v = (p[n >> 1] >> ((n & 1) * 4)) & 15; n++; return v; }
  inline int get() {
    unsigned v = nib();
    if (v != 15) return (int)v - 1;
    unsigned lo = nib(), hi = nib();
    return (int)(int8_t)(uint8_t)(lo | hi << 4);
  }
};
constexpr size_t ROW_MAX = 2 + 3 * (FIXED_BYTES + MAXMSG * sizeof(Msg)) / 2 + 8;
size_t encode_state(const State& s, uint8_t* out) {  // out: u16 length + nibbles
  NibW w{out + 2};
  const int N = C.N;
  w.put(s.nmsg & 255); w.put(s.nmsg >> 8); w.put(s.electionCtr); w.put(s.restartCtr);
  for (int v = 0; v < C.V; v++) w.put(s.acked[v]);
  for (int i = 0; i < N; i++) {
    w.put(s.term[i]); w.put(s.st[i]); w.put(s.voted[i]); w.put(s.voted2[i]); w.put(s.loglen[i]);
    w.put(s.commit[i]); w.put(s.fsync[i]); w.put((int8_t)s.votes[i]); w.put((int8_t)s.pending[i]);
    for (int x = 0; x < s.loglen[i]; x++) { w.put(s.log[i][x].term); w.put(s.log[i][x].value); }
    for (int j = 0; j < N; j++) { w.put(s.next[i][j]); w.put(s.match[i][j]); }
    if (C.spec == PULL2) for (int j = 0; j < N; j++) { w.put(s.vleI[i][j]); w.put(s.vleT[i][j]); }
  }
  for (int k = 0; k < s.nmsg; k++) {
    const int8_t* b = (const int8_t*)&s.msgs[k];
    for (size_t f = 0; f < REC_BYTES; f++) w.put(b[f]);
    w.put((int8_t)s.msgs[k].count);
  }
  const size_t bytes = (w.n + 1) / 2;
  const uint16_t len = (uint16_t)bytes;
  memcpy(out, &len, 2);
  return 2 + bytes;
}
void decode_state(const uint8_t* row, State& s) {
  memset(&s, 0, FIXED_BYTES);
  NibR r{row + 2};
  const int N = C.N;
  int lo = r.get() & 255;
  s.nmsg = (int16_t)(lo | (r.get() << 8));
  s.electionCtr = (int8_t)r.get(); s.restartCtr = (int8_t)r.get();
  for (int v = 0; v < C.V; v++) s.acked[v] = (int8_t)r.get();
  for (int i = 0; i < N; i++) {
    s.term[i] = (int8_t)r.get(); s.st[i] = (int8_t)r.get(); s.voted[i] = (int8_t)r.get(); s.voted2[i] = (int8_t)r.get();
    s.loglen[i] = (int8_t)r.get(); s.commit[i] = (int8_t)r.get(); s.fsync[i] = (int8_t)r.get();
    s.votes[i] = (uint8_t)r.get(); s.pending[i] = (uint8_t)r.get();
    for (int x = 0; x < s.loglen[i]; x++) { s.log[i][x].term = (int8_t)r.get(); s.log[i][x].value = (int8_t)r.get(); }
    for (int j = 0; j < N; j++) { s.next[i][j] = (int8_t)r.get(); s.match[i][j] = (int8_t)r.get(); }
    if (C.spec == PULL2) for (int j = 0; j < N; j++) { s.vleI[i][j] = (int8_t)r.get(); s.vleT[i][j] = (int8_t)r.get(); }
    for (int j = N; j < MAXN; j++) s.vleI[i][j] = -1;  // Init's value for unused peers
  }
  for (int k = 0; k < s.nmsg; k++) {
    int8_t* b = (int8_t*)&s.msgs[k];
    for (size_t f = 0; f < REC_BYTES; f++) b[f] = (int8_t)r.get();
    s.msgs[k].count = (uint8_t)r.get();
  }
}
inline size_t row_len(const uint8_t* row) { uint16_t n; memcpy(&n, row, 2); return 2 + (size_t)n; }

// A BFS level: rows appended in TLC order, either in memory or spilled to a
// file (--spill-dir) and read back through a read-only mapping.
struct Level {
  std::vector<uint8_t> mem;
  std::string path;
  FILE* wf = nullptr;
  const uint8_t* map = nullptr;
  size_t bytes = 0, count = 0;
  std::vector<uint8_t> wbuf;
  void open(const std::string& p) { path = p; }
  void clear() {
    if (map) { munmap((void*)map, bytes); map = nullptr; }
    if (wf) { fclose(wf); wf = nullptr; }
    mem.clear();
    mem.shrink_to_fit();
    bytes = count = 0;
    if (!path.empty()) {
      wf = fopen(path.c_str(), "wb");
      if (!wf) { perror(path.c_str()); exit(3); }
      wbuf.resize(64 << 20);
      setvbuf(wf, (char*)wbuf.data(), _IOFBF, wbuf.size());
    }
  }
  void push(const uint8_t* row, size_t n) {
    if (wf) { if (fwrite(row, 1, n, wf) != n) { perror("spill write"); exit(3); } }
    else mem.insert(mem.end(), row, row + n);
    bytes += n;
    count++;
  }
  void finish() {  // writing done: map for reading
    if (!wf) return;
    if (fflush(wf) != 0) { perror("spill flush"); exit(3); }
    fclose(wf);
    wf = nullptr;
    if (bytes == 0) return;
    int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) { perror(path.c_str()); exit(3); }
    void* m = mmap(nullptr, bytes, PROT_READ, MAP_SHARED, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) { perror("spill mmap"); exit(3); }
    madvise(m, bytes, MADV_SEQUENTIAL);
    map = (const uint8_t*)m;
  }
  const uint8_t* data() const { return map ? map : mem.data(); }
  size_t size() const { return count; }
  ~Level() { if (map) munmap((void*)map, bytes); if (wf) fclose(wf); if (!path.empty()) unlink(path.c_str()); }
};

// ---------------------------------------------------------------- BFS driver
struct Stats {
  uint64_t generated = 0, distinct = 0, left = 0;
  int depth = 0;
  std::string status = "ok", violated, error;
  uint64_t hidden_same = 0, hidden_cross = 0;
  uint64_t act[A_COUNT] = {0};
  int max_msgs = 0;
  std::vector<std::pair<uint64_t, uint64_t>> levels;
  double seconds = 0;
};

std::string state_json(const State& s);

struct Checker {
  Stats st;
  std::vector<FPShard> fps;
  // trace records (parent global index, ordinal within parent's successors)
  std::vector<uint64_t> parent;
  std::vector<uint16_t> ordinal;
  std::vector<uint8_t> actid;
  bool trace = true;
  uint64_t max_distinct = 0;
  uint64_t fp_slots = 0;  // preallocated total slots (0 = start small, grow at 0.5 load)
  double max_seconds = 0;
  int threads = 1;
  bool reverse_order = false;
  bool progress = false;
  std::string spill_dir;
  FILE* fpdump = nullptr;
  int64_t bad_index = -1;

  void run();
};

// a successor candidate of one chunk (expanded by the worker that owns its parent)
enum CandRes : uint8_t { R_NEW = 0, R_DUP = 1, R_DUP_HID_SAME = 2, R_DUP_HID_CROSS = 3 };
struct Cand {
  Key128 key;
  uint32_t parent_local;
  uint32_t row_off;      // into the worker's keep buffer
  uint16_t ordinal;
  uint16_t hidden;
  uint8_t act;
  uint8_t res;           // CandRes, set by the insert pass
  int16_t inv;           // -1 ok, k = index into inv_names, -2 evaluation error (see inv_err)
};

struct Worker {
  std::vector<Cand> cands;
  std::vector<uint8_t> keep;
  std::vector<std::pair<size_t, std::string>> inv_err;  // candidate index -> evaluation error
  std::string err;
  size_t err_parent = 0;
  int maxmsg = 0;
};

std::vector<std::string> inv_names;  // check_invariants' results, interned
int16_t intern_inv(const char* n) {
  for (size_t k = 0; k < inv_names.size(); k++) if (inv_names[k] == n) return (int16_t)k;
  inv_names.push_back(n);
  return (int16_t)(inv_names.size() - 1);
}

struct CandEmit : Emitter {
  Worker* w;
  uint32_t parent_local;
  uint16_t q = 0;
  uint8_t row[ROW_MAX];
  void emit(const State& t, int a) override {
    Ser o;
    canonical(t, o);
    Cand c;
    c.key = hash_ser(o);
    c.hidden = hidden_of(t);
    c.parent_local = parent_local;
    c.ordinal = q++;
    c.act = (uint8_t)a;
    c.res = R_NEW;
    c.inv = -1;
    try {
      if (const char* bad = check_invariants(t)) c.inv = intern_inv(bad);
    } catch (EvalError& e) {
      c.inv = -2;
      w->inv_err.push_back({w->cands.size(), std::string("invariant: ") + e.what()});
    }
    size_t n = encode_state(t, row);
    c.row_off = (uint32_t)w->keep.size();
    w->keep.insert(w->keep.end(), row, row + n);
    w->cands.push_back(c);
  }
};

void expand_range(const uint8_t* const* rows, size_t lo, size_t hi, Worker& W) {
  CandEmit em;
  em.w = &W;
  State s;
  for (size_t k = lo; k < hi; k++) {
    decode_state(rows[k], s);
    W.maxmsg = std::max(W.maxmsg, (int)s.nmsg);
    em.parent_local = (uint32_t)k;
    em.q = 0;
    const size_t before = W.cands.size(), kb = W.keep.size(), eb = W.inv_err.size();
    try {
      Next(s, em);
    } catch (EvalError& e) {
      // the parent's successors are not generated: TLC stops at the error
      W.cands.resize(before);
      W.keep.resize(kb);
      W.inv_err.resize(eb);
      W.err = e.what();
      W.err_parent = k;
      return;
    }
  }
}

template <class F> void parallel(int T, F f) {
  if (T == 1) { f(0); return; }
  std::vector<std::thread> th;
  for (int w = 0; w < T; w++) th.emplace_back([&, w]() { f(w); });
  for (auto& x : th) x.join();
}

void Checker::run() {
  auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
  const int T = std::max(1, threads);
  fps.resize(T);
  for (auto& f : fps) f.init(fp_slots ? (fp_slots + T - 1) / T : (1u << 20), fp_slots ? 0.92 : 0.5);
  auto shard_of = [T](const Key128& k) { return (int)(((k.a >> 32) * (uint64_t)T) >> 32); };
  Level lv[2];
  if (!spill_dir.empty()) {
    lv[0].open(spill_dir + "/level_a.bin");
    lv[1].open(spill_dir + "/level_b.bin");
  }
  Level* cur = &lv[0];
  Level* nxt = &lv[1];
  cur->clear();
  State init = Init();
  st.generated = 1;
  st.distinct = 1;
  {
    Ser o;
    canonical(init, o);
    Key128 k = hash_ser(o);
    fps[shard_of(k)].insert(k, 1, hidden_of(init));
    if (fpdump) fwrite(&k, sizeof k, 1, fpdump);
  }
  if (trace) { parent.push_back(UINT64_MAX); ordinal.push_back(0); actid.push_back(255); }
  {
    uint8_t row[ROW_MAX];
    size_t n = encode_state(init, row);
    cur->push(row, n);
    cur->finish();
  }
  st.levels.push_back({1, 1});
  st.depth = 1;
  try {
    if (const char* bad = check_invariants(init)) { st.status = "violation"; st.violated = bad; bad_index = 0; }
  } catch (EvalError& e) { st.status = "error"; st.error = e.what(); bad_index = 0; }
  uint64_t base = 0;  // global index of cur[0]
  uint32_t level = 1;
  const size_t CHUNK = 8192 * (size_t)T;
  std::vector<Worker> W(T);
  std::vector<const uint8_t*> rows(CHUNK);
  double t_exp = 0, t_ins = 0, t_seq = 0;
  while (st.status == "ok" && cur->size() > 0) {
    const size_t F = cur->size();
    nxt->clear();
    uint64_t gen_lvl = 0;
    bool stop = false;
    const uint8_t* rp = cur->data();
    for (size_t c0 = 0; c0 < F && !stop; c0 += CHUNK) {
      const size_t c1 = std::min(F, c0 + CHUNK);
      for (size_t k = c0; k < c1; k++) { rows[k - c0] = rp; rp += row_len(rp); }
      // 1. expand (parallel over parents): successors, canonical keys, invariants
      auto ta = std::chrono::steady_clock::now();
      parallel(T, [&](int w) {
        const size_t n = c1 - c0, lo = n * w / T, hi = n * (w + 1) / T;
        Worker& X = W[w];
        X.cands.clear(); X.keep.clear(); X.inv_err.clear(); X.err.clear();
        expand_range(rows.data(), lo, hi, X);
        for (auto& c : X.cands) c.parent_local += (uint32_t)c0;
        if (!X.err.empty()) X.err_parent += c0;
      });
      auto tb = std::chrono::steady_clock::now();
      // 2. insert (parallel over fingerprint shards): each shard sees its keys in
      //    (parent, ordinal) order, so the first successor in TLC order wins
      //    (--reverse-order probe: the last one)
      parallel(T, [&](int s) {
        for (int w0 = 0; w0 < T; w0++) {
          const int w = reverse_order ? T - 1 - w0 : w0;
          auto& cs = W[w].cands;
          for (size_t q0 = 0; q0 < cs.size(); q0++) {
            Cand& c = cs[reverse_order ? cs.size() - 1 - q0 : q0];
            if (shard_of(c.key) != s) continue;
            Slot* old = fps[s].insert(c.key, (uint16_t)(level + 1), c.hidden);
            if (!old) c.res = R_NEW;
            else if (old->hidden == c.hidden) c.res = R_DUP;
            else c.res = old->level == level + 1 ? R_DUP_HID_SAME : R_DUP_HID_CROSS;
          }
        }
      });
      auto tc = std::chrono::steady_clock::now();
      // 3. sequential pass in TLC order: counts, next level, trace, first violation
      for (int w0 = 0; w0 < T && !stop; w0++) {
        const int w = reverse_order ? T - 1 - w0 : w0;
        Worker& X = W[w];
        st.max_msgs = std::max(st.max_msgs, X.maxmsg);
        size_t ie = 0;
        for (size_t q0 = 0; q0 < X.cands.size() && !stop; q0++) {
          const size_t q = reverse_order ? X.cands.size() - 1 - q0 : q0;
          const Cand& c = X.cands[q];
          gen_lvl++;
          st.generated++;
          st.act[c.act]++;
          if (c.res != R_NEW) {
            if (c.res == R_DUP_HID_SAME) st.hidden_same++;
            else if (c.res == R_DUP_HID_CROSS) st.hidden_cross++;
            continue;
          }
          st.distinct++;
          if (fpdump) fwrite(&c.key, sizeof c.key, 1, fpdump);
          const uint8_t* row = X.keep.data() + c.row_off;
          nxt->push(row, row_len(row));
          if (trace) { parent.push_back(base + c.parent_local); ordinal.push_back(c.ordinal); actid.push_back(c.act); }
          const int64_t idx = (int64_t)(st.distinct - 1);
          if (c.inv >= 0) {
            st.status = "violation"; st.violated = inv_names[c.inv]; bad_index = idx; stop = true;
          } else if (c.inv == -2) {
            while (ie < X.inv_err.size() && X.inv_err[ie].first != q) ie++;
            st.status = "error";
            st.error = ie < X.inv_err.size() ? X.inv_err[ie].second : "invariant: evaluation error";
            bad_index = idx; stop = true;
          }
        }
        if (!stop && !X.err.empty()) {
          st.status = "error";
          st.error = X.err;
          bad_index = (int64_t)(base + X.err_parent);
          stop = true;
        }
      }
      auto td = std::chrono::steady_clock::now();
      t_exp += std::chrono::duration<double>(tb - ta).count();
      t_ins += std::chrono::duration<double>(tc - tb).count();
      t_seq += std::chrono::duration<double>(td - tc).count();
    }
    nxt->finish();
    if (nxt->size() > 0 || gen_lvl > 0) st.levels.push_back({gen_lvl, nxt->size()});
    if (nxt->size() > 0) st.depth++;
    if (progress)
      fprintf(stderr, "level %u gen %llu new %llu distinct %llu rows %.2f GB t %.1f s (expand %.1f insert %.1f seq %.1f)\n",
              level + 1, (unsigned long long)gen_lvl, (unsigned long long)nxt->size(), (unsigned long long)st.distinct,
              nxt->bytes / 1e9, elapsed(), t_exp, t_ins, t_seq);
    base += F;
    level++;
    std::swap(cur, nxt);
    if (st.status != "ok") { st.left = cur->size(); break; }
    if ((max_distinct && st.distinct >= max_distinct) || (max_seconds > 0 && elapsed() > max_seconds)) {
      st.status = "truncated";
      st.left = cur->size();
      break;
    }
  }
  st.seconds = elapsed();
}

// -------------------------------------------------------------- trace / JSON
std::string state_json(const State& s) {
  std::string o = "{";
  char buf[256];
  auto arr = [&](const char* name, const int8_t* a, int n) {
    o += std::string("\"") + name + "\":[";
    for (int i = 0; i < n; i++) { snprintf(buf, sizeof buf, "%s%d", i ? "," : "", a[i]); o += buf; }
    o += "],";
  };
  arr("currentTerm", s.term, C.N);
  arr("state", s.st, C.N);
  arr(C.pull() ? "leader" : "votedFor", s.voted, C.N);
  if (C.spec == PULL2) arr("votedFor", s.voted2, C.N);
  arr("commitIndex", s.commit, C.N);
  if (C.spec == FSYNC) arr("fsyncIndex", s.fsync, C.N);
  arr("acked", s.acked, C.V);
  o += "\"votesGranted\":[";
  for (int i = 0; i < C.N; i++) { snprintf(buf, sizeof buf, "%s%d", i ? "," : "", s.votes[i]); o += buf; }
  o += "],\"log\":[";
  for (int i = 0; i < C.N; i++) {
    o += i ? ",[" : "[";
    for (int x = 0; x < s.loglen[i]; x++) { snprintf(buf, sizeof buf, "%s[%d,%d]", x ? "," : "", s.log[i][x].term, s.log[i][x].value); o += buf; }
    o += "]";
  }
  o += "],\"nextIndex\":[";
  for (int i = 0; i < C.N; i++) {
    o += i ? ",[" : "[";
    for (int j = 0; j < C.N; j++) { snprintf(buf, sizeof buf, "%s%d", j ? "," : "", s.next[i][j]); o += buf; }
    o += "]";
  }
  o += "],\"matchIndex\":[";
  for (int i = 0; i < C.N; i++) {
    o += i ? ",[" : "[";
    for (int j = 0; j < C.N; j++) { snprintf(buf, sizeof buf, "%s%d", j ? "," : "", s.match[i][j]); o += buf; }
    o += "]";
  }
  snprintf(buf, sizeof buf, "],\"pendingResponse\":[%d,%d,%d,%d,%d],\"electionCtr\":%d,\"restartCtr\":%d,\"messages\":[",
           s.pending[0], s.pending[1], s.pending[2], s.pending[3], s.pending[4], s.electionCtr, s.restartCtr);
  o += buf;
  for (int k = 0; k < s.nmsg; k++) {
    const Msg& m = s.msgs[k];
    snprintf(buf, sizeof buf,
             "%s{\"mtype\":\"%s\",\"mterm\":%d,\"msource\":%d,\"mdest\":%d,\"f\":[%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d],\"count\":%d}",
             k ? "," : "", type_name(m.type), m.term, m.src, m.dst, m.lastLogTerm, m.lastLogIndex, m.voteGranted,
             m.prevLogIndex, m.prevLogTerm, m.nent, m.eterm, m.evalue, m.commit, m.success, m.matchIndex, m.lciIndex,
             m.lciTerm, m.count);
    o += buf;
  }
  o += "]}";
  return o;
}

struct NthCollect : Emitter {
  int want, seen = 0;
  State got;
  int act = -1;
  void emit(const State& t, int a) override {
    if (seen++ == want) { got = t; act = a; }
  }
};

std::vector<std::pair<int, State>> rebuild_trace(const Checker& ck, int64_t idx) {
  std::vector<int64_t> chain;
  for (int64_t x = idx; x >= 0 && (uint64_t)x != UINT64_MAX; x = (int64_t)(ck.parent[x] == UINT64_MAX ? -1 : (int64_t)ck.parent[x])) {
    chain.push_back(x);
    if (ck.parent[x] == UINT64_MAX) break;
  }
  std::reverse(chain.begin(), chain.end());
  std::vector<std::pair<int, State>> out;
  State s = Init();
  out.push_back({-1, s});
  for (size_t k = 1; k < chain.size(); k++) {
    NthCollect nc;
    nc.want = ck.ordinal[chain[k]];
    Next(s, nc);
    s = nc.got;
    out.push_back({nc.act, s});
  }
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  Checker ck;
  bool print_trace = false;
  std::string fpdump;
  for (int a = 1; a < argc; a++) {
    std::string k = argv[a];
    auto val = [&]() { if (a + 1 >= argc) { fprintf(stderr, "missing value for %s\n", k.c_str()); exit(2); } return std::string(argv[++a]); };
    if (k == "--spec") {
      std::string v = val();
      if (v == "Raft") C.spec = RAFT; else if (v == "FlexibleRaft") C.spec = FLEX;
      else if (v == "RaftFsync") C.spec = FSYNC; else if (v == "PullRaft") C.spec = PULL;
      else if (v == "PullRaftVariant2") C.spec = PULL2;
      else { fprintf(stderr, "unknown spec %s\n", v.c_str()); return 2; }
    } else if (k == "--servers") C.N = std::stoi(val());
    else if (k == "--values") C.V = std::stoi(val());
    else if (k == "--max-elections") C.E = std::stoi(val());
    else if (k == "--max-restarts") C.R = std::stoi(val());
    else if (k == "--eq") C.EQ = std::stoi(val());
    else if (k == "--rq") C.RQ = std::stoi(val());
    else if (k == "--lfae") C.lfae = std::stoi(val()) != 0;
    else if (k == "--lfiq") C.lfiq = std::stoi(val()) != 0;
    else if (k == "--ffbr") C.ffbr = std::stoi(val()) != 0;
    else if (k == "--inv") {
      std::string v = val();
      C.inv_order.clear();
      size_t p = 0;
      while (p <= v.size()) {
        size_t q = v.find(',', p);
        if (q == std::string::npos) q = v.size();
        if (q > p) C.inv_order.push_back(v.substr(p, q - p));
        p = q + 1;
      }
    } else if (k == "--max-distinct") ck.max_distinct = std::stoull(val());
    else if (k == "--max-seconds") ck.max_seconds = std::stod(val());
    else if (k == "--threads") ck.threads = std::stoi(val());
    else if (k == "--fp-slots") ck.fp_slots = std::stoull(val());
    else if (k == "--spill-dir") ck.spill_dir = val();
    else if (k == "--no-trace") ck.trace = false;
    else if (k == "--progress") ck.progress = true;
    else if (k == "--trace") print_trace = true;
    else if (k == "--reverse-order") ck.reverse_order = true;
    else if (k == "--dump-fps") fpdump = val();
    else { fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
  }
  if (C.inv_order.empty() && argc > 0) C.inv_order = {"LeaderHasAllAckedValues", "NoLogDivergence"};
  if (C.N < 1 || C.N > MAXN || C.V < 1 || C.V > MAXV) { fprintf(stderr, "bad N/V\n"); return 2; }
  if (C.E > 15 || C.R > 15) { fprintf(stderr, "MaxElections/MaxRestarts > 15 do not fit the hidden-variable key\n"); return 2; }
  if (print_trace && !ck.trace) { fprintf(stderr, "--trace needs the trace records (drop --no-trace)\n"); return 2; }
  if (!fpdump.empty()) ck.fpdump = fopen(fpdump.c_str(), "wb");
  ck.run();
  if (ck.fpdump) fclose(ck.fpdump);
  const Stats& s = ck.st;
  printf("{\"generated\":%llu,\"distinct\":%llu,\"depth\":%d,\"left\":%llu,\"status\":\"%s\",",
         (unsigned long long)s.generated, (unsigned long long)s.distinct, s.depth, (unsigned long long)s.left,
         s.status.c_str());
  printf("\"violated\":\"%s\",\"error\":\"%s\",\"hidden_same_level\":%llu,\"hidden_cross_level\":%llu,",
         s.violated.c_str(), s.error.c_str(), (unsigned long long)s.hidden_same, (unsigned long long)s.hidden_cross);
  printf("\"max_msgs\":%d,\"seconds\":%.3f,\"threads\":%d,\"levels\":[", s.max_msgs, s.seconds, ck.threads);
  for (size_t k = 0; k < s.levels.size(); k++)
    printf("%s[%llu,%llu]", k ? "," : "", (unsigned long long)s.levels[k].first, (unsigned long long)s.levels[k].second);
  printf("],\"action_counts\":{");
  bool first = true;
  uint64_t merged[A_COUNT] = {0};
  for (int a = 0; a < A_COUNT; a++) merged[a] = s.act[a];
  merged[A_REQUESTVOTE] += merged[A_REQUESTVOTE_IJ];
  for (int a = 0; a < A_COUNT; a++) {
    if (a == A_REQUESTVOTE_IJ || !merged[a]) continue;
    printf("%s\"%s\":%llu", first ? "" : ",", act_name(a), (unsigned long long)merged[a]);
    first = false;
  }
  printf("}");
  if (print_trace && ck.bad_index >= 0) {
    auto tr = rebuild_trace(ck, ck.bad_index);
    printf(",\"trace\":[");
    for (size_t k = 0; k < tr.size(); k++)
      printf("%s{\"action\":\"%s\",\"state\":%s}", k ? "," : "", tr[k].first < 0 ? "Initial predicate" : act_name(tr[k].first),
             state_json(tr[k].second).c_str());
    printf("]");
  }
  printf("}\n");
  return 0;
}
