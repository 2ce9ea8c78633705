// kraft_oracle — CPU restatement of pull-raft/KRaft.tla under TLC -workers 1
// semantics.  TEST INFRASTRUCTURE ONLY: the second, independent checker for
// the KRaft fixtures (tests/golden/kraft.json); it shares no code with
// raft-tlaplus_amd/ (the product) or with oracle/pyoracle/kraft.py.
//
// Restated from /root/reference/specifications/pull-raft/KRaft.tla:
// Next :823-840, actions :423-801, helpers :160-392, invariants :887-957.
// TLC semantics: Next split per constant binding (first
// bound variable fastest), DOMAIN messages in TLC value order (records: field
// count, then sorted field names with values; model values by name), FIFO BFS,
// first successor per fingerprint wins, invariants on new states in cfg order,
// VIEW hides electionCtr/restartCtr (:154), SYMMETRY = all server permutations.
// Fingerprints are EXACT canonical forms: the lexicographic minimum over every
// permutation of a complete serialisation of the view, hashed to 128 bits.
//
// Parity unpinned against TLC (absent here and on the GPU box).
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

// ---- model values, ordered by name (TLC compares model values by name)
// servers are "n1".."nN" (lower case: above every capitalised constant)
enum MV {
  MV_DIVERGING, MV_FENCED, MV_NIL, MV_NOTLEADER, MV_NOTOK, MV_OK, MV_UNKNOWN,  // sorted names
  MV_SERVER0 = 100
};
enum St { FOLLOWER, CANDIDATE, LEADER, UNATTACHED, VOTED, ILLEGAL };
enum Type { T_RVREQ, T_RVRESP, T_BQREQ, T_BQRESP, T_FREQ, T_FRESP };

int N = 3, V = 1, E = 2, R = 0;
std::vector<std::string> inv_order = {"LeaderHasAllAckedValues", "NoLogDivergence", "NeverTwoLeadersInSameEpoch",
                                      "NoIllegalState"};

struct Entry {
  int epoch = 0, value = 0;
  bool operator==(const Entry& o) const { return epoch == o.epoch && value == o.value; }
};
// a FetchRequest record (also a FetchResponse's correlation and pendingFetch[i])
struct FReq {
  int epoch = 0, fo = 0, lfe = 0, src = 0, dst = 0;
  bool operator==(const FReq& o) const {
    return epoch == o.epoch && fo == o.fo && lfe == o.lfe && src == o.src && dst == o.dst;
  }
};
struct Msg {
  int type = 0, epoch = 0, src = 0, dst = 0;
  int lle = 0, llo = 0;            // RequestVoteRequest
  int leader = -1, error = MV_NIL;  // responses (leader -1 = Nil)
  bool granted = false;
  FReq fr;                          // FetchRequest fields / FetchResponse correlation
  int result = MV_OK;               // FetchResponse
  int hwm = 0, divend = 0, divepoch = 0;
  bool has_entry = false;
  Entry entry;
};

// TLC key of a value, flattened: records as [#fields, (name id, value...)...],
// sequences as [length, elements...]; a field always holds the same shape, so
// lexicographic comparison of two flattened keys is TLC's compareTo.
enum Name {  // field names in sorted (string) order
  F_CORR, F_EPOCH_E, F_VALUE_E, F_MDEST, F_MDIVEND, F_MDIVEPOCH, F_MENTRIES, F_MEPOCH, F_MERROR, F_MFO, F_MHWM,
  F_MLFE, F_MLLE, F_MLLO, F_MLEADER, F_MRESULT, F_MSOURCE, F_MTYPE, F_MVOTE
};
// names: "correlation" < "epoch" < "value" < "mdest" ... -- compare as strings
const char* NAMES[] = {"correlation", "epoch", "value", "mdest", "mdivergingEndOffset", "mdivergingEpoch", "mentries",
                       "mepoch", "merror", "mfetchOffset", "mhwm", "mlastFetchedEpoch", "mlastLogEpoch",
                       "mlastLogOffset", "mleader", "mresult", "msource", "mtype", "mvoteGranted"};
int name_rank[19];
// the type names are model values too (mtype): their ranks by name
const char* TYPE_NAME[] = {"RequestVoteRequest", "RequestVoteResponse", "BeginQuorumRequest", "BeginQuorumResponse",
                           "FetchRequest", "FetchResponse"};
int type_rank[6];
void init_ranks() {
  std::vector<int> idx(19);
  for (int k = 0; k < 19; k++) idx[k] = k;
  std::sort(idx.begin(), idx.end(), [](int a, int b) { return strcmp(NAMES[a], NAMES[b]) < 0; });
  for (int r = 0; r < 19; r++) name_rank[idx[r]] = r;
  std::vector<int> t(6);
  for (int k = 0; k < 6; k++) t[k] = k;
  std::sort(t.begin(), t.end(), [](int a, int b) { return strcmp(TYPE_NAME[a], TYPE_NAME[b]) < 0; });
  for (int r = 0; r < 6; r++) type_rank[t[r]] = r;
}
int mv_server(int s) { return s < 0 ? MV_NIL : MV_SERVER0 + s; }  // Nil < n1 < n2 (by name)

struct KeyB {
  std::vector<int> k;
  std::vector<std::pair<int, std::vector<int>>> f;  // (name, value key) before sorting
  void field(int name, std::vector<int> v) { f.push_back({name, std::move(v)}); }
  std::vector<int> done() {
    std::sort(f.begin(), f.end(), [](auto& a, auto& b) { return name_rank[a.first] < name_rank[b.first]; });
    std::vector<int> o{(int)f.size()};
    for (auto& x : f) {
      o.push_back(name_rank[x.first]);
      o.insert(o.end(), x.second.begin(), x.second.end());
    }
    return o;
  }
};
std::vector<int> freq_key(const FReq& r, const int* P) {
  KeyB b;
  b.field(F_MTYPE, {type_rank[T_FREQ]});
  b.field(F_MEPOCH, {r.epoch});
  b.field(F_MFO, {r.fo});
  b.field(F_MLFE, {r.lfe});
  b.field(F_MSOURCE, {mv_server(P[r.src])});
  b.field(F_MDEST, {mv_server(P[r.dst])});
  return b.done();
}
// the record exactly as KRaft.tla builds it, relabelled by P
std::vector<int> msg_key(const Msg& m, const int* P) {
  KeyB b;
  b.field(F_MTYPE, {type_rank[m.type]});
  b.field(F_MEPOCH, {m.epoch});
  b.field(F_MSOURCE, {mv_server(P[m.src])});
  b.field(F_MDEST, {mv_server(P[m.dst])});
  switch (m.type) {
    case T_RVREQ: b.field(F_MLLE, {m.lle}); b.field(F_MLLO, {m.llo}); break;        // :450-455
    case T_RVRESP:                                                                   // :498-511
      b.field(F_MLEADER, {mv_server(m.leader < 0 ? -1 : P[m.leader])});
      b.field(F_MVOTE, {m.granted ? 1 : 0});
      b.field(F_MERROR, {m.error});
      break;
    case T_BQREQ: break;                                                             // :553-556
    case T_BQRESP: b.field(F_MERROR, {m.error}); break;                              // :578-587
    case T_FREQ: b.field(F_MFO, {m.fr.fo}); b.field(F_MLFE, {m.fr.lfe}); break;      // :616-621
    case T_FRESP: {                                                                  // :641-649, :667-677, :725-734
      b.field(F_MRESULT, {m.result});
      b.field(F_MERROR, {m.error});
      b.field(F_MLEADER, {mv_server(m.leader < 0 ? -1 : P[m.leader])});
      b.field(F_MHWM, {m.hwm});
      b.field(F_CORR, freq_key(m.fr, P));
      if (m.result == MV_DIVERGING) { b.field(F_MDIVEPOCH, {m.divepoch}); b.field(F_MDIVEND, {m.divend}); }
      if (m.result == MV_OK) {
        std::vector<int> e{m.has_entry ? 1 : 0};
        if (m.has_entry) {
          KeyB eb;
          eb.field(F_EPOCH_E, {m.entry.epoch});
          eb.field(F_VALUE_E, {m.entry.value});
          auto ek = eb.done();
          e.insert(e.end(), ek.begin(), ek.end());
        }
        b.field(F_MENTRIES, e);
      }
      break;
    }
  }
  return b.done();
}
const int IDP[8] = {0, 1, 2, 3, 4, 5, 6, 7};

struct State {
  std::vector<Msg> mrec;  // DOMAIN messages, sorted by TLC key (msg_key) = TLC's enumeration order
  std::vector<int> cnt;   // messages[m]
  int acked[4];                                          // -1 Nil, 0 FALSE, 1 TRUE
  int ectr = 0, rctr = 0;
  int epoch[5], st[5], voted[5], leader[5];              // -1 = Nil
  bool has_pf[5];
  FReq pf[5];
  std::vector<Entry> log[5];
  int hwm[5];
  int votes[5];                                          // bitmask
  int endoff[5][5];
};

// ---- bag helpers (:169-227): binary search in TLC order
// lower bound of m's TLC key in DOMAIN; *hit = the record is there
int lower_msg(const State& s, const Msg& m, bool* hit) {
  const std::vector<int> k = msg_key(m, IDP);
  int lo = 0, hi = (int)s.mrec.size();
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (msg_key(s.mrec[mid], IDP) < k) lo = mid + 1; else hi = mid;
  }
  *hit = lo < (int)s.mrec.size() && msg_key(s.mrec[lo], IDP) == k;
  return lo;
}
int find_msg(const State& s, const Msg& m) {
  bool hit;
  int p = lower_msg(s, m, &hit);
  return hit ? p : -1;
}
void add_msg(State& t, const Msg& m, int count) {
  bool hit;
  int p = lower_msg(t, m, &hit);
  t.mrec.insert(t.mrec.begin() + p, m);
  t.cnt.insert(t.cnt.begin() + p, count);
}
void send_any(State& t, const Msg& m) {
  int k = find_msg(t, m);
  if (k >= 0) t.cnt[k]++;
  else add_msg(t, m, 1);
}
// Reply(response, request): a FetchResponse must be new (:220-227)
bool reply(State& t, const Msg& resp, int req) {
  if (!(t.cnt[req] > 0)) return false;
  int k = find_msg(t, resp);
  if (k >= 0 && resp.type == T_FRESP) return false;
  t.cnt[req]--;
  if (k >= 0) t.cnt[k]++;
  else add_msg(t, resp, 1);
  return true;
}

int last_epoch(const std::vector<Entry>& l) { return l.empty() ? 0 : l.back().epoch; }
int compare_entries(int o1, int e1, int o2, int e2) {  // :247-251
  if (e1 > e2) return 1;
  if (e1 == e2 && o1 > o2) return 1;
  if (e1 == e2 && o1 == o2) return 0;
  return -1;
}
bool quorum(int set) { return __builtin_popcount(set) * 2 > N; }

struct Tr { int st, epoch, leader; };
Tr illegal() { return {ILLEGAL, 0, -1}; }
Tr maybe_transition(const State& s, int i, int leaderId, int epoch) {  // :351-367
  bool consistent;
  if (leaderId == i) consistent = s.st[i] == LEADER;
  else consistent = epoch != s.epoch[i] || leaderId < 0 || s.leader[i] < 0 || s.leader[i] == leaderId;
  if (!consistent) return illegal();
  auto follower = [&]() -> Tr {
    if (s.epoch[i] == epoch && (s.st[i] == FOLLOWER || s.st[i] == LEADER)) return illegal();
    return {FOLLOWER, epoch, leaderId};
  };
  if (epoch > s.epoch[i]) return leaderId < 0 ? Tr{UNATTACHED, epoch, -1} : follower();
  if (leaderId >= 0 && s.leader[i] < 0) return follower();
  return {s.st[i], s.epoch[i], s.leader[i]};
}
Tr common_response(const State& s, int i, int leaderId, int epoch, int err, bool& handled) {  // :369-392
  handled = true;
  if (epoch < s.epoch[i]) return {s.st[i], s.epoch[i], s.leader[i]};
  if (epoch > s.epoch[i] || err != MV_NIL) return maybe_transition(s, i, leaderId, epoch);
  if (leaderId >= 0 && s.leader[i] < 0) return {FOLLOWER, s.epoch[i], leaderId};
  handled = false;
  return {s.st[i], s.epoch[i], s.leader[i]};
}
void apply(State& t, int i, const Tr& x) { t.st[i] = x.st; t.epoch[i] = x.epoch; t.leader[i] = x.leader; }
std::pair<int, int> end_offset_for_epoch(const State& s, int i, int lfe) {  // :285-301
  int off = 0;
  for (int o = 1; o <= (int)s.log[i].size(); o++)
    if (s.log[i][o - 1].epoch <= lfe) off = o;
  return {off, off ? s.log[i][off - 1].epoch : 0};
}

// ---- actions; emit(t, action index)
enum Act { RESTART, REQUESTVOTE, HRVREQ, HRVRESP, BECOMELEADER, CLIENT, REJFETCH, DIVFETCH, ACCFETCH, HBQ,
           SENDFETCH, HSUCC, HDIV, HERR, NACT };
const char* ACT_NAME[] = {"Restart", "RequestVote", "HandleRequestVoteRequest", "HandleRequestVoteResponse",
                          "BecomeLeader", "ClientRequest", "RejectFetchRequest", "DivergingFetchRequest",
                          "AcceptFetchRequest", "HandleBeginQuorumRequest", "SendFetchRequest",
                          "HandleSuccessFetchResponse", "HandleDivergingFetchResponse", "HandleErrorFetchResponse"};

template <class F>
void next(const State& s, F&& emit) {
  for (int i = 0; i < N; i++) {  // Restart (:423-432)
    if (!(s.rctr < R)) break;
    State t = s;
    t.st[i] = FOLLOWER; t.leader[i] = -1; t.votes[i] = 0;
    for (int j = 0; j < N; j++) t.endoff[i][j] = 0;
    t.hwm[i] = 0; t.has_pf[i] = false; t.rctr++;
    emit(t, RESTART);
  }
  for (int i = 0; i < N; i++) {  // RequestVote (:439-456)
    if (!(s.ectr < E)) break;
    if (!(s.st[i] == FOLLOWER || s.st[i] == CANDIDATE || s.st[i] == UNATTACHED)) continue;
    State t = s;
    bool ok = true;
    for (int j = 0; j < N && ok; j++) {
      if (j == i) continue;
      Msg m; m.type = T_RVREQ; m.epoch = s.epoch[i] + 1; m.lle = last_epoch(s.log[i]); m.llo = (int)s.log[i].size();
      m.src = i; m.dst = j;
      if (find_msg(s, m) >= 0) ok = false;
      else add_msg(t, m, 1);
    }
    if (!ok) continue;
    t.st[i] = CANDIDATE; t.epoch[i]++; t.leader[i] = -1; t.voted[i] = i; t.votes[i] = 1 << i; t.has_pf[i] = false;
    t.ectr++;
    emit(t, REQUESTVOTE);
  }
  auto each_msg = [&](int type, auto&& body) {
    for (size_t k = 0; k < s.mrec.size(); k++)
      if (s.cnt[k] > 0 && s.mrec[k].type == type) body((int)k, s.mrec[k]);
  };
  each_msg(T_RVREQ, [&](int k, const Msg& m) {  // HandleRequestVoteRequest (:464-513)
    const int i = m.dst, j = m.src;
    State t = s;
    Msg r; r.type = T_RVRESP; r.src = i; r.dst = j;
    if (m.epoch < s.epoch[i]) {
      r.epoch = s.epoch[i]; r.leader = s.leader[i]; r.granted = false; r.error = MV_FENCED;
    } else {
      Tr s0 = m.epoch > s.epoch[i] ? Tr{UNATTACHED, m.epoch, -1} : Tr{s.st[i], s.epoch[i], s.leader[i]};
      bool logOk = compare_entries(m.llo, m.lle, (int)s.log[i].size(), last_epoch(s.log[i])) >= 0;
      bool grant = (s0.st == UNATTACHED || (s0.st == VOTED && s.voted[i] == j)) && logOk;
      Tr fin = s0;
      if (grant && s0.st == UNATTACHED) fin = (s0.epoch == m.epoch && s0.st != UNATTACHED) ? illegal() : Tr{VOTED, m.epoch, -1};
      apply(t, i, fin);
      if (grant) t.voted[i] = j;
      if (fin.st != s.st[i]) t.has_pf[i] = false;
      r.epoch = m.epoch; r.leader = fin.leader; r.granted = grant; r.error = MV_NIL;
    }
    if (reply(t, r, k)) emit(t, HRVREQ);
  });
  each_msg(T_RVRESP, [&](int k, const Msg& m) {  // HandleRequestVoteResponse (:519-541)
    const int i = m.dst, j = m.src;
    bool handled;
    Tr ns = common_response(s, i, m.leader, m.epoch, m.error, handled);
    State t = s;
    if (handled) apply(t, i, ns);
    else {
      if (s.st[i] != CANDIDATE) return;
      if (m.granted) t.votes[i] |= 1 << j;
    }
    t.cnt[k]--;
    emit(t, HRVRESP);
  });
  for (int i = 0; i < N; i++) {  // BecomeLeader (:546-558)
    if (s.st[i] != CANDIDATE || !quorum(s.votes[i])) continue;
    State t = s;
    bool ok = true;
    for (int j = 0; j < N && ok; j++) {
      if (j == i) continue;
      Msg m; m.type = T_BQREQ; m.epoch = s.epoch[i]; m.src = i; m.dst = j;
      if (find_msg(s, m) >= 0) ok = false;
      else add_msg(t, m, 1);
    }
    if (!ok) continue;
    t.st[i] = LEADER; t.leader[i] = i;
    for (int j = 0; j < N; j++) t.endoff[i][j] = 0;
    emit(t, BECOMELEADER);
  }
  for (int v = 0; v < V; v++)  // ClientRequest (:594-603), i fastest
    for (int i = 0; i < N; i++) {
      if (s.st[i] != LEADER || s.acked[v] != -1) continue;
      State t = s;
      t.log[i].push_back(Entry{s.epoch[i], v});
      t.acked[v] = 0;
      emit(t, CLIENT);
    }
  auto fresp = [&](const Msg& m, int i, int j) {
    Msg r; r.type = T_FRESP; r.src = i; r.dst = j; r.fr = m.fr; r.leader = s.leader[i]; r.epoch = s.epoch[i];
    r.hwm = s.hwm[i];
    return r;
  };
  each_msg(T_FREQ, [&](int k, const Msg& m) {  // RejectFetchRequest (:631-651)
    const int i = m.dst, j = m.src;
    int err = s.st[i] != LEADER ? MV_NOTLEADER : m.epoch < s.epoch[i] ? MV_FENCED : m.epoch > s.epoch[i] ? MV_UNKNOWN : MV_NIL;
    if (err == MV_NIL) return;
    Msg r = fresp(m, i, j); r.result = MV_NOTOK; r.error = err;
    State t = s;
    if (reply(t, r, k)) emit(t, REJFETCH);
  });
  auto valid_pos = [&](int i, const Msg& m) {  // ValidFetchPosition (:305-310)
    if (m.fr.fo == 0 && m.fr.lfe == 0) return true;
    auto e = end_offset_for_epoch(s, i, m.fr.lfe);
    return m.fr.fo <= e.first && m.fr.lfe == e.second;
  };
  each_msg(T_FREQ, [&](int k, const Msg& m) {  // DivergingFetchRequest (:658-679)
    const int i = m.dst, j = m.src;
    if (m.epoch != s.epoch[i] || s.st[i] != LEADER || valid_pos(i, m)) return;
    auto e = end_offset_for_epoch(s, i, m.fr.lfe);
    Msg r = fresp(m, i, j); r.result = MV_DIVERGING; r.error = MV_NIL; r.divepoch = e.second; r.divend = e.first;
    State t = s;
    if (reply(t, r, k)) emit(t, DIVFETCH);
  });
  each_msg(T_FREQ, [&](int k, const Msg& m) {  // AcceptFetchRequest (:703-736)
    const int i = m.dst, j = m.src;
    if (m.epoch != s.epoch[i] || s.st[i] != LEADER || !valid_pos(i, m)) return;
    const int offset = m.fr.fo + 1;
    int ne[5];
    for (int q = 0; q < N; q++) ne[q] = s.endoff[i][q];
    ne[j] = m.fr.fo;
    int best = 0;  // NewHighwaterMark (:689-701)
    for (int o = 1; o <= (int)s.log[i].size(); o++) {
      int set = 1 << i;
      for (int q = 0; q < N; q++)
        if (ne[q] >= o) set |= 1 << q;
      if (quorum(set)) best = o;
    }
    const int nh = (best > 0 && s.log[i][best - 1].epoch == s.epoch[i]) ? best : s.hwm[i];
    Msg r = fresp(m, i, j); r.result = MV_OK; r.error = MV_NIL; r.hwm = std::min(nh, offset);
    if (offset <= (int)s.log[i].size()) { r.has_entry = true; r.entry = s.log[i][offset - 1]; }
    State t = s;
    if (!reply(t, r, k)) return;
    for (int q = 0; q < N; q++) t.endoff[i][q] = ne[q];
    t.hwm[i] = nh;
    for (int v = 0; v < V; v++)
      if (s.acked[v] == 0) {
        bool in = false;
        for (int x = s.hwm[i] + 1; x <= nh; x++)
          if (s.log[i][x - 1].value == v) in = true;
        t.acked[v] = in ? 1 : 0;
      }
    emit(t, ACCFETCH);
  });
  each_msg(T_BQREQ, [&](int k, const Msg& m) {  // HandleBeginQuorumRequest (:563-590)
    const int i = m.dst, j = m.src;
    State t = s;
    Msg r; r.type = T_BQRESP; r.src = i; r.dst = j;
    if (m.epoch < s.epoch[i]) { r.epoch = s.epoch[i]; r.error = MV_FENCED; }
    else {
      apply(t, i, maybe_transition(s, i, m.src, m.epoch));
      t.has_pf[i] = false;
      r.epoch = m.epoch; r.error = MV_NIL;
    }
    if (reply(t, r, k)) emit(t, HBQ);
  });
  for (int j = 0; j < N; j++)  // SendFetchRequest (:607-624), i fastest
    for (int i = 0; i < N; i++) {
      if (i == j || s.st[i] != FOLLOWER || s.leader[i] != j || s.has_pf[i]) continue;
      Msg m; m.type = T_FREQ; m.epoch = s.epoch[i]; m.src = i; m.dst = j;
      m.fr = FReq{s.epoch[i], (int)s.log[i].size(), last_epoch(s.log[i]), i, j};
      State t = s;
      t.has_pf[i] = true; t.pf[i] = m.fr;
      send_any(t, m);
      emit(t, SENDFETCH);
    }
  auto fetch_response = [&](bool want_handled, int result, int act) {
    each_msg(T_FRESP, [&](int k, const Msg& m) {  // :742-801
      const int i = m.dst;
      bool handled;
      Tr ns = common_response(s, i, m.leader, m.epoch, m.error, handled);
      if (handled != want_handled || !s.has_pf[i] || !(s.pf[i] == m.fr)) return;
      if (result >= 0 && m.result != result) return;
      State t = s;
      if (act == HSUCC) {
        t.hwm[i] = m.hwm;
        if (m.has_entry) t.log[i].push_back(m.entry);
      } else if (act == HDIV) {  // TruncateLog / HighestCommonOffset (:255-282)
        int o = 0;
        for (int x = 1; x <= (int)s.log[i].size(); x++)
          if (compare_entries(x, s.log[i][x - 1].epoch, m.divend, m.divepoch) <= 0) o = x;
        t.log[i].resize(o);
      } else {
        apply(t, i, ns);
      }
      t.has_pf[i] = false;
      t.cnt[k]--;
      emit(t, act);
    });
  };
  fetch_response(false, MV_OK, HSUCC);
  fetch_response(false, MV_DIVERGING, HDIV);
  fetch_response(true, -1, HERR);
}

// ---- invariants (:887-957); -1 ok, -2 evaluation error, else the cfg position
int check(const State& s) {
  for (size_t q = 0; q < inv_order.size(); q++) {
    const std::string& n = inv_order[q];
    bool ok = true;
    if (n == "NoIllegalState") {
      for (int i = 0; i < N; i++) if (s.st[i] == ILLEGAL) ok = false;
    } else if (n == "NoLogDivergence") {
      for (int s2 = 0; s2 < N && ok; s2++)
        for (int s1 = 0; s1 < N && ok; s1++) {
          if (s1 == s2) continue;
          int c = std::min(s.hwm[s1], s.hwm[s2]);
          for (int o = 1; o <= c && ok; o++) {
            if (o > (int)s.log[s1].size() || o > (int)s.log[s2].size()) return -2;
            if (!(s.log[s1][o - 1] == s.log[s2][o - 1])) ok = false;
          }
        }
    } else if (n == "NeverTwoLeadersInSameEpoch") {
      for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++)
          if (s.leader[i] >= 0 && s.leader[j] >= 0 && s.leader[i] != s.leader[j] && s.epoch[i] == s.epoch[j]) ok = false;
    } else if (n == "LeaderHasAllAckedValues") {
      for (int v = 0; v < V; v++) {
        if (s.acked[v] != 1) continue;
        for (int i = 0; i < N; i++) {
          if (s.st[i] != LEADER) continue;
          bool newer = false, has = false;
          for (int l = 0; l < N; l++) if (l != i && s.epoch[l] > s.epoch[i]) newer = true;
          for (auto& e : s.log[i]) if (e.value == v) has = true;
          if (!newer && !has) ok = false;
        }
      }
    }
    if (!ok) return (int)q;
  }
  return -1;
}

// ---- exact canonical form of the view (everything but the counters)
std::vector<int> serialise(const State& s, const int* P) {
  int inv[5];
  for (int i = 0; i < N; i++) inv[P[i]] = i;
  std::vector<int> o;
  for (int v = 0; v < V; v++) o.push_back(s.acked[v]);
  for (int pos = 0; pos < N; pos++) {
    const int i = inv[pos];
    o.push_back(s.epoch[i]); o.push_back(s.st[i]);
    o.push_back(s.voted[i] < 0 ? -1 : P[s.voted[i]]);
    o.push_back(s.leader[i] < 0 ? -1 : P[s.leader[i]]);
    o.push_back(s.has_pf[i]);
    if (s.has_pf[i]) { o.push_back(s.pf[i].epoch); o.push_back(s.pf[i].fo); o.push_back(s.pf[i].lfe); o.push_back(P[s.pf[i].dst]); }
    o.push_back((int)s.log[i].size());
    for (auto& e : s.log[i]) { o.push_back(e.epoch); o.push_back(e.value); }
    o.push_back(s.hwm[i]);
    int vg = 0;
    for (int j = 0; j < N; j++) if ((s.votes[i] >> j) & 1) vg |= 1 << P[j];
    o.push_back(vg);
    for (int q = 0; q < N; q++) o.push_back(s.endoff[i][inv[q]]);
  }
  // the messages as a multiset of injective 64-bit codes of the relabelled
  // records (any injective code: only equality of canonical forms matters)
  uint64_t ms[128];
  const int nm = (int)s.mrec.size();
  for (int k = 0; k < nm; k++) {
    const Msg& m = s.mrec[k];
    uint64_t c = 0;
    auto put = [&](int v, int w) { c = (c << w) | ((uint64_t)v & ((1ULL << w) - 1)); };
    put(m.type, 3); put(m.epoch, 3); put(P[m.src], 3); put(P[m.dst], 3); put(m.lle, 3); put(m.llo, 3);
    put(m.leader < 0 ? 0 : P[m.leader] + 1, 3); put(m.granted, 1); put(m.error, 3); put(m.fr.epoch, 3);
    put(m.fr.fo, 3); put(m.fr.lfe, 3); put(m.result, 3); put(m.hwm, 3); put(m.divend, 3); put(m.divepoch, 3);
    put(m.has_entry, 1); put(m.entry.epoch, 3); put(m.entry.value, 2); put(s.cnt[k], 4);
    ms[k] = c;
  }
  std::sort(ms, ms + nm);
  o.push_back(nm);
  for (int k = 0; k < nm; k++) { o.push_back((int)(ms[k] >> 32)); o.push_back((int)(uint32_t)ms[k]); }
  return o;
}
struct Fp { uint64_t a, b; bool operator==(const Fp& o) const { return a == o.a && b == o.b; } };
struct FpH { size_t operator()(const Fp& f) const { return (size_t)(f.a ^ (f.b * 0x9E3779B97F4A7C15ULL)); } };
Fp canon(const State& s) {
  std::vector<int> P(N), best;
  for (int i = 0; i < N; i++) P[i] = i;
  bool first = true;
  do {
    auto x = serialise(s, P.data());
    if (first || x < best) { best.swap(x); first = false; }
  } while (std::next_permutation(P.begin(), P.end()));
  uint64_t a = 0xcbf29ce484222325ULL, b = 0x84222325cbf29ce4ULL;
  for (int v : best) {
    a = (a ^ (uint32_t)v) * 0x100000001b3ULL;
    b = (b + (uint32_t)v + 0x9E3779B97F4A7C15ULL) * 0xBF58476D1CE4E5B9ULL;
    b ^= b >> 31;
  }
  return {a, b};
}

}  // namespace

int main(int argc, char** argv) {
  uint64_t max_states = 0;
  for (int a = 1; a < argc; a++) {
    std::string k = argv[a];
    auto val = [&]() { return std::string(argv[++a]); };
    if (k == "--servers") N = std::stoi(val());
    else if (k == "--values") V = std::stoi(val());
    else if (k == "--max-elections") E = std::stoi(val());
    else if (k == "--max-restarts") R = std::stoi(val());
    else if (k == "--max-states") max_states = std::stoull(val());
    else if (k == "--inv") {
      std::string v = val();
      inv_order.clear();
      size_t p = 0;
      while (p <= v.size()) {
        size_t q = v.find(',', p);
        if (q == std::string::npos) q = v.size();
        if (q > p) inv_order.push_back(v.substr(p, q - p));
        p = q + 1;
      }
    } else { fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
  }
  if (N < 1 || N > 5 || V < 1 || V > 4) { fprintf(stderr, "bad N/V\n"); return 2; }
  init_ranks();
  auto t0 = std::chrono::steady_clock::now();
  State init;
  for (int v = 0; v < V; v++) init.acked[v] = -1;
  for (int i = 0; i < N; i++) {  // Init (:397-415)
    init.epoch[i] = 1; init.st[i] = UNATTACHED; init.voted[i] = init.leader[i] = -1; init.has_pf[i] = false;
    init.hwm[i] = 0; init.votes[i] = 0;
    for (int j = 0; j < N; j++) init.endoff[i][j] = 0;
  }
  struct Seen { int level; int hidden; };
  std::unordered_map<Fp, Seen, FpH> seen;
  std::vector<State> level{init};
  seen[canon(init)] = {1, 0};
  uint64_t generated = 1, distinct = 1, hidden_same = 0, act[NACT] = {0};
  int depth = 1, max_msgs = 0;
  std::vector<std::pair<uint64_t, uint64_t>> levels{{1, 1}};
  std::string status = "ok", violated;
  uint64_t left = 0;
  while (!level.empty() && status == "ok") {
    std::vector<State> nxt;
    uint64_t gl = 0;
    size_t pidx = 0;
    for (; pidx < level.size() && status == "ok"; pidx++) {
      const State& s = level[pidx];
      max_msgs = std::max(max_msgs, (int)s.mrec.size());
      next(s, [&](const State& t, int a) {
        if (status != "ok") return;
        gl++; generated++; act[a]++;
        Fp f = canon(t);
        const int hid = t.ectr * 16 + t.rctr;
        auto it = seen.find(f);
        if (it != seen.end()) {
          if (it->second.hidden != hid && it->second.level == depth + 1) hidden_same++;
          return;
        }
        seen[f] = {depth + 1, hid};
        distinct++;
        nxt.push_back(t);
        int c = check(t);
        if (c == -2) status = "error";
        else if (c >= 0) { status = "violation"; violated = inv_order[c]; }
      });
    }
    if (status != "ok") {
      levels.push_back({gl, nxt.size()});
      depth += nxt.empty() ? 0 : 1;
      left = nxt.size() + (level.size() - pidx);
      break;
    }
    if (!nxt.empty()) { depth++; levels.push_back({gl, nxt.size()}); }
    else if (gl) levels.push_back({gl, 0});
    level.swap(nxt);
    if (max_states && distinct >= max_states) { status = "truncated"; left = level.size(); break; }
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("{\"generated\":%llu,\"distinct\":%llu,\"depth\":%d,\"left\":%llu,\"status\":\"%s\",\"violated\":\"%s\","
         "\"hidden_same_level\":%llu,\"max_msgs\":%d,\"seconds\":%.3f,\"levels\":[",
         (unsigned long long)generated, (unsigned long long)distinct, depth, (unsigned long long)left, status.c_str(),
         violated.c_str(), (unsigned long long)hidden_same, max_msgs, secs);
  for (size_t k = 0; k < levels.size(); k++)
    printf("%s[%llu,%llu]", k ? "," : "", (unsigned long long)levels[k].first, (unsigned long long)levels[k].second);
  printf("],\"action_counts\":{");
  bool first = true;
  for (int a = 0; a < NACT; a++)
    if (act[a]) { printf("%s\"%s\":%llu", first ? "" : ",", ACT_NAME[a], (unsigned long long)act[a]); first = false; }
  printf("}}\n");
  return 0;
}
