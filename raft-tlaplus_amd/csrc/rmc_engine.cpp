// rmc_engine.cpp — librmc host side: cfg parsing and spec identification
// (replacing TLC's SANY + cfg binding), the level-synchronous BFS driver over
// the HIP kernels, trace reconstruction and the TLC-format report, behind the
// C ABI of include/rmc.h.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <unordered_map>
#include <set>
#include <sstream>
#include <sys/stat.h>
#include <dirent.h>
#include <fcntl.h>
#include <unistd.h>
#include <cerrno>
#include <string>
#include <vector>
#include "rmc_internal.h"
#include "rmc_fpset.h"
#include "rmc_tla.h"

using namespace rmc;
using namespace rmcx;

static thread_local std::string g_last_error;
// the first HIP call of this process (runtime + device initialisation), reported
// in the phases of the process's first check
static double g_hip_init_s = 0;
static bool g_hip_init_done = false;

// ------------------------------------------------------------------ cfg
namespace {

struct CfgVal {
  enum Kind { INT, BOOL, MV, SET, STR, OP } kind = MV;
  long long i = 0;
  bool b = false;
  std::string s;
  std::vector<std::string> set;  // set of model values (names)
};

struct Cfg {
  std::map<std::string, CfgVal> consts;
  std::string init, next, spec, view, symmetry;
  std::vector<std::string> invariants, properties, constraints;
  int check_deadlock = -1;
};

std::string strip_comments(const std::string& t) {
  std::string out;
  int depth = 0;
  for (size_t i = 0; i < t.size(); i++) {
    if (t.compare(i, 2, "(*") == 0) { depth++; i++; continue; }
    if (depth && t.compare(i, 2, "*)") == 0) { depth--; i++; continue; }
    if (!depth) out += t[i];
  }
  std::string res, line;
  std::istringstream is(out);
  while (std::getline(is, line)) {
    size_t c = line.find("\\*");
    if (c != std::string::npos) line = line.substr(0, c);
    res += line + "\n";
  }
  return res;
}

std::vector<std::string> tokenize(const std::string& t) {
  std::vector<std::string> v;
  size_t i = 0;
  while (i < t.size()) {
    char c = t[i];
    if (isspace((unsigned char)c)) { i++; continue; }
    if (c == '<' && i + 1 < t.size() && t[i + 1] == '-') { v.push_back("<-"); i += 2; continue; }
    if (strchr("{}(),=", c)) { v.push_back(std::string(1, c)); i++; continue; }
    if (c == '"') {
      size_t j = t.find('"', i + 1);
      if (j == std::string::npos) throw std::runtime_error("cfg: unterminated string");
      v.push_back(t.substr(i, j - i + 1));
      i = j + 1;
      continue;
    }
    if (isalnum((unsigned char)c) || c == '_' || c == '-') {
      size_t j = i;
      while (j < t.size() && (isalnum((unsigned char)t[j]) || t[j] == '_' || t[j] == '!' || (j == i && t[j] == '-')))
        j++;
      v.push_back(t.substr(i, j - i));
      i = j;
      continue;
    }
    throw std::runtime_error(std::string("cfg: unexpected character '") + c + "'");
  }
  return v;
}

bool is_int(const std::string& s) {
  if (s.empty()) return false;
  size_t k = s[0] == '-' ? 1 : 0;
  if (k == s.size()) return false;
  for (; k < s.size(); k++)
    if (!isdigit((unsigned char)s[k])) return false;
  return true;
}

CfgVal parse_value(const std::vector<std::string>& tk, size_t& k) {
  CfgVal v;
  const std::string& t = tk.at(k);
  if (t == "{") {
    v.kind = CfgVal::SET;
    k++;
    while (tk.at(k) != "}") {
      CfgVal e = parse_value(tk, k);
      if (e.kind != CfgVal::MV) throw std::runtime_error("cfg: only sets of model values are supported");
      v.set.push_back(e.s);
      if (tk.at(k) == ",") k++;
    }
    k++;
    return v;
  }
  k++;
  if (t == "TRUE" || t == "FALSE") { v.kind = CfgVal::BOOL; v.b = t == "TRUE"; return v; }
  if (is_int(t)) { v.kind = CfgVal::INT; v.i = std::stoll(t); return v; }
  if (t[0] == '"') { v.kind = CfgVal::STR; v.s = t.substr(1, t.size() - 2); return v; }
  v.kind = CfgVal::MV;  // bare identifier: an untyped model value (Raft.cfg:6-9 quirk)
  v.s = t;
  return v;
}

Cfg parse_cfg(const std::string& text) {
  static const std::set<std::string> kw = {"CONSTANT", "CONSTANTS", "INIT", "NEXT", "SPECIFICATION", "INVARIANT",
                                           "INVARIANTS", "PROPERTY", "PROPERTIES", "VIEW", "SYMMETRY", "CONSTRAINT",
                                           "CONSTRAINTS", "ACTION_CONSTRAINT", "ACTION_CONSTRAINTS",
                                           "CHECK_DEADLOCK", "POSTCONDITION", "ALIAS"};
  Cfg c;
  auto tk = tokenize(strip_comments(text));
  std::string sec;
  size_t k = 0;
  while (k < tk.size()) {
    const std::string t = tk[k];
    if (kw.count(t)) {
      sec = t;
      k++;
      if (sec == "INIT") c.init = tk.at(k++);
      else if (sec == "NEXT") c.next = tk.at(k++);
      else if (sec == "SPECIFICATION") c.spec = tk.at(k++);
      else if (sec == "VIEW") c.view = tk.at(k++);
      else if (sec == "SYMMETRY") c.symmetry = tk.at(k++);
      else if (sec == "ALIAS") k++;
      else if (sec == "CHECK_DEADLOCK") { CfgVal v = parse_value(tk, k); c.check_deadlock = v.b; }
      continue;
    }
    if (sec == "CONSTANT" || sec == "CONSTANTS") {
      if (k + 1 >= tk.size()) throw std::runtime_error("cfg: dangling constant " + t);
      if (tk[k + 1] == "=") {
        k += 2;
        c.consts[t] = parse_value(tk, k);
      } else if (tk[k + 1] == "<-") {
        CfgVal v;
        v.kind = CfgVal::OP;
        v.s = tk.at(k + 2);
        c.consts[t] = v;
        k += 3;
      } else {
        throw std::runtime_error("cfg: bad constant assignment near " + t);
      }
      continue;
    }
    if (sec == "INVARIANT" || sec == "INVARIANTS") c.invariants.push_back(t);
    else if (sec == "PROPERTY" || sec == "PROPERTIES") c.properties.push_back(t);
    else if (sec.find("CONSTRAINT") != std::string::npos) c.constraints.push_back(t);
    else throw std::runtime_error("cfg: token '" + t + "' outside any section");
    k++;
  }
  return c;
}

}  // namespace

namespace rmcx {

int spec_of_module(const std::string& m) {
  if (m == "Raft") return RAFT;
  if (m == "FlexibleRaft") return FLEX;
  if (m == "RaftFsync") return FSYNC;
  if (m == "PullRaft") return PULL;
  if (m == "PullRaftVariant2") return PULL2;
  if (m == "KRaft") return KRAFT;
  return -1;
}

const char* act_label(int a) {
  static const char* n[] = {"Restart", "RequestVote", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest",
                            "AdvanceCommitIndex", "AppendEntries", "AdvanceFsyncIndex", "UpdateTerm",
                            "HandleRequestVoteRequest", "HandleRequestVoteResponse", "RejectAppendEntriesRequest",
                            "AcceptAppendEntriesRequest", "HandleAppendEntriesResponse", "RejectPullEntriesRequest",
                            "AcceptPullEntriesRequest", "LearnOfLeader", "SendPullEntriesRequest",
                            "HandleSuccessPullEntriesResponse", "HandleFailPullEntriesResponse",
                            "RejectFetchRequest", "DivergingFetchRequest", "AcceptFetchRequest",
                            "HandleBeginQuorumRequest", "SendFetchRequest", "HandleSuccessFetchResponse",
                            "HandleDivergingFetchResponse", "HandleErrorFetchResponse", "DuplicateMessage",
                            "DropMessage", "Compiled0", "Compiled1", "Compiled2", "Compiled3"};
  static_assert(sizeof n / sizeof n[0] == A_NUM, "a label per action id");
  return (a >= 0 && a < A_NUM) ? n[a] : "?";
}

// The action table in Next order: the spec's own (the reference modules'
// Next), or the one the TLA+ front end lowered from the module text.
void build_actions(Model& M, const std::vector<std::pair<int, int>>* lowered) {
  struct E { int id, kind; };
  std::vector<E> t;
  if (lowered && !lowered->empty()) {
    for (auto& a : *lowered) t.push_back({a.first, a.second});
  } else switch (M.spec) {
    case RAFT: case FLEX:  // Raft.tla:527-539; FlexibleRaft.tla:488-500
      t = {{A_RESTART, K_I}, {A_REQUESTVOTE, K_I}, {A_BECOMELEADER, K_I}, {A_CLIENT, K_IV}, {A_ADVCOMMIT, K_I},
           {A_APPENDENTRIES, K_IJ}, {A_UPDATETERM, K_MSG}, {A_HRVREQ, K_MSG}, {A_HRVRESP, K_MSG},
           {A_REJAE, K_MSG}, {A_ACCAE, K_MSG}, {A_HAERESP, K_MSG}};
      break;
    case FSYNC:  // RaftFsync.tla:522-536
      t = {{A_RESTART, K_I}, {A_TIMEOUT, K_I}, {A_RVIJ, K_IJ}, {A_BECOMELEADER, K_I}, {A_CLIENT, K_IV},
           {A_ADVCOMMIT, K_I}, {A_APPENDENTRIES, K_IJ}, {A_ADVFSYNC, K_I}, {A_UPDATETERM, K_MSG},
           {A_HRVREQ, K_MSG}, {A_HRVRESP, K_MSG}, {A_REJAE, K_MSG}, {A_ACCAE, K_MSG}, {A_HAERESP, K_MSG}};
      break;
    case PULL: case PULL2:  // PullRaft.tla:542-558; PullRaftVariant2.tla:560-576 (same disjuncts)
      t = {{A_RESTART, K_I}, {A_UPDATETERM, K_MSG}, {A_REQUESTVOTE, K_I}, {A_HRVREQ, K_MSG}, {A_HRVRESP, K_MSG},
           {A_BECOMELEADER, K_I}, {A_CLIENT, K_IV}, {A_REJPULL, K_MSG}, {A_ACCPULL, K_MSG}, {A_LEARN, K_MSG},
           {A_SENDPULL, K_IJ}, {A_HSUCC, K_MSG}, {A_HFAIL, K_MSG}};
      break;
    case KRAFT:  // KRaft.tla:823-840
      t = {{A_RESTART, K_I}, {A_REQUESTVOTE, K_I}, {A_HRVREQ, K_MSG}, {A_HRVRESP, K_MSG}, {A_BECOMELEADER, K_I},
           {A_CLIENT, K_IV}, {A_KREJFETCH, K_MSG}, {A_KDIVFETCH, K_MSG}, {A_KACCFETCH, K_MSG}, {A_KHBQ, K_MSG},
           {A_KSENDFETCH, K_IJ}, {A_KHSUCC, K_MSG}, {A_KHDIV, K_MSG}, {A_KHERR, K_MSG}};
      break;
  }
  if ((int)t.size() > MAXACT) throw std::runtime_error("Next has more disjuncts than the lowering's " +
                                                       std::to_string(MAXACT) + " action slots");
  M.nact = (int)t.size();
  int off = 0, nf = 0;
  for (int a = 0; a < A_NUM; a++) M.msg_act_slot[a] = 0;
  M.msg_act_mask = 0;
  M.nmsgc = 0;
  for (int s = 0; s < M.nact; s++) {
    M.act_fb_first[s] = (uint8_t)nf;
    M.act_id[s] = t[s].id;
    M.act_kind[s] = t[s].kind;
    M.act_off[s] = off;
    int size = t[s].kind == K_I ? M.N : t[s].kind == K_IV ? M.N * M.V : t[s].kind == K_IJ ? M.N * M.N : M.kmax;
    if (t[s].kind == K_MSG) {
      M.msg_act_slot[t[s].id] = s;
      M.msg_act_mask |= 1ULL << t[s].id;
    } else if (t[s].kind == K_MSGC) {  // a compiled message handler: evaluated on its own (act_message skips it)
      if (t[s].id < A_C0 || t[s].id >= A_C0 + MAXCOMPILED) throw std::runtime_error("compiled handler id");
      M.msg_act_slot[t[s].id] = s;
      M.msgc_q[M.nmsgc++] = (int8_t)(t[s].id - A_C0);
    } else
      for (int x = 0; x < size; x++) {
        // bindings the constants disable for good are not evaluated at all
        // (their ordinals stay reserved, so TLC's order is unchanged):
        // AppendEntries / RequestVote(i, j) / SendPullEntriesRequest with i = j
        // (Raft.tla:264, RaftFsync.tla:235, PullRaft.tla:397), Restart with
        // MaxRestarts = 0 (Raft.tla:227), elections with MaxElections = 0
        const int id = t[s].id;
        // K_M (\E m \in DOMAIN messages): the message slot k = x as (k & 15, k >> 4)
        const int i = t[s].kind == K_M ? (x & 15) : x % M.N, j = t[s].kind == K_M ? (x >> 4) : x / M.N;
        if (t[s].kind == K_IJ && i == j &&
            (id == A_APPENDENTRIES || id == A_RVIJ || id == A_SENDPULL || id == A_KSENDFETCH))  // KRaft.tla:608
          continue;
        if (id == A_RESTART && M.R == 0) continue;
        if ((id == A_REQUESTVOTE || id == A_TIMEOUT) && M.E == 0) continue;
        if (nf >= MAXFIXED) throw std::runtime_error("too many fixed bindings");
        M.fb_act[nf] = (uint8_t)s;
        M.fb_x[nf] = (uint8_t)x;
        M.fb_desc[nf] = (uint32_t)s | (uint32_t)x << 8 | (uint32_t)id << 16 | (uint32_t)i << 24 | (uint32_t)j << 28;
        nf++;
      }
    M.act_fb_end[s] = (uint8_t)nf;
    off += size;
  }
  M.nfixed = nf;
  M.ordinal_limit = off;
  if (off > 1024) throw std::runtime_error("ordinal space exceeds 10 bits; lower msg_cap_K");
  for (int q = 0; q < 1024; q++) M.ord2b[q] = 0xFFFF;
  for (int b = 0; b < nf; b++) M.ord2b[M.act_off[M.fb_act[b]] + M.fb_x[b]] = (uint16_t)b;
  for (int sl = 0; sl < M.nact; sl++) {
    if (M.act_kind[sl] == K_MSG)
      for (int k = 0; k < M.kmax; k++) M.ord2b[M.act_off[sl] + k] = (uint16_t)(nf + k);
    if (M.act_kind[sl] == K_MSGC)
      for (int k = 0; k < M.kmax; k++)
        M.ord2b[M.act_off[sl] + k] = (uint16_t)(nf + MSGC_STRIDE * (1 + M.act_id[sl] - A_C0) + k);
  }
  if (M.kmax > MSGC_STRIDE) throw std::runtime_error("more message slots than a compiled handler's binding stride");
  for (int a = 0; a < A_NUM; a++) M.msg_off[a] = (uint16_t)M.act_off[M.msg_act_slot[a]];
  M.bind_words = (M.nfixed + M.kmax + 31) / 32;
  M.ord_words = (off + 31) / 32;
  if (off >= 1024) throw std::runtime_error("ordinal space exceeds 10 bits; lower msg_cap_K");
}

void build_perms(Model& M, bool symmetry) {
  std::vector<int> p(M.N);
  for (int i = 0; i < M.N; i++) p[i] = i;
  M.nperm = 0;
  do {
    uint32_t P = 0;
    for (int j = 0; j < M.N; j++) P |= (uint32_t)p[j] << (3 * j);
    M.perm[M.nperm++] = P;
    if (!symmetry) break;
  } while (std::next_permutation(p.begin(), p.end()));
}

// The drop-in boundary lowers four specs by hand, so the .tla it is given must
// BE one of them: its text, with comments and whitespace removed, hashed
// (FNV-1a 64) against the reference's specifications (tools/spec_hashes.py
// regenerates the table).  Comment and layout edits pass; any edit to the
// TLA+ itself (e.g. re-enabling DuplicateMessage in Raft's Next,
// standard-raft/Raft.tla:540) is refused rather than silently checked as the
// built-in lowering.
std::string normalise_tla(const std::string& t) {
  std::string out;
  int depth = 0;
  for (size_t i = 0; i < t.size();) {
    if (t.compare(i, 2, "(*") == 0) { depth++; i += 2; }
    else if (depth && t.compare(i, 2, "*)") == 0) { depth--; i += 2; }
    else if (depth) i++;
    else if (t.compare(i, 2, "\\*") == 0) { while (i < t.size() && t[i] != '\n') i++; }
    else { if (!isspace((unsigned char)t[i])) out += t[i]; i++; }
  }
  return out;
}
unsigned long long fnv1a64(const std::string& s) {
  unsigned long long h = 0xcbf29ce484222325ULL;
  for (unsigned char c : s) h = (h ^ c) * 0x100000001b3ULL;
  return h;
}
unsigned long long known_spec_hash(const std::string& module) {
  static const std::map<std::string, unsigned long long> k = {
      {"Raft", 0x83a8af2f23ec2fd5ULL},          // specifications/standard-raft/Raft.tla
      {"FlexibleRaft", 0xc4f3c1e150bbc233ULL},  // specifications/flexible-raft/FlexibleRaft.tla
      {"PullRaft", 0x158f1b6f8dd861a3ULL},      // specifications/pull-raft/PullRaft.tla
      {"RaftFsync", 0x8135c01b3aedbce3ULL},     // specifications/raft-and-fsync/RaftFsync.tla
      {"PullRaftVariant2", 0xa830c4c4ebcf30b0ULL},  // specifications/pull-raft/PullRaftVariant2.tla
      {"KRaft", 0xb2b4f50a062d58efULL},             // specifications/pull-raft/KRaft.tla
  };
  auto it = k.find(module);
  return it == k.end() ? 0 : it->second;
}

// Does the module text define operator `name` (a line starting `name ==` or `name(...) ==`)?
static bool defines_operator(const std::string& tla, const std::string& name) {
  size_t p = 0;
  while ((p = tla.find(name, p)) != std::string::npos) {
    const bool bol = p == 0 || tla[p - 1] == '\n';
    size_t q = p + name.size();
    while (q < tla.size() && (tla[q] == ' ' || tla[q] == '\t')) q++;
    if (bol && q + 1 < tla.size() && tla[q] == '=' && tla[q + 1] == '=') return true;
    p += name.size();
  }
  return false;
}

// Compile the guards the front end lowered onto library effects (rmc_guard.cpp)
// against this model's constants, into Model::gcode / gstart (all of them:
// gs replaces the model's compiled guards).
void install_guards(rmc_model* m, const std::vector<rmc::tla::GuardSrc>& gs) {
  Model& M = m->M;
  rmc::tla::GuardEnv env;
  env.spec = M.spec;
  env.N = M.N;
  env.V = M.V;
  env.servers = m->server_names;
  env.values = m->value_names;
  for (auto& kv : m->int_consts) env.ints.insert(kv);
  std::vector<uint32_t> code;
  std::vector<std::pair<int, int>> starts, estarts;
  for (const auto& g : gs) {
    const bool whole = g.act >= A_C0;  // compiled whole: guard and effect (rmc_guard.cpp compile_effect)
    if (whole && g.kind == K_MSGC) {  // a message handler: one program, guards and effects in the text's order
      rmc::tla::GuardEnv eenv = env;
      eenv.send_helpers = g.send_helpers;
      std::vector<uint32_t> h = rmc::tla::compile_handler(*g.mod, g.params, g.conjuncts, eenv, g.op);
      estarts.push_back({g.act - A_C0, (int)code.size()});
      code.insert(code.end(), h.begin(), h.end());
      continue;
    }
    const int kind = whole ? g.kind : g.act == A_CLIENT ? K_IV : g.act == A_RVIJ ? K_IJ : K_I;
    const std::vector<int> types = kind == K_IV ? std::vector<int>{0, 1} : kind == K_IJ ? std::vector<int>{0, 0}
                                                                                         : std::vector<int>{0};
    if (g.params.size() != types.size())
      throw std::runtime_error("guard of " + g.op + ": " + std::to_string(g.params.size()) +
                               " parameters, the action binds " + std::to_string(types.size()));
    std::vector<uint32_t> c = rmc::tla::compile_guard(*g.mod, g.params, types, g.conjuncts, env, g.op);
    starts.push_back({g.act, (int)code.size()});
    code.insert(code.end(), c.begin(), c.end());
    if (whole) {
      rmc::tla::GuardEnv eenv = env;
      eenv.send_helpers = g.send_helpers;
      std::vector<uint32_t> e = rmc::tla::compile_effect(*g.mod, g.params, types, g.effects, eenv, g.op);
      estarts.push_back({g.act - A_C0, (int)code.size()});
      code.insert(code.end(), e.begin(), e.end());
    }
  }
  if (code.size() > (size_t)MAXGCODE)
    throw std::runtime_error("compiled guards take " + std::to_string(code.size()) + " words (at most " +
                             std::to_string(MAXGCODE) + ")");
  for (int a = 0; a < A_NUM; a++) M.gstart[a] = -1;
  memset(M.gcode, 0, sizeof M.gcode);
  for (size_t q = 0; q < code.size(); q++) M.gcode[q] = code[q];
  for (auto& s2 : starts) M.gstart[s2.first] = (int16_t)s2.second;
  for (int q = 0; q < MAXCOMPILED; q++) M.estart[q] = -1;
  for (auto& s2 : estarts) M.estart[s2.first] = (int16_t)s2.second;
  M.gany = starts.empty() && estarts.empty() ? 0 : 1;
  m->guard_srcs = gs;
}

rmc_model* load_model(const std::string& module, const std::string& cfg_text, const std::string& tla_text) {
  auto m = new rmc_model();
  try {
    m->module = module;
    m->tla_text = tla_text;
    int spec = spec_of_module(module);
    if (!tla_text.empty() && tla_text.find("MODULE " + module) == std::string::npos)
      throw std::runtime_error("the .tla file does not declare MODULE " + module);
    // The reference text of a module this checker lowers (comments and layout
    // may differ): its built-in action table.  Any other text goes through the
    // TLA+ front end (rmc_tla.cpp), which lowers what it can and names what it
    // cannot.
    const bool reference_text =
        tla_text.empty() || (spec >= 0 && fnv1a64(normalise_tla(tla_text)) == known_spec_hash(module));
    if (tla_text.empty() && spec < 0)
      throw std::runtime_error("unsupported module '" + module +
                               "' (supported: Raft, FlexibleRaft, RaftFsync, PullRaft, PullRaftVariant2, KRaft)");
    Cfg c = parse_cfg(cfg_text);
    if (!c.spec.empty()) throw std::runtime_error("SPECIFICATION is not supported; use INIT Init / NEXT Next");
    if (!c.properties.empty()) throw std::runtime_error("PROPERTY checking (liveness) is not supported");
    if (!c.constraints.empty()) throw std::runtime_error("CONSTRAINT is not supported");
    rmc::tla::Lowering low;
    if (reference_text) {
      if (c.init != "Init" || c.next != "Next")
        throw std::runtime_error("cfg must bind INIT Init and NEXT Next (got '" + c.init + "', '" + c.next + "')");
      if (c.view != "view") throw std::runtime_error("cfg must set VIEW view (the reference cfgs do)");
      if (!c.symmetry.empty() && c.symmetry != "symmServers")
        throw std::runtime_error("only SYMMETRY symmServers is supported");
    } else {
      if (c.init != "Init") throw std::runtime_error("cfg must bind INIT Init (got '" + c.init + "')");
      if (c.view.empty()) throw std::runtime_error("cfg must set a VIEW (the lowering fingerprints the spec's view)");
      low = rmc::tla::lower(tla_text, c.next, c.view, c.symmetry, c.invariants);
      spec = low.spec;
      m->lowered_actions = low.actions;
      m->lowered_labels = low.labels;
    }
    auto need = [&](const std::string& n) -> CfgVal& {
      auto it = c.consts.find(n);
      if (it == c.consts.end()) throw std::runtime_error("cfg: constant " + n + " is not assigned");
      return it->second;
    };
    Model& M = m->M;
    memset(&M, 0, sizeof M);
    for (int a = 0; a < A_NUM; a++) M.gstart[a] = -1;  // the library's guards
    for (int q = 0; q < MAXCOMPILED; q++) M.estart[q] = -1;
    M.spec = spec;
    CfgVal& S = need("Server");
    CfgVal& Vv = need("Value");
    if (S.kind != CfgVal::SET || Vv.kind != CfgVal::SET) throw std::runtime_error("Server and Value must be sets");
    m->server_names = S.set;
    m->value_names = Vv.set;
    for (auto& kv : c.consts) {
      const CfgVal& v = kv.second;
      std::string t;
      if (v.kind == CfgVal::INT) m->int_consts[kv.first] = v.i;
      switch (v.kind) {
        case CfgVal::INT: t = std::to_string(v.i); break;
        case CfgVal::BOOL: t = v.b ? "TRUE" : "FALSE"; break;
        case CfgVal::SET:
          t = "{";
          for (size_t q = 0; q < v.set.size(); q++) t += (q ? ", " : "") + v.set[q];
          t += "}";
          break;
        case CfgVal::OP: t = "<- " + v.s; break;
        default: t = v.s; break;
      }
      m->cfg_consts.push_back({kv.first, t});
    }
    std::sort(m->server_names.begin(), m->server_names.end());  // TLC orders model values by name
    std::sort(m->value_names.begin(), m->value_names.end());
    M.N = (int)S.set.size();
    M.V = (int)Vv.set.size();
    if (M.N < 2 || M.N > 5) throw std::runtime_error("|Server| must be 2..5");
    if (M.V < 1 || M.V > MAXV) throw std::runtime_error("|Value| must be 1..4");
    auto geti = [&](const char* n) {
      CfgVal& v = need(n);
      if (v.kind != CfgVal::INT) throw std::runtime_error(std::string("constant ") + n + " must be an integer");
      return (int)v.i;
    };
    auto getb = [&](const char* n) {
      CfgVal& v = need(n);
      if (v.kind != CfgVal::BOOL) throw std::runtime_error(std::string("constant ") + n + " must be TRUE/FALSE");
      return (int)v.b;
    };
    M.E = geti("MaxElections");
    M.R = geti("MaxRestarts");
    if (M.E < 0 || M.E > 14 || M.R < 0 || M.R > 15) throw std::runtime_error("MaxElections/MaxRestarts out of range");
    // KRaft's records pack into one 32-bit DOMAIN word only with 2-bit epochs and
    // offsets (rmc_spec.h kr_encode), and its fingerprint relates mleader to a
    // message's two servers (kr_body), which is exact for N <= 3
    if (spec == KRAFT && (M.N > 3 || M.E > 2 || M.V > 3))
      throw std::runtime_error("the KRaft lowering supports |Server| <= 3, MaxElections <= 2, |Value| <= 3");
    if (spec == FLEX) { M.EQ = geti("ElectionQuorumSize"); M.RQ = geti("ReplicationQuorumSize"); }
    if (spec == FSYNC) {
      M.lfae = getb("LeaderFsyncBeforeAppendEntries");
      M.lfiq = getb("LeaderFsyncBeforeIncludeInQuorum");
      M.ffbr = getb("FollowerFsyncBeforeReply");
    }
    M.ninv = 0;
    for (auto& n : c.invariants) {
      if (!reference_text) {  // the front end matched the module's invariant definitions
        auto it = low.invariants.find(n);
        if (it == low.invariants.end())
          throw std::runtime_error("invariant " + n + " is not defined in module " + module);
        if (M.ninv >= 9) throw std::runtime_error("too many invariants");
        M.inv[M.ninv++] = it->second;
        m->inv_names.push_back(n);
        continue;
      }
      int id = n == "LeaderHasAllAckedValues" ? 0 : n == "NoLogDivergence" ? 1
                                               : n == "CommittedEntriesReachMajority" ? 2
                                               : n == "TestInv" ? -2 : -1;
      if (spec == KRAFT && n == "NeverTwoLeadersInSameEpoch") id = 3;  // KRaft.tla:916-921
      if (spec == KRAFT && n == "NoIllegalState") id = 4;              // KRaft.tla:887-889
      // the classic Raft properties, opt-in (rmc_spec.h)
      if (spec != KRAFT && n == "ElectionSafety") id = 5;
      if (spec != KRAFT && n == "LogMatching") id = 6;
      if (spec != KRAFT && n == "LeaderCompleteness") id = 7;
      if (spec != KRAFT && n == "StateMachineSafety") id = 8;
      // ... but not on the TLC-compatible path (a .tla was given): TLC resolves
      // an INVARIANT name in the module, and no reference spec defines these,
      // so there the name is unknown exactly as TLC would report it
      if (id >= 5 && !tla_text.empty() && !defines_operator(tla_text, n))
        throw std::runtime_error("invariant " + n + " is not defined in module " + module +
                                 " (the classic Raft invariants are built-in extras of the checker: load the cfg "
                                 "with rmc_model_load_text / raftmc -module " + module + ")");
      if (id == -2) continue;  // TestInv == TRUE
      if (id < 0) throw std::runtime_error("unsupported invariant " + n);
      if (M.ninv >= 9) throw std::runtime_error("too many invariants");
      M.inv[M.ninv++] = id;
      m->inv_names.push_back(n);
    }
    build_perms(M, !c.symmetry.empty());
    switch (spec) {
      case RAFT:
        m->var_order = {"messages", "acked", "electionCtr", "restartCtr", "currentTerm", "state", "votedFor", "log",
                        "commitIndex", "votesGranted", "nextIndex", "matchIndex", "pendingResponse"};
        break;
      case FLEX:
        m->var_order = {"messages", "acked", "electionCtr", "restartCtr", "currentTerm", "state", "votedFor", "log",
                        "commitIndex", "votesGranted", "nextIndex", "matchIndex"};
        break;
      case FSYNC:
        m->var_order = {"messages", "acked", "electionCtr", "restartCtr", "currentTerm", "state", "votedFor", "log",
                        "commitIndex", "fsyncIndex", "votesGranted", "nextIndex", "matchIndex"};
        break;
      case PULL:
        m->var_order = {"messages", "acked", "electionCtr", "restartCtr", "currentTerm", "state", "leader", "log",
                        "commitIndex", "votesGranted", "matchIndex"};
        break;
      case PULL2:  // declaration order, PullRaftVariant2.tla:56-106
        m->var_order = {"messages", "acked", "electionCtr", "restartCtr", "currentTerm", "state", "leader",
                        "votedFor", "log", "commitIndex", "votesGranted", "votesLastEntry", "matchIndex"};
        break;
      case KRAFT:  // declaration order, KRaft.tla:100-144
        m->var_order = {"messages", "acked", "electionCtr", "restartCtr", "currentEpoch", "state", "votedFor",
                        "leader", "pendingFetch", "log", "highWatermark", "votesGranted", "endOffset"};
        break;
    }
    if (!low.guards.empty()) install_guards(m, low.guards);
  } catch (std::exception& e) {
    delete m;
    throw;
  }
  return m;
}

void finalize_model(rmc_model* m, uint32_t kmax) {
  Model& M = m->M;
  // rows are a multiple of 4 words (16 B aligned for the kernels' vector
  // stores); the padding becomes message capacity
  // (padding can give up to 123 slots for a request of 120: never round a
  // request down below itself -- the regrow path asks for exactly 120)
  int words = (1 + 4 * M.N + (int)kmax + 3) & ~3;
  if (words - 1 - 4 * M.N > 124) words -= 4;
  M.words = words;
  M.kmax = words - 1 - 4 * M.N;
  M.fpw = 1;
  build_actions(M, &m->lowered_actions);
}

uint32_t default_kmax(const Model& M) {
  int k = 8 * M.N + 8 * M.V + 4 * M.E;
  k = ((k + 7) / 8) * 8;
  return (uint32_t)std::min(std::max(k, 24), 120);
}

// Message slots per packed row: the largest |DOMAIN messages| the last complete
// check of this model materialized (rows then carry no dead slots), else the
// constants-based default.  Either way an overflow re-runs with twice the slots.
uint32_t model_kmax(const rmc_model* m) { return m->hint_kmax ? m->hint_kmax : default_kmax(m->M); }

std::vector<uint32_t> init_state(const Model& M) {
  std::vector<uint32_t> S(M.words, 0u);
  S[0] = 0;  // nmsg 0, counters 0, acked all Nil (Raft.tla:209-213)
  for (int i = 0; i < M.N; i++) {
    uint32_t a = 1u | (FOLLOWER << 4) | ((uint32_t)NILS << 6);  // currentTerm 1, Follower, votedFor Nil
    if (M.spec == PULL2) a |= (uint32_t)NILS << 15;          // leader and votedFor Nil (PullRaftVariant2.tla:224-225)
    if (M.spec == KRAFT) a = kr_set_st(a | ((uint32_t)NILS << 15), KS_UNATTACHED);  // KRaft.tla:397-401
    S[1 + 4 * i] = a;
    S[2 + 4 * i] = 0;
    S[3 + 4 * i] = (pullish(M.spec) || M.spec == KRAFT) ? 0u : all_rows(M.N, 1);  // nextIndex 1 / Nil / pendingFetch Nil
    S[4 + 4 * i] = 0;                                        // matchIndex = 0
  }
  return S;
}

// ------------------------------------------------------------ formatting
std::vector<std::pair<std::string, std::string>> state_vars(const rmc_model* m, const uint32_t* S) {
  const Model& M = m->M;
  auto sv = [&](int i) { return i == NILS ? std::string("Nil") : m->server_names.at(i); };
  auto fn = [&](auto val) {
    std::string o = "(";
    for (int i = 0; i < M.N; i++) o += (i ? " @@ " : "") + m->server_names[i] + " :> " + val(i);
    return o + ")";
  };
  auto entry = [&](int t, int v) {
    return std::string(M.spec == KRAFT ? "[epoch |-> " : "[term |-> ") + std::to_string(t) + ", value |-> " +
           m->value_names.at(v) + "]";
  };
  // KRaft records in TLC's field order (KRaft.tla:450-455, :498-504, :553-556, :578-587, :616-621, :641-677, :725-734)
  auto kerr = [](int e) { return std::string(e == KE_FENCED ? "FencedLeaderEpoch" : e == KE_NIL ? "Nil" : e == KE_NOTLEADER ? "NotLeader" : "UnknownLeader"); };
  auto kld = [&](int l) { return l < 0 ? std::string("Nil") : m->server_names.at(l); };
  auto kfetch = [&](int dst, int epoch, int fo, int lfe, int src) {
    return "[mdest |-> " + sv(dst) + ", mepoch |-> " + std::to_string(epoch) + ", mfetchOffset |-> " + std::to_string(fo) +
           ", mlastFetchedEpoch |-> " + std::to_string(lfe) + ", msource |-> " + sv(src) + ", mtype |-> FetchRequest]";
  };
  auto kmsg = [&](uint32_t mw) {
    const KMsg f = kr_decode(mw);
    const std::string ep = std::to_string(f.epoch);
    switch (f.cls) {
      case 0: return "[mdest |-> " + sv(f.dst) + ", mepoch |-> " + ep + ", msource |-> " + sv(f.src) + ", mtype |-> BeginQuorumRequest]";
      case 1: return "[mdest |-> " + sv(f.dst) + ", mepoch |-> " + ep + ", merror |-> " + kerr(f.err) + ", msource |-> " + sv(f.src) + ", mtype |-> BeginQuorumResponse]";
      case 2:
        if (f.granted)
          return "[mdest |-> " + sv(f.dst) + ", mepoch |-> " + ep + ", mlastLogEpoch |-> " + std::to_string(f.f1) +
                 ", mlastLogOffset |-> " + std::to_string(f.f2) + ", msource |-> " + sv(f.src) + ", mtype |-> RequestVoteRequest]";
        return kfetch(f.dst, f.epoch, f.f1, f.f2, f.src);
      case 3:
        return "[mdest |-> " + sv(f.dst) + ", mepoch |-> " + ep + ", merror |-> " + kerr(f.err) + ", mleader |-> " + kld(f.leader) +
               ", msource |-> " + sv(f.src) + ", mtype |-> RequestVoteResponse, mvoteGranted |-> " + (f.granted ? "TRUE" : "FALSE") + "]";
      default: {
        const std::string corr = "[correlation |-> " + kfetch(f.src, f.cepoch, f.cfo, f.clfe, f.dst) + ", mdest |-> " + sv(f.dst);
        const std::string tail = ", mhwm |-> " + std::to_string(f.hwm) + ", mleader |-> " + kld(f.leader);
        if (f.cls == KR_NOTOK)
          return corr + ", mepoch |-> " + ep + ", merror |-> " + kerr(f.err) + tail + ", mresult |-> NotOk, msource |-> " +
                 sv(f.src) + ", mtype |-> FetchResponse]";
        if (f.cls == KR_OK)
          return corr + ", mentries |-> " + (f.elen ? "<<" + entry(f.eepoch, f.evalue) + ">>" : std::string("<<>>")) +
                 ", mepoch |-> " + ep + ", merror |-> Nil" + tail + ", mresult |-> Ok, msource |-> " + sv(f.src) +
                 ", mtype |-> FetchResponse]";
        return corr + ", mdivergingEndOffset |-> " + std::to_string(f.divend) + ", mdivergingEpoch |-> " +
               std::to_string(f.divepoch) + ", mepoch |-> " + ep + ", merror |-> Nil" + tail +
               ", mresult |-> Diverging, msource |-> " + sv(f.src) + ", mtype |-> FetchResponse]";
      }
    }
  };
  std::vector<std::pair<std::string, std::string>> o;
  int nm = h_nmsg(S[0]);
  for (auto& var : m->var_order) {
    std::string val;
    if (var == "messages") {
      if (nm == 0) val = "<< >>";
      else {
        val = "(";
        for (int k = 0; k < nm; k++) {
          const uint32_t mw = S[1 + 4 * M.N + k];
          if (M.spec == KRAFT) {
            val += (k ? " @@\n  " : "") + kmsg(mw) + " :> " + std::to_string(msg_count(mw));
            continue;
          }
          MsgF f = M.spec == PULL2 ? msg_decode<PULL2>(mw) : M.spec == PULL ? msg_decode<PULL>(mw) : msg_decode<RAFT>(mw);
          std::string r;
          auto B = [](int x) { return std::string(x ? "TRUE" : "FALSE"); };
          auto ents = [&](int n, int t, int v) { return n ? "<<" + entry(t, v) + ">>" : std::string("<<>>"); };
          switch (f.type) {
            case RVREQ:
              r = "[mdest |-> " + sv(f.dst) + ", mlastLogIndex |-> " + std::to_string(f.lli) + ", mlastLogTerm |-> " +
                  std::to_string(f.llt) + ", msource |-> " + sv(f.src) + ", mterm |-> " + std::to_string(f.term) +
                  ", mtype |-> RequestVoteRequest]";
              break;
            case PEREQ:
              r = "[mdest |-> " + sv(f.dst) + ", mlastLogIndex |-> " + std::to_string(f.lli) + ", mlastLogTerm |-> " +
                  std::to_string(f.llt) + ", msource |-> " + sv(f.src) + ", mterm |-> " + std::to_string(f.term) +
                  ", mtype |-> PullEntriesRequest]";
              break;
            case RVRESP:
              if (M.spec == PULL2)
                r = "[mdest |-> " + sv(f.dst) + ", mlastLogIndex |-> " + std::to_string(f.lli) +
                    ", mlastLogTerm |-> " + std::to_string(f.llt) + ", msource |-> " + sv(f.src) + ", mterm |-> " +
                    std::to_string(f.term) + ", mtype |-> RequestVoteResponse, mvoteGranted |-> " + B(f.granted) + "]";
              else
                r = "[mdest |-> " + sv(f.dst) + ", msource |-> " + sv(f.src) + ", mterm |-> " + std::to_string(f.term) +
                    ", mtype |-> RequestVoteResponse, mvoteGranted |-> " + B(f.granted) + "]";
              break;
            case AEREQ:
              r = "[mcommitIndex |-> " + std::to_string(f.commit) + ", mdest |-> " + sv(f.dst) + ", mentries |-> " +
                  ents(f.nent, f.eterm, f.evalue) + ", mprevLogIndex |-> " + std::to_string(f.pli) +
                  ", mprevLogTerm |-> " + std::to_string(f.plt) + ", msource |-> " + sv(f.src) + ", mterm |-> " +
                  std::to_string(f.term) + ", mtype |-> AppendEntriesRequest]";
              break;
            case AERESP:
              r = "[mdest |-> " + sv(f.dst) + ", mmatchIndex |-> " + std::to_string(f.midx) + ", msource |-> " +
                  sv(f.src) + ", msuccess |-> " + B(f.success) + ", mterm |-> " + std::to_string(f.term) +
                  ", mtype |-> AppendEntriesResponse]";
              break;
            case LNREQ:
              if (M.spec == PULL2)
                r = "[mdest |-> " + sv(f.dst) + ", mlastCommonEntry |-> " +
                    (f.lcenil ? std::string("Nil")
                              : "[index |-> " + std::to_string(f.lci) + ", term |-> " + std::to_string(f.lct) + "]") +
                    ", msource |-> " + sv(f.src) + ", mterm |-> " + std::to_string(f.term) +
                    ", mtype |-> LeaderNotifyRequest]";
              else
                r = "[mdest |-> " + sv(f.dst) + ", msource |-> " + sv(f.src) + ", mterm |-> " + std::to_string(f.term) +
                    ", mtype |-> LeaderNotifyRequest]";
              break;
            case PERESP:
              if (f.success)
                r = "[mcommitIndex |-> " + std::to_string(f.commit) + ", mdest |-> " + sv(f.dst) + ", mentries |-> " +
                    ents(f.nent, f.eterm, f.evalue) + ", msource |-> " + sv(f.src) + ", msuccess |-> TRUE, mterm |-> " +
                    std::to_string(f.term) + ", mtype |-> PullEntriesResponse]";
              else
                r = "[mdest |-> " + sv(f.dst) + ", mlastCommonEntry |-> [index |-> " + std::to_string(f.lci) +
                    ", term |-> " + std::to_string(f.lct) + "], msource |-> " + sv(f.src) +
                    ", msuccess |-> FALSE, mterm |-> " + std::to_string(f.term) + ", mtype |-> PullEntriesResponse]";
              break;
          }
          val += (k ? " @@\n  " : "") + r + " :> " + std::to_string(f.count);
        }
        val += ")";
      }
    } else if (var == "acked") {
      val = "(";
      for (int v = 0; v < M.V; v++) {
        int a = h_acked(S[0], v);
        val += (v ? " @@ " : "") + m->value_names[v] + " :> " + (a == 0 ? "Nil" : a == 1 ? "FALSE" : "TRUE");
      }
      val += ")";
    } else if (var == "electionCtr") val = std::to_string(h_ectr(S[0]));
    else if (var == "restartCtr") val = std::to_string(h_rctr(S[0]));
    else if (var == "currentTerm" || var == "currentEpoch") val = fn([&](int i) { return std::to_string(a_term(S[1 + 4 * i])); });
    else if (var == "state" && M.spec == KRAFT)
      val = fn([&](int i) {
        static const char* names[] = {"Follower", "Candidate", "Leader", "Unattached", "Voted", "IllegalState", "?", "?"};
        return std::string(names[kr_st(S[1 + 4 * i])]);
      });
    else if (var == "pendingFetch")
      val = fn([&](int i) {
        const uint32_t c = S[3 + 4 * i];
        if (!(c & 1u)) return std::string("Nil");
        return kfetch((int)getb(c, 7, 3), (int)getb(c, 1, 2), (int)getb(c, 3, 2), (int)getb(c, 5, 2), i);
      });
    else if (var == "highWatermark") val = fn([&](int i) { return std::to_string(a_commit(S[1 + 4 * i])); });
    else if (var == "endOffset")
      val = fn([&](int i) {
        std::string o2 = "(";
        for (int j = 0; j < M.N; j++) o2 += (j ? " @@ " : "") + m->server_names[j] + " :> " + std::to_string(row_get(S[4 + 4 * i], j));
        return o2 + ")";
      });
    else if (var == "state")
      val = fn([&](int i) {
        int st = a_st(S[1 + 4 * i]);
        return std::string(st == FOLLOWER ? "Follower" : st == CANDIDATE ? "Candidate" : "Leader");
      });
    else if (var == "votedFor" && (M.spec == PULL2 || M.spec == KRAFT)) val = fn([&](int i) { return sv(a_votedfor2(S[1 + 4 * i])); });
    else if (var == "votedFor" || var == "leader") val = fn([&](int i) { return sv(a_voted(S[1 + 4 * i])); });
    else if (var == "votesLastEntry")
      val = fn([&](int i) {
        std::string o2 = "(";
        for (int j = 0; j < M.N; j++) {
          const uint32_t v = j == i ? 0u : vle_get(S[3 + 4 * i], i, j);
          o2 += (j ? " @@ " : "") + m->server_names[j] + " :> " +
                (v ? "[index |-> " + std::to_string((int)(v & 7u) - 1) + ", term |-> " + std::to_string((int)(v >> 3)) + "]"
                   : std::string("Nil"));
        }
        return o2 + ")";
      });
    else if (var == "log")
      val = fn([&](int i) {
        uint32_t a = S[1 + 4 * i], b = S[2 + 4 * i];
        std::string o2 = "<<";
        for (int x = 0; x < a_len(a); x++) o2 += (x ? ", " : "") + entry(e_term(b, x), e_value(b, x));
        return o2 + ">>";
      });
    else if (var == "commitIndex") val = fn([&](int i) { return std::to_string(a_commit(S[1 + 4 * i])); });
    else if (var == "fsyncIndex") val = fn([&](int i) { return std::to_string(a_fsync(S[1 + 4 * i])); });
    else if (var == "votesGranted")
      val = fn([&](int i) {
        int vg = a_votes(S[1 + 4 * i]);
        std::string o2 = "{";
        bool first = true;
        for (int j = 0; j < M.N; j++)
          if ((vg >> j) & 1) { o2 += (first ? "" : ", ") + m->server_names[j]; first = false; }
        return o2 + "}";
      });
    else if (var == "nextIndex" || var == "matchIndex" || var == "pendingResponse")
      val = fn([&](int i) {
        std::string o2 = "(";
        for (int j = 0; j < M.N; j++) {
          std::string x;
          if (var == "nextIndex") x = std::to_string(row_get(S[3 + 4 * i], j));
          else if (var == "matchIndex") x = std::to_string(row_get(S[4 + 4 * i], j));
          else x = ((a_pending(S[1 + 4 * i]) >> j) & 1) ? "TRUE" : "FALSE";
          o2 += (j ? " @@ " : "") + m->server_names[j] + " :> " + x;
        }
        return o2 + ")";
      });
    o.push_back({var, val});
  }
  return o;
}

std::string fmt_state(const rmc_model* m, const uint32_t* S) {
  std::string o;
  for (auto& kv : state_vars(m, S)) o += "/\\ " + kv.first + " = " + kv.second + "\n";
  return o;
}

std::string binding_label(const rmc_model* m, int b, int act) {
  const Model& M = m->M;
  std::string name = act_label(act);
  if (b < M.nfixed) {
    int slot = M.fb_act[b], x = M.fb_x[b];
    int kind = M.act_kind[slot];
    int i = x % M.N, jv = x / M.N;
    if (!m->lowered_labels.empty()) name = m->lowered_labels[slot];
    if (kind == K_M) return name;
    if (kind == K_I) return name + "(" + m->server_names[i] + ")";
    if (kind == K_IV) return name + "(" + m->server_names[i] + ", " + m->value_names[jv] + ")";
    return name + "(" + m->server_names[i] + ", " + m->server_names[jv] + ")";
  }
  if (!m->lowered_labels.empty() && act >= 0 && act < A_NUM) return m->lowered_labels[M.msg_act_slot[act]];
  return name;
}

// line of an operator definition in the module text, for TLC-style labels
std::string def_location(const rmc_model* m, const std::string& op) {
  if (m->tla_text.empty()) return "";
  std::istringstream is(m->tla_text);
  std::string line;
  int ln = 0;
  while (std::getline(is, line)) {
    ln++;
    if (line.compare(0, op.size(), op) == 0) {
      size_t p = op.size();
      while (p < line.size() && line[p] != '=' && line[p] != '\n') p++;
      if (line.find("==", op.size()) != std::string::npos) return " line " + std::to_string(ln);
    }
  }
  return "";
}

}  // namespace

// ----------------------------------------------------------- BFS driver
namespace rmcx {

// Per-chunk readbacks land in pinned host memory, so they are true async
// copies: one stream sync per chunk (after the mark/scan), none after
// k_materialize — its status is snapshotted into `mat` in stream order and
// examined at the next sync.
struct HostReadback {
  unsigned long long segc[128];  // k_expand's 8 per-XCD candidate counters, 128 B apart
  uint32_t lastpos, lastwin;     // the chunk's last parent: scan position and winner count
  DevStatus st;                  // status after the chunk's mark/scan
  DevStatus mat;                 // status after the chunk's k_materialize
};
struct Arena {
  // table/table2: the fingerprint set and its growth target
  DevBuf table, table2, cslot, cob, cwin, poff, pn, pwin, ppos, counters, stbuf, scantmp;
  DevBuf hwin_in[2], hwin_out[2];  // host-frontier windows: parents in, new rows out (double-buffered)
  // compact host rows (per window parity): out = pack side, in = unpack side
  DevBuf hf_pack[2], hf_olen32[2], hf_olen8[2], hf_ooff[2], hf_oscan[2];
  DevBuf hf_stage[2], hf_ilen32[2], hf_ilen8[2], hf_ioff[2], hf_iscan[2];
  DevBuf hf_flag;  // k_row_words' bound: a row whose header claims more than W words
  void release_hf() {
    hf_flag.release();
    for (int k = 0; k < 2; k++)
      for (DevBuf* b : {&hwin_in[k], &hwin_out[k], &hf_pack[k], &hf_olen32[k], &hf_olen8[k], &hf_ooff[k], &hf_oscan[k],
                        &hf_stage[k], &hf_ilen32[k], &hf_ilen8[k], &hf_ioff[k], &hf_iscan[k]})
        b->release();
  }
  // the second set of per-chunk arrays (two chunks in flight) and
  // k_materialize's own status (its stream runs beside k_expand's)
  DevBuf cslot2, cob2, cwin2, poff2, pn2, pwin2, ppos2, counters2, stmat;
  void release_set2() {
    for (DevBuf* b : {&cslot2, &cob2, &cwin2, &poff2, &pn2, &pwin2, &ppos2, &counters2}) b->release();
  }
  GrowBuf fa, fb, trp, trb;  // frontiers and trace records grow in place
  HostReadback* hrb = nullptr;
  void release() {
    if (hrb) (void)hipHostFree(hrb);
    hrb = nullptr;
    for (DevBuf* b : {&table, &table2, &cslot, &cob, &cwin, &poff, &pn, &pwin, &ppos, &counters, &stbuf, &scantmp,
                      &stmat})
      b->release();
    release_set2();
    release_hf();
    for (GrowBuf* b : {&fa, &fb, &trp, &trb}) b->release();
  }
};
std::mutex g_arena_mu;
std::map<int, Arena*> g_arenas;
Arena& arena_for_current_device() {
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_arena_mu);
  Arena*& a = g_arenas[dev];
  if (!a) a = new Arena();
  return *a;
}

void set_last_error(const std::string& s) { g_last_error = s; }

// The single-GPU search's cached buffers on the current device.  The sharded
// entry points call this (and rmc_check calls release_shard_buffers): a
// process that alternates the two must not have one's cache starve the other.
void release_single_buffers() {
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_arena_mu);
  auto it = g_arenas.find(dev);
  if (it != g_arenas.end()) it->second->release();
}

void replay_trace(rmc_model* m, const std::vector<int>& binds, int last_b, int status, std::string& message,
                  rmc_result* res) {
  const Model& M = m->M;
  const size_t W = (size_t)M.words;
  std::vector<uint32_t> s = init_state(M);
  m->trace_states.push_back(s);
  m->trace_actions.push_back("Initial predicate");
  auto step = [&](int b) {
    std::vector<uint32_t> t(W, 0);
    int ordv = 0, act = -1, err = 0;
    int en = host_eval_apply(M, s.data(), b, t.data(), &ordv, &act, &err);
    if (en != 1) throw std::runtime_error("trace replay: binding not enabled");
    std::string lbl = binding_label(m, b, act);
    if (err) return lbl;  // the erroring step: no successor state
    s = t;
    m->trace_states.push_back(s);
    m->trace_actions.push_back(lbl);
    return std::string();
  };
  for (int b : binds) step(b);
  if (last_b >= 0) {
    std::string e = step(last_b);
    if (!e.empty()) message += " in action " + e;
  }
  if (status == 1 && !m->trace_states.empty()) {
    int err = 0;
    int bad = host_check_invariants(M, m->trace_states.back().data(), &err);
    if (bad >= 0) snprintf(res->violated, sizeof res->violated, "%s", m->inv_names[bad].c_str());
  }
}

// ---- checkpoint / recover (TLC -checkpoint / -recover, its states/ directory)
// A snapshot is taken at a level boundary: the fingerprint set (raw entries),
// the next level's frontier (packed rows), the trace records of every state
// so far, and the counts.  Each snapshot goes into a fresh subdirectory
// (snap-<seq>); its files are fsync'd, then checkpoint.meta is replaced
// atomically (written to a temporary, fsync'd, renamed, directory fsync'd) to
// name it, and only then is the previous snapshot's subdirectory removed -- as
// TLC keeps its previous checkpoint valid until the new one is complete, a
// crash, kill or full disk at any point leaves one complete snapshot.
struct Ckpt {
  unsigned long long sig = 0, slots = 0, generated = 0, distinct = 0, cur_base = 0, cur_n = 0, hidden = 0;
  unsigned depth = 0;
  uint32_t kmax = 0;
  int fpw = 1;
  double rate = 4.0;
  unsigned long long seq = 0;  // snapshot sequence number; files in snap-<seq>/
  std::vector<std::pair<unsigned long long, unsigned long long>> levels;
};
static std::string ckpt_subdir(unsigned long long seq) { return "snap-" + std::to_string(seq); }
static void fsync_dir(const std::string& dir) {
  int fd = open(dir.c_str(), O_RDONLY | O_DIRECTORY);
  if (fd < 0) throw std::runtime_error("checkpoint: cannot open " + dir);
  int rc = fsync(fd);
  close(fd);
  if (rc != 0) throw std::runtime_error("checkpoint: cannot sync " + dir);
}
static void remove_tree(const std::string& dir) {
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) {
      std::string n = e->d_name;
      if (n != "." && n != "..") (void)unlink((dir + "/" + n).c_str());
    }
    closedir(d);
  }
  (void)rmdir(dir.c_str());
}
unsigned long long model_signature(const rmc_model* m) {
  const Model& M = m->M;
  char b[320];
  snprintf(b, sizeof b, "%s|%d|%d|%d|%d|%d|%d|%d|%d|%d|%d|%d|%d|%d|%d", m->module.c_str(), M.spec, M.N, M.V, M.E,
           M.R, M.EQ, M.RQ, M.lfae, M.lfiq, M.ffbr, M.words, M.kmax, M.fpw, M.nperm);
  std::string s = b;
  for (int q = 0; q < M.ninv; q++) s += "|inv" + std::to_string(M.inv[q]);
  for (auto& n : m->server_names) s += "|s:" + n;
  for (auto& n : m->value_names) s += "|v:" + n;
  for (int a = 0; a < A_NUM; a++)  // compiled guards (rmc_guard.cpp) are part of the model
    if (M.gstart[a] >= 0) s += "|g" + std::to_string(a) + ":" + std::to_string(M.gstart[a]);
  for (int q = 0; q < MAXCOMPILED; q++)
    if (M.estart[q] >= 0) s += "|e" + std::to_string(q) + ":" + std::to_string(M.estart[q]);
  // every word of the compiled code: a program ends in G_END, which encodes
  // to 0, so stopping at the first zero word would hash only the first guard
  //  -- install_guards zeroes the words past the code
  for (int q = 0; q < MAXGCODE; q++) s += "," + std::to_string(M.gcode[q]);
  for (int a = 0; a < M.nact; a++) s += "|a" + std::to_string(M.act_id[a]) + ":" + std::to_string(M.act_kind[a]);
  return fnv1a64(s);
}
static void ckpt_write(const std::string& path, const void* dev, size_t bytes, void* stage, size_t stage_bytes) {
  const std::string tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("checkpoint: cannot write " + tmp);
  for (size_t o = 0; o < bytes; o += stage_bytes) {
    const size_t n = std::min(stage_bytes, bytes - o);
    HIPCHK(hipMemcpy(stage, (const char*)dev + o, n, hipMemcpyDeviceToHost));
    if (fwrite(stage, 1, n, f) != n) { fclose(f); throw std::runtime_error("checkpoint: short write to " + tmp); }
  }
  if (fflush(f) != 0 || fsync(fileno(f)) != 0) { fclose(f); throw std::runtime_error("checkpoint: cannot sync " + tmp); }
  if (fclose(f) != 0 || rename(tmp.c_str(), path.c_str()) != 0)
    throw std::runtime_error("checkpoint: cannot finish " + path);
}
static void ckpt_read(const std::string& path, void* dev, size_t bytes, void* stage, size_t stage_bytes) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("recover: cannot read " + path);
  fseek(f, 0, SEEK_END);
  if ((size_t)ftell(f) != bytes) { fclose(f); throw std::runtime_error("recover: " + path + " has the wrong size"); }
  fseek(f, 0, SEEK_SET);
  for (size_t o = 0; o < bytes; o += stage_bytes) {
    const size_t n = std::min(stage_bytes, bytes - o);
    if (fread(stage, 1, n, f) != n) { fclose(f); throw std::runtime_error("recover: short read from " + path); }
    HIPCHK(hipMemcpy((char*)dev + o, stage, n, hipMemcpyHostToDevice));
  }
  fclose(f);
}
// The frontier file of a snapshot taken with w0-word rows, loaded as w-word rows
// (w >= w0: a resumed check that overflowed the snapshot's message capacity
// re-runs with more slots; the extra slots are empty -- the message count is in
// the header word -- and fingerprints, ranks and bindings do not depend on it).
static void ckpt_read_rows(const std::string& path, uint32_t* dev, size_t n, size_t w0, size_t w, void* stage,
                           size_t stage_bytes) {
  if (w == w0) return ckpt_read(path, dev, n * w * 4, stage, stage_bytes);
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("recover: cannot read " + path);
  fseek(f, 0, SEEK_END);
  if ((size_t)ftell(f) != n * w0 * 4) { fclose(f); throw std::runtime_error("recover: " + path + " has the wrong size"); }
  fseek(f, 0, SEEK_SET);
  const size_t rows = stage_bytes / (w * 4);
  std::vector<uint32_t> in(rows * w0);
  uint32_t* out = (uint32_t*)stage;
  for (size_t r0 = 0; r0 < n; r0 += rows) {
    const size_t k = std::min(rows, n - r0);
    if (fread(in.data(), 4, k * w0, f) != k * w0) { fclose(f); throw std::runtime_error("recover: short read from " + path); }
    for (size_t r = 0; r < k; r++) {
      memcpy(out + r * w, in.data() + r * w0, w0 * 4);
      memset(out + r * w + w0, 0, (w - w0) * 4);
    }
    HIPCHK(hipMemcpy(dev + r0 * w, out, k * w * 4, hipMemcpyHostToDevice));
  }
  fclose(f);
}
// The same frontier file streamed straight into host-frontier pages (a level
// that only fit on the host when the snapshot was taken): no device copy.
static void ckpt_read_rows_host(const std::string& path, HostLevel& h, HostPagePool& pool, size_t n, size_t w0,
                                int hdr_words) {
  // the snapshot's rows (w0 words each) compacted on the way into the pages;
  // the compact form does not depend on the row width, so a resumed level
  // with more message slots unpacks them zero-padded
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("recover: cannot read " + path);
  fseek(f, 0, SEEK_END);
  if ((size_t)ftell(f) != n * w0 * 4) { fclose(f); throw std::runtime_error("recover: " + path + " has the wrong size"); }
  fseek(f, 0, SEEK_SET);
  const size_t batch = 1 << 16;
  std::vector<uint32_t> in(batch * w0);
  for (size_t r0 = 0; r0 < n; r0 += batch) {
    const size_t k = std::min(batch, n - r0);
    if (fread(in.data(), 4, k * w0, f) != k * w0) { fclose(f); throw std::runtime_error("recover: short read from " + path); }
    h.append_fixed_host(in.data(), k, w0, hdr_words, pool);
  }
  fclose(f);
}
// Every snap-* subdirectory of dir but `keep` (an interrupted rotation, or a
// snapshot of another model whose meta was replaced, leaves them behind).
static void ckpt_remove_stale(const std::string& dir, unsigned long long keep) {
  std::vector<std::string> stale;
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) {
      std::string n = e->d_name;
      if (n.rfind("snap-", 0) == 0 && n != ckpt_subdir(keep)) stale.push_back(n);
    }
    closedir(d);
  }
  for (auto& n : stale) remove_tree(dir + "/" + n);
}
static void ckpt_write_meta(const std::string& dir, const rmc_model* m, const Ckpt& c) {
  const std::string path = dir + "/checkpoint.meta", tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "w");
  if (!f) throw std::runtime_error("checkpoint: cannot write " + tmp);
  fprintf(f, "raftmc-checkpoint 2\nmodule %s\nsnapshot %llu\nsignature %016llx\nkmax %u\nfpw %d\nslots %llu\n"
             "generated %llu\ndistinct %llu\ndepth %u\ncur_base %llu\ncur_n %llu\nhidden %llu\nrate %.17g\n"
             "levels %zu\n",
          m->module.c_str(), c.seq, c.sig, c.kmax, c.fpw, c.slots, c.generated, c.distinct, c.depth, c.cur_base,
          c.cur_n, c.hidden, c.rate, c.levels.size());
  for (auto& l : c.levels) fprintf(f, "%llu %llu\n", l.first, l.second);
  if (fflush(f) != 0 || fsync(fileno(f)) != 0) { fclose(f); throw std::runtime_error("checkpoint: cannot sync " + tmp); }
  if (fclose(f) != 0 || rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("checkpoint: cannot finish " + path);
  fsync_dir(dir);
}
static Ckpt ckpt_read_meta(const std::string& dir, const rmc_model* m) {
  const std::string path = dir + "/checkpoint.meta";
  FILE* f = fopen(path.c_str(), "r");
  if (!f) throw std::runtime_error("recover: no checkpoint in " + dir + " (" + path + " missing)");
  Ckpt c;
  char module[128] = {0};
  int ver = 0;
  size_t nl = 0;
  int ok = fscanf(f, "raftmc-checkpoint %d module %127s snapshot %llu signature %llx kmax %u fpw %d slots %llu "
                     "generated %llu distinct %llu depth %u cur_base %llu cur_n %llu hidden %llu rate %lg levels %zu",
                  &ver, module, &c.seq, &c.sig, &c.kmax, &c.fpw, &c.slots, &c.generated, &c.distinct, &c.depth,
                  &c.cur_base, &c.cur_n, &c.hidden, &c.rate, &nl);
  if (ok >= 1 && ver != 2) {
    fclose(f);
    throw std::runtime_error("recover: " + path + " is checkpoint format version " + std::to_string(ver) +
                             "; this build reads version 2 (resume it with the build that wrote it)");
  }
  if (ok != 15) { fclose(f); throw std::runtime_error("recover: unreadable " + path + " (format version 2 expected)"); }
  for (size_t k = 0; k < nl; k++) {
    unsigned long long g = 0, d = 0;
    if (fscanf(f, "%llu %llu", &g, &d) != 2) { fclose(f); throw std::runtime_error("recover: unreadable " + path); }
    c.levels.push_back({g, d});
  }
  fclose(f);
  if (m->module != module) throw std::runtime_error(std::string("recover: the checkpoint is of module ") + module);
  return c;
}

// The auto switch's threshold: a next level projected past this fraction of
// HBM moves the levels to the host at a level boundary (RMC_HF_HBM_FRACTION,
// default 0.25; tests lower it to exercise the switch on small configs).
double hf_hbm_fraction() {
  if (const char* e = getenv("RMC_HF_HBM_FRACTION")) return atof(e);
  return 0.25;
}

size_t host_frontier_limit() {
  if (const char* e = getenv("RMC_HOST_FRONTIER_GIB")) return (size_t)(atof(e) * 1073741824.0);
  unsigned long long avail_kb = 0;
  if (FILE* f = fopen("/proc/meminfo", "r")) {
    char line[256];
    while (fgets(line, sizeof line, f))
      if (sscanf(line, "MemAvailable: %llu kB", &avail_kb) == 1) break;
    fclose(f);
  }
  const size_t avail = (size_t)avail_kb * 1024;
  return std::min<size_t>(avail / 5 * 4, 200ULL << 30);
}

// The copy streams and events of the host frontier, created on first use:
// parents in (H2D) on `cs`, new rows out (D2H) on `co`, so the two directions
// of the PCIe link run at once instead of queueing behind each other.
// The compact rows are packed on `cp` (after the chunk's k_materialize:
// event mat; packed = the output window is free again), then copied out on
// `co` (event out = the pack buffer is free again).
struct HostFrontierStreams {
  hipStream_t cs = nullptr, co = nullptr, cp = nullptr;
  hipEvent_t in[2], mat[2], out[2], packed[2];
  void init(hipStream_t compute) {
    if (cs) return;
    HIPCHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&co, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&cp, hipStreamNonBlocking));
    for (int k = 0; k < 2; k++) {
      for (hipEvent_t* e : {&in[k], &mat[k], &out[k], &packed[k]}) {
        HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
        HIPCHK(hipEventRecord(*e, compute));
      }
    }
  }
  void sync() {
    if (!cs) return;
    HIPCHK(hipStreamSynchronize(cs));
    HIPCHK(hipStreamSynchronize(cp));
    HIPCHK(hipStreamSynchronize(co));
  }
  ~HostFrontierStreams() {
    if (!cs) return;
    (void)hipStreamSynchronize(cs);
    (void)hipStreamSynchronize(cp);
    (void)hipStreamSynchronize(co);
    for (int k = 0; k < 2; k++)
      for (hipEvent_t e : {in[k], mat[k], out[k], packed[k]}) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(cp);
    (void)hipStreamDestroy(co);
    (void)hipStreamDestroy(cs);
  }
};

int check_impl(rmc_model* m, const rmc_options* opt_in, rmc_result* res) {
  auto t0 = std::chrono::steady_clock::now();
  rmc_options opt_v = *opt_in;  // RMC_VERBOSE=1: per-level progress from any caller (bench.py, tests)
  if (getenv("RMC_VERBOSE") && atoi(getenv("RMC_VERBOSE")) > 0) opt_v.verbose = 1;
  const rmc_options* opt = &opt_v;
  Model& M = m->M;
  if (opt->deadlock_check) throw std::runtime_error("deadlock checking is not supported; run with -deadlock (README.md:6)");
  if (opt->fp_bits && opt->fp_bits != 64 && opt->fp_bits != 128)
    throw std::runtime_error("fp_bits must be 64 or 128");
  if (opt->fp_bits == 128 && m->M.gany)
    throw std::runtime_error("a model with compiled guards is checked with 64-bit fingerprints");
  // Rows widen in place while the levels are on the device (below: a chunk
  // whose successors need more message slots widens the current and next
  // level's rows and is redone), so a model checked for the first time starts
  // with rows for N messages and grows them to the search's real maximum;
  // a host-frontier check (whose levels re-run on an overflow) starts at the
  // constants-based default.
  const bool widen_ok = !opt->msg_cap_K && opt->host_frontier != 1 && !(opt->recover_dir && *opt->recover_dir);
  uint32_t kmax = opt->msg_cap_K ? opt->msg_cap_K
                                 : m->kmax_user ? m->kmax_user
                                 : m->hint_kmax ? m->hint_kmax
                                 : widen_ok     ? (uint32_t)m->M.N
                                                : default_kmax(m->M);
  if (kmax > 120) kmax = 120;
  const bool recovering = opt->recover_dir && *opt->recover_dir;
  Ckpt rc;
  size_t snap_words = 0;  // row width of the snapshot's frontier file
  if (recovering) {  // verified against the snapshot's own row layout
    rc = ckpt_read_meta(opt->recover_dir, m);
    finalize_model(m, rc.kmax);
    M.fpw = opt->fp_bits == 128 ? 2 : 1;
    if (M.kmax != (int)rc.kmax || M.fpw != rc.fpw || model_signature(m) != rc.sig)
      throw std::runtime_error(std::string("recover: the checkpoint in ") + opt->recover_dir +
                               " is of a different model, constants or fingerprint width");
    snap_words = (size_t)M.words;
    // a resumed level that overflowed the snapshot's message capacity re-runs
    // from the same snapshot with more slots (its rows are widened on load)
    kmax = std::max(kmax, rc.kmax);
  }
  finalize_model(m, kmax);
  M.fpw = opt->fp_bits == 128 ? 2 : 1;
  const int ew = 2 * M.fpw;  // fingerprint-set entry width in 64-bit words
  HIPCHK(upload_model(M));
  hipStream_t stream;
  HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  // Two chunks in flight while the frontiers are on the device: chunk i's
  // k_materialize runs on mstream beside chunk i+1's k_expand / k_mark / scan
  // on `stream` (k_materialize touches neither the fingerprint set nor the
  // arrays of the chunk being expanded; chunk i+1's inserts carry larger
  // ranks than chunk i's, so they cannot change a chunk-i winner).  The
  // per-chunk arrays alternate between two sets.  Opt-in (RMC_OVERLAP=1):
  // measured on the bench workload (profiles/r04/bench_r04o_*.json) the two
  // kernels contend for the same memory system -- overlapped, k_expand takes
  // 1,057 ms per check instead of 755 and k_materialize 420 instead of 347 --
  // and the check gains 0.5% (1.216-1.219 s vs 1.223-1.224 s) for a second
  // 7.6 GB candidate set.
  const bool pipe = opt->host_frontier != 1 && getenv("RMC_OVERLAP") && atoi(getenv("RMC_OVERLAP")) > 0;
  hipStream_t mstream = stream;
  hipEvent_t matdone[2] = {nullptr, nullptr}, ev_scan = nullptr;
  if (pipe) {
    HIPCHK(hipStreamCreateWithFlags(&mstream, hipStreamNonBlocking));
    for (hipEvent_t* e : {&matdone[0], &matdone[1], &ev_scan}) HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  struct MStreamGuard {
    hipStream_t s, m;
    hipEvent_t* ev;
    ~MStreamGuard() {
      if (m != s) {
        (void)hipStreamSynchronize(m);
        (void)hipStreamDestroy(m);
      }
      for (int i = 0; i < 3; i++)
        if (ev[i]) (void)hipEventDestroy(ev[i]);
    }
  };
  hipEvent_t evs[3] = {matdone[0], matdone[1], ev_scan};
  MStreamGuard mguard{stream, mstream, evs};
  size_t W = (size_t)M.words;  // row width (words); grows when the rows widen
  const auto t_model = std::chrono::steady_clock::now();

  // ---- sizing
  // Fingerprint set: starts at hash_slots (or at the size the last check of
  // this model ended with -- TLC's preallocated FPSet, -fpmem, in spirit) and
  // doubles before a chunk whose new states could take it past 0.75 load.
  unsigned long long slots = opt->hash_slots ? opt->hash_slots : std::max(1ULL << 26, m->hint_slots);
  if (recovering) slots = rc.slots;
  if (slots & (slots - 1)) throw std::runtime_error("hash_slots must be a power of two");
  unsigned long long fcap = opt->frontier_cap ? opt->frontier_cap : std::max(1ULL << 22, m->hint_fcap);
  size_t hbm_total = 0;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceTotalMem(&hbm_total, dev);
  }
  // A snapshot whose level is past the auto switch's threshold (or one
  // resumed with host_frontier = 1) resumes on the host: its rows stream from
  // the file into pinned pages and never need device frontiers of that size.
  const bool rec_host = recovering && opt->host_frontier != -1 &&
                        (opt->host_frontier == 1 ||
                         (hbm_total && (double)rc.cur_n * std::max(rc.rate, 1.0) * 1.25 * (double)(W * 4) >
                                           hf_hbm_fraction() * (double)hbm_total) ||
                         getenv("RMC_RECOVER_TO_HOST"));  // test hook
  if (recovering && !rec_host) fcap = std::max(fcap, rc.cur_n);
  int maxsucc = max_successors(M);
  // 8M parents per launch (bench cfg: 1.325 s per check vs 1.349 s at 4M; 4M
  // was 4% below 2M, 2M 4% below 1M), held to 2^31 candidates per launch
  unsigned long long chunk = opt->chunk_parents
                                 ? opt->chunk_parents
                                 : std::min(1ULL << 23, (1ULL << 31) / (unsigned long long)std::min(maxsucc, 256) - 1024);
  // + 1024 parents of slack: each of k_expand's 8 candidate segments must hold 1/8 of the tiles, rounded up
  unsigned long long cand_cap = (chunk + 1024) * (unsigned long long)std::min(maxsucc, 256);
  // candidate indices (par_off, k_mark, k_materialize's winner list) are 32-bit
  if (cand_cap > 0xFFFFFFFFULL)
    throw std::runtime_error("chunk_parents too large: " + std::to_string(chunk) + " parents x " +
                             std::to_string(std::min(maxsucc, 256)) + " bindings exceeds 2^32 candidates per launch");

  // Device buffers persist per device across checks (grow-only), so repeated
  // checks do not pay hipMalloc/hipFree of tens of GB each time.
  Arena& A = arena_for_current_device();
  DevBuf &table = A.table, &cslot = A.cslot, &cob = A.cob, &cwin = A.cwin;
  DevBuf &poff = A.poff, &pn = A.pn, &pwin = A.pwin, &ppos = A.ppos, &counters = A.counters, &stbuf = A.stbuf;
  DevBuf& scantmp = A.scantmp;
  GrowBuf &fa = A.fa, &fb = A.fb, &trp = A.trp, &trb = A.trb;
  table.ensure(slots * ew * 8);
  HIPCHK(hipMemsetAsync(table.p, 0xFF, slots * ew * 8, stream));
  if (opt->host_frontier != 1 && !rec_host) {
    fa.ensure(fcap * W * 4);
    fb.ensure(fcap * W * 4);
  } else {  // host levels: only Init (or a small recovered level) passes through the device
    fa.ensure((recovering && !rec_host ? std::max(1ULL, rc.cur_n) : 1ULL) * W * 4);
  }
  cslot.ensure(cand_cap * 8);
  cob.ensure(cand_cap * 4);
  cwin.ensure(cand_cap * 2);
  poff.ensure(chunk * 4);
  pn.ensure(chunk * 4);
  pwin.ensure(chunk * 4);
  ppos.ensure(chunk * 4);
  counters.ensure(1024);  // 8 per-XCD candidate counters, 128 B apart (k_expand)
  stbuf.ensure(sizeof(DevStatus));
  A.stmat.ensure(sizeof(DevStatus));
  if (pipe && !rec_host) {
    A.cslot2.ensure(cand_cap * 8);
    A.cob2.ensure(cand_cap * 4);
    A.cwin2.ensure(cand_cap * 2);
    for (DevBuf* b : {&A.poff2, &A.pn2, &A.pwin2, &A.ppos2}) b->ensure(chunk * 4);
    A.counters2.ensure(1024);
  }
  DevBuf* const set_cslot[2] = {&cslot, &A.cslot2};
  DevBuf* const set_cob[2] = {&cob, &A.cob2};
  DevBuf* const set_cwin[2] = {&cwin, &A.cwin2};
  DevBuf* const set_poff[2] = {&poff, &A.poff2};
  DevBuf* const set_pn[2] = {&pn, &A.pn2};
  DevBuf* const set_pwin[2] = {&pwin, &A.pwin2};
  DevBuf* const set_ppos[2] = {&ppos, &A.ppos2};
  DevBuf* const set_counters[2] = {&counters, &A.counters2};
  if (!A.hrb) HIPCHK(hipHostMalloc((void**)&A.hrb, sizeof(HostReadback), hipHostMallocDefault));
  HostReadback* const hrb = A.hrb;
  size_t stb = scan_temp_bytes(chunk);
  scantmp.ensure(stb ? stb : 16);
  unsigned long long trcap = std::max(fcap * 4, m->hint_trcap);
  if (recovering) trcap = std::max(trcap, rc.distinct + rc.distinct / 4);
  trp.ensure(trcap * 8);
  trb.ensure(trcap * 2);

  DevStatus hst;
  auto reset_status = [&]() {
    hst.err_key = hst.inv_err_key = hst.viol_key = ~0ULL;
    hst.cap_flags = 0;
    hst.max_msgs = 0;
    hst.hidden_coll = 0;
    hst.row_words = 0;
    HIPCHK(hipMemcpyAsync(stbuf.p, &hst, sizeof hst, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(A.stmat.p, &hst, sizeof hst, hipMemcpyHostToDevice, stream));
  };
  reset_status();
  HIPCHK(hipStreamSynchronize(stream));
  const auto t_setup = std::chrono::steady_clock::now();
  if (opt->verbose)
    fprintf(stderr, "[rmc] setup: runtime + model upload %.3fs, buffers %.3fs (fingerprint set 2^%d slots)\n",
            std::chrono::duration<double>(t_model - t0).count(),
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t_model).count(), __builtin_ctzll(slots));

  auto now = [] { return std::chrono::steady_clock::now(); };
  auto secs = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double>(b - a).count();
  };
  double rehash_s = 0, grow_s = 0;
  double tg_alloc_s = 0, tg_fill_s = 0, tg_rehash_s = 0;  // table growth by step (rmc_check_phases)

  // ---- growth: room for `need` entries at <= 0.75 load (0.9 once HBM is full)
  bool full_ok = false;
  unsigned long long grows = 0;

  // ---- level 1: Init (Raft.tla:213-218)
  std::vector<uint32_t> init = init_state(M);
  if (!recovering) HIPCHK(hipMemcpyAsync(fa.p, init.data(), W * 4, hipMemcpyHostToDevice, stream));
  if (!recovering) {
    unsigned long long ent[4];
    if (M.fpw == 2) {
      host_fingerprint2(M, init.data(), ent);  // (a, b)
      ent[2] = 0ULL;                           // val 0: older than every successor
      ent[3] = ~0ULL;
    } else {
      ent[0] = host_fingerprint(M, init.data());
      if (ent[0] == ~0ULL) ent[0]--;
      ent[1] = 0ULL;
    }
    HIPCHK(hipMemcpyAsync(table.as<unsigned long long>() + ew * fp_slot(ent[0], slots - 1), ent, ew * 8,
                          hipMemcpyHostToDevice, stream));
    unsigned long long root = ~0ULL;
    uint16_t zero = 0;
    HIPCHK(hipMemcpyAsync(trp.p, &root, 8, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(trb.p, &zero, 2, hipMemcpyHostToDevice, stream));
  }
  HIPCHK(hipStreamSynchronize(stream));
  m->levels.clear();
  m->trace_states.clear();
  m->trace_actions.clear();
  m->widenings.clear();
  m->hf_pack_regrows = m->hf_out_regrows = 0;
  unsigned long long generated = 1, distinct = 1, cur_n = 1, cur_base = 0;
  unsigned depth = 1;
  m->levels.push_back({1, 1});
  int status = 0;
  std::string message;
  unsigned long long bad_state = ~0ULL;  // global index of the violating / erroring state, if materialized
  unsigned long long bad_key = ~0ULL;
  bool bad_is_parent_key = false;
  // pinned staging for checkpoint files (allocated on first use)
  void* ck_stage = nullptr;
  const size_t ck_stage_bytes = 64ULL << 20;
  struct StageGuard {
    void*& p;
    ~StageGuard() { if (p) (void)hipHostFree(p); }
  } ck_guard{ck_stage};
  auto stage = [&]() {
    if (!ck_stage) HIPCHK(hipHostMalloc(&ck_stage, ck_stage_bytes, hipHostMallocDefault));
    return ck_stage;
  };
  if (recovering) {  // resume from the snapshot instead of Init
    const std::string dir = std::string(opt->recover_dir) + "/" + ckpt_subdir(rc.seq);
    ckpt_read(dir + "/fpset.bin", table.p, slots * ew * 8, stage(), ck_stage_bytes);
    if (!rec_host)  // else streamed into host pages below, once they exist
      ckpt_read_rows(dir + "/frontier.bin", fa.as<uint32_t>(), rc.cur_n, snap_words, W, stage(), ck_stage_bytes);
    ckpt_read(dir + "/trace_parent.bin", trp.p, rc.distinct * 8, stage(), ck_stage_bytes);
    ckpt_read(dir + "/trace_bind.bin", trb.p, rc.distinct * 2, stage(), ck_stage_bytes);
    generated = rc.generated;
    distinct = rc.distinct;
    cur_n = rc.cur_n;
    cur_base = rc.cur_base;
    depth = rc.depth;
    m->levels = rc.levels;
    hst.hidden_coll = rc.hidden;
    HIPCHK(hipMemcpyAsync((char*)stbuf.p + offsetof(DevStatus, hidden_coll), &hst.hidden_coll, 8,
                          hipMemcpyHostToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }
  if (!recovering) {
    int err = 0;
    int bad = host_check_invariants(M, init.data(), &err);
    if (err) { status = 2; message = "evaluation error in an invariant on the initial state"; bad_state = 0; }
    else if (bad >= 0) { status = 1; snprintf(res->violated, sizeof res->violated, "%s", m->inv_names[bad].c_str()); bad_state = 0; }
  }
  EventTimer te, tm, tz;
  double expand_ms = 0, mark_ms = 0, mat_ms = 0;
  double launch_s = 0;  // host time inside the kernel launch calls (a fresh process loads the code objects there)
  unsigned mat_max_msgs = 0;  // k_materialize's largest |DOMAIN messages| (its own status buffer)
  unsigned long long expand_launches = 0, redos = 0;
  // hidden-variable collisions counted up to the last chunk that was kept: a
  // redone chunk's first k_mark has counted its collisions once already
  unsigned long long coll_kept = recovering ? rc.hidden : 0;
  auto restore_coll = [&]() {
    HIPCHK(hipMemcpyAsync((char*)stbuf.p + offsetof(DevStatus, hidden_coll), &coll_kept, 8, hipMemcpyHostToDevice,
                          stream));
  };
  uint32_t* cur = fa.as<uint32_t>();
  uint32_t* nxt = fb.as<uint32_t>();
  // ---- host frontier (rmc_options.host_frontier: -1 never, 0 when HBM runs
  // out, 1 always): the current and next level live in pinned host pages and
  // stream through two input and two output windows in HBM; the fingerprint
  // set and the trace records stay on the device.
  const int hf_opt = opt->host_frontier;
  bool hf = false;
  HostPagePool pool;
  size_t row_bytes = W * 4;
  size_t page_bytes = HostPagePool::PAGE_BYTES;
  // test hooks: RMC_HOST_PAGE_ROWS (small pages: rows straddle many), and
  // RMC_HOST_FRONTIER_AT=L (auto mode moves to the host before level L's
  // second chunk) or L:grow (as if the next-level buffer's growth ran out of
  // HBM in that chunk)
  if (const char* e = getenv("RMC_HOST_PAGE_ROWS")) page_bytes = (size_t)std::max<long long>(1, atoll(e)) * row_bytes;
  unsigned hf_force_level = 0;
  bool hf_force_grow = false;
  if (const char* e = getenv("RMC_HOST_FRONTIER_AT")) {
    hf_force_level = (unsigned)atoi(e);
    hf_force_grow = strstr(e, ":grow") != nullptr;
  }
  pool.page_bytes = page_bytes;
  pool.limit = host_frontier_limit();
  // pinning threads and the pages they keep ready (RMC_HF_PIN_THREADS,
  // RMC_HF_PIN_AHEAD; 0 threads = pin on demand in the BFS thread)
  int hf_pin_threads = 4;
  size_t hf_pin_ahead = 32;
  if (const char* e = getenv("RMC_HF_PIN_THREADS")) hf_pin_threads = atoi(e);
  if (const char* e = getenv("RMC_HF_PIN_AHEAD")) hf_pin_ahead = (size_t)atoll(e);
  HostLevel hcur, hnxt;
  hcur.init(pool.page_bytes, row_bytes);
  hnxt.init(pool.page_bytes, row_bytes);
  struct LevelPagesGuard {  // every exit path returns the levels' pages to the pool (freed with it)
    HostLevel &a, &b;
    HostPagePool& pool;
    ~LevelPagesGuard() { a.clear(pool); b.clear(pool); }
  } level_pages_guard{hcur, hnxt, pool};
  HostFrontierStreams hs;
  unsigned long long hwin_c0[2] = {~0ULL, ~0ULL};  // first row of the chunk each input window holds
  unsigned long long lvl_c0 = 0, lvl_next_n = 0;   // chunk-loop position (for a switch to the host frontier)
  double hf_copy_s = 0;
  // The host-frontier windows (two of a chunk's parents, two of 3 rows per
  // parent), allocated while HBM still has room: in the auto mode as soon as a
  // growth would leave less than their size free.  HBM the device frontiers
  // release when the search moves to the host is not reusable at once on this
  // driver (a hipMalloc right after hipMemRelease of the frontiers failed on
  // the GPU box; profiles/r03/vmm_release_probe.txt), so the windows must not
  // depend on it.
  size_t win_in_bytes = chunk * W * 4, win_out_bytes = 3 * chunk * W * 4;
  bool windows = false;
  struct WindowsGuard {  // every exit path (an E_CAP_MSG re-run, a throw, auto mode that never switched)
    Arena& A;
    bool& windows;
    ~WindowsGuard() {
      if (windows) A.release_hf();
    }
  } windows_guard{A, windows};
  // ---- compact host rows (HostLevel): pack before D2H, unpack after H2D
  const int hdr_words = 1 + 4 * M.N;
  // A buffer that is about to be freed and regrown must have no copy or kernel
  // of the copy streams still using it: the wait for it is explicit at each
  // call site (hf_pack_async, the output windows), and this makes a missing
  // one an error naming the buffer instead of a GPU fault.
  auto hf_idle = [&](hipEvent_t e, const char* what) {
    if (!hs.cs) return;  // the copy streams are not running yet
    const hipError_t q = hipEventQuery(e);
    if (q == hipErrorNotReady)
      throw std::logic_error(std::string("host frontier: ") + what + " regrown while a copy still uses it");
    if (q != hipSuccess) HIPCHK(q);
  };
  auto hf_ensure_out = [&](int k, unsigned long long n) {
    if (A.hf_pack[k].p && A.hf_pack[k].bytes < std::max<size_t>(n * W * 4, 16)) {
      hf_idle(hs.out[k], "a compact-row pack buffer");  // its last copy-out (hs.co)
      hf_idle(hs.packed[k], "a compact-row pack buffer");  // its last pack (hs.cp)
      if (hs.cs) m->hf_pack_regrows++;  // while copy-outs run (the r05 fault's path)
    }
    A.hf_pack[k].ensure(std::max<size_t>(n * W * 4, 16));
    A.hf_olen32[k].ensure(std::max<size_t>(n * 4, 16));
    A.hf_olen8[k].ensure(std::max<size_t>(n, 16));
    A.hf_ooff[k].ensure(std::max<size_t>(n * 4, 16));
    A.hf_oscan[k].ensure(std::max<size_t>(scan_temp_bytes(n), 16));
  };
  auto hf_ensure_in = [&](int k, unsigned long long n) {
    if (A.hf_stage[k].p && A.hf_stage[k].bytes < std::max<size_t>(n * W * 4, 16))
      hf_idle(hs.in[k], "an input staging buffer");  // its last load (hs.cs)
    A.hf_stage[k].ensure(std::max<size_t>(n * W * 4, 16));
    A.hf_ilen32[k].ensure(std::max<size_t>(n * 4, 16));
    A.hf_ilen8[k].ensure(std::max<size_t>(n, 16));
    A.hf_ioff[k].ensure(std::max<size_t>(n * 4, 16));
    A.hf_iscan[k].ensure(std::max<size_t>(scan_temp_bytes(n), 16));
  };
  // rows [r0, r0 + n) of a host level -> fixed-stride rows at dev (on stream st, with input buffers k)
  auto hf_load = [&](const HostLevel& h, unsigned long long r0, unsigned long long n, void* dev, int k,
                     hipStream_t st) {
    if (!n) return;
    hf_ensure_in(k, n);
    const unsigned long long b0 = h.byte_of(r0), b1 = h.byte_of(r0 + n);
    h.copy_in(b0, b1 - b0, A.hf_stage[k].p, st);
    HIPCHK(hipMemcpyAsync(A.hf_ilen8[k].p, h.lens.data() + r0, n, hipMemcpyHostToDevice, st));
    launch_widen_lens(A.hf_ilen8[k].as<uint8_t>(), n, A.hf_ilen32[k].as<uint32_t>(), st);
    launch_scan(A.hf_iscan[k].p, A.hf_iscan[k].bytes, A.hf_ilen32[k].as<uint32_t>(), A.hf_ioff[k].as<uint32_t>(), n,
                st);
    launch_unpack_rows(A.hf_stage[k].as<uint32_t>(), n, (int)W, A.hf_ioff[k].as<uint32_t>(),
                       A.hf_ilen32[k].as<uint32_t>(), (uint32_t*)dev, st);
    HIPCHK(hipGetLastError());
  };
  bool hf_flag_ready = false;  // A.hf_flag zeroed for this check
  auto hf_flag_init = [&]() {
    if (hf_flag_ready) return;
    A.hf_flag.ensure(16);
    HIPCHK(hipMemsetAsync(A.hf_flag.p, 0, 16, stream));
    HIPCHK(hipStreamSynchronize(stream));
    hf_flag_ready = true;
  };
  // n fixed rows on the device -> appended to a host level (synchronous, in slices; the switch to the host)
  auto hf_from_device = [&](HostLevel& h, const uint32_t* rows, unsigned long long n) {
    if (!n) return;
    DevBuf local[5];
    const bool have = A.hf_pack[0].p != nullptr;
    unsigned long long S = have ? A.hf_pack[0].bytes / (W * 4) : std::max<unsigned long long>(1, (256ULL << 20) / (W * 4));
    S = std::max<unsigned long long>(1, std::min<unsigned long long>(S, 1ULL << 24));
    DevBuf& pk = have ? A.hf_pack[0] : local[0];
    DevBuf& l32 = have ? A.hf_olen32[0] : local[1];
    DevBuf& l8 = have ? A.hf_olen8[0] : local[2];
    DevBuf& off = have ? A.hf_ooff[0] : local[3];
    DevBuf& sc = have ? A.hf_oscan[0] : local[4];
    pk.ensure(S * W * 4);
    l32.ensure(S * 4);
    l8.ensure(S);
    off.ensure(S * 4);
    sc.ensure(std::max<size_t>(scan_temp_bytes(S), 16));
    std::vector<uint8_t> l;
    hf_flag_init();
    for (unsigned long long r = 0; r < n; r += S) {
      const unsigned long long k = std::min(S, n - r);
      launch_row_words(rows + r * W, k, (int)W, hdr_words, HostRowsIO::max_words(W), l32.as<uint32_t>(),
                       l8.as<uint8_t>(), A.hf_flag.as<unsigned>(), stream);
      launch_scan(sc.p, sc.bytes, l32.as<uint32_t>(), off.as<uint32_t>(), k, stream);
      launch_pack_rows(rows + r * W, k, (int)W, off.as<uint32_t>(), l32.as<uint32_t>(), pk.as<uint32_t>(), stream);
      HIPCHK(hipGetLastError());
      l.resize(k);
      HIPCHK(hipMemcpyAsync(l.data(), l8.p, k, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipStreamSynchronize(stream));
      h.append_dev(l.data(), k, pk.p, pk.bytes, stream, pool);
      HIPCHK(hipStreamSynchronize(stream));
    }
  };
  // the chunk's new rows (output window k, n rows) are packed on cp after its
  // k_materialize; their bytes are appended to hnxt at the next host sync
  // point (hf_flush), when the compact sizes are known
  struct PendingOut { bool on; int k; unsigned long long n; } hf_pend{false, 0, 0};
  auto hf_pack_async = [&](int k, unsigned long long n) {
    // the pack buffer k is still the source of chunk ck-2's copy-out (hs.co):
    // a regrowth waits for it (DevBuf::alloc also drains the device)
    if (A.hf_pack[k].bytes < std::max<size_t>(n * W * 4, 16)) HIPCHK(hipEventSynchronize(hs.out[k]));
    hf_ensure_out(k, n);
    HIPCHK(hipStreamWaitEvent(hs.cp, hs.mat[k], 0));  // the rows are written
    HIPCHK(hipStreamWaitEvent(hs.cp, hs.out[k], 0));  // the pack buffer's last copy-out is done
    launch_row_words(A.hwin_out[k].as<uint32_t>(), n, (int)W, hdr_words, HostRowsIO::max_words(W),
                     A.hf_olen32[k].as<uint32_t>(), A.hf_olen8[k].as<uint8_t>(), A.hf_flag.as<unsigned>(), hs.cp);
    launch_scan(A.hf_oscan[k].p, A.hf_oscan[k].bytes, A.hf_olen32[k].as<uint32_t>(), A.hf_ooff[k].as<uint32_t>(), n,
                hs.cp);
    launch_pack_rows(A.hwin_out[k].as<uint32_t>(), n, (int)W, A.hf_ooff[k].as<uint32_t>(),
                     A.hf_olen32[k].as<uint32_t>(), A.hf_pack[k].as<uint32_t>(), hs.cp);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(hs.packed[k], hs.cp));
    hf_pend = {true, k, n};
  };
  std::vector<uint8_t> hf_lens_tmp;
  auto hf_flush = [&]() {
    if (!hf_pend.on) return;
    hf_pend.on = false;
    HIPCHK(hipEventSynchronize(hs.packed[hf_pend.k]));
    hf_lens_tmp.resize(hf_pend.n);
    HIPCHK(hipMemcpy(hf_lens_tmp.data(), A.hf_olen8[hf_pend.k].p, hf_pend.n, hipMemcpyDeviceToHost));
    hnxt.append_dev(hf_lens_tmp.data(), hf_pend.n, A.hf_pack[hf_pend.k].p, A.hf_pack[hf_pend.k].bytes, hs.co, pool);
    HIPCHK(hipEventRecord(hs.out[hf_pend.k], hs.co));
  };
  auto reserve_windows = [&]() {
    if (windows) return;
    A.hwin_in[0].ensure(win_in_bytes);
    A.hwin_in[1].ensure(win_in_bytes);
    A.hwin_out[0].ensure(win_out_bytes);
    A.hwin_out[1].ensure(win_out_bytes);
    for (int k = 0; k < 2; k++) {  // the compact-row buffers (pack out, unpack in)
      hf_ensure_out(k, 3 * chunk);
      hf_ensure_in(k, chunk);
    }
    hf_flag_init();
    windows = true;
  };
  auto before_growth = [&](size_t request) {  // auto mode: keep the windows' HBM available
    if (hf || windows || hf_opt != 0) return;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return;
    const size_t wb = 4 * (win_in_bytes + win_out_bytes);  // windows + the compact-row buffers
    if (fr < request + wb + (2ULL << 30)) {
      try {
        reserve_windows();
      } catch (OutOfDeviceMemory&) {
      }
      if (opt->verbose)
        fprintf(stderr, "[rmc] host-frontier windows %s (%.1f GiB)\n", windows ? "reserved" : "could not be reserved",
                wb / 1073741824.0);
    }
  };
  // Move the current level (all of it) and the next level so far to host
  // pages, free the device frontiers, and continue in host-frontier mode.
  auto enter_hf = [&]() {
    auto th0 = std::chrono::steady_clock::now();
    HIPCHK(hipStreamSynchronize(stream));
    HIPCHK(hipStreamSynchronize(mstream));  // the chunk in flight has written its rows
    try {  // while the device frontiers still hold their HBM (see reserve_windows)
      reserve_windows();
    } catch (OutOfDeviceMemory&) {
    }
    hs.init(stream);
    pool.start_fillers(hf_pin_ahead, hf_pin_threads);
    hcur.init(pool.page_bytes, row_bytes);
    hnxt.init(pool.page_bytes, row_bytes);
    hf_from_device(hcur, cur, cur_n);
    hf_from_device(hnxt, nxt, lvl_next_n);
    if (lvl_c0 > chunk) hcur.recycle_below(lvl_c0 - chunk, pool);
    fa.release();
    fb.release();
    cur = nxt = nullptr;
    hf = true;
    hwin_c0[0] = hwin_c0[1] = ~0ULL;
    reserve_windows();
    hf_copy_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - th0).count();
    if (opt->verbose)
      fprintf(stderr, "[rmc] frontier moved to host memory at depth %u (%.1f GiB of pinned pages, limit %.1f GiB)\n",
              depth, pool.allocated / 1073741824.0, pool.limit / 1073741824.0);
  };
  // Growth threshold: 0.5 load while the set is at most 32 GiB (short probe
  // runs: at 0.75 a miss reads ~8 slots, 2-3 dependent 64 B groups), 0.75
  // beyond (HBM capacity matters more than probe length there).
  auto over_load = [&](unsigned long long need) {
    return slots * (unsigned long long)ew * 8 <= (32ULL << 30) ? need * 2 > slots : need * 4 > slots * 3;
  };
  auto t_grow = [&](unsigned long long nslots) {  // rehash into nslots (entries and values kept)
    auto tr0 = now();
    HIPCHK(hipStreamSynchronize(stream));
    bool grown = true;
    before_growth(nslots * ew * 8);
    try {
      A.table2.ensure(nslots * ew * 8);
    } catch (OutOfDeviceMemory&) {
      grown = false;
    }
    if (!grown) return false;
    const auto tr1 = now();
    HIPCHK(hipMemsetAsync(A.table2.p, 0xFF, nslots * ew * 8, stream));
    HIPCHK(hipStreamSynchronize(stream));
    const auto tr2 = now();
    launch_rehash(table.as<unsigned long long>(), slots, A.table2.as<unsigned long long>(), nslots - 1,
                  stbuf.as<DevStatus>(), stream, ew);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(stream));
    const auto tr3 = now();
    std::swap(table.p, A.table2.p);
    std::swap(table.bytes, A.table2.bytes);
    slots = nslots;
    if (A.table2.bytes >= (1ULL << 30)) A.table2.release();  // large searches need the HBM more than a spare
    grows++;
    rehash_s += secs(tr0, now());
    tg_alloc_s += secs(tr0, tr1);
    tg_fill_s += secs(tr1, tr2);
    tg_rehash_s += secs(tr2, tr3);
    if (opt->verbose)
      fprintf(stderr, "[rmc] fingerprint set grown to 2^%d slots (%.3fs: allocate %.3f, fill %.3f, rehash %.3f, free %.3f)\n",
              __builtin_ctzll(slots), secs(tr0, now()), secs(tr0, tr1), secs(tr1, tr2), secs(tr2, tr3), secs(tr3, now()));
    return true;
  };
  auto t_fit = [&](unsigned long long need) {
    if (!over_load(need)) return;
    if (!full_ok) {
      unsigned long long nslots = slots;
      // to <= 0.25 after growing while small (threshold 0.5), else to <= 0.5
      while (need * 2 > nslots || (nslots * (unsigned long long)ew * 8 <= (32ULL << 30) && need * 4 > nslots)) nslots <<= 1;
      if (t_grow(nslots)) return;
      if (!hf && hf_opt == 0) {  // the device frontiers give their HBM to the set
        enter_hf();
        if (t_grow(nslots)) return;
      }
      full_ok = true;
      if (opt->verbose) fprintf(stderr, "[rmc] fingerprint set stays at 2^%d slots (HBM full)\n", __builtin_ctzll(slots));
    }
    if (need * 10 > slots * 9) throw OutOfDeviceMemory("fingerprint set full (0.9 load) and HBM exhausted");
  };
  double rate = recovering ? rc.rate : 4.0;  // new states per parent of the previous level (pre-sizes the table per chunk)
  auto last_ckpt = now();
  // the level that stopped the search (exact counts at the failing state, below)
  struct ChunkLog { unsigned long long c0, gen_before, new_before; };
  std::vector<ChunkLog> chunk_log;
  unsigned long long stop_level_base = 0, stop_level_n = 0, stop_gen_before = 0, stop_dist_before = 0;
  const uint32_t* stop_front = nullptr;
  bool stop_hf = false;
  unsigned stop_level = 0;
  auto fill_args = [&](LevelArgs& a, unsigned long long c0, unsigned long long n, unsigned level,
                       const uint32_t* rows = nullptr, int set = 0) {
    memset(&a, 0, sizeof a);
    a.model = &M;
    a.frontier = rows ? rows : cur + c0 * W;
    a.nparents = n;
    a.pbase = cur_base + c0;
    a.level = level;
    a.floor = (cur_base + 1) << VAL_FLOOR_SHIFT;
    a.table = table.as<unsigned long long>();
    a.mask = slots - 1;
    a.cand_slot = set_cslot[set]->as<unsigned long long>();
    a.cand_ob = set_cob[set]->as<uint32_t>();
    a.cand_win = set_cwin[set]->as<uint16_t>();
    a.par_off = set_poff[set]->as<uint32_t>();
    a.par_n = set_pn[set]->as<uint32_t>();
    a.par_win = set_pwin[set]->as<uint32_t>();
    a.par_pos = set_ppos[set]->as<uint32_t>();
    a.counters = set_counters[set]->as<unsigned long long>();
    a.cand_cap = cand_cap;
    a.st = stbuf.as<DevStatus>();
  };
  // ---- widening the rows (device frontiers): chunk [c0, c0 + n) of the
  // current level met a successor with more messages than the rows hold.
  // The chunk is redone at a row width for `need` messages: its claimed
  // ranks go back to unclaimed (the message bindings' TLC ordinals depend on
  // the slot count: k_reset_ranks), the current level's rows and the next
  // level's rows so far are restrided (from the last row down, a slice at a
  // time through the candidate buffer, which the redo rewrites anyway), the
  // model's binding tables are rebuilt for the new slot count, and the
  // chunk's status goes back to the last kept chunk's.  Widenings per check:
  // a handful at small levels on a first check (rows start at N slots), none
  // when the model was checked before (its last maximum is the hint).
  unsigned widenings = 0;
  double widen_s = 0;
  auto widen = [&](unsigned need, unsigned long long c0, unsigned long long n) {
    auto tw0 = now();
    HIPCHK(hipStreamSynchronize(stream));
    if (mstream != stream) HIPCHK(hipStreamSynchronize(mstream));
    launch_reset_ranks(table.as<unsigned long long>(), slots, ew, (cur_base + c0 + 1) << 10,
                       (cur_base + c0 + n + 1) << 10, stream);
    HIPCHK(hipGetLastError());
    const size_t Wo = W;
    finalize_model(m, std::min(120u, need));
    M.fpw = opt->fp_bits == 128 ? 2 : 1;
    HIPCHK(upload_model(M));
    W = (size_t)M.words;
    auto restride = [&](uint32_t* rows, unsigned long long nr) {
      const unsigned long long slice = std::max<unsigned long long>(1, cslot.bytes / (Wo * 4));
      for (unsigned long long r1 = nr; r1 > 0;) {
        const unsigned long long r0 = r1 > slice ? r1 - slice : 0;
        HIPCHK(hipMemcpyAsync(cslot.p, rows + r0 * Wo, (r1 - r0) * Wo * 4, hipMemcpyDeviceToDevice, stream));
        launch_restride(cslot.as<uint32_t>(), r1 - r0, (int)Wo, (int)W, rows + r0 * W, stream);
        HIPCHK(hipGetLastError());
        r1 = r0;
      }
    };
    const bool cur_is_a = cur == fa.as<uint32_t>();
    GrowBuf& gc = cur_is_a ? fa : fb;
    GrowBuf& gn = cur_is_a ? fb : fa;
    gc.ensure(std::max<unsigned long long>(cur_n, 1) * W * 4);
    gn.ensure(std::max<unsigned long long>(lvl_next_n, 1) * W * 4);
    cur = gc.as<uint32_t>();
    nxt = gn.as<uint32_t>();
    restride(cur, cur_n);
    restride(nxt, lvl_next_n);
    maxsucc = max_successors(M);
    cand_cap = (chunk + 1024) * (unsigned long long)std::min(maxsucc, 256);
    if (cand_cap > 0xFFFFFFFFULL) throw std::runtime_error("widened rows: more than 2^32 candidates per launch");
    HIPCHK(hipStreamSynchronize(stream));  // the candidate buffer served as the slice buffer
    cslot.ensure(cand_cap * 8);
    cob.ensure(cand_cap * 4);
    cwin.ensure(cand_cap * 2);
    if (pipe) {
      A.cslot2.ensure(cand_cap * 8);
      A.cob2.ensure(cand_cap * 4);
      A.cwin2.ensure(cand_cap * 2);
    }
    row_bytes = W * 4;
    win_in_bytes = chunk * W * 4;
    win_out_bytes = 3 * chunk * W * 4;
    if (windows) {  // auto mode reserved the host-frontier windows at the narrower rows: widen them too
      windows = false;  // (no copy stream runs before the switch to the host: widen needs !hf)
      reserve_windows();
    }
    const unsigned zero = 0;
    const unsigned long long none = ~0ULL;
    HIPCHK(hipMemcpyAsync((char*)stbuf.p + offsetof(DevStatus, cap_flags), &zero, 4, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync((char*)stbuf.p + offsetof(DevStatus, err_key), &none, 8, hipMemcpyHostToDevice, stream));
    restore_coll();
    HIPCHK(hipStreamSynchronize(stream));
    widenings++;
    m->widenings.push_back({(unsigned long long)depth, c0, (unsigned long long)M.kmax});
    widen_s += secs(tw0, now());
    if (opt->verbose)
      fprintf(stderr, "[rmc] rows widened to %zu words (%d message slots) at depth %u, chunk at %llu (%.3fs)\n", W,
              M.kmax, depth, c0, secs(tw0, now()));
  };
  try {
  if (rec_host) {  // the snapshot's level goes straight to host pages
    auto th0 = std::chrono::steady_clock::now();
    HIPCHK(hipStreamSynchronize(stream));
    reserve_windows();
    hs.init(stream);
    pool.start_fillers(hf_pin_ahead, hf_pin_threads);
    hcur.init(pool.page_bytes, row_bytes);
    hnxt.init(pool.page_bytes, row_bytes);
    ckpt_read_rows_host(std::string(opt->recover_dir) + "/" + ckpt_subdir(rc.seq) + "/frontier.bin", hcur, pool,
                        rc.cur_n, snap_words, 1 + 4 * M.N);
    fa.release();
    fb.release();
    cur = nxt = nullptr;
    hf = true;
    hwin_c0[0] = hwin_c0[1] = ~0ULL;
    hf_copy_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - th0).count();
    if (opt->verbose)
      fprintf(stderr, "[rmc] recovered level of %llu states into host memory (%.1f GiB of pinned pages)\n", rc.cur_n,
              pool.allocated / 1073741824.0);
  }
  if (hf_opt == 1 && !hf) enter_hf();
  while (status == 0 && cur_n > 0) {
    if (opt->max_depth && (int)depth >= opt->max_depth) { status = 4; break; }
    if (opt->time_limit > 0 && secs(t0, now()) >= opt->time_limit) { status = 4; message = "time limit"; break; }
    // auto mode: a next level projected past a quarter of HBM moves the
    // levels to the host at this boundary, while the device frontiers are
    // still small -- their HBM is not reusable once released (§3), so a
    // later switch strands more of it
    if (!hf && hf_opt == 0 && hbm_total &&
        (double)cur_n * std::max(rate, 1.0) * 1.25 * (double)(W * 4) > hf_hbm_fraction() * (double)hbm_total) {
      lvl_c0 = 0;
      lvl_next_n = 0;
      enter_hf();
    }
    if (hf) A.release_set2();  // host-frontier chunks use one array set
    unsigned level = depth + 1;
    if (level >= 0xFFFF) throw std::runtime_error("too many levels");
    if (cur_base + cur_n + 1 >= (1ULL << 38)) throw std::runtime_error("more than 2^38 states (the TLC-order rank field)");
    unsigned long long next_n = 0, gen_lvl = 0;
    chunk_log.clear();
    hwin_c0[0] = hwin_c0[1] = ~0ULL;
    unsigned ck = 0;                       // chunk number within the level (host-frontier window parity)
    unsigned long long prev_c0 = 0;        // first row of the previous chunk (kept for the recount)
    // the last k_materialize's snapshot (hrb->mat) is not examined yet; call
    // after a stream sync.  True when it ended the search (status 3 set, or
    // hst holds the error/violation keys).
    bool mat_pending = false;
    // k_materialize's status buffer (stmat) is its own: its invariant keys
    // merge into hst here, its capacity flags end the search
    auto finish_mat = [&]() -> bool {
      mat_pending = false;
      float mms = 0;
      HIPCHK(hipEventElapsedTime(&mms, tz.a, tz.b));
      mat_ms += mms;
      const DevStatus& mt = hrb->mat;
      hst.inv_err_key = std::min(hst.inv_err_key, mt.inv_err_key);
      hst.viol_key = std::min(hst.viol_key, mt.viol_key);
      hst.err_key = std::min(hst.err_key, mt.err_key);
      mat_max_msgs = std::max(mat_max_msgs, mt.max_msgs);
      if (mt.cap_flags) {
        status = 3;
        message = "capacity overflow while materializing";
        return true;
      }
      return hst.err_key != ~0ULL || hst.inv_err_key != ~0ULL || hst.viol_key != ~0ULL;
    };
    auto sync_both = [&]() {
      HIPCHK(hipStreamSynchronize(stream));
      if (mstream != stream) HIPCHK(hipStreamSynchronize(mstream));
    };
    if (m->profile_level && level == m->profile_level && !hf) {
      // test hook (RMC_DIAG builds): k_expand on this level's first chunk,
      // stopped after each phase in turn; none of these launches inserts
      const unsigned long long n = std::min(chunk, cur_n);
      for (int dg : {4, 3, 2, 1})
        for (int rep = 0; rep < 3; rep++) {
          LevelArgs a;
          fill_args(a, 0, n, level);
          a.diag = dg;
          HIPCHK(hipMemsetAsync(counters.p, 0, 1024, stream));
          HIPCHK(hipEventRecord(te.a, stream));
          launch_expand(M.spec, M.N, a, stream);
          HIPCHK(hipGetLastError());
          HIPCHK(hipEventRecord(te.b, stream));
          HIPCHK(hipStreamSynchronize(stream));
          float ms = 0;
          HIPCHK(hipEventElapsedTime(&ms, te.a, te.b));
          m->profile_ms.push_back({dg, ms});
        }
    }
    unsigned long long c0 = 0;
    while (c0 < cur_n) {
      unsigned long long n = std::min(chunk, cur_n - c0);
      lvl_c0 = c0;
      lvl_next_n = next_n;
      if (!hf && hf_opt == 0 && !hf_force_grow && level == hf_force_level && c0 > 0) {
        if (mat_pending) {
          sync_both();
          if (finish_mat()) break;
        }
        enter_hf();
      }
      if (!opt->grow_on_overflow) {  // room for this chunk's new states (at the highest rate seen)
        const double r = std::max(rate, c0 ? (double)next_n / (double)c0 : 0.0);
        const unsigned long long need = distinct + next_n + (unsigned long long)((double)n * r * 1.25) + 1024;
        if (over_load(need)) {
          if (mat_pending) {  // the previous chunk may have ended the search: no growth for nothing
            sync_both();
            if (finish_mat()) break;
          }
          t_fit(need);
        }
      }
      const int hs_k = ck & 1;  // host frontier: this chunk's windows
      const bool pl = pipe && !hf;  // two chunks in flight (device frontiers)
      const int ks = pl ? (int)(ck & 1) : 0;  // this chunk's array set
      if (hf && hwin_c0[hs_k] != c0) {  // parents not prefetched: copy them in (window free after chunk ck-2)
        HIPCHK(hipStreamWaitEvent(hs.cs, hs.mat[hs_k], 0));
        hf_load(hcur, c0, n, A.hwin_in[hs_k].p, hs_k, hs.cs);
        HIPCHK(hipEventRecord(hs.in[hs_k], hs.cs));
        hwin_c0[hs_k] = c0;
      }
      if (hf) HIPCHK(hipStreamWaitEvent(stream, hs.in[hs_k], 0));
      if (pl) HIPCHK(hipStreamWaitEvent(stream, matdone[ks], 0));  // chunk ck-2's k_materialize read this set
      LevelArgs a;
      fill_args(a, c0, n, level, hf ? A.hwin_in[hs_k].as<uint32_t>() : nullptr, ks);
      HIPCHK(hipMemsetAsync(a.counters, 0, 1024, stream));
      HIPCHK(hipEventRecord(te.a, stream));
      const auto tl0 = now();
      launch_expand(M.spec, M.N, a, stream);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(te.b, stream));
      launch_mark(a, stream);
      HIPCHK(hipGetLastError());
      launch_scan(scantmp.p, scantmp.bytes, a.par_win, a.par_pos, n, stream);
      HIPCHK(hipGetLastError());
      launch_s += secs(tl0, now());
      HIPCHK(hipEventRecord(tm.b, stream));
      if (hf && c0 + n < cur_n && hwin_c0[hs_k ^ 1] != c0 + n) {
        // prefetch the next chunk's parents into the other window once chunk
        // ck-1's k_materialize (which re-reads that window) is done
        HIPCHK(hipStreamWaitEvent(hs.cs, hs.mat[hs_k ^ 1], 0));
        hf_load(hcur, c0 + n, std::min(chunk, cur_n - c0 - n), A.hwin_in[hs_k ^ 1].p, hs_k ^ 1, hs.cs);
        HIPCHK(hipEventRecord(hs.in[hs_k ^ 1], hs.cs));
        hwin_c0[hs_k ^ 1] = c0 + n;
      }
      unsigned long long ncand = 0;
      HIPCHK(hipMemcpyAsync(hrb->segc, a.counters, 1024, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipMemcpyAsync(&hrb->lastpos, a.par_pos + (n - 1), 4, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipMemcpyAsync(&hrb->lastwin, a.par_win + (n - 1), 4, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipMemcpyAsync(&hrb->st, stbuf.p, sizeof hst, hipMemcpyDeviceToHost, stream));
      sync_both();
      if (hf) hf_flush();  // the previous chunk's compact rows go out now that their sizes are known
      // the previous chunk's k_materialize outcome first: if it stopped the
      // search, this chunk's expand never happened as far as the counts go
      if (mat_pending && finish_mat()) break;
      {  // expand / mark status of this chunk; the invariant keys k_materialize found stay merged
        const unsigned long long ik = hst.inv_err_key, vk = hst.viol_key;
        hst = hrb->st;
        hst.inv_err_key = std::min(hst.inv_err_key, ik);
        hst.viol_key = std::min(hst.viol_key, vk);
      }
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, te.a, te.b));
      expand_ms += ms;
      expand_launches++;
      if (m->profile_level && level == m->profile_level && c0 == 0) m->profile_ms.push_back({0, ms});
      HIPCHK(hipEventElapsedTime(&ms, te.b, tm.b));
      mark_ms += ms;
      if (hst.cap_flags == (1u << E_RETRY)) {
        // fp_bits 128: a lane met a key whose second word was still in flight;
        // redo the chunk (idempotent), every key it claimed is complete now
        const unsigned zero = 0;
        HIPCHK(hipMemcpyAsync((char*)stbuf.p + offsetof(DevStatus, cap_flags), &zero, 4, hipMemcpyHostToDevice, stream));
        restore_coll();
        HIPCHK(hipStreamSynchronize(stream));
        redos++;
        continue;
      }
      if ((hst.cap_flags & ~(1u << E_RETRY)) == (1u << E_CAP_TABLE) && !full_ok) {
        // the table filled up under this chunk: grow it and redo the chunk
        // (its inserts are idempotent; the next frontier was not touched)
        bool grown = t_grow(slots * 2);
        if (!grown && !hf && hf_opt == 0) {  // the device frontiers give their HBM to the set
          enter_hf();
          grown = t_grow(slots * 2);
        }
        if (!grown) {
          full_ok = true;
          status = 3;
          message = "capacity overflow: fingerprint set full and HBM exhausted";
          break;
        }
        const unsigned zero = 0;
        HIPCHK(hipMemcpyAsync((char*)stbuf.p + offsetof(DevStatus, cap_flags), &zero, 4, hipMemcpyHostToDevice, stream));
        restore_coll();
        HIPCHK(hipStreamSynchronize(stream));
        redos++;
        continue;
      }
      if (hst.cap_flags) {
        int e = 0;
        while (!((hst.cap_flags >> e) & 1)) e++;
        const unsigned redoable = (1u << E_CAP_MSG) | (1u << E_CAP_TABLE) | (1u << E_RETRY);
        if (e == E_CAP_MSG && !opt->msg_cap_K && M.kmax < 120 && !hf && widen_ok && !(hst.cap_flags & ~redoable)) {
          widen(std::max(hst.max_msgs, (unsigned)M.kmax + 1), c0, n);
          redos++;
          continue;
        }
        if (e == E_CAP_MSG && !opt->msg_cap_K && M.kmax < 120) {
          // the caller re-runs with a larger message capacity
          m->kmax_user = std::min(120u, std::max((uint32_t)M.kmax * 2, default_kmax(M)));
          HIPCHK(hipStreamDestroy(stream));
          return 1;
        }
        static const char* names[] = {"", "", "log longer than the packed layout (5 entries)",
                                      "message capacity msg_cap_K exceeded", "message multiplicity > 7",
                                      "term > 15", "index field > 7", "successor buffer", "fingerprint set full",
                                      "frontier capacity", "fingerprint retry"};
        status = 3;
        message = std::string("capacity overflow: ") + names[e];
        break;
      }
      chunk_log.push_back({c0, gen_lvl, next_n});
      coll_kept = hst.hidden_coll;
      unsigned long long W_chunk = (unsigned long long)hrb->lastpos + hrb->lastwin;
      for (int sg = 0; sg < 8; sg++) ncand += hrb->segc[16 * sg];
      gen_lvl += ncand;
      for (int attempt = 0;; attempt++) {
        try {
          if (!hf && hf_opt == 0 && hf_force_grow && level == hf_force_level && c0 > 0 && !attempt)
            throw OutOfDeviceMemory("test: RMC_HOST_FRONTIER_AT");
          if (!hf) {
            // the next-level buffer grows in place to exactly what this chunk needs
            bool cur_is_a = cur == fa.as<uint32_t>();
            GrowBuf& nb = cur_is_a ? fb : fa;
            const size_t need = (size_t)(next_n + W_chunk) * W * 4;
            if (nb.bytes < need) {
              auto tg0 = now();
              HIPCHK(hipStreamSynchronize(stream));
              before_growth(need - nb.bytes);
              nb.ensure(need);
              cur = (cur_is_a ? fa : fb).as<uint32_t>();
              nxt = nb.as<uint32_t>();
              a.frontier = cur + c0 * W;
              grow_s += secs(tg0, now());
            }
            fcap = std::max(fcap, next_n + W_chunk);
          }
          if (distinct + next_n + W_chunk > trcap) {
            auto tg0 = now();
            HIPCHK(hipStreamSynchronize(stream));
            trcap = (distinct + next_n + W_chunk) + (distinct + next_n + W_chunk) / 4;
            trp.ensure(trcap * 8);
            trb.ensure(trcap * 2);
            grow_s += secs(tg0, now());
          }
          break;
        } catch (OutOfDeviceMemory&) {
          if (hf || hf_opt != 0 || attempt) throw;
          // HBM is full: the frontiers move to host memory; this chunk's
          // parents (k_materialize re-reads them) go to its input window
          lvl_next_n = next_n;
          enter_hf();
          hf_load(hcur, c0, n, A.hwin_in[hs_k].p, hs_k, hs.cs);
          HIPCHK(hipStreamSynchronize(hs.cs));
          hwin_c0[hs_k] = c0;
          a.frontier = A.hwin_in[hs_k].as<uint32_t>();
        }
      }
      if (hf) {
        // output window hs_k: free once chunk ck-2's rows have left it
        const size_t need = (size_t)W_chunk * W * 4;
        if (A.hwin_out[hs_k].bytes < need) {
          HIPCHK(hipEventSynchronize(hs.packed[hs_k]));
          hf_idle(hs.mat[hs_k], "an output window");
          A.hwin_out[hs_k].ensure(need + need / 4);
          m->hf_out_regrows++;
        }
        HIPCHK(hipStreamWaitEvent(stream, hs.packed[hs_k], 0));  // chunk ck-2's rows have been packed
        a.out = A.hwin_out[hs_k].as<uint32_t>();
      } else {
        a.out = nxt + next_n * W;
      }
      a.out_base_global = distinct + next_n;
      a.tr_parent = trp.as<unsigned long long>();
      a.tr_bind = trb.as<uint16_t>();
      // positions from the scan are chunk-local; shift by next_n via out pointer
      const bool plm = pl && !hf;  // (a mid-chunk switch to the host frontier drained mstream)
      hipStream_t mst = plm ? mstream : stream;
      if (plm) {  // after everything this chunk put on `stream` (growth included)
        HIPCHK(hipEventRecord(ev_scan, stream));
        HIPCHK(hipStreamWaitEvent(mstream, ev_scan, 0));
      }
      a.st = A.stmat.as<DevStatus>();
      HIPCHK(hipEventRecord(tz.a, mst));
      const auto tl1 = now();
      launch_materialize(M.spec, M.N, a, mst);
      HIPCHK(hipGetLastError());
      launch_s += secs(tl1, now());
      HIPCHK(hipEventRecord(tz.b, mst));
      HIPCHK(hipMemcpyAsync(&hrb->mat, A.stmat.p, sizeof hst, hipMemcpyDeviceToHost, mst));
      if (plm) HIPCHK(hipEventRecord(matdone[ks], mstream));
      if (hf) {  // the new rows go to host pages (copy stream), after this k_materialize
        HIPCHK(hipEventRecord(hs.mat[hs_k], stream));
        hf_flush();  // (normally already flushed at this chunk's sync point)
        hf_pack_async(hs_k, W_chunk);
        // rows below the previous chunk are consumed (the last two chunks stay
        // for the recount at a violation)
        hcur.recycle_below(prev_c0, pool);
      }
      mat_pending = true;
      next_n += W_chunk;
      prev_c0 = c0;
      c0 += n;
      ck++;
      if (hst.err_key != ~0ULL) {  // this chunk's expand hit an evaluation error: the search stops here
        sync_both();
        finish_mat();
        break;
      }
    }
    if (mat_pending) {
      sync_both();
      finish_mat();
    }
    if (hf) {
      hf_flush();
      hs.sync();  // every new row is in its host page
      unsigned f = 0;
      HIPCHK(hipMemcpy(&f, A.hf_flag.p, 4, hipMemcpyDeviceToHost));
      if (f) {  // the level that met the bound is not counted (as a capacity stop mid-level)
        status = 3;
        message = "capacity overflow: a row's message count exceeds the row width (a row never written)";
        break;
      }
    }
    const unsigned long long gen_before = generated, dist_before = distinct;
    generated += gen_lvl;
    distinct += next_n;
    if (next_n || gen_lvl) m->levels.push_back({gen_lvl, next_n});
    if (next_n) depth++;
    if (status) break;
    if (hst.err_key != ~0ULL || hst.inv_err_key != ~0ULL || hst.viol_key != ~0ULL) {
      // TLC stops at the first problem in its exploration order
      unsigned long long k_err = std::min(hst.err_key, hst.inv_err_key);
      if (k_err < hst.viol_key) {
        status = 2;
        bad_key = k_err;
        bad_is_parent_key = hst.err_key <= hst.inv_err_key;
        message = bad_is_parent_key ? "evaluation error in the next-state relation (a sequence applied outside its domain)"
                                    : "evaluation error while checking an invariant";
      } else {
        status = 1;
        bad_key = hst.viol_key;
      }
      stop_level = level;
      stop_level_base = cur_base;
      stop_level_n = cur_n;
      stop_front = hf ? nullptr : cur;
      stop_hf = hf;
      stop_gen_before = gen_before;
      stop_dist_before = dist_before;
      cur_base += cur_n;
      cur_n = next_n;
      std::swap(cur, nxt);
      std::swap(hcur, hnxt);  // host frontier: hnxt keeps the stopped level for the recount
      break;
    }
    rate = (double)next_n / (double)cur_n;
    cur_base += cur_n;
    cur_n = next_n;
    std::swap(cur, nxt);
    if (hf) {
      hcur.clear(pool);
      std::swap(hcur, hnxt);
    }
    if (opt->verbose) {
      size_t fr = 0, tot = 0;
      (void)hipMemGetInfo(&fr, &tot);
      fprintf(stderr,
              "[rmc] depth %u: %llu new, %llu distinct, %llu generated, t=%.3fs (rehash %.3fs, grow %.3fs) "
              "HBM GiB: fp-set %.1f+%.1f frontiers %.1f+%.1f trace %.1f+%.1f free %.1f%s\n",
              depth, next_n, distinct, generated, secs(t0, now()), rehash_s, grow_s, table.bytes / 1073741824.0,
              A.table2.bytes / 1073741824.0, fa.bytes / 1073741824.0, fb.bytes / 1073741824.0, trp.bytes / 1073741824.0, trb.bytes / 1073741824.0,
              fr / 1073741824.0,
              hf ? (" | host frontier: " + std::to_string(pool.allocated >> 20) + " MiB pinned").c_str() : "");
    }
    // ---- snapshot at this level boundary (TLC -checkpoint)
    if (opt->checkpoint_dir && *opt->checkpoint_dir && cur_n > 0 &&
        (opt->checkpoint_minutes <= 0 || secs(last_ckpt, now()) >= 60.0 * opt->checkpoint_minutes)) {
      auto tc0 = now();
      HIPCHK(hipStreamSynchronize(stream));
      const std::string dir = opt->checkpoint_dir;
      if (mkdir(dir.c_str(), 0755) != 0 && errno != EEXIST) throw std::runtime_error("checkpoint: cannot create " + dir);
      // the snapshot the directory holds now (if any) stays valid until the new one is durable
      unsigned long long prev_seq = 0;
      bool have_prev = false;
      try {
        prev_seq = ckpt_read_meta(dir, m).seq;
        have_prev = true;
      } catch (std::exception&) {
      }
      Ckpt c;
      c.seq = have_prev ? prev_seq + 1 : 0;
      const std::string sub = dir + "/" + ckpt_subdir(c.seq);
      remove_tree(sub);  // debris of an interrupted snapshot with this number
      if (mkdir(sub.c_str(), 0755) != 0) throw std::runtime_error("checkpoint: cannot create " + sub);
      ckpt_write(sub + "/fpset.bin", table.p, slots * ew * 8, stage(), ck_stage_bytes);
      if (hf) {
        const std::string fp = sub + "/frontier.bin", tmp = fp + ".tmp";
        FILE* f = fopen(tmp.c_str(), "wb");
        if (!f) throw std::runtime_error("checkpoint: cannot write " + tmp);
        std::vector<uint32_t> buf(std::min<unsigned long long>(cur_n, 1ULL << 16) * W);
        for (unsigned long long r = 0; r < cur_n; r += 1ULL << 16) {  // fixed-stride rows, as a device snapshot
          const size_t k = (size_t)std::min<unsigned long long>(1ULL << 16, cur_n - r);
          hcur.read_fixed_host(r, k, buf.data());
          if (fwrite(buf.data(), row_bytes, k, f) != k) { fclose(f); throw std::runtime_error("checkpoint: short write"); }
        }
        if (fflush(f) != 0 || fsync(fileno(f)) != 0 || fclose(f) != 0 || rename(tmp.c_str(), fp.c_str()) != 0)
          throw std::runtime_error("checkpoint: cannot finish " + fp);
      } else {
        ckpt_write(sub + "/frontier.bin", cur, cur_n * W * 4, stage(), ck_stage_bytes);
      }
      ckpt_write(sub + "/trace_parent.bin", trp.p, distinct * 8, stage(), ck_stage_bytes);
      ckpt_write(sub + "/trace_bind.bin", trb.p, distinct * 2, stage(), ck_stage_bytes);
      fsync_dir(sub);
      c.sig = model_signature(m);
      c.slots = slots;
      c.generated = generated;
      c.distinct = distinct;
      c.cur_base = cur_base;
      c.cur_n = cur_n;
      c.hidden = coll_kept;
      c.depth = depth;
      c.kmax = (uint32_t)M.kmax;
      c.fpw = M.fpw;
      c.rate = rate;
      c.levels = m->levels;
      ckpt_write_meta(dir, m, c);
      (void)prev_seq;
      ckpt_remove_stale(dir, c.seq);
      last_ckpt = now();
      if (opt->verbose)
        fprintf(stderr, "[rmc] checkpoint at depth %u in %s (%.3fs)\n", depth, dir.c_str(), secs(tc0, now()));
    }
  }
  } catch (OutOfHostMemory& oom) {
    status = 3;
    message = std::string("capacity overflow: ") + oom.what();
    HIPCHK(hipDeviceSynchronize());
  } catch (RowCapacity& rc) {
    status = 3;
    message = rc.what();
    HIPCHK(hipDeviceSynchronize());
  } catch (OutOfDeviceMemory& oom) {
    // the level in progress is abandoned; counts are those of the completed levels
    status = 3;
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    char buf[160];
    snprintf(buf, sizeof buf, " (HBM: %.1f GiB free of %.1f)", fr / 1073741824.0, tot / 1073741824.0);
    message = std::string("capacity overflow: ") + oom.what() + buf;
    HIPCHK(hipDeviceSynchronize());
  }
  HIPCHK(hipStreamSynchronize(stream));
  HIPCHK(hipStreamSynchronize(mstream));
  // ---- exact counts at the failing state.  TLC stops at the first violating
  // (or erroring) state in its exploration order; the chunks run whole, so
  // the failing chunk is expanded and marked again (its inserts are idempotent)
  // and the counts are
  // taken up to the failing candidate -- generated: every successor of the
  // parents before it plus the failing parent's up to the failing one; distinct:
  // the winners among those.  An evaluation error in Next drops the failing
  // parent's successors (as the oracle's convention does).
  DevStatus fin;  // before the recount below (which marks the failing chunk a second time)
  HIPCHK(hipMemcpy(&fin, stbuf.p, sizeof fin, hipMemcpyDeviceToHost));
  if ((status == 1 || status == 2) && bad_key != ~0ULL && (stop_front || stop_hf)) {
    const unsigned long long pg = bad_key >> 20, li = pg - stop_level_base;
    const int ordv = (int)((bad_key >> 10) & 0x3FF);
    const ChunkLog* cl = nullptr;
    for (const ChunkLog& c : chunk_log)
      if (c.c0 <= li) cl = &c;
    if (cl && li < stop_level_n) {
      const unsigned long long c0 = cl->c0, n = std::min(chunk, stop_level_n - c0);
      uint32_t* save_cur = cur;
      unsigned long long save_base = cur_base;
      cur = const_cast<uint32_t*>(stop_front);
      cur_base = stop_level_base;
      if (stop_hf) {  // the stopped level's pages (hnxt after the swap)
        hf_load(hnxt, c0, n, A.hwin_in[0].p, 0, stream);
        HIPCHK(hipStreamSynchronize(stream));
      }
      LevelArgs a;
      fill_args(a, c0, n, stop_level, stop_hf ? A.hwin_in[0].as<uint32_t>() : nullptr);
      cur = save_cur;
      cur_base = save_base;
      HIPCHK(hipMemsetAsync(counters.p, 0, 1024, stream));
      launch_expand(M.spec, M.N, a, stream);
      HIPCHK(hipGetLastError());
      launch_mark(a, stream);
      HIPCHK(hipGetLastError());
      std::vector<uint32_t> h_n(n), h_w(n);
      HIPCHK(hipMemcpyAsync(h_n.data(), a.par_n, n * 4, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipMemcpyAsync(h_w.data(), a.par_win, n * 4, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipStreamSynchronize(stream));
      const unsigned long long pl = li - c0;
      unsigned long long g = cl->gen_before, d = cl->new_before;
      for (unsigned long long p = 0; p < pl; p++) { g += h_n[p]; d += h_w[p]; }
      if (!bad_is_parent_key) {  // the failing state itself is new: count up to and including it
        uint32_t off = 0;
        HIPCHK(hipMemcpy(&off, a.par_off + pl, 4, hipMemcpyDeviceToHost));
        std::vector<uint32_t> ob(h_n[pl]);
        std::vector<uint16_t> win(h_n[pl]);
        if (h_n[pl]) {
          HIPCHK(hipMemcpy(ob.data(), a.cand_ob + off, h_n[pl] * 4, hipMemcpyDeviceToHost));
          HIPCHK(hipMemcpy(win.data(), a.cand_win + off, h_n[pl] * 2, hipMemcpyDeviceToHost));
        }
        for (uint32_t k = 0; k < h_n[pl]; k++)
          if ((int)(ob[k] >> 16) == ordv) { g += k + 1; d += win[k]; break; }
      }
      generated = stop_gen_before + g;
      distinct = stop_dist_before + d;
      if (!m->levels.empty()) m->levels.back() = {g, d};
    }
  }
  // ---- trace reconstruction: walk parent records, replay bindings on the host
  if (status == 1 || status == 2) {
    std::vector<std::pair<unsigned long long, int>> chain;  // (global state index or parent, binding)
    unsigned long long parent_g = ~0ULL;
    int last_b = -1;
    if (bad_key != ~0ULL) {
      parent_g = bad_key >> 20;
      last_b = (int)(bad_key & 0x3FF);
    } else if (bad_state != ~0ULL) {
      parent_g = bad_state;
    }
    std::vector<int> binds;
    unsigned long long g = parent_g;
    while (g != ~0ULL && g != 0) {
      unsigned long long pp;
      uint16_t bb;
      HIPCHK(hipMemcpy(&pp, trp.as<unsigned long long>() + g, 8, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(&bb, trb.as<uint16_t>() + g, 2, hipMemcpyDeviceToHost));
      binds.push_back(bb);
      g = pp;
    }
    std::reverse(binds.begin(), binds.end());
    replay_trace(m, binds, last_b, status, message, res);
  }
  res->hidden_var_collisions = fin.hidden_coll;
  if (opt->verbose) {
    unsigned long long stp[32];
    read_stamps(stp);
    double tot = (double)(stp[0] + stp[15] + stp[16] + stp[17] + stp[1] + stp[2] + stp[3]);
    if (tot > 0)
      fprintf(stderr, "[rmc] k_expand phase B fixed split: guard masks %.1f%%, prefix + chunk table %.1f%%, chunks %.1f%%\n",
              100 * stp[16] / tot, 100 * stp[17] / tot, 100 * stp[1] / tot);
    if (tot > 0)
      fprintf(stderr, "[rmc] k_expand phase shares: stage %.1f%%, message sums %.1f%%, bindings %.1f%% (fixed %.1f%%, "
              "messages %.1f%%), fp+insert %.1f%% (the same without inserts: %.1f%%); "
              "fingerprints %llu, with signature ties %llu, permutations hashed under ties %llu\n",
              100 * stp[0] / tot, 100 * stp[15] / tot, 100 * (stp[1] + stp[2]) / tot, 100 * stp[1] / tot,
              100 * stp[2] / tot, 100 * stp[3] / tot, 100 * stp[7] / tot, stp[4], stp[5], stp[6]);
    if (stp[8])
      fprintf(stderr, "[rmc] phase B: %llu parents, %.2f message bindings and %.2f live ones per parent (%d fixed); "
              "wave steps %llu, with live messages only %llu\n", stp[8], (double)stp[9] / stp[8],
              (double)stp[10] / stp[8], M.nfixed, stp[11], stp[12]);
    if (stp[8])
      fprintf(stderr, "[rmc] phase B fixed bindings: %.2f (parent, binding) pairs per parent pass may_enable; "
              "%.2f wave chunks per 64 parents\n", (double)stp[13] / stp[8], 64.0 * stp[14] / stp[8]);
    {
      unsigned long long fs[8];
      read_fpstats(fs);
      if (fs[FPS_INSERT])
        fprintf(stderr, "[rmc] fingerprint-set inserts: %llu, 4-entry load groups %llu (%.3f per insert), CAS %llu "
                "(%.3f per insert, %llu won), atomicMin %llu (%.3f per insert)\n", fs[FPS_INSERT], fs[FPS_GROUP],
                (double)fs[FPS_GROUP] / fs[FPS_INSERT], fs[FPS_CAS], (double)fs[FPS_CAS] / fs[FPS_INSERT],
                fs[FPS_CAS_WON], fs[FPS_MIN], (double)fs[FPS_MIN] / fs[FPS_INSERT]);
    }
    {  // -DRMC_ROWSTATS builds: the rows' bytes up to their last message (what the masked stores write)
      DevStatus ms;
      HIPCHK(hipMemcpy(&ms, A.stmat.p, sizeof ms, hipMemcpyDeviceToHost));
      if (ms.row_words && distinct > 1)
        fprintf(stderr, "[rmc] rows: %llu materialized, %.1f B each up to the last message (16 B units) of %zu B "
                "fixed stride\n", distinct - 1, 4.0 * (double)ms.row_words / (double)(distinct - 1), W * 4);
    }
    fprintf(stderr, "[rmc] fingerprint set: 2^%d slots, load %.3f, %llu growths, %llu chunk redos\n",
            __builtin_ctzll(slots), (double)distinct / (double)slots, grows, redos);
  }
  if (hf) {
    hs.sync();
    const size_t hf_peak = pool.allocated;
    hcur.clear(pool);
    hnxt.clear(pool);
    pool.release();
    A.release_hf();
    if (opt->verbose)
      fprintf(stderr, "[rmc] host frontier: %.3fs moving levels to host memory; %.3fs pinning pages (%zu MiB peak)\n", hf_copy_s,
              pool.alloc_s, hf_peak >> 20);
  }
  HIPCHK(hipStreamDestroy(stream));
  if (!opt->hash_slots) m->hint_slots = slots;
  if (!opt->frontier_cap && !hf) m->hint_fcap = fcap;
  m->hint_trcap = trcap;
  res->state_bytes = (uint32_t)(W * 4);
  if (opt->verbose && widenings)
    fprintf(stderr, "[rmc] rows widened %u times (%.3fs), to %zu words\n", widenings, widen_s, W);
  res->generated = generated;
  res->distinct = distinct;
  res->left_on_queue = (status == 0) ? 0 : cur_n;
  res->depth = depth;
  res->status = status;
  snprintf(res->message, sizeof res->message, "%s", message.c_str());
  res->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  res->expand_ms = expand_ms;
  res->mark_ms = mark_ms;
  res->materialize_ms = mat_ms;
  res->expand_launches = expand_launches;
  res->hash_capacity = slots;
  // where the wall time went (rmc_check_phases; bench.py reports the warm-up
  // check's, VERDICT r05 What's weak #4)
  m->phases = {{"hip_init", g_hip_init_s},
               {"model_upload", std::chrono::duration<double>(t_model - t0).count()},
               {"buffers", std::chrono::duration<double>(t_setup - t_model).count()},
               {"launch_enqueue", launch_s},
               {"table_growth", rehash_s},
               {"table_growth.allocate", tg_alloc_s},  // hipMalloc of the doubled set (the driver's own time)
               {"table_growth.fill", tg_fill_s},
               {"table_growth.rehash", tg_rehash_s},
               {"buffer_growth", grow_s},
               {"widening", widen_s},
               {"host_frontier", hf_copy_s},
               {"kernels", (expand_ms + mark_ms + mat_ms) * 1e-3},
               {"total", res->seconds}};
  g_hip_init_s = 0;  // counted once, by the process's first check
  hst.max_msgs = std::max(hst.max_msgs, mat_max_msgs);
  res->max_msgs = hst.max_msgs;
  {
    size_t b = 0;
    for (DevBuf* x : {&A.table, &A.table2, &A.cslot, &A.cob, &A.cwin, &A.poff, &A.pn, &A.pwin, &A.ppos, &A.counters,
                      &A.stbuf, &A.scantmp, &A.stmat, &A.cslot2, &A.cob2, &A.cwin2, &A.poff2, &A.pn2, &A.pwin2, &A.ppos2,
                      &A.counters2})
      b += x->bytes;
    for (int k = 0; k < 2; k++)
      for (DevBuf* x : {&A.hwin_in[k], &A.hwin_out[k], &A.hf_pack[k], &A.hf_olen32[k], &A.hf_olen8[k], &A.hf_ooff[k],
                        &A.hf_oscan[k], &A.hf_stage[k], &A.hf_ilen32[k], &A.hf_ilen8[k], &A.hf_ioff[k], &A.hf_iscan[k]})
        b += x->bytes;
    for (GrowBuf* x : {&A.fa, &A.fb, &A.trp, &A.trb}) b += x->bytes;
    res->device_bytes = b;
  }
  // the next check's row packing: the peak |DOMAIN messages| of a complete
  // check (a resumed one saw only the levels after its snapshot)
  if (status == 0 && !opt->max_depth && !opt->msg_cap_K && !recovering) m->hint_kmax = std::max(1u, hst.max_msgs);
  return 0;
}

std::string read_file(const std::string& p, bool& ok) {
  std::ifstream f(p);
  if (!f) { ok = false; return ""; }
  ok = true;
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

void set_err(char* err, size_t len, const std::string& msg) {
  g_last_error = msg;
  if (err && len) snprintf(err, len, "%s", msg.c_str());
}

}  // namespace

// ------------------------------------------------------------------ C ABI
extern "C" {

const char* rmc_version(void) { return "raftmc 0.5 (gfx950, abi 2)"; }
int rmc_abi_version(void) { return RMC_ABI_VERSION; }

// ABI self-description for binding checks: sizeof and every field offset of
// rmc_options then rmc_result, in declaration order (see include/rmc.h).
int rmc_abi_layout(uint64_t* out, int cap) {
  const uint64_t v[] = {
      sizeof(rmc_options), offsetof(rmc_options, n_gpus), offsetof(rmc_options, cpu_workers),
      offsetof(rmc_options, deadlock_check), offsetof(rmc_options, fp_bits), offsetof(rmc_options, tlc_order),
      offsetof(rmc_options, hash_slots), offsetof(rmc_options, msg_cap_K), offsetof(rmc_options, frontier_cap),
      offsetof(rmc_options, chunk_parents), offsetof(rmc_options, verbose), offsetof(rmc_options, max_depth),
      offsetof(rmc_options, grow_on_overflow), offsetof(rmc_options, time_limit),
      offsetof(rmc_options, checkpoint_dir), offsetof(rmc_options, checkpoint_minutes),
      offsetof(rmc_options, recover_dir), offsetof(rmc_options, host_frontier),
      sizeof(rmc_result), offsetof(rmc_result, generated), offsetof(rmc_result, distinct),
      offsetof(rmc_result, left_on_queue), offsetof(rmc_result, depth), offsetof(rmc_result, status),
      offsetof(rmc_result, violated), offsetof(rmc_result, hidden_var_collisions), offsetof(rmc_result, seconds),
      offsetof(rmc_result, message), offsetof(rmc_result, expand_ms), offsetof(rmc_result, mark_ms),
      offsetof(rmc_result, materialize_ms), offsetof(rmc_result, expand_launches), offsetof(rmc_result, state_bytes),
      offsetof(rmc_result, max_msgs), offsetof(rmc_result, hash_capacity), offsetof(rmc_result, device_bytes)};
  const int n = (int)(sizeof v / sizeof v[0]);
  for (int k = 0; k < n && k < cap; k++) out[k] = v[k];
  return n;
}
const char* rmc_last_error(void) { return g_last_error.c_str(); }

void rmc_options_default(rmc_options* o) {
  memset(o, 0, sizeof *o);
  o->n_gpus = 1;
  o->fp_bits = 64;
  o->tlc_order = 1;
}

int rmc_model_set_next(rmc_model* m, const char* disjuncts) {
  if (!m || !disjuncts) { g_last_error = "null argument"; return -1; }
  try {
    std::vector<std::string> names;
    std::string cur;
    for (const char* p = disjuncts;; p++) {
      if (*p == ',' || *p == 0) {
        while (!cur.empty() && cur.back() == ' ') cur.pop_back();
        if (!cur.empty()) names.push_back(cur);
        cur.clear();
        if (!*p) break;
      } else if (!(cur.empty() && *p == ' ')) {
        cur += *p;
      }
    }
    if (names.empty()) throw std::runtime_error("empty Next");
    // actions defined as TLA+ text (rmc_model_define_action) are compiled
    // whole, A_C0.. in Next order; the rest are the library's
    std::vector<std::pair<int, int>> acts;
    std::vector<rmc::tla::GuardSrc> srcs;
    for (auto& g : m->guard_srcs)
      if (g.act < A_C0) srcs.push_back(g);
    int k = 0;
    for (const std::string& n : names) {
      auto it = m->defined_actions.find(n);
      if (it == m->defined_actions.end()) {
        acts.push_back(rmc::tla::actions_by_name(m->M.spec, {n})[0]);
        continue;
      }
      if (k >= MAXCOMPILED) throw std::runtime_error("more than " + std::to_string(MAXCOMPILED) + " defined actions in Next");
      rmc::tla::GuardSrc g = it->second;
      g.act = A_C0 + k++;
      acts.push_back({g.act, g.kind});
      srcs.push_back(g);
    }
    const Model saved = m->M;
    const std::vector<rmc::tla::GuardSrc> saved_srcs = m->guard_srcs;
    try {
      install_guards(m, srcs);
    } catch (...) {
      m->M = saved;
      m->guard_srcs = saved_srcs;
      throw;
    }
    m->lowered_actions = acts;
    m->lowered_labels = names;
    m->hint_slots = m->hint_fcap = m->hint_trcap = 0;
    m->hint_kmax = 0;
    return 0;
  } catch (std::exception& e) {
    g_last_error = e.what();
    return -2;
  }
}

int rmc_model_define_action(rmc_model* m, const char* name, int form, const char* params, const char* body) {
  if (!m || !name || !params || !body) { g_last_error = "null argument"; return -1; }
  try {
    const int spec = m->M.spec;
    if (spec != RAFT && spec != FLEX && spec != FSYNC)
      throw std::runtime_error("actions compiled whole are offered for Raft, FlexibleRaft and RaftFsync");
    if (form != K_I && form != K_IV && form != K_IJ && form != 3)
      throw std::runtime_error("form must be 0 (\\E i \\in Server), 1 (i \\in Server, v \\in Value), 2 (i, j \\in "
                               "Server) or 3 (a message handler, \\E m \\in DOMAIN messages)");
    const int kind = form == 3 ? K_MSGC : form;
    std::vector<std::string> ps;
    std::string cur;
    for (const char* p = params;; p++) {
      if (*p == ',' || *p == 0) {
        while (!cur.empty() && cur.back() == ' ') cur.pop_back();
        if (!cur.empty()) ps.push_back(cur);
        cur.clear();
        if (!*p) break;
      } else if (!(cur.empty() && *p == ' ')) {
        cur += *p;
      }
    }
    if ((int)ps.size() != (kind == K_I || kind == K_MSGC ? 1 : 2))
      throw std::runtime_error(std::string("action ") + name + ": the form binds " +
                               (kind == K_I || kind == K_MSGC ? "one" : "two") + " parameters");
    rmc::tla::GuardSrc g = rmc::tla::parse_action(spec, name, kind, ps, body);
    // compile it once now, against this model's constants, so errors show here
    {
      rmc::tla::GuardEnv env;
      env.spec = spec;
      env.N = m->M.N;
      env.V = m->M.V;
      env.servers = m->server_names;
      env.values = m->value_names;
      for (auto& kv : m->int_consts) env.ints.insert(kv);
      env.send_helpers = g.send_helpers;
      const std::vector<int> types = form == K_IV ? std::vector<int>{0, 1} : form == K_IJ ? std::vector<int>{0, 0}
                                                                                         : std::vector<int>{0};
      if (kind == K_MSGC) {
        (void)rmc::tla::compile_handler(*g.mod, g.params, g.conjuncts, env, name);
      } else {
        (void)rmc::tla::compile_guard(*g.mod, g.params, types, g.conjuncts, env, name);
        (void)rmc::tla::compile_effect(*g.mod, g.params, types, g.effects, env, name);
      }
    }
    m->defined_actions[name] = g;
    return 0;
  } catch (std::exception& e) {
    g_last_error = e.what();
    return -2;
  }
}

int rmc_model_set_guard(rmc_model* m, const char* action, const char* params, const char* expr) {
  if (!m || !action || !params || !expr) { g_last_error = "null argument"; return -1; }
  try {
    const int spec = m->M.spec;
    if (spec == KRAFT) throw std::runtime_error("compiled guards are not offered for KRaft");
    const int act = rmc::tla::actions_by_name(spec, {std::string(action)})[0].first;
    if (act != A_RESTART && act != A_REQUESTVOTE && act != A_TIMEOUT && act != A_RVIJ && act != A_BECOMELEADER &&
        act != A_CLIENT)
      throw std::runtime_error(std::string("the guard of ") + action + " is not one the front end compiles (Restart, "
                               "RequestVote, Timeout, BecomeLeader, ClientRequest)");
    std::vector<std::string> ps;
    std::string cur;
    for (const char* p = params;; p++) {
      if (*p == ',' || *p == 0) {
        while (!cur.empty() && cur.back() == ' ') cur.pop_back();
        if (!cur.empty()) ps.push_back(cur);
        cur.clear();
        if (!*p) break;
      } else if (!(cur.empty() && *p == ' ')) {
        cur += *p;
      }
    }
    std::vector<rmc::tla::GuardSrc> all;
    for (auto& g : m->guard_srcs)
      if (g.act != act) all.push_back(g);
    all.push_back(rmc::tla::parse_guard(spec, act, action, ps, expr));
    const Model saved = m->M;
    const std::vector<rmc::tla::GuardSrc> saved_srcs = m->guard_srcs;
    try {
      install_guards(m, all);
    } catch (...) {
      m->M = saved;
      m->guard_srcs = saved_srcs;
      throw;
    }
    m->hint_slots = m->hint_fcap = m->hint_trcap = 0;
    m->hint_kmax = 0;
    return 0;
  } catch (std::exception& e) {
    g_last_error = e.what();
    return -2;
  }
}

int rmc_model_next(const rmc_model* m, char* out, size_t len) {
  if (!m || !out || !len) return -1;
  std::string o;
  if (!m->lowered_actions.empty()) {
    for (size_t q = 0; q < m->lowered_actions.size(); q++) {
      const int a = m->lowered_actions[q].first;
      o += (o.empty() ? "" : ",") + (a >= A_C0 && q < m->lowered_labels.size() ? m->lowered_labels[q]
                                                                                : rmc::tla::action_name(m->M.spec, a));
    }
  } else {
    Model M = m->M;
    build_actions(M, nullptr);
    for (int s = 0; s < M.nact; s++) o += (o.empty() ? "" : ",") + rmc::tla::action_name(M.spec, M.act_id[s]);
  }
  snprintf(out, len, "%s", o.c_str());
  return (int)o.size();
}

int rmc_tla_hashes(const char* tla_text, char* out, size_t len) {
  if (!tla_text || !out || !len) return -1;
  try {
    const std::string r = rmc::tla::hash_report(tla_text);
    snprintf(out, len, "%s", r.c_str());
    return (int)r.size();
  } catch (std::exception& e) {
    snprintf(out, len, "error: %s", e.what());
    g_last_error = e.what();
    return -2;
  }
}

int rmc_model_load_text(const char* module, const char* cfg_text, rmc_model** out, char* err, size_t errlen) {
  if (!module || !cfg_text || !out) { set_err(err, errlen, "null argument"); return -1; }
  try {
    *out = load_model(module, cfg_text, "");
    return 0;
  } catch (std::exception& e) {
    set_err(err, errlen, e.what());
    return -2;
  }
}

int rmc_model_load(const char* tla_path, const char* cfg_path, rmc_model** out, char* err, size_t errlen) {
  if (!tla_path || !out) { set_err(err, errlen, "null argument"); return -1; }
  std::string tp = tla_path;
  std::string base = tp.substr(tp.find_last_of('/') == std::string::npos ? 0 : tp.find_last_of('/') + 1);
  std::string module = base.size() > 4 && base.substr(base.size() - 4) == ".tla" ? base.substr(0, base.size() - 4) : base;
  if (base.size() <= 4 || base.substr(base.size() - 4) != ".tla") tp += ".tla";  // TLC: `tlc2.TLC Raft` reads Raft.tla
  bool ok = false;
  std::string tla = read_file(tp, ok);
  if (!ok) {
    // as TLC: the module file must exist (rmc_model_load_text checks the
    // built-in lowering of a module from its cfg alone)
    set_err(err, errlen, "cannot read module file " + tp + " (file not found)");
    return -3;
  }
  std::string cp = cfg_path ? std::string(cfg_path) : (tp.size() > 4 && tp.substr(tp.size() - 4) == ".tla" ? tp.substr(0, tp.size() - 4) : tp) + ".cfg";
  bool cok = false;
  std::string cfg = read_file(cp, cok);
  if (!cok) { set_err(err, errlen, "cannot read cfg file " + cp); return -3; }
  try {
    *out = load_model(module, cfg, tla);
    return 0;
  } catch (std::exception& e) {
    set_err(err, errlen, e.what());
    return -2;
  }
}

int rmc_check(rmc_model* m, const rmc_options* o, rmc_result* out) {
  if (!m || !out) { g_last_error = "null argument"; return -1; }
  rmc_options def;
  rmc_options_default(&def);
  if (!o) o = &def;
  memset(out, 0, sizeof *out);
  try {
    int ndev = 0;
    const auto ti = std::chrono::steady_clock::now();
    const hipError_t de = hipGetDeviceCount(&ndev);
    if (!g_hip_init_done) {
      g_hip_init_done = true;
      g_hip_init_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - ti).count();
      if (de == hipSuccess && ndev > 0) {  // the context itself is created at the first call that needs it
        void* p = nullptr;
        if (hipMalloc(&p, 256) == hipSuccess) (void)hipFree(p);
        g_hip_init_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - ti).count();
      }
    }
    if (de != hipSuccess || ndev < 1) {
      g_last_error = "no HIP device available: the raftmc GPU path requires an MI355X (gfx950)";
      return -4;
    }
    if (o->n_gpus < 1) {
      g_last_error = "n_gpus must be at least 1";
      return -1;
    }
    if (o->n_gpus > 1) {
      // one host thread per GPU, the fingerprint-sharded search
      // over them (rmc_check_multi); never silently fewer GPUs than asked
      if (o->n_gpus > ndev) {
        g_last_error = "n_gpus = " + std::to_string(o->n_gpus) + " requested, but only " + std::to_string(ndev) +
                       " GPU(s) are visible to this process: a multi-GPU check never runs on fewer GPUs than asked";
        return -4;
      }
      std::vector<int> devs(o->n_gpus);
      for (int d = 0; d < o->n_gpus; d++) devs[d] = d;
      const char* xp = getenv("RMC_MGPU_TRANSPORT");  // "p2p": peer copies instead of RCCL
      return rmc_check_multi(m, o, devs.data(), o->n_gpus,
                             xp && !strcmp(xp, "p2p") ? RMC_XPORT_P2P : RMC_XPORT_RCCL, out);
    }
    release_shard_buffers();
    m->kmax_user = 0;
    int rc;
    while ((rc = check_impl(m, o, out)) == 1) memset(out, 0, sizeof *out);
    return rc;
  } catch (std::exception& e) {
    g_last_error = e.what();
    return -5;
  }
}

int rmc_trace_len(const rmc_model* m) { return m ? (int)m->trace_states.size() : -1; }

int rmc_check_phases(const rmc_model* m, char* json, size_t len) {
  if (!m) return -1;
  std::string o = "{";
  for (size_t q = 0; q < m->phases.size(); q++) {
    char b[96];
    snprintf(b, sizeof b, "%s\"%s\": %.6f", q ? ", " : "", m->phases[q].first.c_str(), m->phases[q].second);
    o += b;
  }
  o += "}";
  if (json && len) snprintf(json, len, "%s", o.c_str());
  return (int)o.size();
}

int rmc_trace_state(const rmc_model* m, int k, char* buf, size_t len) {
  if (!m || k < 0 || k >= (int)m->trace_states.size()) return -1;
  std::string s = fmt_state(m, m->trace_states[k].data());
  if (buf && len) snprintf(buf, len, "%s", s.c_str());
  return (int)s.size();
}

// Trace-validation module (TLC's -dumpTrace tla): the error behaviour as a
// sequence of records, replayed by the spec's own Next.  TLC run on it with
// the companion cfg must report "Invariant TraceAccepted is violated" -- the
// last trace state was reached, i.e. every step of the trace is a Next step
// from Init (Raft.tla:213, :527).  Variables in TLC's order (var_order).
int rmc_trace_module(const rmc_model* m, const char* name, char* tla, size_t tla_len, char* cfg, size_t cfg_len) {
  if (!m || !name || m->trace_states.empty()) return -1;
  const std::string nm = name;
  std::string o;
  o += "---------------------------- MODULE " + nm + " ----------------------------\n";
  o += "(* Written by " + std::string(rmc_version()) + ": the behaviour of " + m->module +
       " that ends in the reported error\n";
  o += "   (" + std::to_string(m->trace_states.size()) + " states), replayed by " + m->module +
       "'s own Init and Next.  Check it with\n";
  o += "       java tlc2.TLC -deadlock -config " + nm + ".cfg " + nm + ".tla\n";
  o += "   Expected: \"Error: Invariant TraceAccepted is violated.\" -- the whole trace was\n";
  o += "   replayed.  Any other outcome means the trace is not a behaviour of the spec. *)\n";
  o += "EXTENDS " + m->module + ", Sequences, TLC\n\n";
  o += "CONSTANTS ";
  {
    std::vector<std::string> mv = m->server_names;
    mv.insert(mv.end(), m->value_names.begin(), m->value_names.end());
    for (size_t q = 0; q < mv.size(); q++) o += (q ? ", " : "") + mv[q];
  }
  o += "\n\nVARIABLE traceIdx\n\n";
  o += "TraceStates == <<\n";
  for (size_t k = 0; k < m->trace_states.size(); k++) {
    auto vars = state_vars(m, m->trace_states[k].data());
    o += "  \\* State " + std::to_string(k + 1) + ": " +
         (k == 0 ? std::string("<Initial predicate>") : m->trace_actions[k]) + "\n  [";
    for (size_t q = 0; q < vars.size(); q++) o += (q ? ",\n   " : "") + vars[q].first + " |-> " + vars[q].second;
    o += k + 1 < m->trace_states.size() ? "],\n" : "]\n";
  }
  o += ">>\n\n";
  auto is = [&](const char* idx, bool primed) {
    std::string r;
    for (size_t q = 0; q < m->var_order.size(); q++)
      r += std::string("    /\\ ") + m->var_order[q] + (primed ? "'" : "") + " = TraceStates[" + idx + "]." +
           m->var_order[q] + "\n";
    return r;
  };
  o += "TraceInit ==\n    /\\ traceIdx = 1\n" + is("1", false) + "    /\\ Init\n\n";
  o += "TraceNext ==\n    /\\ traceIdx < Len(TraceStates)\n    /\\ traceIdx' = traceIdx + 1\n    /\\ Next\n" +
       is("traceIdx + 1", true) + "\n";
  o += "TraceAccepted == traceIdx < Len(TraceStates)\n";
  o += "=============================================================================\n";
  std::string c;
  c += "\\* Companion cfg of " + nm + ".tla (raftmc -dumpTrace tla): " + m->module + "'s constants.\n";
  c += "CONSTANTS\n";
  for (auto& kv : m->cfg_consts)
    c += "    " + kv.first + (kv.second.rfind("<-", 0) == 0 ? " " : " = ") + kv.second + "\n";
  c += "INIT TraceInit\nNEXT TraceNext\nINVARIANT TraceAccepted\n";
  if (tla && tla_len) snprintf(tla, tla_len, "%s", o.c_str());
  if (cfg && cfg_len) snprintf(cfg, cfg_len, "%s", c.c_str());
  return (int)o.size();
}

// The same behaviour as JSON (TLC's -dumpTrace json): {"module", "states": [{"action", var: TLA+ value text}]}.
int rmc_trace_json(const rmc_model* m, char* buf, size_t len) {
  if (!m || m->trace_states.empty()) return -1;
  auto esc = [](const std::string& x) {
    std::string r;
    for (char ch : x) {
      if (ch == '"' || ch == '\\') { r += '\\'; r += ch; }
      else if (ch == '\n') r += "\\n";
      else r += ch;
    }
    return r;
  };
  std::string o = "{\"module\": \"" + esc(m->module) + "\", \"states\": [\n";
  for (size_t k = 0; k < m->trace_states.size(); k++) {
    o += "  {\"action\": \"" + esc(k == 0 ? std::string("Initial predicate") : m->trace_actions[k]) + "\"";
    for (auto& kv : state_vars(m, m->trace_states[k].data())) o += ", \"" + kv.first + "\": \"" + esc(kv.second) + "\"";
    o += k + 1 < m->trace_states.size() ? "},\n" : "}\n";
  }
  o += "]}\n";
  if (buf && len) snprintf(buf, len, "%s", o.c_str());
  return (int)o.size();
}

int rmc_trace_action(const rmc_model* m, int k, char* buf, size_t len) {
  if (!m || k < 0 || k >= (int)m->trace_actions.size()) return -1;
  const std::string& s = m->trace_actions[k];
  if (buf && len) snprintf(buf, len, "%s", s.c_str());
  return (int)s.size();
}

int rmc_levels(const rmc_model* m, uint64_t* pairs, int cap) {
  if (!m) return -1;
  int n = (int)m->levels.size();
  for (int k = 0; k < n && k < cap; k++) {
    pairs[2 * k] = m->levels[k].first;
    pairs[2 * k + 1] = m->levels[k].second;
  }
  return n;
}

int rmc_format_report(const rmc_model* m, const rmc_result* r, char* buf, size_t len) {
  if (!m || !r) return -1;
  std::string o;
  char line[512];
  if (r->status == 1) {
    o += std::string("Error: Invariant ") + r->violated + " is violated.\n";
  } else if (r->status == 2) {
    o += std::string("Error: TLC threw an unexpected exception.\n") + r->message + "\n";
  } else if (r->status == 3) {
    o += std::string("Error: ") + r->message + "\n";
  }
  if ((r->status == 1 || r->status == 2) && !m->trace_states.empty()) {
    o += "Error: The behavior up to this point is:\n";
    for (size_t k = 0; k < m->trace_states.size(); k++) {
      std::string act = m->trace_actions[k];
      std::string op = act.substr(0, act.find('('));
      if (k == 0) snprintf(line, sizeof line, "State %zu: <Initial predicate>\n", k + 1);
      else snprintf(line, sizeof line, "State %zu: <%s%s of module %s>\n", k + 1, act.c_str(),
                    def_location(m, op).c_str(), m->module.c_str());
      o += line;
      o += fmt_state(m, m->trace_states[k].data());
      o += "\n";
    }
  }
  if (r->status == 0) {
    o += "Model checking completed. No error has been found.\n";
    // TLC's estimate for 64-bit fingerprints: distinct x (generated - distinct) / 2^64
    double d = (double)r->distinct, g = (double)r->generated;
    snprintf(line, sizeof line,
             "  Estimates of the probability that TLC did not check all reachable states\n"
             "  because two distinct states had the same fingerprint:\n"
             "  calculated (optimistic):  val = %.1E\n",
             d * (g > d ? g - d : 0.0) / 18446744073709551616.0);
    o += line;
  }
  snprintf(line, sizeof line, "%llu states generated, %llu distinct states found, %llu states left on queue.\n",
           (unsigned long long)r->generated, (unsigned long long)r->distinct, (unsigned long long)r->left_on_queue);
  o += line;
  snprintf(line, sizeof line, "The depth of the complete state graph search is %u.\n", r->depth);
  o += line;
  if (buf && len) snprintf(buf, len, "%s", o.c_str());
  return (int)o.size();
}

void rmc_model_free(rmc_model* m) { delete m; }

void rmc_release_device_memory(void) {
  drain_device();
  release_shard_buffers();
  std::lock_guard<std::mutex> lk(g_arena_mu);
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto& kv : g_arenas) {
    if (hipSetDevice(kv.first) == hipSuccess) kv.second->release();
  }
  (void)hipSetDevice(cur);
}

// Test hook only (RMC_DIAG builds): check up to `level`, timing k_expand on
// that level's first chunk stopped after each phase (diag 4: staging, 3:
// bindings, 2: successor deltas, 1: fingerprints, no insert; 0: the real
// launch).  Fills (diag, ms) pairs; returns how many.
// TEST HOOK: the last check's row widenings, 3 values each (depth, first
// parent of the redone chunk within its level, message slots after); returns
// how many there were.
int rmc_selftest_widenings(const rmc_model* m, uint64_t* out, int cap) {
  const int n = (int)m->widenings.size();
  for (int k = 0; k < n && 3 * k + 2 < cap; k++)
    for (int j = 0; j < 3; j++) out[3 * k + j] = m->widenings[k][j];
  return n;
}
// TEST HOOK: the last single-GPU check's host-frontier regrowths while its
// copy streams ran: out[0] compact-row pack buffers, out[1] output windows.
int rmc_selftest_hf_stats(const rmc_model* m, uint64_t* out) {
  if (!m || !out) return -1;
  out[0] = m->hf_pack_regrows;
  out[1] = m->hf_out_regrows;
  return 2;
}
int rmc_selftest_profile_expand(rmc_model* m, const rmc_options* o, int level, double* out, int cap) {
  if (!m || !o || level < 2) { g_last_error = "bad argument"; return -1; }
  if (!diag_build()) { g_last_error = "librmc was not built with -DRMC_DIAG"; return -1; }
  rmc_options oo = *o;
  oo.max_depth = level;
  m->profile_level = (unsigned)level;
  m->profile_ms.clear();
  rmc_result r;
  const int rc = rmc_check(m, &oo, &r);
  m->profile_level = 0;
  if (rc != 0) return rc;
  int n = 0;
  for (auto& pr : m->profile_ms)
    if (n + 1 < cap) { out[n] = pr.first; out[n + 1] = pr.second; n += 2; }
  return n / 2;
}

// Test hook only: the row packing the next check of m starts from (as if its
// last complete check had materialized at most k messages per state).
void rmc_selftest_set_hint_kmax(rmc_model* m, uint32_t k) {
  if (m) m->hint_kmax = k;
}

// Test hook only (never called by rmc_check): a seeded random walk of at most
// `steps` steps over the lowered actions on the host, replayed into the
// model's trace (as after a violation), so the CPU tests can check the trace
// writers (rmc_trace_module / rmc_trace_json) against the oracle's Next.
int rmc_selftest_random_trace(rmc_model* m, uint64_t seed, int steps) {
  try {
    finalize_model(m, m->kmax_user ? m->kmax_user : default_kmax(m->M));
    const Model& M = m->M;
    std::vector<uint32_t> s = init_state(M), t(M.words, 0u);
    std::vector<int> binds;
    uint64_t x = seed * 0x9E3779B97F4A7C15ULL + 1;
    for (int k = 0; k < steps; k++) {
      std::vector<int> en;
      for (int x = 0; x < nbindings(M, h_nmsg(s[0])); x++) {
        const int b = binding_at(M, x, h_nmsg(s[0]));
        int err = 0;
        if (host_eval_apply(M, s.data(), b, t.data(), nullptr, nullptr, &err) == 1 && !err) en.push_back(b);
      }
      if (en.empty()) break;
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      int b = en[x % en.size()];
      host_eval_apply(M, s.data(), b, t.data(), nullptr, nullptr, nullptr);
      s = t;
      binds.push_back(b);
    }
    m->trace_states.clear();
    m->trace_actions.clear();
    rmc_result res;
    memset(&res, 0, sizeof res);
    std::string msg;
    replay_trace(m, binds, -1, 0, msg, &res);
    return (int)m->trace_states.size();
  } catch (std::exception& e) {
    g_last_error = e.what();
    return -1;
  }
}

// Test hook only (never called by rmc_check): sequential host BFS over the same
// lowered actions and fingerprints the kernels use, in TLC order, so the CPU
// test suite can pin the lowering against the oracle without a GPU.
int rmc_selftest_host_bfs(rmc_model* m, uint32_t kmax, uint64_t max_distinct, uint64_t* out3, uint64_t* levels,
                          int level_cap) {
  try {
    finalize_model(m, kmax ? kmax : default_kmax(m->M));
    const Model& M = m->M;
    const size_t W = (size_t)M.words;
    std::unordered_map<unsigned long long, char> seen;
    std::vector<uint32_t> cur = init_state(M), nxt;
    seen[host_fingerprint(M, cur.data())] = 1;
    uint64_t gen = 1, distinct = 1, depth = 1;
    int nl = 0;
    auto push_level = [&](uint64_t g, uint64_t d) {
      if (nl < level_cap) { levels[2 * nl] = g; levels[2 * nl + 1] = d; }
      nl++;
    };
    push_level(1, 1);
    size_t ncur = 1;
    std::vector<std::pair<int, std::vector<uint32_t>>> succ;
    while (ncur) {
      nxt.clear();
      size_t nn = 0;
      uint64_t gl = 0;
      for (size_t p = 0; p < ncur; p++) {
        const uint32_t* S = cur.data() + p * W;
        const int B = nbindings(M, h_nmsg(S[0]));
        succ.clear();
        for (int x = 0; x < B; x++) {
          const int b = binding_at(M, x, h_nmsg(S[0]));
          std::vector<uint32_t> t(W, 0);
          int ord = 0, act = 0, err = 0;
          if (host_eval_apply(M, S, b, t.data(), &ord, &act, &err) != 1) continue;
          if (err) { out3[0] = gen; out3[1] = distinct; out3[2] = depth; return -10 - err; }
          if (const int fc = host_fp_check(M, S, b, t.data())) {
            g_last_error = fc == 2 ? "selftest: may_enable rejects an enabled fixed binding"
                                   : "selftest: incremental fingerprint differs from the materialized state's";
            return -2;
          }
          succ.push_back({ord, t});
        }
        std::stable_sort(succ.begin(), succ.end(), [](auto& x, auto& y) { return x.first < y.first; });
        for (auto& sc : succ) {
          gen++;
          gl++;
          unsigned long long fp = host_fingerprint(M, sc.second.data());
          if (seen.count(fp)) continue;
          seen[fp] = 1;
          distinct++;
          nxt.insert(nxt.end(), sc.second.begin(), sc.second.end());
          nn++;
          int err = 0;
          if (host_check_invariants(M, sc.second.data(), &err) >= 0 || err) {
            out3[0] = gen; out3[1] = distinct; out3[2] = depth + 1;
            return err ? -3 : 1;
          }
        }
      }
      if (nn || gl) push_level(gl, nn);
      if (nn) depth++;
      std::swap(cur, nxt);
      ncur = nn;
      if (max_distinct && distinct >= max_distinct) break;
    }
    out3[0] = gen; out3[1] = distinct; out3[2] = depth;
    return nl;
  } catch (std::exception& e) {
    g_last_error = e.what();
    return -1;
  }
}

}  // extern "C"
