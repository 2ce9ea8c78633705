// rmc_guard.cpp — the TLA+ front end's guard compiler.
//
// A Next disjunct whose operator differs from every library action, but whose
// EFFECT -- the conjuncts that prime a variable, say UNCHANGED or call an
// operator that does -- is a library action's effect exactly (same effect
// hash, rmc_tla.cpp effect_hash), is checked with the library's effect run
// unguarded behind ITS OWN guard, compiled here from the module's guard
// conjuncts into the stack-machine code rmc_spec.h guard_vm runs on the
// device (and in the CPU engine: the same code).  E.g. Raft.tla:242-257's
// RequestVote with `electionCtr <= MaxElections`, or a BecomeLeader
// (Raft.tla:289-300) that wants every vote.
//
// The guard language is the specs' expression subset over the state, typed
// as the packed layout stores it: per-server variables (state, currentTerm,
// votedFor / leader, commitIndex, fsyncIndex, votesGranted, Len(log[x]),
// log[x][k].term / .value, nextIndex / matchIndex / pendingResponse rows),
// electionCtr, restartCtr, acked[v]; the cfg's constants and model values;
// integers (+ - *, comparisons), booleans (/\ \/ ~ => short-circuit, as TLC
// evaluates them), sets of servers / values / states as bitmasks (\in,
// \notin, \subseteq, \cup, \cap, \, Cardinality, SUBSET, set filters such as
// Quorum), IF/THEN/ELSE, LET, \E / \A over constant sets (unrolled), and the
// module's own operators (inlined).  Anything else is refused, naming it.
#include <functional>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "rmc_spec.h"
#include "rmc_tla.h"

namespace rmc {
namespace tla {
namespace {

enum Ty { T_INT, T_BOOL, T_SRV, T_VAL, T_STATE, T_ACK, T_SET_SRV, T_SET_VAL, T_SET_STATE, T_NIL, T_TRUE, T_FALSE,
          // compiled message handlers: a record type (RequestVoteRequest, ...), a term-match model value
          // (EqualTerm / LessOrEqualTerm), a message's entries sequence (<<>> or one entry)
          T_MTYPE, T_TMATCH, T_ENTRIES };

const char* ty_name(Ty t) {
  static const char* n[] = {"an integer", "a boolean", "a server", "a value", "a server state", "an acked value",
                            "a set of servers", "a set of values", "a set of states", "Nil", "TRUE", "FALSE",
                            "a message type", "a term-match value", "a sequence of entries"};
  return n[t];
}

// The fields of the Raft family's records (Raft.tla:243-505) a compiled
// handler reads from its bound message: G_MF operand and type.
bool msg_field_of(const std::string& f, int& mf, Ty& ty) {
  static const struct { const char* name; int mf; Ty ty; } t[] = {
      {"mtype", MF_TYPE, T_MTYPE},          {"mterm", MF_TERM, T_INT},           {"msource", MF_SRC, T_SRV},
      {"mdest", MF_DST, T_SRV},             {"mvoteGranted", MF_GRANTED, T_BOOL}, {"mlastLogIndex", MF_LLI, T_INT},
      {"mlastLogTerm", MF_LLT, T_INT},      {"mprevLogIndex", MF_PLI, T_INT},    {"mprevLogTerm", MF_PLT, T_INT},
      {"mentries", MF_NENT, T_ENTRIES},     {"mcommitIndex", MF_COMMIT, T_INT},  {"msuccess", MF_SUCCESS, T_BOOL},
      {"mmatchIndex", MF_MIDX, T_INT}};
  for (auto& x : t)
    if (f == x.name) { mf = x.mf; ty = x.ty; return true; }
  return false;
}

struct Compiler;

// A name in scope: an action parameter (ARG n), a constant of an unrolled
// quantifier, or a macro (an operator of the module / LET, inlined at use).
struct Binding {
  enum K { ARG, CONSTV, MACRO, MSG } k = ARG;  // MSG: a compiled handler's bound message
  int v = 0;
  Ty ty = T_INT;
  const Def* def = nullptr;  // MACRO: its definition
  std::weak_ptr<struct Scope> defsc;  // MACRO from a LET: the scope it was defined in (its body's free names)
  // MACRO arguments bound to expressions in the caller's scope
  std::vector<std::pair<std::string, std::pair<NodeP, std::shared_ptr<struct Scope>>>> args;
};
struct Scope {
  std::map<std::string, Binding> names;
  std::shared_ptr<Scope> up;
  const Binding* find(const std::string& n) const {
    for (const Scope* s = this; s; s = s->up.get()) {
      auto it = s->names.find(n);
      if (it != s->names.end()) return &it->second;
    }
    return nullptr;
  }
};
using ScopeP = std::shared_ptr<Scope>;

// An expression argument of an inlined operator, evaluated in its caller's scope.
struct Arg {
  NodeP n;
  ScopeP sc;
};

struct Compiler {
  const Module& m;
  const GuardEnv& env;
  std::vector<uint32_t> code;
  std::string where;  // the action, for messages
  // parameters of inlined operators: name -> argument (innermost last)
  std::vector<std::pair<std::string, Arg>> params;
  int depth = 0;
  // effects: `@` inside [x EXCEPT ![i] = ...] -- the old x[i], emitted by this
  std::function<Ty()> at;

  Compiler(const Module& mod, const GuardEnv& e) : m(mod), env(e) {}

  [[noreturn]] void fail(const NodeP& n, const std::string& what) {
    throw std::runtime_error("guard of " + where + " (line " + std::to_string(n ? n->line : 0) + "): " + what);
  }
  void emit(uint32_t op, int imm = 0) { code.push_back(g_ins(op, imm)); }
  size_t jump(uint32_t op) {
    code.push_back(g_ins(op, 0));
    return code.size() - 1;
  }
  void patch(size_t at) { code[at] = (code[at] & 0xFFu) | ((uint32_t)((int)(code.size() - at - 1)) << 8); }

  const Arg* param(const std::string& s) const {
    for (size_t q = params.size(); q-- > 0;)
      if (params[q].first == s) return &params[q].second;
    return nullptr;
  }

  // emit code for a symbolic constant (Nil / TRUE / FALSE) compared with a value of type t
  int sym_code(Ty sym, Ty t, const NodeP& n) {
    if (sym == T_NIL) {
      if (t == T_SRV) return NILS;
      if (t == T_ACK) return 0;
      fail(n, std::string("Nil compared with ") + ty_name(t));
    }
    if (t == T_ACK) return sym == T_TRUE ? 2 : 1;
    if (t == T_BOOL) return sym == T_TRUE ? 1 : 0;
    fail(n, std::string("TRUE/FALSE compared with ") + ty_name(t));
  }
  static bool is_sym(Ty t) { return t == T_NIL || t == T_TRUE || t == T_FALSE; }
  // a symbolic constant where a value is needed on its own (a boolean TRUE/FALSE)
  Ty concrete(Ty t, const NodeP& n) {
    if (t == T_TRUE || t == T_FALSE) {
      emit(G_CONST, t == T_TRUE);
      return T_BOOL;
    }
    if (t == T_NIL) fail(n, "Nil outside a comparison");
    return t;
  }
  Ty elem_of(Ty set, const NodeP& n) {
    if (set == T_SET_SRV) return T_SRV;
    if (set == T_SET_VAL) return T_VAL;
    if (set == T_SET_STATE) return T_STATE;
    fail(n, std::string("membership in ") + ty_name(set));
  }
  Ty set_of(Ty e, const NodeP& n) {
    if (e == T_SRV) return T_SET_SRV;
    if (e == T_VAL) return T_SET_VAL;
    if (e == T_STATE) return T_SET_STATE;
    fail(n, std::string("a set of ") + ty_name(e));
  }

  // variables indexed by one server: the load op and the value type
  bool server_var(const std::string& v, uint32_t& op, Ty& ty) {
    const int spec = env.spec;
    if (v == "state") { op = G_ST; ty = T_STATE; return true; }
    if (v == "currentTerm") { op = G_TERM; ty = T_INT; return true; }
    if (v == "commitIndex") { op = G_COMMIT; ty = T_INT; return true; }
    if (v == "fsyncIndex" && spec == FSYNC) { op = G_FSYNC; ty = T_INT; return true; }
    if (v == "votesGranted") { op = G_VOTES; ty = T_SET_SRV; return true; }
    if (v == "votedFor" && spec != PULL) { op = spec == PULL2 ? G_VOTED2 : G_VOTED; ty = T_SRV; return true; }
    if (v == "leader" && pullish(spec)) { op = G_VOTED; ty = T_SRV; return true; }
    return false;
  }
  bool pair_var(const std::string& v, uint32_t& op, Ty& ty) {
    if (v == "nextIndex" && !pullish(env.spec)) { op = G_NEXT; ty = T_INT; return true; }
    if (v == "matchIndex") { op = G_MATCH; ty = T_INT; return true; }
    if (v == "pendingResponse" && env.spec == RAFT) { op = G_PEND; ty = T_BOOL; return true; }
    return false;
  }

  // log[x] as an operand of Len / indexing: the server expression
  bool log_of(const NodeP& n, ScopeP sc, Arg& x) {
    if (n->kind == N_ID) {
      if (const Arg* a = param(n->s)) return log_of(a->n, a->sc, x);
      if (sc->find(n->s)) return false;
    }
    if (n->kind == N_FAPP && n->k.size() == 2 && n->k[0]->kind == N_ID && n->k[0]->s == "log" && !sc->find("log")) {
      x = {n->k[1], sc};
      return true;
    }
    return false;
  }

  Ty sub(const Arg& a) { return expr(a.n, a.sc); }

  // Does n denote the handler's bound message (through operator parameters
  // and parameterless LET definitions)?
  bool is_msg(const NodeP& n, ScopeP sc, int depth_ = 0) {
    if (depth_ > 32 || !n || n->kind != N_ID) return false;
    if (const Binding* b = sc->find(n->s)) {
      if (b->k == Binding::MSG) return true;
      if (b->k == Binding::MACRO && b->def && b->def->params.empty())
        return is_msg(b->def->body, b->defsc.lock() ? b->defsc.lock() : sc, depth_ + 1);
      return false;
    }
    if (const Arg* a = param(n->s)) {
      std::vector<std::pair<std::string, Arg>> save = params;
      while (!params.empty() && &params.back().second != a) params.pop_back();
      params.pop_back();
      const bool r = is_msg(a->n, a->sc, depth_ + 1);
      params = save;
      return r;
    }
    return false;
  }
  // Does n denote the bound message's mdest (the server a handler's effects act on)?
  bool is_mdest(const NodeP& n, ScopeP sc, int depth_ = 0) {
    if (depth_ > 32 || !n) return false;
    if (n->kind == N_FIELD && n->s == "mdest") return is_msg(n->k[0], sc);
    if (n->kind != N_ID) return false;
    if (const Binding* b = sc->find(n->s)) {
      if (b->k == Binding::MACRO && b->def && b->def->params.empty())
        return is_mdest(b->def->body, b->defsc.lock() ? b->defsc.lock() : sc, depth_ + 1);
      return false;
    }
    if (const Arg* a = param(n->s)) {
      std::vector<std::pair<std::string, Arg>> save = params;
      while (!params.empty() && &params.back().second != a) params.pop_back();
      params.pop_back();
      const bool r = is_mdest(a->n, a->sc, depth_ + 1);
      params = save;
      return r;
    }
    return false;
  }

  Ty bin_int(const NodeP& n, ScopeP sc, uint32_t op) {
    Ty a = concrete(expr(n->k[0], sc), n), b = concrete(expr(n->k[1], sc), n);
    if (a != T_INT || b != T_INT) fail(n, "arithmetic on " + std::string(ty_name(a)) + " and " + ty_name(b));
    emit(op);
    return T_INT;
  }
  Ty compare(const NodeP& n, ScopeP sc, const std::string& op) {
    {  // m.mentries = <<>> (or /=, #): the message carries no entry
      const bool e0 = n->k[0]->kind == N_TUPLE && n->k[0]->k.empty(), e1 = n->k[1]->kind == N_TUPLE && n->k[1]->k.empty();
      if (e0 || e1) {
        if (concrete(expr(e0 ? n->k[1] : n->k[0], sc), n) != T_ENTRIES) fail(n, "<<>> compared with something other than a message's entries");
        emit(G_CONST, 0);
        if (op == "=") emit(G_EQ);
        else if (op == "/=" || op == "#") emit(G_NE);
        else fail(n, "order comparison with <<>>");
        return T_BOOL;
      }
    }
    // a symbolic operand takes its code from the other side's type
    const size_t mark = code.size();
    Ty a = expr(n->k[0], sc);
    Ty b;
    if (is_sym(a)) {
      code.resize(mark);
      b = concrete(expr(n->k[1], sc), n);
      emit(G_CONST, sym_code(a, b, n));
      if (op == "<" || op == ">" || op == "<=" || op == ">=") fail(n, "order comparison with a symbolic constant");
      a = b;
    } else {
      b = expr(n->k[1], sc);
      if (is_sym(b)) {
        emit(G_CONST, sym_code(b, a, n));
        b = a;
      }
    }
    a = concrete(a, n);
    b = concrete(b, n);
    if (a != b && !(a == T_INT && b == T_INT)) fail(n, std::string("comparison of ") + ty_name(a) + " and " + ty_name(b));
    if (a == T_ENTRIES) fail(n, "comparison of message entries other than with <<>>");
    if ((op == "<" || op == ">" || op == "<=" || op == ">=") && a != T_INT) fail(n, "order comparison of non-integers");
    if (op == "=") emit(G_EQ);
    else if (op == "/=" || op == "#") emit(G_NE);
    else if (op == "<") emit(G_LT);
    else if (op == "<=" || op == "=<" || op == "\\leq") emit(G_LE);
    else if (op == ">") { emit(G_LE); emit(G_NOT); }
    else if (op == ">=" || op == "\\geq") { emit(G_LT); emit(G_NOT); }
    return T_BOOL;
  }

  // x \in S: filters and SUBSET are rewritten (e \in {y \in S : P} is e \in S /\ P[y := e])
  Ty member(const NodeP& n, const NodeP& e, const NodeP& set, ScopeP sc, ScopeP esc) {
    NodeP S = set;
    ScopeP ssc = sc;
    // unfold names of the module / parameters until the set's own form shows
    for (int guard = 0; guard < 16; guard++) {
      if (S->kind == N_ID) {
        if (const Arg* a = param(S->s)) { S = a->n; ssc = a->sc; continue; }
        if (!ssc->find(S->s) && S->s != "Server" && S->s != "Value") {
          const Def* d = m.find(S->s);
          if (d && d->params.empty() && !d->error.empty()) fail(n, "definition " + S->s + " does not parse");
          if (d && d->params.empty()) { S = d->body; ssc = std::make_shared<Scope>(); continue; }
        }
      }
      break;
    }
    if (S->kind == N_SETFILTER && S->bounds.size() == 1 && S->bounds[0].vars.size() == 1) {
      // e \in S' /\ P[y := e]
      NodeP inner = S->bounds[0].set;
      Ty t = member(n, e, inner, ssc, esc);
      (void)t;
      const size_t j = jump(G_JZ);
      params.push_back({S->bounds[0].vars[0], Arg{e, esc}});
      Ty p = concrete(expr(S->k[0], ssc), n);
      params.pop_back();
      if (p != T_BOOL) fail(n, "set filter predicate is not a boolean");
      const size_t k = jump(G_JMP);
      patch(j);
      emit(G_CONST, 0);
      patch(k);
      return T_BOOL;
    }
    if (S->kind == N_UNARY && S->s == "SUBSET") {  // e \subseteq S
      Ty a = concrete(expr(e, esc), n);
      Ty b = concrete(expr(S->k[0], ssc), n);
      if (a != b || (a != T_SET_SRV && a != T_SET_VAL && a != T_SET_STATE)) fail(n, "SUBSET membership of mismatched sets");
      emit(G_SUBSETEQ);
      return T_BOOL;
    }
    Ty a = concrete(expr(e, esc), n);
    Ty b = concrete(expr(S, ssc), n);
    if (elem_of(b, n) != a) fail(n, std::string(ty_name(a)) + " \\in " + ty_name(b));
    emit(G_BIT);
    return T_BOOL;
  }

  Ty junction(const std::vector<NodeP>& items, ScopeP sc, bool conj, const NodeP& n) {
    // /\: the first false item ends it with 0; \/: the first true one with 1 (TLC's short circuit)
    std::vector<size_t> exits;
    for (size_t q = 0; q < items.size(); q++) {
      Ty t = concrete(expr(items[q], sc), n);
      if (t != T_BOOL) fail(items[q], std::string("junction item is ") + ty_name(t));
      if (q + 1 < items.size()) exits.push_back(jump(conj ? G_JZ : G_JNZ));
    }
    if (exits.empty()) return T_BOOL;
    const size_t done = jump(G_JMP);
    for (size_t x : exits) patch(x);
    emit(G_CONST, conj ? 0 : 1);
    patch(done);
    return T_BOOL;
  }
  void flatten(const NodeP& n, const std::string& op, std::vector<NodeP>& out) {
    if ((n->kind == N_JUNCT || n->kind == N_BIN) && n->s == op) {
      for (auto& c : n->k) flatten(c, op, out);
    } else {
      out.push_back(n);
    }
  }

  // the elements of a constant set (for unrolled quantifiers)
  std::vector<int> const_set(const NodeP& S, ScopeP sc, Ty& elem) {
    if (S->kind == N_ID && !sc->find(S->s) && !param(S->s)) {
      if (S->s == "Server") { elem = T_SRV; std::vector<int> v; for (int x = 0; x < env.N; x++) v.push_back(x); return v; }
      if (S->s == "Value") { elem = T_VAL; std::vector<int> v; for (int x = 0; x < env.V; x++) v.push_back(x); return v; }
    }
    fail(S, "quantifier over a set other than Server or Value");
  }

  Ty quant(const NodeP& n, ScopeP sc) {
    const bool ex = n->s == "\\E";
    std::vector<std::pair<std::string, std::vector<int>>> vars;
    std::vector<Ty> tys;
    for (auto& b : n->bounds) {
      if (!b.set) fail(n, "unbounded quantifier");
      Ty et;
      std::vector<int> els = const_set(b.set, sc, et);
      for (auto& v : b.vars) { vars.push_back({v, els}); tys.push_back(et); }
    }
    // all combinations, first variable fastest
    std::vector<size_t> idx(vars.size(), 0);
    std::vector<size_t> exits;
    bool any = false;
    for (;;) {
      for (size_t q = 0; q < vars.size(); q++)
        if (vars[q].second.empty()) goto done;
      {
        auto s2 = std::make_shared<Scope>();
        s2->up = sc;
        for (size_t q = 0; q < vars.size(); q++) {
          Binding b;
          b.k = Binding::CONSTV;
          b.v = vars[q].second[idx[q]];
          b.ty = tys[q];
          s2->names[vars[q].first] = b;
        }
        Ty t = concrete(expr(n->k[0], s2), n);
        if (t != T_BOOL) fail(n, "quantified body is not a boolean");
        exits.push_back(jump(ex ? G_JNZ : G_JZ));  // \E: a true instance decides; \A: a false one
        any = true;
      }
      {
        size_t q = 0;
        while (q < vars.size() && ++idx[q] == vars[q].second.size()) idx[q++] = 0;
        if (q == vars.size()) break;
      }
    }
  done:
    emit(G_CONST, ex ? 0 : 1);
    const size_t end = jump(G_JMP);
    for (size_t x : exits) patch(x);
    emit(G_CONST, ex ? 1 : 0);
    patch(end);
    (void)any;
    return T_BOOL;
  }

  Ty expr(const NodeP& n, ScopeP sc) {
    if (++depth > 200) fail(n, "expression nested too deeply (a recursive operator?)");
    struct D { int& d; ~D() { d--; } } dd{depth};
    switch (n->kind) {
      case N_NUM: emit(G_CONST, std::stoi(n->s)); return T_INT;
      case N_ID: {
        const std::string& s = n->s;
        if (const Binding* b = sc->find(s)) {
          if (b->k == Binding::ARG) { emit(G_ARG, b->v); return b->ty; }
          if (b->k == Binding::CONSTV) { emit(G_CONST, b->v); return b->ty; }
          if (b->k == Binding::MSG) fail(n, "the message " + s + " itself as a value (its fields are read as " + s + ".f)");
          return inline_def(n, b->def, {}, sc, b->defsc.lock());
        }
        if (const Arg* a = param(s)) {
          // evaluate the argument in its own scope, without the parameters bound after it
          std::vector<std::pair<std::string, Arg>> save = params;
          while (!params.empty() && &params.back().second != a) params.pop_back();
          params.pop_back();
          Ty t = sub(*a);
          params = save;
          return t;
        }
        if (s == "TRUE") return T_TRUE;
        if (s == "FALSE") return T_FALSE;
        if (s == "Nil") return T_NIL;
        if (s == "RequestVoteRequest") { emit(G_CONST, RVREQ); return T_MTYPE; }
        if (s == "RequestVoteResponse") { emit(G_CONST, RVRESP); return T_MTYPE; }
        if (s == "AppendEntriesRequest") { emit(G_CONST, AEREQ); return T_MTYPE; }
        if (s == "AppendEntriesResponse") { emit(G_CONST, AERESP); return T_MTYPE; }
        if (s == "EqualTerm") { emit(G_CONST, 0); return T_TMATCH; }
        if (s == "LessOrEqualTerm") { emit(G_CONST, 1); return T_TMATCH; }
        if (s == "Follower") { emit(G_CONST, FOLLOWER); return T_STATE; }
        if (s == "Candidate") { emit(G_CONST, CANDIDATE); return T_STATE; }
        if (s == "Leader") { emit(G_CONST, LEADER); return T_STATE; }
        if (s == "Server") { emit(G_CONST, (1 << env.N) - 1); return T_SET_SRV; }
        if (s == "Value") { emit(G_CONST, (1 << env.V) - 1); return T_SET_VAL; }
        if (s == "electionCtr") { emit(G_ECTR); return T_INT; }
        if (s == "restartCtr") { emit(G_RCTR); return T_INT; }
        for (size_t q = 0; q < env.servers.size(); q++)
          if (env.servers[q] == s) { emit(G_CONST, (int)q); return T_SRV; }
        for (size_t q = 0; q < env.values.size(); q++)
          if (env.values[q] == s) { emit(G_CONST, (int)q); return T_VAL; }
        auto ci = env.ints.find(s);
        if (ci != env.ints.end()) { emit(G_CONST, (int)ci->second); return T_INT; }
        if (const Def* d = m.find(s)) return inline_def(n, d, {}, sc);
        fail(n, "'" + s + "' is not a state variable, constant or operator the guard compiler knows");
      }
      case N_APP: {
        const std::string& s = n->s;
        if (const Binding* b = sc->find(s))
          if (b->k == Binding::MACRO) return inline_def(n, b->def, n->k, sc, b->defsc.lock());
        int mm = -1;
        if (!sc->find(s) && n->k.size() == 1 && (mm = minmax_def(m.find(s))) >= 0) return minmax(n, n->k[0], mm, sc);
        if (!m.find(s) || sc->find(s)) {
          if (s == "Len" && n->k.size() == 1) {
            Arg x;
            if (!log_of(n->k[0], sc, x)) fail(n, "Len of something other than log[x]");
            if (sub(x) != T_SRV) fail(n, "log indexed by a non-server");
            emit(G_LEN);
            return T_INT;
          }
          if (s == "Len" && n->k.size() == 1 && n->k[0]->kind == N_FIELD && n->k[0]->s == "mentries" &&
              is_msg(n->k[0]->k[0], sc)) {
            emit(G_MF, MF_NENT);
            return T_INT;
          }
          if (s == "Cardinality" && n->k.size() == 1) {
            Ty t = concrete(expr(n->k[0], sc), n);
            if (t != T_SET_SRV && t != T_SET_VAL && t != T_SET_STATE) fail(n, "Cardinality of a non-set");
            emit(G_POPC);
            return T_INT;
          }
          fail(n, "operator '" + s + "' is not one the guard compiler knows");
        }
        return inline_def(n, m.find(s), n->k, sc);
      }
      case N_FAPP: {
        if (n->k.size() != 2) fail(n, "function application with several arguments");
        const NodeP& f = n->k[0];
        if (f->kind == N_ID && f->s == "messages" && !sc->find("messages") && !param("messages")) {
          if (!is_msg(n->k[1], sc)) fail(n, "messages[x] of something other than the handler's message");
          emit(G_MF, MF_COUNT);
          return T_INT;
        }
        if (f->kind == N_ID && !sc->find(f->s) && !param(f->s)) {
          uint32_t op;
          Ty ty;
          if (server_var(f->s, op, ty)) {
            if (concrete(expr(n->k[1], sc), n) != T_SRV) fail(n, f->s + " indexed by a non-server");
            emit(op);
            return ty;
          }
          if (f->s == "acked") {
            if (concrete(expr(n->k[1], sc), n) != T_VAL) fail(n, "acked indexed by a non-value");
            emit(G_ACKED);
            return T_ACK;
          }
        }
        if (f->kind == N_FAPP && f->k.size() == 2 && f->k[0]->kind == N_ID && !sc->find(f->k[0]->s)) {
          uint32_t op;
          Ty ty;
          if (pair_var(f->k[0]->s, op, ty)) {
            if (concrete(expr(f->k[1], sc), n) != T_SRV || concrete(expr(n->k[1], sc), n) != T_SRV)
              fail(n, f->k[0]->s + " indexed by a non-server");
            emit(op);
            return ty;
          }
        }
        fail(n, "this function application (only the state variables' own indexing is compiled)");
      }
      case N_FIELD: {  // log[x][k].term / .value, and a compiled handler's m.f / m.mentries[1].term / .value
        const NodeP& e = n->k[0];
        if (is_msg(e, sc)) {
          int mf;
          Ty ty;
          if (!msg_field_of(n->s, mf, ty)) fail(n, "a message has no field " + n->s);
          emit(G_MF, mf);
          return ty;
        }
        if (e->kind == N_FAPP && e->k.size() == 2 && e->k[0]->kind == N_FIELD && e->k[0]->s == "mentries" &&
            is_msg(e->k[0]->k[0], sc) && (n->s == "term" || n->s == "value")) {
          if (e->k[1]->kind != N_NUM || e->k[1]->s != "1") fail(n, "a message entry other than mentries[1]");
          emit(G_MF, MF_NENT);  // mentries[1] of <<>>: TLC's evaluation error
          const size_t ok = jump(G_JNZ);
          emit(G_ERR);
          patch(ok);
          emit(G_MF, n->s == "term" ? MF_ETERM : MF_EVALUE);
          return n->s == "term" ? T_INT : T_VAL;
        }
        if (e->kind == N_FAPP && e->k.size() == 2 && (n->s == "term" || n->s == "value")) {
          Arg x;
          if (log_of(e->k[0], sc, x)) {
            if (sub(x) != T_SRV) fail(n, "log indexed by a non-server");
            if (concrete(expr(e->k[1], sc), n) != T_INT) fail(n, "log index is not an integer");
            emit(n->s == "term" ? G_LOGTERM : G_LOGVAL);
            return n->s == "term" ? T_INT : T_VAL;
          }
        }
        fail(n, "field access other than log[x][k].term / .value");
      }
      case N_UNARY: {
        if (n->s == "~" || n->s == "\\lnot" || n->s == "\\neg") {
          if (concrete(expr(n->k[0], sc), n) != T_BOOL) fail(n, "~ of a non-boolean");
          emit(G_NOT);
          return T_BOOL;
        }
        if (n->s == "-") {
          if (concrete(expr(n->k[0], sc), n) != T_INT) fail(n, "- of a non-integer");
          emit(G_NEG);
          return T_INT;
        }
        fail(n, "unary " + n->s);
      }
      case N_JUNCT:
      case N_BIN: {
        const std::string& op = n->s;
        if (op == "/\\" || op == "\\/" || op == "\\land" || op == "\\lor") {
          const bool conj = op == "/\\" || op == "\\land";
          std::vector<NodeP> items;
          flatten(n, op, items);
          return junction(items, sc, conj, n);
        }
        if (op == "=>") {  // ~a \/ b
          if (concrete(expr(n->k[0], sc), n) != T_BOOL) fail(n, "=> of a non-boolean");
          const size_t j = jump(G_JZ);
          if (concrete(expr(n->k[1], sc), n) != T_BOOL) fail(n, "=> of a non-boolean");
          const size_t e = jump(G_JMP);
          patch(j);
          emit(G_CONST, 1);
          patch(e);
          return T_BOOL;
        }
        if (op == "+") return bin_int(n, sc, G_ADD);
        if (op == "-") return bin_int(n, sc, G_SUB);
        if (op == "*") return bin_int(n, sc, G_MUL);
        if (op == "=" || op == "/=" || op == "#" || op == "<" || op == ">" || op == "<=" || op == "=<" ||
            op == ">=" || op == "\\leq" || op == "\\geq")
          return compare(n, sc, op);
        if (op == "\\in") return member(n, n->k[0], n->k[1], sc, sc);
        if (op == "\\notin") {
          member(n, n->k[0], n->k[1], sc, sc);
          emit(G_NOT);
          return T_BOOL;
        }
        if (op == "\\subseteq") {
          Ty a = concrete(expr(n->k[0], sc), n), b = concrete(expr(n->k[1], sc), n);
          if (a != b || (a != T_SET_SRV && a != T_SET_VAL && a != T_SET_STATE)) fail(n, "\\subseteq of mismatched sets");
          emit(G_SUBSETEQ);
          return T_BOOL;
        }
        if (op == "\\cup" || op == "\\union" || op == "\\cap" || op == "\\intersect" || op == "\\") {
          Ty a = concrete(expr(n->k[0], sc), n), b = concrete(expr(n->k[1], sc), n);
          if (a != b || (a != T_SET_SRV && a != T_SET_VAL && a != T_SET_STATE)) fail(n, op + " of mismatched sets");
          emit(op == "\\cup" || op == "\\union" ? G_BOR : op == "\\" ? G_BDIFF : G_BAND);
          return a;
        }
        fail(n, "operator " + op);
      }
      case N_SETENUM: {
        emit(G_CONST, 0);
        Ty et = T_SRV;
        bool first = true;
        for (auto& c : n->k) {
          Ty t = expr(c, sc);
          if (t == T_NIL) {  // {Nil, j} (Raft.tla:372): a set of servers with Nil's code (votedFor's Nil)
            emit(G_CONST, NILS);
            t = T_SRV;
          }
          t = concrete(t, n);
          if (!first && t != et) fail(n, "set literal of mixed types");
          et = t;
          first = false;
          emit(G_SETADD);
        }
        if (first) fail(n, "empty set literal (its type is not known)");
        return set_of(et, n);
      }
      case N_IF: {
        if (concrete(expr(n->k[0], sc), n) != T_BOOL) fail(n, "IF condition is not a boolean");
        const size_t j = jump(G_JZ);
        Ty a = concrete(expr(n->k[1], sc), n);
        const size_t e = jump(G_JMP);
        patch(j);
        Ty b = concrete(expr(n->k[2], sc), n);
        patch(e);
        if (a != b) fail(n, "IF branches of different types");
        return a;
      }
      case N_LET: {
        auto s2 = std::make_shared<Scope>();
        s2->up = sc;
        for (auto& d : n->defs) {
          Binding b;
          b.k = Binding::MACRO;
          b.def = &d;
          b.defsc = s2;
          s2->names[d.name] = b;
        }
        return expr(n->k[0], s2);
      }
      case N_QUANT: return quant(n, sc);
      case N_AT:
        if (!at) fail(n, "@ outside an EXCEPT the effect compiler knows");
        return at();
      case N_SETFILTER: {  // {y \in S : P} over a constant set: the bitmask of the elements P holds for
        if (n->bounds.size() != 1 || n->bounds[0].vars.size() != 1) fail(n, "set filter over several variables");
        Ty et;
        const std::vector<int> els = const_set(n->bounds[0].set, sc, et);
        emit(G_CONST, 0);
        for (int e : els) {
          auto s2 = std::make_shared<Scope>();
          s2->up = sc;
          Binding b;
          b.k = Binding::CONSTV;
          b.v = e;
          b.ty = et;
          s2->names[n->bounds[0].vars[0]] = b;
          if (concrete(expr(n->k[0], s2), n) != T_BOOL) fail(n, "set filter predicate is not a boolean");
          const size_t skip = jump(G_JZ);
          emit(G_CONST, e);
          emit(G_SETADD);
          patch(skip);
        }
        return set_of(et, n);
      }
      default: break;
    }
    fail(n, "this construct");
  }

  // (defsc: a LET definition's own scope -- TLA+ LET bodies see the names
  // bound around them, e.g. a handler's message; a module operator sees none)
  // The specs' Min / Max (Raft.tla:190-192: CHOOSE x \in s : \A y \in s : x <= y,
  // resp. x >= y) -- recognised by that shape, whatever the name: 0 Min, 1 Max,
  // -1 another definition.
  static int minmax_def(const Def* d) {
    if (!d || d->params.size() != 1 || !d->body || d->body->kind != N_CHOOSE) return -1;
    const Node& c = *d->body;
    auto is_id = [](const NodeP& n, const std::string& s) { return n && n->kind == N_ID && n->s == s; };
    if (c.bounds.size() != 1 || c.bounds[0].vars.size() != 1 || !is_id(c.bounds[0].set, d->params[0]) || c.k.size() != 1)
      return -1;
    const NodeP& q = c.k[0];
    if (q->kind != N_QUANT || q->s != "\\A" || q->bounds.size() != 1 || q->bounds[0].vars.size() != 1 ||
        !is_id(q->bounds[0].set, d->params[0]) || q->k.size() != 1)
      return -1;
    const NodeP& b = q->k[0];
    const std::string& x = c.bounds[0].vars[0];
    const std::string& y = q->bounds[0].vars[0];
    if (b->kind != N_BIN || b->k.size() != 2 || x == y) return -1;
    const bool xy = is_id(b->k[0], x) && is_id(b->k[1], y), yx = is_id(b->k[0], y) && is_id(b->k[1], x);
    if (!xy && !yx) return -1;
    const std::string& op = b->s;
    const bool le = op == "<=" || op == "=<" || op == "\\leq", ge = op == ">=" || op == "\\geq";
    if (!le && !ge) return -1;
    return (le == xy) ? 0 : 1;
  }
  // Min / Max of a set literal of one or two integers: IF a <= b THEN a ELSE b
  // (its operands are pure, so each is evaluated again where it is chosen).
  Ty minmax(const NodeP& at, const NodeP& set, int is_max, ScopeP sc) {
    if (set->kind != N_SETENUM || set->k.empty() || set->k.size() > 2)
      fail(at, "Min / Max of something other than a literal of one or two integers");
    if (concrete(expr(set->k[0], sc), at) != T_INT) fail(at, "Min / Max of a non-integer");
    if (set->k.size() == 1) return T_INT;
    if (concrete(expr(set->k[1], sc), at) != T_INT) fail(at, "Min / Max of a non-integer");
    emit(is_max ? G_LE : G_LT);  // Max: a <= b picks b; Min: a < b picks a
    const size_t j = jump(is_max ? G_JNZ : G_JZ);
    expr(set->k[0], sc);
    const size_t e = jump(G_JMP);
    patch(j);
    expr(set->k[1], sc);
    patch(e);
    return T_INT;
  }
  Ty inline_def(const NodeP& at, const Def* d, const std::vector<NodeP>& args, ScopeP sc, ScopeP defsc = nullptr) {
    if (!d->error.empty()) fail(at, "definition " + d->name + " does not parse: " + d->error);
    if (d->params.size() != args.size()) fail(at, "operator " + d->name + " applied to the wrong number of arguments");
    const size_t base = params.size();
    for (size_t q = 0; q < args.size(); q++) params.push_back({d->params[q], Arg{args[q], sc}});
    // the body sees only its parameters (and the module), not the caller's bound names
    auto s2 = std::make_shared<Scope>();
    s2->up = defsc;
    Ty t = expr(d->body, s2);
    params.resize(base);
    return t;
  }
};

}  // namespace

namespace {
// The stack-depth check of every compiled program, guards and effects alike:
// guard_vm / effect_vm keep the stack in eight registers, so each path's depth
// is followed (the code is structured: each instruction has one depth on all
// paths).  A guard (guard_end) must leave its value on the stack at G_END.
void check_depth(const std::vector<uint32_t>& code, const std::string& where, bool guard_end = false) {
  std::vector<int> at(code.size() + 1, -1);
  std::vector<size_t> work{0};
  at[0] = 0;
  auto flow = [&](size_t to, int d) {
    if (to > code.size()) throw std::runtime_error(where + ": a jump leaves the code (compiler bug)");
    if (at[to] < 0) { at[to] = d; work.push_back(to); }
    else if (at[to] != d) throw std::runtime_error(where + ": stack depths disagree at a join (compiler bug)");
  };
  while (!work.empty()) {
    const size_t pc = work.back();
    work.pop_back();
    if (pc == code.size()) continue;
    const uint32_t op = code[pc] & 0xFFu;
    const int imm = (int)code[pc] >> 8;
    int d = at[pc], need = 0, delta = 0;
    switch (op) {
      case G_END:
        if (guard_end && d < 1) throw std::runtime_error(where + ": empty stack at the end");
        continue;
      case E_END: case G_ERR: continue;  // (G_ERR: the program ends with an evaluation error)
      case G_MF: delta = 1; break;
      case E_DISCARD: break;
      case E_REPLY: need = imm == AERESP ? 5 : 4; delta = -need; break;
      case G_CONST: case G_ARG: case G_ECTR: case G_RCTR: delta = 1; break;
      case G_ST: case G_TERM: case G_VOTED: case G_VOTED2: case G_LEN: case G_COMMIT: case G_FSYNC: case G_VOTES:
      case G_ACKED: case G_NEG: case G_NOT: case G_POPC: need = 1; break;
      case G_JZ: case G_JNZ: need = 1; delta = -1; break;
      case G_JMP: break;
      case G_POP: case E_ST: case E_TERM: case E_VOTED: case E_VOTES: case E_COMMIT: case E_ECTR: case E_RCTR:
        need = 1; delta = -1; break;
      case E_ACKED: case E_APPEND: case E_NEXT: case E_MATCH: case E_PEND: need = 2; delta = -2; break;
      case E_RVREQ: need = 5; delta = -5; break;
      default: need = 2; delta = -1; break;  // binary operators
    }
    if (d < need) throw std::runtime_error(where + ": stack underflow (compiler bug)");
    d += delta;
    if (d > 8)
      throw std::runtime_error(where + " nests deeper than the machine's 8-value stack: split it into helper conjuncts");
    if (op == G_JMP) { flow(pc + 1 + imm, d); continue; }
    if (op == G_JZ || op == G_JNZ) flow(pc + 1 + imm, d);
    flow(pc + 1, d);
  }
}
}  // namespace

std::vector<uint32_t> compile_guard(const Module& m, const std::vector<std::string>& action_params,
                                    const std::vector<int>& param_types, const std::vector<NodeP>& conjuncts,
                                    const GuardEnv& env, const std::string& where) {
  Compiler c(m, env);
  c.where = where;
  auto sc = std::make_shared<Scope>();
  for (size_t q = 0; q < action_params.size(); q++) {
    Binding b;
    b.k = Binding::ARG;
    b.v = (int)q;
    b.ty = param_types[q] == 1 ? T_VAL : T_SRV;
    sc->names[action_params[q]] = b;
  }
  if (conjuncts.empty()) {
    c.emit(G_CONST, 1);
  } else {
    NodeP root = conjuncts[0];
    Ty t = c.junction(conjuncts, sc, true, root);
    if (t != T_BOOL) c.fail(root, "the guard is not a boolean");
  }
  c.emit(G_END);
  // guard_vm keeps its stack in eight registers: every path's depth is checked
  check_depth(c.code, "guard of " + where, true);
  return c.code;
}


namespace {
// The effect conjuncts of a compiled action, shared by compile_effect (a
// fixed-binding action: its server is its first parameter) and
// compile_handler (a message handler: its server is the bound message's
// mdest).  Each item emits effect_vm stores after the expression machine's
// code for its values; `done` / `kept` track every VARIABLE (assigned,
// UNCHANGED) for the completeness check.
struct EffectGen {
  Compiler& c;
  const Module& m;
  const GuardEnv& env;
  std::string where;
  std::function<bool(const NodeP&, ScopeP)> own;  // the action's own server?
  std::string own_name;                            // ... as the text names it (messages)
  bool handler = false;                            // a message handler (Discard / Reply allowed)
  std::set<std::string> vars, done, kept;
  bool sent = false;
  EffectGen(Compiler& c_, const Module& m_, const GuardEnv& e_, const std::string& w)
      : c(c_), m(m_), env(e_), where(w), vars(m_.variables.begin(), m_.variables.end()) {}

  [[noreturn]] void fail(const NodeP& n, const std::string& what) {
    throw std::runtime_error("effect of " + where + " (line " + std::to_string(n ? n->line : 0) + "): " + what);
  }
  void mark(const std::string& v, const NodeP& n) {
    if (!vars.count(v)) fail(n, v + " is not a variable of the module");
    if (done.count(v)) fail(n, v + " is changed twice");
    if (kept.count(v)) fail(n, v + " is both changed and UNCHANGED");
    done.insert(v);
  }
  // UNCHANGED e: variables, tuples of them, and definitions naming them (a
  // variable may be named twice: RaftFsync.tla:116 lists fsyncIndex twice)
  void unchanged(const NodeP& n, int depth) {
    if (depth > 16) fail(n, "UNCHANGED nests too deeply");
    if (n->kind == N_TUPLE) { for (auto& k : n->k) unchanged(k, depth + 1); return; }
    if (n->kind == N_ID) {
      if (vars.count(n->s)) {
        if (done.count(n->s)) fail(n, n->s + " is both changed and UNCHANGED");
        kept.insert(n->s);
        return;
      }
      const Def* d = m.find(n->s);
      if (d && d->params.empty() && d->body) { unchanged(d->body, depth + 1); return; }
    }
    fail(n, "UNCHANGED of something other than variables");
  }
  void value(const NodeP& e, Ty want, ScopeP sc) {
    if (e->kind == N_SETENUM && e->k.empty() && (want == T_SET_SRV || want == T_SET_VAL || want == T_SET_STATE)) {
      c.emit(G_CONST, 0);  // {} takes the variable's set type
      return;
    }
    Ty t = c.expr(e, sc);
    if (t == T_NIL || t == T_TRUE || t == T_FALSE) {
      c.emit(G_CONST, c.sym_code(t, want, e));
      t = want;
    }
    if (t != want) fail(e, std::string("the new value is ") + ty_name(t) + ", the variable holds " + ty_name(want));
  }
  // [v EXCEPT ![p] = e]: the single path element and its value
  void except1(const NodeP& rhs, const std::string& v, NodeP& path, NodeP& val) {
    if (rhs->kind != N_EXCEPT || rhs->k.size() != 2 || rhs->k[0]->kind != N_ID || rhs->k[0]->s != v ||
        rhs->paths.size() != 1 || rhs->paths[0].size() != 1 || rhs->paths[0][0].field ||
        rhs->paths[0][0].args.size() != 1)
      fail(rhs, v + "' must be [" + v + " EXCEPT ![x] = e]");
    path = rhs->paths[0][0].args[0];
    val = rhs->k[1];
  }
  // One effect conjunct; false when n is not one (the caller reports it).
  bool item(const NodeP& n, ScopeP sc) {
    if (n->kind == N_UNARY && n->s == "UNCHANGED") { unchanged(n->k[0], 0); return true; }
    if (n->kind == N_BIN && n->s == "=" && n->k[0]->kind == N_PRIME && n->k[0]->k[0]->kind == N_ID) {
      const std::string v = n->k[0]->k[0]->s;
      const NodeP& rhs = n->k[1];
      mark(v, n);
      uint32_t load = 0, store = 0;
      Ty ty = T_INT;
      if (v == "state") { load = G_ST; store = E_ST; ty = T_STATE; }
      else if (v == "currentTerm") { load = G_TERM; store = E_TERM; ty = T_INT; }
      else if (v == "votedFor") { load = G_VOTED; store = E_VOTED; ty = T_SRV; }
      else if (v == "votesGranted") { load = G_VOTES; store = E_VOTES; ty = T_SET_SRV; }
      else if (v == "commitIndex") { load = G_COMMIT; store = E_COMMIT; ty = T_INT; }
      if (store) {
        NodeP path, val;
        except1(rhs, v, path, val);
        if (!own(path, sc)) fail(path, v + " may change at the action's own server (" + own_name + ") only");
        Compiler& cc = c;
        c.at = [&cc, load, ty]() { cc.emit(G_ARG, 0); cc.emit(load); return ty; };
        value(val, ty, sc);
        c.at = nullptr;
        c.emit(store);
        return true;
      }
      // the leader's rows: [v EXCEPT ![i] = [j \in Server |-> e]] (unrolled over
      // Server) or [v EXCEPT ![i][q] = e]
      uint32_t rstore = 0;
      Ty rty = T_INT;
      if (v == "nextIndex") { rstore = E_NEXT; }
      else if (v == "matchIndex") { rstore = E_MATCH; }
      else if (v == "pendingResponse" && env.spec == RAFT) { rstore = E_PEND; rty = T_BOOL; }
      if (rstore) {
        if (rhs->kind != N_EXCEPT || rhs->k.size() != 2 || rhs->k[0]->kind != N_ID || rhs->k[0]->s != v ||
            rhs->paths.size() != 1 || rhs->paths[0].empty() || rhs->paths[0].size() > 2 || rhs->paths[0][0].field ||
            rhs->paths[0][0].args.size() != 1 || (rhs->paths[0].size() == 2 && (rhs->paths[0][1].field ||
                                                                                 rhs->paths[0][1].args.size() != 1)))
          fail(rhs, v + "' must be [" + v + " EXCEPT ![i] = [j \\in Server |-> e]] or [" + v + " EXCEPT ![i][j] = e]");
        if (!own(rhs->paths[0][0].args[0], sc))
          fail(rhs->paths[0][0].args[0], v + " may change at the action's own server (" + own_name + ") only");
        const NodeP& val = rhs->k[1];
        if (rhs->paths[0].size() == 2) {  // one entry: ![i][q] = e
          const NodeP& q = rhs->paths[0][1].args[0];
          if (c.concrete(c.expr(q, sc), q) != T_SRV) fail(q, v + " indexed by a non-server");
          value(val, rty, sc);
          c.emit(rstore);
          return true;
        }
        if (val->kind != N_FUNC || val->bounds.size() != 1 || val->bounds[0].vars.size() != 1 || !val->bounds[0].set ||
            val->bounds[0].set->kind != N_ID || val->bounds[0].set->s != "Server")
          fail(val, v + "[i]' must be a function [j \\in Server |-> e]");
        for (int x = 0; x < env.N; x++) {
          auto s2 = std::make_shared<Scope>();
          s2->up = sc;
          Binding b;
          b.k = Binding::CONSTV;
          b.v = x;
          b.ty = T_SRV;
          s2->names[val->bounds[0].vars[0]] = b;
          c.emit(G_CONST, x);
          Ty t = c.expr(val->k[0], s2);
          if (t == T_NIL || t == T_TRUE || t == T_FALSE) {
            c.emit(G_CONST, c.sym_code(t, rty, val->k[0]));
            t = rty;
          }
          if (t != rty) fail(val->k[0], std::string("the new value is ") + ty_name(t) + ", " + v + " holds " + ty_name(rty));
          c.emit(rstore);
        }
        return true;
      }
      if (v == "electionCtr" || v == "restartCtr") {
        value(rhs, T_INT, sc);
        c.emit(v == "electionCtr" ? E_ECTR : E_RCTR);
        return true;
      }
      if (v == "acked") {
        NodeP path, val;
        except1(rhs, v, path, val);
        if (c.concrete(c.expr(path, sc), path) != T_VAL) fail(path, "acked indexed by a non-value");
        value(val, T_ACK, sc);  // (no @ here: the compiler refuses it)
        c.emit(E_ACKED);
        return true;
      }
      if (v == "log") {
        NodeP path, val;
        except1(rhs, v, path, val);
        if (!own(path, sc)) fail(path, "log may change at the action's own server only");
        const bool app = val->kind == N_APP && val->s == "Append" && val->k.size() == 2 && !m.find("Append");
        const NodeP base = app ? val->k[0] : nullptr;
        const bool on_own = base && (base->kind == N_AT || (base->kind == N_FAPP && base->k.size() == 2 &&
                                                            base->k[0]->kind == N_ID && base->k[0]->s == "log" &&
                                                            own(base->k[1], sc)));
        if (!app || !on_own) fail(val, "log[i]' must be Append(@, entry) or Append(log[i], entry)");
        const NodeP& rec = val->k[1];
        if (rec->kind != N_RECORD || rec->names.size() != 2) fail(rec, "a log entry is [term |-> t, value |-> v]");
        NodeP tv, vv;
        for (size_t q = 0; q < 2; q++) (rec->names[q] == "term" ? tv : vv) = rec->k[q];
        if (!tv || !vv) fail(rec, "a log entry is [term |-> t, value |-> v]");
        value(tv, T_INT, sc);
        value(vv, T_VAL, sc);
        c.emit(E_APPEND);
        return true;
      }
      fail(n, "the effect compiler does not assign " + v + " (it may stay UNCHANGED)");
    }
    // the bag helpers (the lowering checked each is the family's own, by closure
    // hash): a set of RequestVoteRequest records {[...] : j \in S} sent all new
    // (class 0), or one record sent new (1) or with its count + 1 (2); in a
    // message handler, Discard(m) (3) and Reply(response, m) (4)
    if (n->kind == N_APP && env.send_helpers.count(n->s)) {
      const int cls = env.send_helpers.at(n->s);
      if (cls >= 3) {
        if (!handler) fail(n, n->s + " outside a message handler (no bound message)");
        if (n->k.size() != (cls == 3 ? 1u : 2u) || !c.is_msg(n->k.back(), sc))
          fail(n, n->s + " of something other than the handler's message");
        if (sent) fail(n, "messages are changed twice");
        sent = true;
        mark("messages", n);
        if (cls == 3) {
          c.emit(E_DISCARD);
          return true;
        }
        const NodeP& rec = n->k[0];
        if (rec->kind != N_RECORD) fail(rec, "Reply of something other than a record literal");
        std::map<std::string, NodeP> f;
        for (size_t q = 0; q < rec->names.size(); q++) f[rec->names[q]] = rec->k[q];
        const bool rv = f.size() == 5 && f.count("mtype") && f["mtype"]->kind == N_ID &&
                        f["mtype"]->s == "RequestVoteResponse" && f.count("mterm") && f.count("mvoteGranted") &&
                        f.count("msource") && f.count("mdest");
        const bool ae = f.size() == 6 && f.count("mtype") && f["mtype"]->kind == N_ID &&
                        f["mtype"]->s == "AppendEntriesResponse" && f.count("mterm") && f.count("msuccess") &&
                        f.count("mmatchIndex") && f.count("msource") && f.count("mdest");
        if (!rv && !ae) fail(rec, "the handler compiler replies with RequestVoteResponse or AppendEntriesResponse records");
        auto field = [&](const char* name, Ty t) { value(f[name], t, sc); };
        field("mterm", T_INT);
        field(rv ? "mvoteGranted" : "msuccess", T_BOOL);
        if (ae) field("mmatchIndex", T_INT);
        field("msource", T_SRV);
        field("mdest", T_SRV);
        c.emit(E_REPLY, rv ? RVRESP : AERESP);
        return true;
      }
      if (sent) fail(n, "messages are sent twice");
      sent = true;
      mark("messages", n);
      NodeP rec = n->k[0];
      const NodeP S = cls == 0 ? n->k[0] : nullptr;
      if (cls == 0) {
        if (S->kind != N_SETMAP || S->bounds.size() != 1 || S->bounds[0].vars.size() != 1)
          fail(S, n->s + " of something other than {record : j \\in S}");
        rec = S->k[0];
      }
      if (rec->kind != N_RECORD) fail(rec, n->s + " of something other than a record literal");
      std::map<std::string, NodeP> f;
      for (size_t q = 0; q < rec->names.size(); q++) f[rec->names[q]] = rec->k[q];
      const char* want[] = {"mtype", "mterm", "mlastLogTerm", "mlastLogIndex", "msource", "mdest"};
      bool rv = f.size() == 6 && f.count("mtype") && f["mtype"]->kind == N_ID && f["mtype"]->s == "RequestVoteRequest";
      for (const char* w : want) rv = rv && f.count(w);
      if (!rv) fail(rec, "the effect compiler sends RequestVoteRequest records only");
      auto send = [&](ScopeP s2) {
        auto field = [&](const char* name, Ty t) {
          Ty got = c.concrete(c.expr(f[name], s2), f[name]);
          if (got != t) fail(f[name], std::string(name) + " is " + ty_name(got));
        };
        field("mterm", T_INT);
        field("mlastLogTerm", T_INT);
        field("mlastLogIndex", T_INT);
        field("msource", T_SRV);
        field("mdest", T_SRV);
        c.emit(E_RVREQ, cls == 2 ? 1 : 0);
      };
      if (cls != 0) {
        send(sc);
        return true;
      }
      const std::string jv = S->bounds[0].vars[0];
      // TLC's set {rec : j \in S} holds each distinct record once; one E_RVREQ
      // per member is that set only when the records are pairwise distinct,
      // which mdest = j guarantees -- any other form could send a
      // record twice where TLC's set has it once, so it is refused
      if (f["mdest"]->kind != N_ID || f["mdest"]->s != jv)
        fail(f["mdest"], n->s + " of {record : " + jv + " \\in S} whose mdest is not " + jv +
                             " (the records must be distinct per member)");
      // over every server x: if x \in S, send the record with j = x
      for (int x = 0; x < env.N; x++) {
        auto s2 = std::make_shared<Scope>();
        s2->up = sc;
        Binding b;
        b.k = Binding::CONSTV;
        b.v = x;
        b.ty = T_SRV;
        s2->names[jv] = b;
        auto xnode = std::make_shared<Node>();
        xnode->kind = N_ID;
        xnode->s = jv;
        xnode->line = S->line;
        if (c.member(S, xnode, S->bounds[0].set, sc, s2) != T_BOOL) fail(S, "the message set's domain");
        const size_t skip = c.jump(G_JZ);
        send(s2);
        c.patch(skip);
      }
      return true;
    }
    return false;
  }
  // every VARIABLE assigned, UNCHANGED or (messages) sent to
  void complete() {
    for (const std::string& v : vars)
      if (!done.count(v) && !kept.count(v))
        throw std::runtime_error("effect of " + where + ": " + v + " is neither assigned nor UNCHANGED");
  }
};
}  // namespace

// An action's EFFECT compiled for effect_vm (rmc_spec.h): the conjuncts that
// prime a variable, say UNCHANGED, or send messages, over the same typed
// expression language as the guards (they read the unprimed state).  Server
// variables may change at the action's own server only ([v EXCEPT ![i] = e],
// with @), as every action of these specs does; the forms are those of the
// specs' fixed-binding actions (Raft.tla:226-313): state, currentTerm,
// votedFor, votesGranted, commitIndex, electionCtr, restartCtr, acked[v],
// log[i] = Append(@, [term |-> t, value |-> v]), and SendMultipleOnce of a set
// of RequestVoteRequest records {[...] : j \in S}.  Every VARIABLE must be
// assigned, left UNCHANGED or (messages) sent to; anything else is refused
// naming it.
std::vector<uint32_t> compile_effect(const Module& m, const std::vector<std::string>& action_params,
                                     const std::vector<int>& param_types, const std::vector<NodeP>& effects,
                                     const GuardEnv& env, const std::string& where) {
  Compiler c(m, env);
  c.where = where;
  if (env.spec != RAFT && env.spec != FLEX && env.spec != FSYNC)
    throw std::runtime_error("effect of " + where + ": the effect compiler knows the Raft, FlexibleRaft and RaftFsync "
                             "layouts only");
  auto sc = std::make_shared<Scope>();
  for (size_t q = 0; q < action_params.size(); q++) {
    Binding b;
    b.k = Binding::ARG;
    b.v = (int)q;
    b.ty = param_types[q] == 1 ? T_VAL : T_SRV;
    sc->names[action_params[q]] = b;
  }
  EffectGen g(c, m, env, where);
  g.own_name = action_params.empty() ? "?" : action_params[0];
  g.own = [&](const NodeP& n, ScopeP) { return n->kind == N_ID && !action_params.empty() && n->s == action_params[0]; };
  std::vector<NodeP> items;
  for (auto& e : effects) c.flatten(e, "/\\", items);
  for (auto& n : items)
    if (!g.item(n, sc))
      g.fail(n, "this effect conjunct (the effect compiler knows v' = ..., UNCHANGED and the module's send helpers)");
  g.complete();
  c.emit(E_END);
  check_depth(c.code, "effect of " + where);
  return c.code;
}

// A message handler compiled whole (K_MSGC): the body of \E m \in DOMAIN
// messages : body as ONE effect_vm program, its conjuncts in the text's order
// -- a guard conjunct jumps to the disabled exit when false, an effect
// conjunct stores into the successor -- so a guard after an effect still
// disables (the partial successor is dropped).  The effects act on the bound
// message's mdest (effect_vm's server i, what the reference handlers name
// LET i == m.mdest, Raft.tla:364, :388, :416): an EXCEPT path must denote
// m.mdest.  LET definitions are macros; an operator of the module whose body
// has effects is inlined; a disjunction of effects is taken when it has two
// branches whose leading guards are complementary (p and ~p, x = y and
// x # y), each branch's guards before its effects -- the form of
// Raft.tla:375-376 and :394-397; any other disjunction of effects would give
// TLC one successor per true branch and is refused.
std::vector<uint32_t> compile_handler(const Module& m, const std::vector<std::string>& params,
                                      const std::vector<NodeP>& body, const GuardEnv& env, const std::string& where) {
  Compiler c(m, env);
  c.where = where;
  if (env.spec != RAFT && env.spec != FLEX && env.spec != FSYNC)
    throw std::runtime_error("handler " + where + ": the handler compiler knows the Raft, FlexibleRaft and RaftFsync "
                             "layouts only");
  if (params.size() != 1) throw std::runtime_error("handler " + where + ": binds one message");
  auto sc = std::make_shared<Scope>();
  {
    Binding b;
    b.k = Binding::MSG;
    sc->names[params[0]] = b;
  }
  EffectGen g(c, m, env, where);
  g.handler = true;
  g.own_name = params[0] + ".mdest";
  g.own = [&c](const NodeP& n, ScopeP s2) { return c.is_mdest(n, s2); };
  auto fail = [&](const NodeP& n, const std::string& what) -> void { g.fail(n, what); };
  // does n change the state (a prime, UNCHANGED, a bag helper, or an operator of the module whose body does)?
  std::function<bool(const NodeP&, int)> effectful = [&](const NodeP& n, int depth) -> bool {
    if (!n || depth > 64) return false;
    if (n->kind == N_PRIME) return true;
    if (n->kind == N_UNARY && n->s == "UNCHANGED") return true;
    if ((n->kind == N_APP || n->kind == N_ID) && env.send_helpers.count(n->s)) return true;
    if ((n->kind == N_APP || n->kind == N_ID) && !sc->find(n->s)) {
      const Def* d = m.find(n->s);
      if (d && d->error.empty() && d->body && effectful(d->body, depth + 1)) return true;
    }
    for (auto& k : n->k)
      if (effectful(k, depth + 1)) return true;
    for (auto& d : n->defs)
      if (effectful(d.body, depth + 1)) return true;
    return false;
  };
  // structural equality (the complementary-guard test)
  std::function<bool(const NodeP&, const NodeP&)> same = [&](const NodeP& a, const NodeP& b) -> bool {
    if (!a || !b) return a == b;
    if (a->kind != b->kind || a->s != b->s || a->k.size() != b->k.size() || a->names != b->names) return false;
    for (size_t q = 0; q < a->k.size(); q++)
      if (!same(a->k[q], b->k[q])) return false;
    return true;
  };
  auto negation_of = [&](const NodeP& a, const NodeP& b) {  // b == ~a (or a and b a complementary comparison)
    if (b->kind == N_UNARY && (b->s == "~" || b->s == "\\lnot" || b->s == "\\neg") && same(a, b->k[0])) return true;
    const bool ca = a->kind == N_BIN && a->s == "=", cb = b->kind == N_BIN && (b->s == "#" || b->s == "/=");
    return ca && cb && same(a->k[0], b->k[0]) && same(a->k[1], b->k[1]);
  };
  std::vector<size_t> disabled;  // jumps to the disabled exit
  std::function<void(const NodeP&, ScopeP, std::vector<size_t>&)> stmt;
  auto guard = [&](const NodeP& n, ScopeP s2, std::vector<size_t>& exits) {
    const Ty t = c.concrete(c.expr(n, s2), n);
    if (t != T_BOOL) fail(n, std::string("a guard conjunct is ") + ty_name(t));
    exits.push_back(c.jump(G_JZ));
  };
  stmt = [&](const NodeP& n, ScopeP s2, std::vector<size_t>& exits) {
    if ((n->kind == N_JUNCT || n->kind == N_BIN) && (n->s == "/\\" || n->s == "\\land")) {
      std::vector<NodeP> items;
      c.flatten(n, n->s, items);
      for (auto& x : items) stmt(x, s2, exits);
      return;
    }
    if (!effectful(n, 0)) { guard(n, s2, exits); return; }
    if (n->kind == N_LET) {
      auto s3 = std::make_shared<Scope>();
      s3->up = s2;
      for (auto& d : n->defs) {
        Binding b;
        b.k = Binding::MACRO;
        b.def = &d;
        b.defsc = s3;
        s3->names[d.name] = b;
      }
      stmt(n->k[0], s3, exits);
      return;
    }
    if ((n->kind == N_JUNCT || n->kind == N_BIN) && (n->s == "\\/" || n->s == "\\lor")) {
      std::vector<NodeP> br;
      c.flatten(n, n->s, br);
      if (br.size() != 2) fail(n, "a disjunction of effects with other than two branches");
      std::vector<NodeP> items[2], guards[2];
      for (int q = 0; q < 2; q++) {
        c.flatten(br[q], "/\\", items[q]);
        bool eff = false;
        for (auto& x : items[q]) {
          if (effectful(x, 0)) eff = true;
          else if (eff) fail(x, "a guard after an effect inside a disjunction of effects");
          else guards[q].push_back(x);
        }
      }
      if (guards[0].size() != 1 || guards[1].size() != 1 ||
          !(negation_of(guards[0][0], guards[1][0]) || negation_of(guards[1][0], guards[0][0])))
        fail(n, "a disjunction of effects whose branches do not start with complementary guards (p and ~p): TLC "
                "would take every branch whose guard holds");
      const auto d0 = g.done, k0 = g.kept;
      const bool s0 = g.sent;
      std::set<std::string> cover[2], chg[2];
      bool snt[2];
      std::vector<size_t> to_next, to_end;
      for (int q = 0; q < 2; q++) {
        g.done = d0;
        g.kept = k0;
        g.sent = s0;
        std::vector<size_t>& gx = q == 0 ? to_next : exits;  // branch 0's guard false: try branch 1
        guard(guards[q][0], s2, gx);
        for (size_t x = 1; x < items[q].size(); x++)
          if (!g.item(items[q][x], s2)) fail(items[q][x], "this effect conjunct");
        chg[q] = g.done;
        cover[q] = g.done;
        cover[q].insert(g.kept.begin(), g.kept.end());
        snt[q] = g.sent;
        if (q == 0) {
          to_end.push_back(c.jump(G_JMP));
          for (size_t x : to_next) c.patch(x);
        }
      }
      for (size_t x : to_end) c.patch(x);
      for (const std::string& v : g.vars)
        if (!d0.count(v) && !k0.count(v) && cover[0].count(v) != cover[1].count(v))
          fail(n, v + " is assigned or UNCHANGED in one branch of the disjunction only");
      g.done = chg[0];
      g.done.insert(chg[1].begin(), chg[1].end());
      g.kept = k0;
      for (const std::string& v : cover[0])
        if (cover[1].count(v) && !g.done.count(v)) g.kept.insert(v);
      g.sent = snt[0] || snt[1];
      return;
    }
    if ((n->kind == N_APP || n->kind == N_ID) && !env.send_helpers.count(n->s) && !s2->find(n->s) &&
        m.find(n->s)) {  // an operator of the module with effects: inlined
      const Def* d = m.find(n->s);
      if (!d->error.empty()) fail(n, "definition " + d->name + " does not parse: " + d->error);
      const std::vector<NodeP> args = n->kind == N_APP ? n->k : std::vector<NodeP>{};
      if (d->params.size() != args.size()) fail(n, "operator " + d->name + " applied to the wrong number of arguments");
      const size_t base = c.params.size();
      for (size_t q = 0; q < args.size(); q++) c.params.push_back({d->params[q], Arg{args[q], s2}});
      // the body sees its parameters and the module only (the message through a parameter)
      stmt(d->body, std::make_shared<Scope>(), exits);
      c.params.resize(base);
      return;
    }
    if (!g.item(n, s2))
      fail(n, "this effect conjunct (the handler compiler knows v' = ..., UNCHANGED, Discard, Reply, the send "
              "helpers, LET and a two-way disjunction of effects)");
  };
  for (auto& n : body) stmt(n, sc, disabled);
  g.complete();
  c.emit(E_END);
  for (size_t x : disabled) c.patch(x);  // the disabled exit: no successor
  c.emit(G_CONST, 0);
  c.emit(G_END);
  check_depth(c.code, "handler " + where);
  return c.code;
}

}  // namespace tla
}  // namespace rmc
