// rmc_tla.cpp — the TLA+ front end (see rmc_tla.h): lexer, parser, closure
// hashes, Next decomposition and the lowering onto the action library.
#include "rmc_tla.h"

#include <algorithm>
#include <cstring>
#include <functional>
#include <set>

#include "rmc_spec.h"

namespace rmc {
namespace tla {
namespace {

// ------------------------------------------------------------------ lexer
enum TokK { T_ID, T_NUM, T_STR, T_OP, T_SEP, T_END, T_EOF };
struct Tok {
  TokK k;
  std::string s;
  int line, col;
};

bool is_id_char(char c) { return isalnum((unsigned char)c) || c == '_'; }

std::vector<Tok> lex(const std::string& src) {
  std::vector<Tok> out;
  size_t i = 0, n = src.size();
  int line = 1;
  size_t line_start = 0;
  auto col = [&](size_t p) { return (int)(p - line_start) + 1; };
  auto newline = [&](size_t p) { line++; line_start = p + 1; };
  while (i < n) {
    char c = src[i];
    if (c == '\n') { newline(i); i++; continue; }
    if (c == ' ' || c == '\t' || c == '\r') { i++; continue; }
    if (c == '(' && i + 1 < n && src[i + 1] == '*') {  // nested block comment
      int depth = 0;
      while (i < n) {
        if (src[i] == '(' && i + 1 < n && src[i + 1] == '*') { depth++; i += 2; continue; }
        if (src[i] == '*' && i + 1 < n && src[i + 1] == ')') { depth--; i += 2; if (!depth) break; continue; }
        if (src[i] == '\n') newline(i);
        i++;
      }
      continue;
    }
    if (c == '\\' && i + 1 < n && src[i + 1] == '*') {  // line comment
      while (i < n && src[i] != '\n') i++;
      continue;
    }
    const int cl = col(i);
    if (c == '-' && i + 3 < n && src.compare(i, 4, "----") == 0) {
      while (i < n && src[i] == '-') i++;
      out.push_back({T_SEP, "----", line, cl});
      continue;
    }
    if (c == '=' && i + 3 < n && src.compare(i, 4, "====") == 0) {
      while (i < n && src[i] == '=') i++;
      out.push_back({T_END, "====", line, cl});
      break;  // the module ends here
    }
    if (isdigit((unsigned char)c)) {
      size_t j = i;
      while (j < n && isdigit((unsigned char)src[j])) j++;
      if (j < n && (isalpha((unsigned char)src[j]) || src[j] == '_')) {  // identifiers may start with digits
        while (j < n && is_id_char(src[j])) j++;
        out.push_back({T_ID, src.substr(i, j - i), line, cl});
      } else {
        out.push_back({T_NUM, src.substr(i, j - i), line, cl});
      }
      i = j;
      continue;
    }
    if (isalpha((unsigned char)c) || c == '_') {
      size_t j = i;
      while (j < n && is_id_char(src[j])) j++;
      out.push_back({T_ID, src.substr(i, j - i), line, cl});
      i = j;
      continue;
    }
    if (c == '"') {
      size_t j = i + 1;
      std::string s;
      while (j < n && src[j] != '"') {
        if (src[j] == '\\' && j + 1 < n) j++;
        s += src[j++];
      }
      out.push_back({T_STR, s, line, cl});
      i = j + 1;
      continue;
    }
    if (c == '\\' && i + 1 < n && isalpha((unsigned char)src[i + 1])) {  // \in, \E, \cup, ...
      size_t j = i + 1;
      while (j < n && isalpha((unsigned char)src[j])) j++;
      out.push_back({T_OP, src.substr(i, j - i), line, cl});
      i = j;
      continue;
    }
    static const char* ops[] = {"<=>", "|->", "\\/", "/\\", "==", "=>", "=<", "<=", ">=", "/=", "->", "<-", "<<", ">>",
                                "..", "@@", ":>", "[]", "<>", "~>", "::"};
    bool done = false;
    for (const char* o : ops) {
      size_t L = strlen(o);
      if (src.compare(i, L, o) == 0) {
        out.push_back({T_OP, o, line, cl});
        i += L;
        done = true;
        break;
      }
    }
    if (done) continue;
    out.push_back({T_OP, std::string(1, c), line, cl});
    i++;
  }
  out.push_back({T_EOF, "", line + 1, 0});
  return out;
}

// ------------------------------------------------------------------ parser
bool is_kw(const std::string& s) {
  static const std::set<std::string> kw = {"LET", "IN", "IF", "THEN", "ELSE", "CASE", "OTHER", "CHOOSE", "EXCEPT",
                                           "DOMAIN", "SUBSET", "UNION", "UNCHANGED", "ENABLED", "EXTENDS", "CONSTANT",
                                           "CONSTANTS", "VARIABLE", "VARIABLES", "ASSUME", "THEOREM", "LOCAL",
                                           "INSTANCE", "RECURSIVE", "MODULE", "WITH", "LAMBDA"};
  return kw.count(s) > 0;
}

struct Parser {
  const std::vector<Tok>& t;
  size_t pos, end;
  std::vector<int> limit;  // junction-item column limits: a token at column <= the innermost one ends the item

  Parser(const std::vector<Tok>& toks, size_t b, size_t e) : t(toks), pos(b), end(e) {}

  bool visible(size_t i) const {
    if (i >= end) return false;
    if (t[i].k == T_EOF || t[i].k == T_END) return false;
    if (!limit.empty() && t[i].col <= limit.back()) return false;
    return true;
  }
  const Tok& peek(size_t o = 0) const {
    static const Tok eof{T_EOF, "", 0, 0};
    for (size_t q = 0; q <= o; q++)
      if (!visible(pos + q)) return eof;
    return t[pos + o];
  }
  bool at_op(const char* s, size_t o = 0) const { const Tok& x = peek(o); return x.k == T_OP && x.s == s; }
  bool at_id(const char* s, size_t o = 0) const { const Tok& x = peek(o); return x.k == T_ID && x.s == s; }
  [[noreturn]] void fail(const std::string& msg) const {
    const Tok& x = pos < t.size() ? t[pos] : t.back();
    throw ParseError("line " + std::to_string(x.line) + ", col " + std::to_string(x.col) + ": " + msg +
                     (x.s.empty() ? "" : " (at '" + x.s + "')"));
  }
  Tok next() {
    if (!visible(pos)) fail("unexpected end of expression");
    return t[pos++];
  }
  void expect_op(const char* s) {
    if (!at_op(s)) fail(std::string("expected '") + s + "'");
    pos++;
  }
  void expect_id(const char* s) {
    if (!at_id(s)) fail(std::string("expected ") + s);
    pos++;
  }
  std::string ident() {
    const Tok& x = peek();
    if (x.k != T_ID || is_kw(x.s)) fail("expected an identifier");
    pos++;
    return x.s;
  }
  NodeP mk(Kind k, const Tok& at, const std::string& s = "") {
    auto n = std::make_shared<Node>();
    n->kind = k;
    n->s = s;
    n->line = at.line;
    n->col = at.col;
    return n;
  }

  // binding powers: (left, right) of infix operators
  static int infix_bp(const Tok& x, int& rbp) {
    if (x.k != T_OP && !(x.k == T_ID && false)) {
      if (x.k != T_OP) return -1;
    }
    const std::string& s = x.s;
    auto lr = [&](int l, int r) { rbp = r; return l; };
    if (s == "=>") return lr(1, 1);
    if (s == "<=>" || s == "\\equiv") return lr(2, 3);
    if (s == "/\\" || s == "\\/" || s == "\\land" || s == "\\lor") return lr(3, 4);
    if (s == "=" || s == "#" || s == "/=" || s == "<" || s == ">" || s == "<=" || s == "=<" || s == ">=" ||
        s == "\\leq" || s == "\\geq" || s == "\\in" || s == "\\notin" || s == "\\subseteq" || s == "\\subset" ||
        s == "\\supseteq")
      return lr(5, 6);
    if (s == "@@") return lr(6, 7);
    if (s == ":>") return lr(7, 8);
    if (s == "\\cup" || s == "\\cap" || s == "\\union" || s == "\\intersect" || s == "\\") return lr(8, 9);
    if (s == "..") return lr(9, 10);
    if (s == "+" || s == "-") return lr(10, 11);
    if (s == "%") return lr(11, 12);
    if (s == "*" || s == "\\o" || s == "\\div" || s == "\\circ") return lr(13, 14);
    if (s == "^") return lr(14, 15);
    return -1;
  }

  NodeP expr(int min_bp = 0) {
    NodeP lhs = prefix();
    for (;;) {
      const Tok& x = peek();
      if (x.k == T_EOF) break;
      if (x.k == T_OP && x.s == "'") {  // postfix prime
        if (15 < min_bp) break;
        pos++;
        auto n = mk(N_PRIME, x);
        n->k.push_back(lhs);
        lhs = n;
        continue;
      }
      if (x.k == T_OP && x.s == ".") {
        pos++;
        auto n = mk(N_FIELD, x, ident());
        n->k.push_back(lhs);
        lhs = n;
        continue;
      }
      if (x.k == T_OP && x.s == "[") {  // function application
        pos++;
        auto n = mk(N_FAPP, x);
        n->k.push_back(lhs);
        n->k.push_back(expr());
        while (at_op(",")) { pos++; n->k.push_back(expr()); }
        expect_op("]");
        lhs = n;
        continue;
      }
      int rbp = 0;
      const int lbp = infix_bp(x, rbp);
      if (lbp < 0 || lbp < min_bp) break;
      pos++;
      NodeP rhs = expr(rbp);
      auto n = mk(N_BIN, x, x.s == "\\land" ? "/\\" : x.s == "\\lor" ? "\\/" : x.s);
      n->k = {lhs, rhs};
      lhs = n;
    }
    return lhs;
  }

  std::vector<Bound> bounds(bool need_set) {
    std::vector<Bound> bs;
    for (;;) {
      Bound b;
      b.vars.push_back(ident());
      while (at_op(",")) { pos++; b.vars.push_back(ident()); }
      if (at_op("\\in")) {
        pos++;
        b.set = expr(5);  // stops at ',' and ':'
      } else if (need_set) {
        fail("expected \\in");
      }
      bs.push_back(b);
      if (at_op(",")) { pos++; continue; }
      break;
    }
    return bs;
  }

  NodeP junction(const Tok& bullet) {
    auto n = mk(N_JUNCT, bullet, bullet.s);
    const int c = bullet.col;
    for (;;) {
      pos++;  // the bullet
      limit.push_back(c);
      n->k.push_back(expr());
      limit.pop_back();
      const Tok& x = peek();
      if (x.k == T_OP && x.s == bullet.s && x.col == c) continue;
      break;
    }
    return n;
  }

  Def letdef() {
    Def d;
    d.line = peek().line;
    d.name = ident();
    if (at_op("(")) {
      pos++;
      d.params.push_back(ident());
      while (at_op(",")) { pos++; d.params.push_back(ident()); }
      expect_op(")");
    }
    expect_op("==");
    d.body = expr();
    return d;
  }

  NodeP prefix() {
    const Tok x = peek();
    if (x.k == T_EOF) fail("unexpected end of expression");
    if (x.k == T_NUM) { pos++; return mk(N_NUM, x, x.s); }
    if (x.k == T_STR) { pos++; return mk(N_STR, x, x.s); }
    if (x.k == T_OP) {
      if (x.s == "/\\" || x.s == "\\/") return junction(x);
      if (x.s == "(") {
        pos++;
        NodeP e = expr();
        expect_op(")");
        return e;
      }
      if (x.s == "<<") {
        pos++;
        auto n = mk(N_TUPLE, x);
        if (!at_op(">>")) {
          n->k.push_back(expr());
          while (at_op(",")) { pos++; n->k.push_back(expr()); }
        }
        expect_op(">>");
        return n;
      }
      if (x.s == "{") return brace(x);
      if (x.s == "[") return bracket(x);
      if (x.s == "@") { pos++; return mk(N_AT, x); }
      if (x.s == "~" || x.s == "\\lnot" || x.s == "\\neg") {
        pos++;
        auto n = mk(N_UNARY, x, "~");
        n->k.push_back(expr(4));
        return n;
      }
      if (x.s == "-") {
        pos++;
        auto n = mk(N_UNARY, x, "-");
        n->k.push_back(expr(12));
        return n;
      }
      if (x.s == "\\E" || x.s == "\\A") {
        pos++;
        auto n = mk(N_QUANT, x, x.s);
        n->bounds = bounds(false);
        expect_op(":");
        n->k.push_back(expr());
        return n;
      }
      fail("unsupported syntax");
    }
    // identifiers and keywords
    if (x.s == "TRUE" || x.s == "FALSE") { pos++; return mk(N_ID, x, x.s); }
    if (x.s == "IF") {
      pos++;
      auto n = mk(N_IF, x);
      n->k.push_back(expr());
      expect_id("THEN");
      n->k.push_back(expr());
      expect_id("ELSE");
      n->k.push_back(expr());
      return n;
    }
    if (x.s == "CASE") {
      pos++;
      auto n = mk(N_CASE, x);
      for (;;) {
        if (at_id("OTHER")) {
          pos++;
          expect_op("->");
          n->k.push_back(expr());
          n->has_other = true;
          break;
        }
        n->k.push_back(expr());
        expect_op("->");
        n->k.push_back(expr());
        if (at_op("[]")) { pos++; continue; }
        break;
      }
      return n;
    }
    if (x.s == "LET") {
      pos++;
      auto n = mk(N_LET, x);
      while (!at_id("IN")) n->defs.push_back(letdef());
      pos++;
      n->k.push_back(expr());
      return n;
    }
    if (x.s == "CHOOSE") {
      pos++;
      auto n = mk(N_CHOOSE, x);
      n->bounds = bounds(false);
      expect_op(":");
      n->k.push_back(expr());
      return n;
    }
    if (x.s == "DOMAIN" || x.s == "SUBSET" || x.s == "UNION" || x.s == "UNCHANGED" || x.s == "ENABLED") {
      pos++;
      auto n = mk(N_UNARY, x, x.s);
      n->k.push_back(expr(x.s == "DOMAIN" ? 9 : x.s == "UNCHANGED" ? 15 : x.s == "ENABLED" ? 4 : 8));
      return n;
    }
    if (is_kw(x.s)) fail("unexpected keyword");
    pos++;
    if (at_op("(")) {  // operator application
      pos++;
      auto n = mk(N_APP, x, x.s);
      if (!at_op(")")) {
        n->k.push_back(expr());
        while (at_op(",")) { pos++; n->k.push_back(expr()); }
      }
      expect_op(")");
      return n;
    }
    return mk(N_ID, x, x.s);
  }

  NodeP brace(const Tok& x) {
    pos++;
    if (at_op("}")) { pos++; return mk(N_SETENUM, x); }
    if (peek().k == T_ID && !is_kw(peek().s) && at_op("\\in", 1)) {
      const size_t save = pos;
      std::string v = ident();
      pos++;  // \in
      NodeP set = expr(5);
      if (at_op(":")) {  // {x \in S : P}
        pos++;
        auto n = mk(N_SETFILTER, x);
        n->bounds.push_back(Bound{{v}, set});
        n->k.push_back(expr());
        expect_op("}");
        return n;
      }
      pos = save;  // an enumeration whose first element is `x \in S`
    }
    NodeP first = expr();
    if (at_op(":")) {  // {e : x \in S, ...}
      pos++;
      auto n = mk(N_SETMAP, x);
      n->k.push_back(first);
      n->bounds = bounds(true);
      expect_op("}");
      return n;
    }
    auto n = mk(N_SETENUM, x);
    n->k.push_back(first);
    while (at_op(",")) { pos++; n->k.push_back(expr()); }
    expect_op("}");
    return n;
  }

  NodeP bracket(const Tok& x) {
    pos++;
    const Tok& a = peek();
    if (a.k == T_ID && !is_kw(a.s) && at_op("|->", 1)) {  // record
      auto n = mk(N_RECORD, x);
      for (;;) {
        n->names.push_back(ident());
        expect_op("|->");
        n->k.push_back(expr());
        if (at_op(",")) { pos++; continue; }
        break;
      }
      expect_op("]");
      return n;
    }
    if (a.k == T_ID && !is_kw(a.s) && at_op(":", 1)) {  // set of records
      auto n = mk(N_RECSET, x);
      for (;;) {
        n->names.push_back(ident());
        expect_op(":");
        n->k.push_back(expr());
        if (at_op(",")) { pos++; continue; }
        break;
      }
      expect_op("]");
      return n;
    }
    if (a.k == T_ID && !is_kw(a.s) && (at_op("\\in", 1) || at_op(",", 1))) {  // [x \in S |-> e]
      const size_t save = pos;
      try {
        auto n = mk(N_FUNC, x);
        n->bounds = bounds(true);
        expect_op("|->");
        n->k.push_back(expr());
        expect_op("]");
        return n;
      } catch (ParseError&) {
        pos = save;
      }
    }
    NodeP e = expr();
    if (at_id("EXCEPT")) {
      pos++;
      auto n = mk(N_EXCEPT, x);
      n->k.push_back(e);
      for (;;) {
        expect_op("!");
        std::vector<PathStep> path;
        for (;;) {
          if (at_op(".")) {
            pos++;
            path.push_back(PathStep{true, ident(), {}});
          } else if (at_op("[")) {
            pos++;
            PathStep st{false, "", {}};
            st.args.push_back(expr());
            while (at_op(",")) { pos++; st.args.push_back(expr()); }
            expect_op("]");
            path.push_back(st);
          } else {
            break;
          }
        }
        if (path.empty()) fail("empty EXCEPT path");
        expect_op("=");
        n->paths.push_back(path);
        n->k.push_back(expr());
        if (at_op(",")) { pos++; continue; }
        break;
      }
      expect_op("]");
      return n;
    }
    if (at_op("->")) {
      pos++;
      auto n = mk(N_FUNCSET, x);
      n->k.push_back(e);
      n->k.push_back(expr());
      expect_op("]");
      return n;
    }
    fail("unsupported [...] form");
  }
};

// Is token i the start of a top-level unit?  (A definition `Name ==` or
// `Name(p, ...) ==` at column 1, a declaration keyword, a separator.)
bool unit_start(const std::vector<Tok>& t, size_t i) {
  const Tok& x = t[i];
  if (x.k == T_SEP || x.k == T_END || x.k == T_EOF) return true;
  if (x.col != 1) return false;
  if (x.k != T_ID) return false;
  if (x.s == "EXTENDS" || x.s == "CONSTANT" || x.s == "CONSTANTS" || x.s == "VARIABLE" || x.s == "VARIABLES" ||
      x.s == "ASSUME" || x.s == "THEOREM" || x.s == "LOCAL" || x.s == "INSTANCE" || x.s == "RECURSIVE" ||
      x.s == "AXIOM" || x.s == "LEMMA")
    return true;
  if (i + 1 < t.size() && t[i + 1].k == T_OP && t[i + 1].s == "==") return true;
  if (i + 1 < t.size() && t[i + 1].k == T_OP && t[i + 1].s == "(") {
    size_t j = i + 2;
    int depth = 1;
    while (j < t.size() && depth) {
      if (t[j].k == T_OP && t[j].s == "(") depth++;
      if (t[j].k == T_OP && t[j].s == ")") depth--;
      j++;
    }
    return j < t.size() && t[j].k == T_OP && t[j].s == "==";
  }
  return false;
}

// ------------------------------------------------------------------ hashing
uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
uint64_t hcomb(uint64_t h, uint64_t x) { return mix64(h ^ (x + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2))); }
uint64_t hstr(const std::string& s) {
  uint64_t h = 1469598103934665603ULL;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ULL;
  return mix64(h);
}

struct Hasher {
  const Module& m;
  std::map<std::string, uint64_t> memo;
  std::set<std::string> active;
  // identifiers and applied operators that are neither bound, nor defined in
  // the module, nor declared: they must be standard-module operators (lower())
  std::set<std::string> unresolved;
  // innermost last: (name, is_local_def, local def hash)
  struct Ent { std::string name; bool def; uint64_t h; size_t nparams; };
  std::vector<Ent> env;

  explicit Hasher(const Module& mod) : m(mod) {}

  uint64_t def_hash(const std::string& name) {
    auto it = memo.find(name);
    if (it != memo.end()) return it->second;
    const Def* d = m.find(name);
    if (!d) throw std::runtime_error("unknown operator " + name);
    if (!d->error.empty())
      throw std::runtime_error("definition " + name + " (line " + std::to_string(d->line) + ") does not parse: " +
                               d->error);
    if (active.count(name)) throw std::runtime_error("recursive definition " + name + " is not supported");
    active.insert(name);
    std::vector<Ent> save;
    save.swap(env);
    for (auto& p : d->params) env.push_back({p, false, 0, 0});
    uint64_t h = hcomb(hstr("def"), d->params.size());
    h = hcomb(h, node(d->body));
    env.swap(save);
    active.erase(name);
    memo[name] = h;
    return h;
  }

  // lookup: bound variable -> de Bruijn index; local definition -> its hash
  bool lookup(const std::string& name, uint64_t& out, bool& is_def) {
    for (size_t q = env.size(); q-- > 0;) {
      if (env[q].name != name) continue;
      is_def = env[q].def;
      out = is_def ? env[q].h : hcomb(hstr("bv"), env.size() - 1 - q);
      return true;
    }
    return false;
  }

  bool is_declared(const std::string& s) const {
    return std::find(m.constants.begin(), m.constants.end(), s) != m.constants.end() ||
           std::find(m.variables.begin(), m.variables.end(), s) != m.variables.end();
  }

  void flatten(const NodeP& n, const std::string& op, std::vector<NodeP>& out) {
    if ((n->kind == N_JUNCT && n->s == op)) {
      for (auto& c : n->k) flatten(c, op, out);
    } else if (n->kind == N_BIN && n->s == op) {
      flatten(n->k[0], op, out);
      flatten(n->k[1], op, out);
    } else {
      out.push_back(n);
    }
  }

  uint64_t bounds_push(const std::vector<Bound>& bs, uint64_t h) {
    for (auto& b : bs) {
      h = hcomb(h, b.vars.size());
      h = hcomb(h, b.set ? node(b.set) : hstr("unbounded"));
      for (auto& v : b.vars) env.push_back({v, false, 0, 0});
    }
    return h;
  }
  void bounds_pop(const std::vector<Bound>& bs) {
    for (auto& b : bs) env.resize(env.size() - b.vars.size());
  }

  uint64_t node(const NodeP& n) {
    uint64_t h = hcomb(hstr("k"), (uint64_t)n->kind);
    switch (n->kind) {
      case N_NUM: case N_STR: return hcomb(h, hstr(n->s));
      case N_AT: return h;
      case N_ID: {
        uint64_t r;
        bool d;
        if (lookup(n->s, r, d)) return d ? hcomb(hstr("ldef"), r) : r;
        if (!is_declared(n->s) && m.find(n->s)) return hcomb(hstr("ref"), def_hash(n->s));
        if (!is_declared(n->s)) unresolved.insert(n->s);
        return hcomb(hstr("name"), hstr(n->s));
      }
      case N_APP: {
        uint64_t r;
        bool d;
        if (lookup(n->s, r, d) && d) h = hcomb(hstr("lapp"), r);
        else if (m.find(n->s) && !is_declared(n->s)) h = hcomb(hstr("app"), def_hash(n->s));
        else {
          if (!is_declared(n->s)) unresolved.insert(n->s);
          h = hcomb(hstr("builtin"), hstr(n->s));
        }
        for (auto& c : n->k) h = hcomb(h, node(c));
        return h;
      }
      case N_JUNCT: case N_BIN: {
        const std::string op = n->s;
        if (op == "/\\" || op == "\\/") {
          std::vector<NodeP> items;
          flatten(n, op, items);
          h = hcomb(hstr(op == "/\\" ? "and" : "or"), items.size());
          for (auto& c : items) h = hcomb(h, node(c));
          return h;
        }
        h = hcomb(h, hstr(op == "/=" ? "#" : op == "=<" || op == "\\leq" ? "<=" : op == "\\geq" ? ">=" :
                          op == "\\union" ? "\\cup" : op == "\\intersect" ? "\\cap" : op));
        h = hcomb(h, node(n->k[0]));
        return hcomb(h, node(n->k[1]));
      }
      case N_FIELD: return hcomb(hcomb(h, hstr(n->s)), node(n->k[0]));
      case N_PRIME: case N_UNARY: case N_FAPP: case N_IF: case N_TUPLE: case N_SETENUM: case N_FUNCSET:
        h = hcomb(h, hstr(n->s));
        for (auto& c : n->k) h = hcomb(h, node(c));
        return h;
      case N_CASE:
        h = hcomb(h, n->has_other);
        for (auto& c : n->k) h = hcomb(h, node(c));
        return h;
      case N_LET: {
        const size_t base = env.size();
        for (auto& d : n->defs) {
          // a local definition is hashed where it is defined, its parameters bound
          for (auto& p : d.params) env.push_back({p, false, 0, 0});
          uint64_t dh = hcomb(hcomb(hstr("ldef"), d.params.size()), node(d.body));
          env.resize(env.size() - d.params.size());
          env.push_back({d.name, true, dh, d.params.size()});
        }
        h = hcomb(h, node(n->k[0]));
        env.resize(base);
        return h;
      }
      case N_QUANT: case N_CHOOSE: case N_SETFILTER: case N_FUNC: {
        h = hcomb(h, hstr(n->s));
        h = bounds_push(n->bounds, h);
        h = hcomb(h, node(n->k[0]));
        bounds_pop(n->bounds);
        return h;
      }
      case N_SETMAP: {
        h = bounds_push(n->bounds, h);
        h = hcomb(h, node(n->k[0]));
        bounds_pop(n->bounds);
        return h;
      }
      case N_RECORD: case N_RECSET: {  // field order is immaterial (TLC sorts record fields)
        std::vector<std::pair<std::string, uint64_t>> f;
        for (size_t q = 0; q < n->names.size(); q++) f.push_back({n->names[q], node(n->k[q])});
        std::sort(f.begin(), f.end());
        for (auto& x : f) h = hcomb(hcomb(h, hstr(x.first)), x.second);
        return h;
      }
      case N_EXCEPT: {
        h = hcomb(h, node(n->k[0]));
        for (size_t q = 0; q < n->paths.size(); q++) {
          for (auto& st : n->paths[q]) {
            h = hcomb(h, st.field ? hstr("." + st.name) : hstr("[]"));
            for (auto& a : st.args) h = hcomb(h, node(a));
          }
          h = hcomb(h, node(n->k[q + 1]));
        }
        return h;
      }
    }
    return h;
  }

  // Does n change the state: a primed variable, UNCHANGED, or an operator of
  // the module whose body does (Send, Reply, ...)?  Bound names shadow
  // definitions.
  std::map<std::string, bool> eff_memo;
  // operators that change the state although the text does not define them
  // (parse_action: the family's send helpers, restated by the effect compiler)
  std::set<std::string> effect_ops;
  bool has_effect(const NodeP& n, std::set<std::string>& bound) {
    if (!n) return false;
    if (n->kind == N_PRIME) return true;
    if (n->kind == N_UNARY && n->s == "UNCHANGED") return true;
    if ((n->kind == N_ID || n->kind == N_APP) && effect_ops.count(n->s) && !bound.count(n->s)) return true;
    if ((n->kind == N_ID || n->kind == N_APP) && !bound.count(n->s)) {
      const Def* d = m.find(n->s);
      if (d && !is_declared(n->s)) {
        auto it = eff_memo.find(n->s);
        bool e;
        if (it != eff_memo.end()) {
          e = it->second;
        } else {
          eff_memo[n->s] = false;  // (recursion guard)
          std::set<std::string> b2(d->params.begin(), d->params.end());
          e = d->error.empty() ? has_effect(d->body, b2) : true;
          eff_memo[n->s] = e;
        }
        if (e) return true;
      }
    }
    std::vector<std::string> added;
    auto bind = [&](const std::string& v) {
      if (bound.insert(v).second) added.push_back(v);
    };
    for (auto& b : n->bounds) {
      if (has_effect(b.set, bound)) return true;
      for (auto& v : b.vars) bind(v);
    }
    bool e = false;
    for (auto& d : n->defs) {
      std::set<std::string> b2 = bound;
      for (auto& p : d.params) b2.insert(p);
      if (has_effect(d.body, b2)) e = true;
      bind(d.name);
    }
    for (auto& c : n->k)
      if (!e && has_effect(c, bound)) e = true;
    for (auto& path : n->paths)
      for (auto& st : path)
        for (auto& a : st.args)
          if (!e && has_effect(a, bound)) e = true;
    for (auto& v : added) bound.erase(v);
    return e;
  }
  // The top-level conjuncts of definition `name`: guards (no effect) and effects.
  bool split(const std::string& name, std::vector<NodeP>& guards, std::vector<NodeP>& effects) {
    const Def* d = m.find(name);
    if (!d || !d->error.empty() || !d->body) return false;
    std::vector<NodeP> items;
    flatten(d->body, "/\\", items);
    std::set<std::string> bound(d->params.begin(), d->params.end());
    for (auto& c : items) (has_effect(c, bound) ? effects : guards).push_back(c);
    return !effects.empty();
  }
  // Hash of an action's EFFECT: its effect conjuncts in order, parameters
  // bound by position as in def_hash.  Two actions with equal effect hashes
  // differ at most in their guards.
  bool effect_hash(const std::string& name, uint64_t& out, std::vector<NodeP>* guards_out = nullptr,
                   std::vector<NodeP>* effects_out = nullptr) {
    std::vector<NodeP> g, e;
    if (!split(name, g, e)) return false;
    if (effects_out) *effects_out = e;
    const Def* d = m.find(name);
    std::vector<Ent> save;
    save.swap(env);
    for (auto& p : d->params) env.push_back({p, false, 0, 0});
    uint64_t h = hcomb(hstr("effect"), d->params.size());
    for (auto& c : e) h = hcomb(h, node(c));
    env.swap(save);
    out = h;
    if (guards_out) *guards_out = g;
    return true;
  }
};

}  // namespace

// ------------------------------------------------------------------ module
Module parse_module(const std::string& text) {
  std::vector<Tok> t = lex(text);
  Module m;
  size_t i = 0;
  // ---- MODULE Name ----
  while (i < t.size() && !(t[i].k == T_ID && t[i].s == "MODULE")) i++;
  if (i + 1 >= t.size() || t[i + 1].k != T_ID) throw ParseError("no MODULE header");
  m.name = t[i + 1].s;
  i += 2;
  if (i < t.size() && t[i].k == T_SEP) i++;
  auto id_list = [&](std::vector<std::string>& out) {
    while (i < t.size() && t[i].k == T_ID) {
      out.push_back(t[i].s);
      i++;
      if (i < t.size() && t[i].k == T_OP && t[i].s == "(") {  // CONSTANT Op(_, _)
        while (i < t.size() && !(t[i].k == T_OP && t[i].s == ")")) i++;
        i++;
      }
      if (i < t.size() && t[i].k == T_OP && t[i].s == ",") { i++; continue; }
      break;
    }
  };
  while (i < t.size() && t[i].k != T_END && t[i].k != T_EOF) {
    const Tok& x = t[i];
    if (x.k == T_SEP) { i++; continue; }
    if (x.k == T_ID && x.s == "EXTENDS") { i++; id_list(m.extends); continue; }
    if (x.k == T_ID && (x.s == "CONSTANT" || x.s == "CONSTANTS")) { i++; id_list(m.constants); continue; }
    if (x.k == T_ID && (x.s == "VARIABLE" || x.s == "VARIABLES")) { i++; id_list(m.variables); continue; }
    if (x.k == T_ID && unit_start(t, i) && !is_kw(x.s)) {
      Def d;
      d.name = x.s;
      d.line = x.line;
      i++;
      if (t[i].k == T_OP && t[i].s == "(") {
        i++;
        while (i < t.size() && !(t[i].k == T_OP && t[i].s == ")")) {
          if (t[i].k == T_ID) d.params.push_back(t[i].s);
          i++;
        }
        i++;
      }
      i++;  // ==
      size_t e = i;
      while (e < t.size() && !unit_start(t, e)) e++;
      try {
        Parser p(t, i, e);
        d.body = p.expr();
        if (p.pos != e) p.fail("unexpected token after the definition");
      } catch (ParseError& pe) {
        d.error = pe.what();
      }
      m.index[d.name] = m.defs.size();
      m.defs.push_back(d);
      i = e;
      continue;
    }
    // ASSUME, THEOREM, INSTANCE, ...: skipped to the next unit
    if (x.k == T_ID) m.skipped.push_back({x.s, x.line});
    i++;
    while (i < t.size() && !unit_start(t, i)) i++;
  }
  return m;
}

std::map<std::string, uint64_t> closure_hashes(const Module& m) {
  Hasher h(m);
  std::map<std::string, uint64_t> out;
  for (auto& d : m.defs) {
    if (!d.error.empty()) continue;
    try {
      out[d.name] = h.def_hash(d.name);
    } catch (std::exception&) {
      // depends on a definition that does not parse (e.g. a temporal formula)
    }
  }
  return out;
}

std::vector<Disjunct> next_disjuncts(const Module& m, const std::string& next) {
  const Def* d = m.find(next);
  if (!d) throw std::runtime_error("the module defines no " + next);
  if (!d->error.empty()) throw std::runtime_error(next + " does not parse: " + d->error);
  std::vector<NodeP> items;
  std::function<void(const NodeP&)> flat = [&](const NodeP& n) {
    if ((n->kind == N_JUNCT || n->kind == N_BIN) && n->s == "\\/") {
      for (auto& c : n->k) flat(c);
    } else {
      items.push_back(n);
    }
  };
  flat(d->body);
  std::vector<Disjunct> out;
  auto is_id = [](const NodeP& n, const std::string& s) { return n && n->kind == N_ID && n->s == s; };
  for (auto& n : items) {
    Disjunct dj;
    dj.line = n->line;
    if (n->kind == N_ID) {  // a bare action: its body ranges over DOMAIN messages
      dj.form = B_MSG;
      dj.op = n->s;
      out.push_back(dj);
      continue;
    }
    if (n->kind == N_QUANT && n->s == "\\E" && n->k[0]->kind == N_APP) {
      const NodeP& app = n->k[0];
      std::vector<std::string> vars;
      std::vector<NodeP> sets;
      for (auto& b : n->bounds)
        for (auto& v : b.vars) { vars.push_back(v); sets.push_back(b.set); }
      bool args_ok = app->k.size() == vars.size();
      for (size_t q = 0; args_ok && q < vars.size(); q++) args_ok = is_id(app->k[q], vars[q]);
      if (args_ok) {
        dj.op = app->s;
        if (vars.size() == 1 && is_id(sets[0], "Server")) { dj.form = B_I; out.push_back(dj); continue; }
        if (vars.size() == 2 && is_id(sets[0], "Server") && is_id(sets[1], "Server")) {
          dj.form = B_IJ;
          out.push_back(dj);
          continue;
        }
        if (vars.size() == 2 && is_id(sets[0], "Server") && is_id(sets[1], "Value")) {
          dj.form = B_IV;
          out.push_back(dj);
          continue;
        }
        if (vars.size() == 1 && sets[0] && sets[0]->kind == N_UNARY && sets[0]->s == "DOMAIN" &&
            is_id(sets[0]->k[0], "messages")) {
          dj.form = B_M;
          out.push_back(dj);
          continue;
        }
      }
    }
    throw std::runtime_error("Next disjunct at line " + std::to_string(n->line) +
                             " has a form the lowering does not bind (supported: \\E i \\in Server : A(i), "
                             "\\E i, j \\in Server : A(i, j), \\E i \\in Server, v \\in Value : A(i, v), "
                             "\\E m \\in DOMAIN messages : A(m), or an action A over DOMAIN messages)");
  }
  return out;
}

// ------------------------------------------------------------------ lowering
namespace {
enum Role { R_INIT = 0, R_ACTION = 1, R_INV = 2, R_VIEW = 3, R_SYMM = 4, R_VARS = 5, R_EFFECT = 6, R_HELPER = 7 };
struct Known {
  int spec, role, id, kind;
  unsigned long long hash;
  const char* name;
};
const Known kKnown[] = {
#include "rmc_tla_known.inc"
    {-1, -1, 0, 0, 0ULL, ""}};

uint64_t vars_hash(const Module& m) {
  std::vector<std::string> v = m.variables;
  std::sort(v.begin(), v.end());
  uint64_t h = hstr("vars");
  for (auto& s : v) h = hcomb(h, hstr(s));
  return h;
}
const char* spec_name(int s) {
  static const char* n[] = {"Raft", "FlexibleRaft", "RaftFsync", "PullRaft", "PullRaftVariant2", "KRaft"};
  return s >= 0 && s < 6 ? n[s] : "?";
}
}  // namespace

// hashes of every definition (tools/gen_tla_known.py; the tests): "name hash" lines
std::string hash_report(const std::string& text) {
  Module m = parse_module(text);
  std::string o = "#module " + m.name + "\n";
  char b[64];
  snprintf(b, sizeof b, "%016llx", (unsigned long long)vars_hash(m));
  o += std::string("#vars ") + b + "\n";
  for (auto& kv : closure_hashes(m)) {
    snprintf(b, sizeof b, "%016llx", (unsigned long long)kv.second);
    o += kv.first + " " + b + "\n";
  }
  {  // "effect:name hash": the effect hash of each action-shaped definition
    Hasher H(m);
    for (auto& d : m.defs) {
      uint64_t h = 0;
      try {
        if (!H.effect_hash(d.name, h)) continue;
      } catch (std::exception&) {
        continue;
      }
      snprintf(b, sizeof b, "%016llx", (unsigned long long)h);
      o += "effect:" + d.name + " " + b + "\n";
    }
  }
  for (auto& d : m.defs)
    if (!d.error.empty()) o += "#unparsed " + d.name + " " + d.error + "\n";
  return o;
}

std::vector<std::pair<int, int>> actions_by_name(int spec, const std::vector<std::string>& names) {
  std::vector<std::pair<int, int>> out;
  for (const std::string& n : names) {
    const Known* hit = nullptr;
    for (const Known& k : kKnown)
      if (k.spec == spec && k.role == R_ACTION && n == k.name) hit = &k;
    if (!hit) throw std::runtime_error(std::string("the ") + spec_name(spec) + " lowering has no action " + n);
    out.push_back({hit->id, hit->kind});
  }
  return out;
}

std::string action_name(int spec, int act) {
  for (const Known& k : kKnown)
    if (k.spec == spec && k.role == R_ACTION && k.id == act) return k.name;
  return "?";
}

// The standard modules a lowered spec may EXTEND, and the operators they (and
// the TLA+ core) give an identifier that no definition of the module binds.
// An identifier outside this list is an operator the hashing cannot see into
// (a user module's, a LOCAL or INSTANCE'd one): an edit to it would leave the
// action hashes unchanged, so the lowering refuses it.
static const std::set<std::string> kStdModules = {"Naturals", "Integers", "Sequences", "FiniteSets", "TLC", "Bags"};
static const std::set<std::string> kStdOps = {
    "TRUE", "FALSE", "BOOLEAN", "STRING", "Nat", "Int",                                  // core, Naturals, Integers
    "Seq", "Len", "Append", "Head", "Tail", "SubSeq", "SelectSeq",                         // Sequences
    "IsFiniteSet", "Cardinality",                                                           // FiniteSets
    "Print", "PrintT", "Assert", "JavaTime", "TLCGet", "TLCSet", "Permutations", "SortSeq",  // TLC
    "RandomElement", "Any", "ToString", "TLCEval",
    "IsABag", "BagToSet", "SetToBag", "BagIn", "EmptyBag", "CopiesIn", "BagCup", "BagDiff",  // Bags
    "BagUnion", "SubBag", "BagOfAll", "BagCardinality"};

Lowering lower(const std::string& text, const std::string& next, const std::string& view,
               const std::string& symmetry, const std::vector<std::string>& invariants) {
  auto mp = std::make_shared<Module>(parse_module(text));
  Module& m = *mp;
  for (const std::string& e : m.extends)
    if (!kStdModules.count(e))
      throw std::runtime_error("module " + m.name + " EXTENDS " + e + ": the lowering reads a module's own text and "
                               "the standard modules (Naturals, Integers, Sequences, FiniteSets, TLC, Bags) only");
  for (auto& u : m.skipped)
    if (u.first == "LOCAL" || u.first == "INSTANCE" || u.first == "RECURSIVE")
      throw std::runtime_error("module " + m.name + ": " + u.first + " (line " + std::to_string(u.second) +
                               ") is not supported by the lowering (its operators would not be seen by the closure "
                               "hashes)");
  Hasher H(m);
  auto hash_of = [&](const std::string& name) -> uint64_t {
    if (!m.find(name)) throw std::runtime_error("module " + m.name + " defines no " + name);
    return H.def_hash(name);
  };
  // the spec family: Init's closure hash and the variable set decide the packed layout
  const uint64_t hi = hash_of("Init"), hv = vars_hash(m);
  Lowering L;
  for (const Known& k : kKnown)
    if (k.role == R_INIT && k.hash == hi) {
      bool vars = false;
      for (const Known& q : kKnown) vars |= q.role == R_VARS && q.spec == k.spec && q.hash == hv;
      if (vars) { L.spec = k.spec; break; }
    }
  if (L.spec < 0)
    throw std::runtime_error("module " + m.name + ": its VARIABLES and Init are not those of a spec family the "
                             "checker lowers (Raft, FlexibleRaft, RaftFsync, PullRaft, PullRaftVariant2, KRaft): the "
                             "packed state layout is derived from them");
  auto find = [&](int role, uint64_t h) -> const Known* {
    for (const Known& k : kKnown)
      if (k.spec == L.spec && k.role == role && k.hash == h) return &k;
    return nullptr;
  };
  const std::vector<Disjunct> djs = next_disjuncts(m, next);
  {  // hash everything the cfg names first: an unresolved identifier is reported as such
    for (const Disjunct& dj : djs) (void)hash_of(dj.op);
    for (const std::string& inv : invariants)
      if (m.find(inv)) (void)hash_of(inv);
    if (!view.empty()) (void)hash_of(view);
    if (!symmetry.empty()) (void)hash_of(symmetry);
    for (const std::string& u : H.unresolved)
      if (!kStdOps.count(u))
        throw std::runtime_error("module " + m.name + " uses " + u + ", which it neither defines nor declares and no "
                                 "standard module the lowering knows defines");
  }
  L.module = mp;
  for (const Disjunct& dj : djs) {
    const uint64_t h = hash_of(dj.op);
    const Known* k = find(R_ACTION, h);
    if (!k) {
      // the library's effect behind the module's own guard (rmc_guard.cpp)?
      uint64_t eh = 0;
      std::vector<NodeP> g;
      if (H.effect_hash(dj.op, eh, &g)) k = find(R_EFFECT, eh);
      if (k) {
        for (const GuardSrc& q : L.guards)
          if (q.act == k->id)
            throw std::runtime_error("Next disjunct " + dj.op + " (line " + std::to_string(dj.line) + ") and " + q.op +
                                     " both guard the library's " + k->name + " effect: one guard per action");
        GuardSrc gs;
        gs.act = k->id;
        gs.op = dj.op;
        gs.params = m.find(dj.op)->params;
        gs.conjuncts = g;
        gs.mod = mp;
        L.guards.push_back(gs);
      }
    }
    if (!k && (L.spec == RAFT || L.spec == FLEX || L.spec == FSYNC) &&
        (dj.form == B_I || dj.form == B_IJ || dj.form == B_IV)) {
      // compiled whole: its guard and its effect (rmc_guard.cpp compile_effect)
      uint64_t eh = 0;
      std::vector<NodeP> g, e;
      if (H.effect_hash(dj.op, eh, &g, &e)) {
        int ncomp = 0;
        for (const GuardSrc& q : L.guards) ncomp += q.act >= A_C0;
        if (ncomp >= MAXCOMPILED)
          throw std::runtime_error("Next disjunct " + dj.op + " (line " + std::to_string(dj.line) + "): more than " +
                                   std::to_string(MAXCOMPILED) + " actions to compile");
        // the bag helpers an effect calls must be the family's own (by closure hash)
        std::map<std::string, int> helpers;
        for (const NodeP& c : e)
          if (c->kind == N_APP && m.find(c->s)) {
            const Known* hk = nullptr;
            const uint64_t hh = hash_of(c->s);
            for (const Known& q : kKnown)
              if (q.spec == L.spec && q.role == R_HELPER && q.hash == hh && c->s == q.name) hk = &q;
            if (!hk)
              throw std::runtime_error("Next disjunct " + dj.op + " (line " + std::to_string(dj.line) + ") calls " + c->s +
                                       ", which is not one of the " + spec_name(L.spec) + " module's own bag helpers");
            helpers[c->s] = hk->id;
          }
        GuardSrc gs;
        gs.send_helpers = helpers;
        gs.act = A_C0 + ncomp;
        gs.op = dj.op;
        gs.params = m.find(dj.op)->params;
        gs.conjuncts = g;
        gs.effects = e;
        gs.kind = dj.form == B_I ? K_I : dj.form == B_IJ ? K_IJ : K_IV;
        gs.mod = mp;
        L.guards.push_back(gs);
        L.actions.push_back({gs.act, gs.kind});
        L.labels.push_back(dj.op);
        continue;
      }
    }
    if (!k && (L.spec == RAFT || L.spec == FLEX || L.spec == FSYNC) && (dj.form == B_MSG || dj.form == B_M)) {
      // a message handler compiled whole (rmc_guard.cpp compile_handler): the
      // bare action's body \E m \in DOMAIN messages : body (Raft.tla:384-401),
      // or the operator A of \E m \in DOMAIN messages : A(m)
      const Def* d = m.find(dj.op);
      GuardSrc gs;
      if (dj.form == B_MSG) {
        const NodeP& b = d->body;
        if (!d->params.empty() || !b || b->kind != N_QUANT || b->s != "\\E" || b->bounds.size() != 1 ||
            b->bounds[0].vars.size() != 1 || !b->bounds[0].set || b->bounds[0].set->kind != N_UNARY ||
            b->bounds[0].set->s != "DOMAIN" || b->bounds[0].set->k[0]->kind != N_ID ||
            b->bounds[0].set->k[0]->s != "messages")
          throw std::runtime_error("Next disjunct " + dj.op + " (line " + std::to_string(dj.line) + ") is neither a "
                                   "lowered handler nor of the form \\E m \\in DOMAIN messages : body");
        gs.params = b->bounds[0].vars;
        gs.conjuncts = {b->k[0]};
      } else {
        if (d->params.size() != 1)
          throw std::runtime_error("Next disjunct " + dj.op + " (line " + std::to_string(dj.line) + "): a handler "
                                   "bound by \\E m \\in DOMAIN messages takes one parameter");
        gs.params = d->params;
        gs.conjuncts = {d->body};
      }
      int ncomp = 0;
      for (const GuardSrc& q : L.guards) ncomp += q.act >= A_C0;
      if (ncomp >= MAXCOMPILED)
        throw std::runtime_error("Next disjunct " + dj.op + " (line " + std::to_string(dj.line) + "): more than " +
                                 std::to_string(MAXCOMPILED) + " actions to compile");
      // the bag helpers it may call are the family's own (by closure hash); a
      // redefined one is refused where it is used
      std::map<std::string, int> helpers;
      std::set<std::string> redefined;
      for (const Known& q : kKnown)
        if (q.spec == L.spec && q.role == R_HELPER && m.find(q.name)) {
          if (hash_of(q.name) == q.hash) helpers[q.name] = q.id;
          else redefined.insert(q.name);
        }
      std::set<std::string> seen;
      std::function<void(const NodeP&, int)> uses = [&](const NodeP& n, int depth) {
        if (!n || depth > 64) return;
        if ((n->kind == N_APP || n->kind == N_ID) && redefined.count(n->s))
          throw std::runtime_error("Next disjunct " + dj.op + " (line " + std::to_string(dj.line) + ") calls " + n->s +
                                   ", which is not the " + spec_name(L.spec) + " module's own bag helper");
        if ((n->kind == N_APP || n->kind == N_ID) && !helpers.count(n->s) && seen.insert(n->s).second)
          if (const Def* od = m.find(n->s)) uses(od->body, depth + 1);
        for (auto& c : n->k) uses(c, depth + 1);
        for (auto& dd : n->defs) uses(dd.body, depth + 1);
      };
      for (auto& c : gs.conjuncts) uses(c, 0);
      gs.send_helpers = helpers;
      gs.act = A_C0 + ncomp;
      gs.op = dj.op;
      gs.kind = K_MSGC;
      gs.mod = mp;
      L.guards.push_back(gs);
      L.actions.push_back({gs.act, gs.kind});
      L.labels.push_back(dj.op);
      continue;
    }
    if (!k)
      throw std::runtime_error("Next disjunct " + dj.op + " (line " + std::to_string(dj.line) + ") computes an action "
                               "the " + spec_name(L.spec) + " lowering does not have (its definition differs from "
                               "every lowered action of the spec family, and its effect -- the conjuncts that change "
                               "the state -- from every effect whose guard the front end compiles, and it is not a "
                               "fixed-binding action of the Raft / FlexibleRaft / RaftFsync families the effect "
                               "compiler takes); adding it needs a lowering in rmc_spec.h");
    static const int form_of_kind[] = {B_I, B_IV, B_IJ, B_MSG, B_M};
    if (form_of_kind[k->kind] != dj.form)
      throw std::runtime_error("Next disjunct " + dj.op + " (line " + std::to_string(dj.line) +
                               ") binds its arguments differently from the lowered " + k->name);
    L.actions.push_back({k->id, k->kind});
    L.labels.push_back(dj.op);
  }
  for (const std::string& inv : invariants) {
    if (!m.find(inv)) continue;  // the caller reports it (TLC: undefined operator)
    const Known* k = find(R_INV, hash_of(inv));
    if (!k)
      throw std::runtime_error("invariant " + inv + " differs from every invariant the " + std::string(spec_name(L.spec)) +
                               " lowering checks");
    L.invariants[inv] = k->id;
  }
  if (!view.empty()) {
    if (!find(R_VIEW, hash_of(view))) throw std::runtime_error("VIEW " + view + " is not the view the lowering fingerprints");
    L.view_ok = true;
  }
  if (!symmetry.empty()) {
    if (!find(R_SYMM, hash_of(symmetry)))
      throw std::runtime_error("SYMMETRY " + symmetry + " is not the server symmetry the lowering canonicalises");
    L.symmetry_ok = true;
  }
  return L;
}

GuardSrc parse_action(int spec, const std::string& op, int kind, const std::vector<std::string>& params,
                      const std::string& body) {
  // the family's state (Raft.tla:58-107, FlexibleRaft.tla:63-109, RaftFsync.tla:62-110), restated
  std::string vars = "messages, acked, electionCtr, restartCtr, currentTerm, state, votedFor, log, commitIndex, "
                     "votesGranted, nextIndex, matchIndex";
  std::string leader = "<<nextIndex, matchIndex>>", logv = "<<log, commitIndex>>";
  std::map<std::string, int> helpers;
  if (spec == RAFT) {
    vars += ", pendingResponse";
    leader = "<<nextIndex, matchIndex, pendingResponse>>";
    helpers = {{"SendMultipleOnce", 0}, {"_SendOnce", 1}, {"Send", 2}, {"_SendNoRestriction", 2}};
  } else if (spec == FLEX) {
    helpers = {{"SendMultiple", 0}, {"Send", 1}};
  } else if (spec == FSYNC) {
    vars += ", fsyncIndex";
    logv = "<<log, commitIndex, fsyncIndex>>";
    helpers = {{"Send", 1}};
  } else {
    throw std::runtime_error("actions compiled whole are offered for Raft, FlexibleRaft and RaftFsync");
  }
  std::string ps;
  for (size_t q = 0; q < params.size(); q++) ps += (q ? ", " : "") + params[q];
  const std::string text = "---- MODULE ActionText ----\n"
                           "VARIABLES " + vars + "\n"
                           "auxVars == <<acked, electionCtr, restartCtr>>\n"
                           "serverVars == <<currentTerm, state, votedFor>>\n"
                           "candidateVars == <<votesGranted>>\n"
                           "leaderVars == " + leader + "\n"
                           "logVars == " + logv + "\n"
                           "Quorum == {i \\in SUBSET(Server) : Cardinality(i) * 2 > Cardinality(Server)}\n"
                           "LastTerm(xlog) == IF Len(xlog) = 0 THEN 0 ELSE xlog[Len(xlog)].term\n"
                           "Min(s) == CHOOSE x \\in s : \\A y \\in s : x <= y\n"
                           "Max(s) == CHOOSE x \\in s : \\A y \\in s : x >= y\n" +
                           // a message handler's guard helper, restated (Raft.tla:180-186)
                           std::string(kind == K_MSGC ? "ReceivableMessage(m, mtype, term_match) ==\n"
                                                        "    /\\ messages[m] > 0\n"
                                                        "    /\\ m.mtype = mtype\n"
                                                        "    /\\ \\/ /\\ term_match = EqualTerm\n"
                                                        "          /\\ m.mterm = currentTerm[m.mdest]\n"
                                                        "       \\/ /\\ term_match = LessOrEqualTerm\n"
                                                        "          /\\ m.mterm <= currentTerm[m.mdest]\n"
                                                      : "") +
                           op + (params.empty() ? "" : "(" + ps + ")") + " ==\n    " + body + "\n====\n";
  auto mod = std::make_shared<Module>(parse_module(text));
  const Def* d = mod->find(op);
  if (!d) throw ParseError("action text did not parse");
  if (!d->error.empty()) throw ParseError("action text: " + d->error);
  Hasher H(*mod);
  GuardSrc g;
  g.act = -1;
  g.op = op;
  g.params = params;
  g.kind = kind;
  g.mod = mod;
  g.send_helpers = helpers;
  if (kind == K_MSGC) {  // a message handler: Discard / Reply too, one program in the text's order
    g.send_helpers["Discard"] = 3;
    g.send_helpers["Reply"] = 4;
    g.conjuncts = {d->body};
    return g;
  }
  // the send helpers are not defined in the text: mark them as effects for the split
  for (auto& h : helpers) H.effect_ops.insert(h.first);
  if (!H.split(op, g.conjuncts, g.effects)) throw std::runtime_error("action " + op + " changes nothing");
  return g;
}

GuardSrc parse_guard(int spec, int act, const std::string& op, const std::vector<std::string>& params,
                     const std::string& expr) {
  // the family's standard helpers, restated (Raft.tla:123 Quorum, :126 LastTerm, :190-192 Min / Max)
  std::string ps;
  for (size_t q = 0; q < params.size(); q++) ps += (q ? ", " : "") + params[q];
  const std::string text = "---- MODULE GuardText ----\n"
                           "Quorum == {i \\in SUBSET(Server) : Cardinality(i) * 2 > Cardinality(Server)}\n"
                           "LastTerm(xlog) == IF Len(xlog) = 0 THEN 0 ELSE xlog[Len(xlog)].term\n"
                           "Min(s) == CHOOSE x \\in s : \\A y \\in s : x <= y\n"
                           "Max(s) == CHOOSE x \\in s : \\A y \\in s : x >= y\n"
                           "GuardOf" + op + (params.empty() ? "" : "(" + ps + ")") + " ==\n    " + expr + "\n====\n";
  auto helpers = std::make_shared<Module>(parse_module(text));
  const Def* d = helpers->find("GuardOf" + op);
  if (!d) throw ParseError("guard text did not parse");
  if (!d->error.empty()) throw ParseError("guard text: " + d->error);
  (void)spec;
  GuardSrc g;
  g.act = act;
  g.op = op;
  g.params = params;
  g.conjuncts = {d->body};
  g.mod = helpers;
  return g;
}

}  // namespace tla
}  // namespace rmc
