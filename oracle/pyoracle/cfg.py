"""TLC model-config (.cfg) reader for the oracle.

TEST INFRASTRUCTURE ONLY: this package is the CPU checker that the HIP path
is compared against.  Nothing in the product path imports it.

The grammar is TLC's config language as used by the reference cfgs, e.g.
`specifications/standard-raft/Raft.cfg:5-36`: CONSTANT(S) blocks of
`Name = value` lines, INIT/NEXT, VIEW, SYMMETRY, INVARIANT(S), PROPERTY.
Quirks accepted: self-assignments of undeclared identifiers
(`n1 = n1`, Raft.cfg:6-9) and model values used without any declaration
(`v2` in `Value = { v1, v2 }`, PullRaft.cfg:11).  Bare identifiers on the
right-hand side are untyped model values.
"""
import re

KEYWORDS = {
    "CONSTANT", "CONSTANTS", "INIT", "NEXT", "SPECIFICATION", "INVARIANT",
    "INVARIANTS", "PROPERTY", "PROPERTIES", "VIEW", "SYMMETRY", "CONSTRAINT",
    "CONSTRAINTS", "ACTION_CONSTRAINT", "ACTION_CONSTRAINTS", "CHECK_DEADLOCK",
    "POSTCONDITION", "ALIAS",
}


class ModelValue(str):
    """An untyped TLC model value (bare cfg identifier)."""
    __slots__ = ()

    def __repr__(self):
        return "MV(%s)" % str(self)


def _strip_comments(text):
    # block comments (* ... *) may nest in TLA+; the cfgs only use line comments
    out, depth, i = [], 0, 0
    while i < len(text):
        if text.startswith("(*", i):
            depth += 1
            i += 2
            continue
        if depth and text.startswith("*)", i):
            depth -= 1
            i += 2
            continue
        if not depth:
            out.append(text[i])
        i += 1
    text = "".join(out)
    return "\n".join(line.split("\\*", 1)[0] for line in text.splitlines())


_TOK = re.compile(r"\s*(<-|[{}(),=]|\"[^\"]*\"|-?\d+|[A-Za-z_][A-Za-z0-9_!]*)")


def _tokens(text):
    pos, toks = 0, []
    text = text.rstrip()
    while pos < len(text):
        m = _TOK.match(text, pos)
        if not m:
            if text[pos:].strip() == "":
                break
            raise ValueError("cfg: cannot tokenize near %r" % text[pos:pos + 20])
        toks.append(m.group(1))
        pos = m.end()
    return toks


def _parse_value(toks, k):
    t = toks[k]
    if t == "{":
        k += 1
        elems = []
        while toks[k] != "}":
            v, k = _parse_value(toks, k)
            elems.append(v)
            if toks[k] == ",":
                k += 1
        return frozenset(elems), k + 1
    if t == "TRUE":
        return True, k + 1
    if t == "FALSE":
        return False, k + 1
    if re.fullmatch(r"-?\d+", t):
        return int(t), k + 1
    if t.startswith('"'):
        return t[1:-1], k + 1
    return ModelValue(t), k + 1


def parse_cfg(text):
    """Return dict(constants, init, next, view, symmetry, invariants, properties)."""
    toks = _tokens(_strip_comments(text))
    cfg = dict(constants={}, init=None, next=None, spec=None, view=None,
               symmetry=None, invariants=[], properties=[], constraints=[],
               check_deadlock=None)
    k, section = 0, None
    while k < len(toks):
        t = toks[k]
        if t in KEYWORDS:
            section = t
            k += 1
            if section in ("INIT", "NEXT", "SPECIFICATION", "VIEW", "SYMMETRY", "ALIAS"):
                key = {"INIT": "init", "NEXT": "next", "SPECIFICATION": "spec",
                       "VIEW": "view", "SYMMETRY": "symmetry", "ALIAS": "alias"}[section]
                cfg[key] = toks[k]
                k += 1
            elif section == "CHECK_DEADLOCK":
                v, k = _parse_value(toks, k)
                cfg["check_deadlock"] = v
            continue
        if section in ("CONSTANT", "CONSTANTS"):
            name = t
            op = toks[k + 1]
            if op == "=":
                v, k = _parse_value(toks, k + 2)
                cfg["constants"][name] = v
            elif op == "<-":
                cfg["constants"][name] = ("<-", toks[k + 2])
                k += 3
            else:
                raise ValueError("cfg: bad constant line at %r" % name)
            continue
        if section in ("INVARIANT", "INVARIANTS"):
            cfg["invariants"].append(t)
        elif section in ("PROPERTY", "PROPERTIES"):
            cfg["properties"].append(t)
        elif section in ("CONSTRAINT", "CONSTRAINTS", "ACTION_CONSTRAINT", "ACTION_CONSTRAINTS"):
            cfg["constraints"].append(t)
        else:
            raise ValueError("cfg: token %r outside any section" % t)
        k += 1
    return cfg


def load_cfg(path):
    with open(path) as f:
        return parse_cfg(f.read())
