"""TLC semantics for the oracle: values, ordering, and the breadth-first driver.

TEST INFRASTRUCTURE ONLY (the checker, never the thing measured or shipped).

What is restated here is TLC's documented behaviour (SURVEY.md §3(1),
Appendix A), which the reference relies on when it says "run all these
specifications with the -deadlock argument" (/root/reference/README.md:6):

* Next is split into actions at start-up: top-level disjuncts in order, and
  a top-level `\\E x \\in S` over a constant set S becomes one action per
  binding (the FIRST bound variable varies fastest).  `\\E m \\in DOMAIN
  messages` is not constant, so it stays one action whose successors are
  produced in DOMAIN order at run time.
* Values are ordered like TLC's `compareTo`: records by field count, then
  field names (sorted) interleaved with their values; sequences by length,
  then elements; model values by name; FALSE < TRUE.  Function domains are
  kept sorted in this order, so DOMAIN messages is enumerated in it.
* One worker, FIFO queue: the first successor reaching a fingerprint wins;
  later successors with the same fingerprint are dropped.  VIEW + SYMMETRY:
  the fingerprint key is the view of the state minimised over all server
  permutations; the stored (and expanded) state is the actual one.
* Invariants are checked (in cfg order) on every NEW state, actual values.
* "states generated" counts every successor plus the initial states;
  "distinct" counts fingerprint inserts; depth counts levels with Init = 1.
"""
import itertools
import time

NIL = -1  # the model value Nil (Raft.tla:41) where a server or value is expected


class EvalError(Exception):
    """A TLC evaluation error (e.g. a sequence applied outside its domain)."""


class Rec(tuple):
    """A TLA+ record value, normalised like TLC: fields sorted by name."""
    __slots__ = ()

    def __new__(cls, **kw):
        return tuple.__new__(cls, tuple(sorted(kw.items())))

    def __getattr__(self, name):
        for k, v in self:
            if k == name:
                return v
        raise AttributeError("record has no field %s" % name)

    # record fields named like tuple methods (mlastCommonEntry.index,
    # PullRaft.tla:187) must read the field, not tuple.index / tuple.count
    @property
    def index(self):
        return self.__getattr__("index")

    @property
    def count(self):
        return self.__getattr__("count")

    def replace(self, **kw):
        d = dict(tuple.__iter__(self))
        d.update(kw)
        return Rec(**d)

    def __reduce__(self):  # picklable (the sharded-protocol test ships states between ranks)
        return (_rec_from_items, (tuple(tuple.__iter__(self)),))


def _rec_from_items(items):
    return Rec(**dict(items))


def tlc_key(v):
    """Sort key reproducing TLC's compareTo for the value kinds the specs use."""
    if isinstance(v, Rec):
        return (len(v), tuple((k, _field_key(x)) for k, x in v))
    if isinstance(v, tuple):  # sequence: length first, then elements
        return (len(v), tuple(tlc_key(x) for x in v))
    return v  # ints, bools (False < True), model-value names / indices


def _field_key(x):
    """A record field's key.  A field that holds either the model value Nil or a
    record (PullRaftVariant2.tla:369-375, mlastCommonEntry) compares Nil below
    every record: TLC's untyped model value is less than any non-model value and
    a record greater than a model value.  A field holding Nil or a server
    (KRaft.tla:500, mleader) compares by model-value name: Nil below n1, n2, ...  Record-valued fields of the other
    specs keep their relative order (both sides wrapped the same way)."""
    if isinstance(x, Rec):
        return (1, tlc_key(x))
    if type(x) is int:  # Nil (the model value) below the servers in a server-or-Nil field (KRaft mleader)
        return (0,) if x == NIL else (1, x)
    return tlc_key(x)


def seq_get(s, i):
    """s[i] for a TLA+ sequence (1-based); out of domain -> evaluation error."""
    if not isinstance(i, int) or i < 1 or i > len(s):
        raise EvalError("sequence of length %d applied to %r" % (len(s), i))
    return s[i - 1]


def fset(f, i, v):
    """[f EXCEPT ![i] = v] for a function over 0..n-1 stored as a tuple."""
    return f[:i] + (v,) + f[i + 1:]


def fset2(f, i, j, v):
    """[f EXCEPT ![i][j] = v]."""
    return fset(f, i, fset(f[i], j, v))


def freeze_msgs(d):
    """A messages function (dict record -> count), domain sorted as TLC keeps it."""
    return tuple(sorted(d.items(), key=lambda kv: _msg_key(kv[0])))


_KEYCACHE = {}


def _msg_key(m):
    k = _KEYCACHE.get(m)
    if k is None:
        k = tlc_key(m)
        _KEYCACHE[m] = k
    return k


def msg_dom(msgs):
    """DOMAIN messages, in TLC order (msgs is the frozen tuple)."""
    return [m for m, _ in msgs]


def msg_count(msgs, m):
    for x, c in msgs:
        if x == m:
            return c
    raise EvalError("messages applied outside its domain")


def msg_in(msgs, m):
    for x, _ in msgs:
        if x == m:
            return True
    return False


class Result:
    def __init__(self):
        self.generated = 0
        self.distinct = 0
        self.depth = 0
        self.left = 0
        self.status = "ok"          # ok | violation | error
        self.violated = None
        self.error = None
        self.levels = []            # [(generated_into_level, new_in_level)]
        self.action_counts = {}     # action name -> successors generated
        self.hidden_same_level = 0  # dup whose hidden vars differ, same level
        self.hidden_cross_level = 0
        self.trace = None           # list of (action label, state) on violation/error
        self.seconds = 0.0
        self.max_msgs = 0

    def as_dict(self):
        return dict(generated=self.generated, distinct=self.distinct,
                    depth=self.depth, left=self.left, status=self.status,
                    violated=self.violated, error=self.error,
                    levels=self.levels, action_counts=self.action_counts,
                    hidden_same_level=self.hidden_same_level,
                    hidden_cross_level=self.hidden_cross_level,
                    max_msgs=self.max_msgs)


def bfs(spec, max_states=None, keep_states=False, progress=False, max_depth=None):
    """Exhaustive BFS of `spec` with TLC -workers 1 semantics.

    spec must provide: init_states(), actions() -> [(label, fn(state) -> iterable)],
    invariants -> [(name, fn(state) -> bool)], canonical(state) -> hashable,
    hidden(state) -> hashable.
    """
    t0 = time.time()
    res = Result()
    seen = {}  # canonical view -> (level, hidden, index)
    parent = []
    states = []
    actions = spec.actions()
    level = []

    def check(s):
        for name, inv in spec.invariants:
            if not inv(s):
                return name
        return None

    def make_trace(idx, last=None):
        chain = []
        while idx is not None:
            chain.append(idx)
            idx = parent[idx][0]
        chain.reverse()
        tr = [(parent[i][1], states[i]) for i in chain]
        if last is not None:
            tr.append(last)
        return tr

    for s in spec.init_states():
        res.generated += 1
        key = spec.canonical(s)
        if key in seen:
            continue
        seen[key] = (1, spec.hidden(s), len(states))
        states.append(s)
        parent.append((None, "Initial predicate"))
        level.append(len(states) - 1)
        try:
            bad = check(s)
        except EvalError as e:
            res.status, res.error = "error", str(e)
            res.trace = make_trace(len(states) - 1)
            bad = None
        if bad:
            res.status, res.violated = "violation", bad
            res.trace = make_trace(len(states) - 1)
        if res.status != "ok":
            res.distinct = len(states)
            res.depth = 1
            res.levels.append((res.generated, len(level)))
            res.seconds = time.time() - t0
            return res
    res.levels.append((res.generated, len(level)))
    depth = 1
    while level:
        if max_depth and depth >= max_depth:  # as rmc_options.max_depth: stop after that many levels
            res.status = "stopped"
            res.left = len(level)
            break
        nxt = []
        gen_lvl = 0
        for pidx in level:
            s = states[pidx]
            res.max_msgs = max(res.max_msgs, len(s["messages"]))
            for label, fn in actions:
                try:
                    succs = list(fn(s))
                except EvalError as e:
                    res.status, res.error = "error", "%s: %s" % (label, e)
                    res.trace = make_trace(pidx)
                    res.trace.append((label, None))
                    break
                for t in succs:
                    gen_lvl += 1
                    res.generated += 1
                    res.action_counts[label.split("(")[0]] = res.action_counts.get(label.split("(")[0], 0) + 1
                    key = spec.canonical(t)
                    old = seen.get(key)
                    if old is not None:
                        if old[1] != spec.hidden(t):
                            if old[0] == depth + 1:
                                res.hidden_same_level += 1
                            else:
                                res.hidden_cross_level += 1
                        continue
                    seen[key] = (depth + 1, spec.hidden(t), len(states))
                    states.append(t)
                    parent.append((pidx, label))
                    nxt.append(len(states) - 1)
                    try:
                        bad = check(t)
                    except EvalError as e:
                        res.status, res.error = "error", "invariant: %s" % e
                        res.trace = make_trace(len(states) - 1)
                        break
                    if bad:
                        res.status, res.violated = "violation", bad
                        res.trace = make_trace(len(states) - 1)
                        break
                if res.status != "ok":
                    break
            if res.status != "ok":
                break
        if res.status != "ok":
            res.levels.append((gen_lvl, len(nxt)))
            res.depth = depth + (1 if nxt else 0)
            # TLC: states left on queue = unexplored states still queued
            res.left = len(nxt) + (len(level) - level.index(pidx) - 1)
            break
        if nxt:
            depth += 1
            res.levels.append((gen_lvl, len(nxt)))
        elif gen_lvl:
            res.levels.append((gen_lvl, 0))
        if progress:
            print("level %d: %d new, %d distinct, %d generated, %.1fs" %
                  (depth, len(nxt), len(states), res.generated, time.time() - t0), flush=True)
        level = nxt
        if max_states and len(states) >= max_states:
            res.status = "truncated"
            res.left = len(level)
            break
    res.distinct = len(states)
    res.depth = max(res.depth, depth)
    res.seconds = time.time() - t0
    if keep_states:
        res.states = states
        res.parent = parent
    return res


def permutations(n):
    return list(itertools.permutations(range(n)))
