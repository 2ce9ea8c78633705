"""Literal restatement of /root/reference/specifications/standard-raft/Raft.tla.

TEST INFRASTRUCTURE ONLY.  Every operator below cites the TLA+ lines it
restates.  Encoding: servers are indices 0..N-1 in model-value name order
(so index order is TLC's enumeration order), values are indices 0..V-1, Nil
is NIL (-1), booleans are Python bools, records are `Rec`, sequences are
tuples, functions over Server/Value are tuples, `messages` is a tuple of
(record, count) pairs sorted in TLC's value order.
"""
from .tlc import (NIL, EvalError, Rec, seq_get, fset, fset2, freeze_msgs,
                  msg_in, permutations)

FOLLOWER, CANDIDATE, LEADER = "Follower", "Candidate", "Leader"
RVREQ, RVRESP = "RequestVoteRequest", "RequestVoteResponse"
AEREQ, AERESP = "AppendEntriesRequest", "AppendEntriesResponse"
EQUAL, LEQ = "EqualTerm", "LessOrEqualTerm"


def _sorted_names(s):
    return sorted(str(x) for x in s)


class RaftSpec:
    """MODULE Raft (Raft.tla:1-638) bound to a cfg (Raft.cfg:5-36)."""
    module = "Raft"
    # declaration order of VARIABLES, Raft.tla:58-106
    variables = ("messages", "acked", "electionCtr", "restartCtr", "currentTerm",
                 "state", "votedFor", "log", "commitIndex", "votesGranted",
                 "nextIndex", "matchIndex", "pendingResponse")
    # view == <<messages, serverVars, candidateVars, leaderVars, logVars>> (Raft.tla:115)
    hidden_vars = ("acked", "electionCtr", "restartCtr")

    def __init__(self, consts, invariants=("LeaderHasAllAckedValues", "NoLogDivergence"), next_order=None,
                 guards=None, defined=None):
        # defined: {name: (form, f(spec, s, *args) -> successors)}: actions
        # written in Python for next_order to name, bound as a Next disjunct
        # \E i \in Server (form "i"), \E i \in Server, v \in Value ("iv"),
        # \E i, j \in Server ("ij") or over DOMAIN messages ("m": f(spec, s)):
        # the oracle side of actions the front end compiles whole (rmc_guard.cpp
        # compile_effect, compile_handler)
        self.defined = dict(defined or {})
        # guards: {action name: g(spec, s, *args) -> bool} replacing the
        # reference's guard of that action (its effect unchanged): the oracle
        # side of the front end's compiled guards (rmc_guard.cpp)
        self.guards = dict(guards or {})
        # next_order: Next's disjuncts by operator name, in order (default: the
        # module's own Next); may drop disjuncts or add the network actions the
        # module defines but leaves commented out of Next (Raft.tla:540-541)
        self.next_order = tuple(next_order) if next_order else None
        self.server_names = _sorted_names(consts["Server"])
        self.value_names = _sorted_names(consts["Value"])
        self.N = len(self.server_names)
        self.V = len(self.value_names)
        self.Server = range(self.N)
        self.Value = range(self.V)
        self.MaxElections = int(consts["MaxElections"])
        self.MaxRestarts = int(consts["MaxRestarts"])
        self.setup(consts)
        self.perms = permutations(self.N)
        table = {"LeaderHasAllAckedValues": self.LeaderHasAllAckedValues,
                 "NoLogDivergence": self.NoLogDivergence,
                 "CommittedEntriesReachMajority": self.CommittedEntriesReachMajority,
                 "ElectionSafety": self.ElectionSafety, "LogMatching": self.LogMatching,
                 "LeaderCompleteness": self.LeaderCompleteness, "StateMachineSafety": self.StateMachineSafety}
        self.invariants = [(n, table[n]) for n in invariants]

    def setup(self, consts):
        pass

    def _guard(self, name, s, args, reference):
        """The action's guard: an override from `guards`, else the reference's (a thunk)."""
        g = self.guards.get(name)
        return g(self, s, *args) if g is not None else reference()

    # ---------------------------------------------------------------- helpers
    def IsQuorum(self, s):
        # Quorum == {i \in SUBSET(Server) : Cardinality(i) * 2 > Cardinality(Server)}  (Raft.tla:123)
        return len(s) * 2 > self.N

    @staticmethod
    def LastTerm(xlog):
        # Raft.tla:126
        return 0 if len(xlog) == 0 else seq_get(xlog, len(xlog)).term

    @staticmethod
    def _SendNoRestriction(msgs, m):
        # Raft.tla:129-132
        d = dict(msgs)
        d[m] = d.get(m, 0) + 1
        return freeze_msgs(d)

    @staticmethod
    def _SendOnce(msgs, m):
        # Raft.tla:136-138; None = disabled
        if msg_in(msgs, m):
            return None
        d = dict(msgs)
        d[m] = 1
        return freeze_msgs(d)

    def Send(self, msgs, m):
        # Raft.tla:145-149
        if m.mtype == AEREQ and m.mentries == ():
            return self._SendOnce(msgs, m)
        return self._SendNoRestriction(msgs, m)

    @staticmethod
    def SendMultipleOnce(msgs, ms):
        # Raft.tla:153-155
        for m in ms:
            if msg_in(msgs, m):
                return None
        d = dict(msgs)
        for m in ms:
            d[m] = 1
        return freeze_msgs(d)

    @staticmethod
    def Discard(msgs, m):
        # Raft.tla:164-167
        d = dict(msgs)
        if m not in d or not d[m] > 0:
            return None
        d[m] -= 1
        return freeze_msgs(d)

    def Reply(self, msgs, response, request):
        # Raft.tla:170-176: adds the response, or increments an existing one
        d = dict(msgs)
        if not d[request] > 0:
            return None
        d[request] -= 1
        d[response] = d.get(response, 0) + 1
        return freeze_msgs(d)

    @staticmethod
    def ReceivableMessage(s, m, count, mtype, term_match):
        # Raft.tla:181-187
        if not count > 0:
            return False
        if m.mtype != mtype:
            return False
        cur = s["currentTerm"][m.mdest]
        if term_match == EQUAL:
            return m.mterm == cur
        return m.mterm <= cur

    # ------------------------------------------------------------------- Init
    def init_states(self):
        # Raft.tla:197-218
        N = self.N
        yield dict(
            messages=(),
            acked=tuple(NIL for _ in self.Value),
            electionCtr=0,
            restartCtr=0,
            currentTerm=tuple(1 for _ in range(N)),
            state=tuple(FOLLOWER for _ in range(N)),
            votedFor=tuple(NIL for _ in range(N)),
            log=tuple(() for _ in range(N)),
            commitIndex=tuple(0 for _ in range(N)),
            votesGranted=tuple(frozenset() for _ in range(N)),
            nextIndex=tuple(tuple(1 for _ in range(N)) for _ in range(N)),
            matchIndex=tuple(tuple(0 for _ in range(N)) for _ in range(N)),
            pendingResponse=tuple(tuple(False for _ in range(N)) for _ in range(N)),
        )

    # ---------------------------------------------------------------- actions
    def Restart(self, s, i):
        # Raft.tla:226-235
        if not self._guard("Restart", s, (i,), lambda: s["restartCtr"] < self.MaxRestarts):
            return
        N = self.N
        t = dict(s)
        t["state"] = fset(s["state"], i, FOLLOWER)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset())
        t["nextIndex"] = fset(s["nextIndex"], i, tuple(1 for _ in range(N)))
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(0 for _ in range(N)))
        t["pendingResponse"] = fset(s["pendingResponse"], i, tuple(False for _ in range(N)))
        t["commitIndex"] = fset(s["commitIndex"], i, 0)
        t["restartCtr"] = s["restartCtr"] + 1
        yield t

    def RequestVote(self, s, i):
        # Raft.tla:242-257
        if not self._guard("RequestVote", s, (i,), lambda: s["electionCtr"] < self.MaxElections and
                           s["state"][i] in (FOLLOWER, CANDIDATE)):
            return
        term = s["currentTerm"][i] + 1
        ms = [Rec(mtype=RVREQ, mterm=term, mlastLogTerm=self.LastTerm(s["log"][i]),
                  mlastLogIndex=len(s["log"][i]), msource=i, mdest=j)
              for j in self.Server if j != i]
        msgs = self.SendMultipleOnce(s["messages"], ms)
        if msgs is None:
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, CANDIDATE)
        t["currentTerm"] = fset(s["currentTerm"], i, term)
        t["votedFor"] = fset(s["votedFor"], i, i)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset([i]))
        t["electionCtr"] = s["electionCtr"] + 1
        t["messages"] = msgs
        yield t

    def AppendEntries(self, s, i, j):
        # Raft.tla:263-285
        if i == j or s["state"][i] != LEADER:
            return
        if s["pendingResponse"][i][j] is not False:
            return
        log_i = s["log"][i]
        nxt = s["nextIndex"][i][j]
        prevLogIndex = nxt - 1
        prevLogTerm = seq_get(log_i, prevLogIndex).term if prevLogIndex > 0 else 0
        lastEntry = min(len(log_i), nxt)
        # SubSeq(log[i], nextIndex[i][j], lastEntry)
        entries = tuple(seq_get(log_i, k) for k in range(nxt, lastEntry + 1))
        m = Rec(mtype=AEREQ, mterm=s["currentTerm"][i], mprevLogIndex=prevLogIndex,
                mprevLogTerm=prevLogTerm, mentries=entries,
                mcommitIndex=min(s["commitIndex"][i], lastEntry), msource=i, mdest=j)
        msgs = self.Send(s["messages"], m)
        if msgs is None:
            return
        t = dict(s)
        t["pendingResponse"] = fset2(s["pendingResponse"], i, j, True)
        t["messages"] = msgs
        yield t

    def BecomeLeader(self, s, i):
        # Raft.tla:289-300
        if not self._guard("BecomeLeader", s, (i,), lambda: s["state"][i] == CANDIDATE and
                           self.IsQuorum(s["votesGranted"][i])):
            return
        N = self.N
        t = dict(s)
        t["state"] = fset(s["state"], i, LEADER)
        t["nextIndex"] = fset(s["nextIndex"], i, tuple(len(s["log"][i]) + 1 for _ in range(N)))
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(0 for _ in range(N)))
        t["pendingResponse"] = fset(s["pendingResponse"], i, tuple(False for _ in range(N)))
        yield t

    def ClientRequest(self, s, i, v):
        # Raft.tla:304-313
        if not self._guard("ClientRequest", s, (i, v), lambda: s["state"][i] == LEADER and s["acked"][v] == NIL):
            return
        entry = Rec(term=s["currentTerm"][i], value=v)
        t = dict(s)
        t["log"] = fset(s["log"], i, s["log"][i] + (entry,))
        t["acked"] = fset(s["acked"], v, False)
        yield t

    def agree_set(self, s, i, index):
        # Agree(index) == {i} \cup {k \in Server : matchIndex[i][k] >= index}  (Raft.tla:323-324)
        return frozenset([i]) | frozenset(k for k in self.Server if s["matchIndex"][i][k] >= index)

    def agree_ok(self, s, i, index):
        return self.IsQuorum(self.agree_set(s, i, index))

    def AdvanceCommitIndex(self, s, i):
        # Raft.tla:320-344
        if s["state"][i] != LEADER:
            return
        log_i = s["log"][i]
        agreeIndexes = [index for index in range(1, len(log_i) + 1) if self.agree_ok(s, i, index)]
        if agreeIndexes and seq_get(log_i, max(agreeIndexes)).term == s["currentTerm"][i]:
            newCommitIndex = max(agreeIndexes)
        else:
            newCommitIndex = s["commitIndex"][i]
        if not s["commitIndex"][i] < newCommitIndex:
            return
        t = dict(s)
        t["commitIndex"] = fset(s["commitIndex"], i, newCommitIndex)
        committed = {seq_get(log_i, index).value
                     for index in range(s["commitIndex"][i] + 1, newCommitIndex + 1)}
        t["acked"] = tuple((v in committed) if s["acked"][v] is False else s["acked"][v]
                           for v in self.Value)
        self.after_commit(s, t, i)
        yield t

    def after_commit(self, s, t, i):
        pass

    def DuplicateMessage(self, s):
        # Raft.tla:512-514 with Duplicate (:157-160): \E m \in DOMAIN messages, messages[m] + 1
        for m, c in s["messages"]:
            d = dict(s["messages"])
            d[m] = c + 1
            t = dict(s)
            t["messages"] = freeze_msgs(d)
            yield t

    def DropMessage(self, s):
        # Raft.tla:519-521 with Discard (:164-167): messages[m] > 0, messages[m] - 1
        for m, _ in s["messages"]:
            nm = self.Discard(s["messages"], m)
            if nm is None:
                continue
            t = dict(s)
            t["messages"] = nm
            yield t

    def UpdateTerm(self, s):
        # Raft.tla:348-355
        for m, _ in s["messages"]:
            d = m.mdest
            if m.mterm > s["currentTerm"][d]:
                t = dict(s)
                t["currentTerm"] = fset(s["currentTerm"], d, m.mterm)
                t["state"] = fset(s["state"], d, FOLLOWER)
                t["votedFor"] = fset(s["votedFor"], d, NIL)
                yield t

    def HandleRequestVoteRequest(self, s):
        # Raft.tla:360-381
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, RVREQ, LEQ):
                continue
            i, j = m.mdest, m.msource
            lt = self.LastTerm(s["log"][i])
            logOk = (m.mlastLogTerm > lt or
                     (m.mlastLogTerm == lt and m.mlastLogIndex >= len(s["log"][i])))
            grant = (m.mterm == s["currentTerm"][i] and logOk and
                     s["votedFor"][i] in (NIL, j))
            if not m.mterm <= s["currentTerm"][i]:
                continue
            resp = Rec(mtype=RVRESP, mterm=s["currentTerm"][i], mvoteGranted=grant,
                       msource=i, mdest=j)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t = dict(s)
            if grant:
                t["votedFor"] = fset(s["votedFor"], i, j)
            t["messages"] = msgs
            yield t

    def HandleRequestVoteResponse(self, s):
        # Raft.tla:386-401
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, RVRESP, EQUAL):
                continue
            i, j = m.mdest, m.msource
            msgs = self.Discard(s["messages"], m)
            if msgs is None:
                continue
            t = dict(s)
            if m.mvoteGranted:
                t["votesGranted"] = fset(s["votesGranted"], i, s["votesGranted"][i] | {j})
            t["messages"] = msgs
            yield t

    def LogOk(self, s, i, m):
        # Raft.tla:406-410
        if m.mprevLogIndex == 0:
            return True
        return (m.mprevLogIndex > 0 and m.mprevLogIndex <= len(s["log"][i]) and
                m.mprevLogTerm == seq_get(s["log"][i], m.mprevLogIndex).term)

    def RejectAppendEntriesRequest(self, s):
        # Raft.tla:412-430
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, AEREQ, LEQ):
                continue
            i, j = m.mdest, m.msource
            cur = s["currentTerm"][i]
            if not (m.mterm < cur or
                    (m.mterm == cur and s["state"][i] == FOLLOWER and not self.LogOk(s, i, m))):
                continue
            resp = Rec(mtype=AERESP, mterm=cur, msuccess=False, mmatchIndex=0,
                       msource=i, mdest=j)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t = dict(s)
            t["messages"] = msgs
            yield t

    # CanAppend / NeedsTruncation / TruncateLog (Raft.tla:438-452)
    @staticmethod
    def CanAppend(s, m, i):
        return m.mentries != () and len(s["log"][i]) == m.mprevLogIndex

    def NeedsTruncation(self, s, m, i, index):
        L = len(s["log"][i])
        return ((m.mentries != () and L >= index) or
                (m.mentries == () and L > m.mprevLogIndex))

    @staticmethod
    def TruncateLog(s, m, i):
        return tuple(seq_get(s["log"][i], k) for k in range(1, m.mprevLogIndex + 1))

    def new_log(self, s, m, i, index):
        # the CASE of Raft.tla:464-470 (arms tried in order)
        log_i = s["log"][i]
        if self.CanAppend(s, m, i):
            return log_i + (seq_get(m.mentries, 1),)
        if self.NeedsTruncation(s, m, i, index) and m.mentries != ():
            return self.TruncateLog(s, m, i) + (seq_get(m.mentries, 1),)
        if self.NeedsTruncation(s, m, i, index) and m.mentries == ():
            return self.TruncateLog(s, m, i)
        return log_i

    def AcceptAppendEntriesRequest(self, s):
        # Raft.tla:454-485
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, AEREQ, EQUAL):
                continue
            i, j = m.mdest, m.msource
            index = m.mprevLogIndex + 1
            if s["state"][i] not in (FOLLOWER, CANDIDATE):
                continue
            if not self.LogOk(s, i, m):
                continue
            nl = self.new_log(s, m, i, index)
            resp = Rec(mtype=AERESP, mterm=s["currentTerm"][i], msuccess=True,
                       mmatchIndex=m.mprevLogIndex + len(m.mentries), msource=i, mdest=j)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t = dict(s)
            t["state"] = fset(s["state"], i, FOLLOWER)
            t["commitIndex"] = fset(s["commitIndex"], i, m.mcommitIndex)
            t["log"] = fset(s["log"], i, nl)
            t["messages"] = msgs
            self.after_accept(s, t, i, nl)
            yield t

    def after_accept(self, s, t, i, nl):
        pass

    def HandleAppendEntriesResponse(self, s):
        # Raft.tla:490-505
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, AERESP, EQUAL):
                continue
            i, j = m.mdest, m.msource
            msgs = self.Discard(s["messages"], m)
            if msgs is None:
                continue
            t = dict(s)
            if m.msuccess:
                t["nextIndex"] = fset2(s["nextIndex"], i, j, m.mmatchIndex + 1)
                t["matchIndex"] = fset2(s["matchIndex"], i, j, m.mmatchIndex)
            else:
                t["nextIndex"] = fset2(s["nextIndex"], i, j, max(s["nextIndex"][i][j] - 1, 1))
            self.after_aeresp(s, t, i, j)
            t["messages"] = msgs
            yield t

    def after_aeresp(self, s, t, i, j):
        t["pendingResponse"] = fset2(s["pendingResponse"], i, j, False)

    # ------------------------------------------------------------------- Next
    def pairs(self):
        # \E i, j \in Server : the first bound variable varies fastest (TLC)
        return [(i, j) for j in self.Server for i in self.Server]

    def actions(self):
        """Next (Raft.tla:527-539) split into TLC actions, in TLC order."""
        if self.next_order:
            return self.ordered_actions(self.next_order)
        return self.default_actions()

    def ordered_actions(self, order):
        r"""Next with the given disjuncts (by operator name) in the given order:
        each disjunct's TLC actions as in the module's own Next, plus the network
        actions \E m \in DOMAIN messages : DuplicateMessage(m) / DropMessage(m)."""
        groups = {}
        for label, fn in self.default_actions():
            groups.setdefault(label.split("(")[0], []).append((label, fn))
        groups["DuplicateMessage"] = [("DuplicateMessage", self.DuplicateMessage)]
        groups["DropMessage"] = [("DropMessage", self.DropMessage)]
        n, vn = self.server_names, self.value_names
        for name, (form, f) in self.defined.items():
            # TLC order: the first bound variable varies fastest
            if form == "i":
                groups[name] = [("%s(%s)" % (name, n[i]), lambda s, f=f, i=i: f(self, s, i)) for i in self.Server]
            elif form == "iv":
                groups[name] = [("%s(%s,%s)" % (name, n[i], vn[v]), lambda s, f=f, i=i, v=v: f(self, s, i, v))
                                for v in self.Value for i in self.Server]
            elif form == "ij":
                groups[name] = [("%s(%s,%s)" % (name, n[i], n[j]), lambda s, f=f, i=i, j=j: f(self, s, i, j))
                                for i, j in self.pairs()]
            elif form == "m":
                # a message handler (\E m \in DOMAIN messages : ...): f ranges over
                # DOMAIN messages itself, in TLC's order, as the module's handlers do
                groups[name] = [(name, lambda s, f=f: f(self, s))]
            else:
                raise ValueError("form %r" % form)
        out = []
        for name in order:
            if name not in groups:
                raise ValueError("no disjunct %s in %s" % (name, self.module))
            out.extend(groups[name])
        return out

    def default_actions(self):
        A = []
        n = self.server_names
        vn = self.value_names
        for i in self.Server:
            A.append(("Restart(%s)" % n[i], lambda s, i=i: self.Restart(s, i)))
        for i in self.Server:
            A.append(("RequestVote(%s)" % n[i], lambda s, i=i: self.RequestVote(s, i)))
        for i in self.Server:
            A.append(("BecomeLeader(%s)" % n[i], lambda s, i=i: self.BecomeLeader(s, i)))
        for v in self.Value:
            for i in self.Server:
                A.append(("ClientRequest(%s,%s)" % (n[i], vn[v]),
                          lambda s, i=i, v=v: self.ClientRequest(s, i, v)))
        for i in self.Server:
            A.append(("AdvanceCommitIndex(%s)" % n[i], lambda s, i=i: self.AdvanceCommitIndex(s, i)))
        for i, j in self.pairs():
            A.append(("AppendEntries(%s,%s)" % (n[i], n[j]),
                      lambda s, i=i, j=j: self.AppendEntries(s, i, j)))
        A.append(("UpdateTerm", self.UpdateTerm))
        A.append(("HandleRequestVoteRequest", self.HandleRequestVoteRequest))
        A.append(("HandleRequestVoteResponse", self.HandleRequestVoteResponse))
        A.append(("RejectAppendEntriesRequest", self.RejectAppendEntriesRequest))
        A.append(("AcceptAppendEntriesRequest", self.AcceptAppendEntriesRequest))
        A.append(("HandleAppendEntriesResponse", self.HandleAppendEntriesResponse))
        return A

    # ------------------------------------------------------------- invariants
    def NoLogDivergence(self, s):
        # Raft.tla:580-596; \A s1, s2 enumerated with s1 fastest
        ci, lg = s["commitIndex"], s["log"]
        for s2 in self.Server:
            for s1 in self.Server:
                if s1 == s2:
                    continue
                c = ci[s1] if ci[s1] < ci[s2] else ci[s2]
                if c > 0:
                    for index in range(1, c + 1):
                        if seq_get(lg[s1], index) != seq_get(lg[s2], index):
                            return False
        return True

    def LeaderHasAllAckedValues(self, s):
        # Raft.tla:604-620
        for v in self.Value:
            if s["acked"][v] is True:
                for i in self.Server:
                    if (s["state"][i] == LEADER and
                            not any(l != i and s["currentTerm"][l] > s["currentTerm"][i]
                                    for l in self.Server) and
                            not any(e.value == v for e in s["log"][i])):
                        return False
        return True

    def CommittedEntriesReachMajority(self, s):
        # Raft.tla:625-636 (not enabled by any shipped cfg; offered as an extra)
        import itertools
        lead = [i for i in self.Server if s["state"][i] == LEADER and s["commitIndex"][i] > 0]
        if not lead:
            return True
        size = self.N // 2 + 1
        for i in lead:
            ci = s["commitIndex"][i]
            for q in itertools.combinations(self.Server, size):
                if i not in q:
                    continue
                if all(len(s["log"][j]) >= ci and
                       seq_get(s["log"][j], ci) == seq_get(s["log"][i], ci) for j in q):
                    return True
        return False

    # The classic Raft safety properties (Ongaro, Fig. 3.2), opt-in extras: the
    # reference's specs do not define them.  Restated from the
    # TLA+ text given in INTEGRATION.md, literally (sets of servers, SubSeq).
    def ElectionSafety(self, s):
        # \A s1, s2 : s1 # s2 /\ both Leader => currentTerm[s1] # currentTerm[s2]
        return not any(s1 != s2 and s["state"][s1] == LEADER and s["state"][s2] == LEADER and
                       s["currentTerm"][s1] == s["currentTerm"][s2]
                       for s1 in self.Server for s2 in self.Server)

    def LogMatching(self, s):
        # \A s1, s2, i \in 1..Min(Len, Len) : same term at i => SubSeq(.., 1, i) equal
        lg = s["log"]
        for s1 in self.Server:
            for s2 in self.Server:
                for i in range(1, min(len(lg[s1]), len(lg[s2])) + 1):
                    if seq_get(lg[s1], i).term == seq_get(lg[s2], i).term and lg[s1][:i] != lg[s2][:i]:
                        return False
        return True

    def LeaderCompleteness(self, s):
        # a leader whose term no server exceeds holds every committed entry
        lg, ci = s["log"], s["commitIndex"]
        for l in self.Server:
            if s["state"][l] != LEADER or any(s["currentTerm"][k] > s["currentTerm"][l] for k in self.Server):
                continue
            for k in self.Server:
                for i in range(1, min(ci[k], len(lg[k])) + 1):
                    if not (i <= len(lg[l]) and seq_get(lg[l], i) == seq_get(lg[k], i)):
                        return False
        return True

    def StateMachineSafety(self, s):
        # committed prefixes (bounded by Len) agree
        lg, ci = s["log"], s["commitIndex"]
        for s1 in self.Server:
            for s2 in self.Server:
                for i in range(1, min(ci[s1], ci[s2], len(lg[s1]), len(lg[s2])) + 1):
                    if seq_get(lg[s1], i) != seq_get(lg[s2], i):
                        return False
        return True

    # ----------------------------------------------------- VIEW and SYMMETRY
    def view_vars(self):
        return [v for v in self.variables if v not in self.hidden_vars]

    def permute_value(self, var, val, p):
        """Apply server permutation p (old index -> new index) to one variable."""
        N = self.N
        inv = [0] * N
        for a, b in enumerate(p):
            inv[b] = a

        def srv(x):
            return x if x == NIL else p[x]

        if var == "messages":
            out = []
            for m, c in val:
                out.append((m.replace(msource=p[m.msource], mdest=p[m.mdest]), c))
            out.sort()
            return tuple(out)
        if var in ("votedFor", "leader"):
            return tuple(srv(val[inv[k]]) for k in range(N))
        if var == "votesGranted":
            return tuple(tuple(sorted(p[x] for x in val[inv[k]])) for k in range(N))
        if var in ("nextIndex", "matchIndex", "pendingResponse"):
            return tuple(tuple(val[inv[k]][inv[q]] for q in range(N)) for k in range(N))
        if var in ("currentTerm", "state", "log", "commitIndex", "fsyncIndex"):
            return tuple(val[inv[k]] for k in range(N))
        return val  # acked, electionCtr, restartCtr contain no servers

    def canonical(self, s):
        vv = self.view_vars()
        best = None
        for p in self.perms:
            cand = tuple(self.permute_value(v, s[v], p) for v in vv)
            if best is None or cand < best:
                best = cand
        return best

    def hidden(self, s):
        return tuple(s[v] for v in self.hidden_vars)
