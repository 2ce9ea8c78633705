"""Literal restatements of FlexibleRaft.tla, RaftFsync.tla, PullRaft.tla and
PullRaftVariant2.tla.

TEST INFRASTRUCTURE ONLY.  The Raft-derived variants subclass RaftSpec and
override exactly the operators whose TLA+ text differs (cited per method);
PullRaft is restated in full, PullRaftVariant2 as its differences from it.
"""
from .tlc import NIL, Rec, seq_get, fset, fset2, freeze_msgs, msg_in, tlc_key
from .raft import (RaftSpec, FOLLOWER, CANDIDATE, LEADER, RVREQ, RVRESP, AEREQ,
                   AERESP, EQUAL, LEQ)


class _SendOnceOnly:
    """Send/SendMultiple/Reply of FlexibleRaft.tla:127-151 and RaftFsync.tla:132-152:
    every send is once-only and Reply needs a response not yet in DOMAIN."""

    def Send(self, msgs, m):
        return self._SendOnce(msgs, m)

    def SendMultipleOnce(self, msgs, ms):  # SendMultiple (FlexibleRaft.tla:131-133)
        return RaftSpec.SendMultipleOnce(msgs, ms)

    def Reply(self, msgs, response, request):
        d = dict(msgs)
        if not d[request] > 0:
            return None
        if response in d:
            return None
        d[request] -= 1
        d[response] = 1
        return freeze_msgs(d)

    def NeedsTruncation(self, s, m, i, index):
        # FlexibleRaft.tla:413-416 / RaftFsync.tla:441-444
        return (m.mentries != () and len(s["log"][i]) >= index and
                seq_get(s["log"][i], index).term != seq_get(m.mentries, 1).term)

    def new_log(self, s, m, i, index):
        # FlexibleRaft.tla:431-435 / RaftFsync.tla:459-463 (IF/ELSE, no empty-AE arm)
        if self.CanAppend(s, m, i):
            return s["log"][i] + (seq_get(m.mentries, 1),)
        if self.NeedsTruncation(s, m, i, index):
            return self.TruncateLog(s, m, i) + (seq_get(m.mentries, 1),)
        return s["log"][i]


class FlexibleRaftSpec(_SendOnceOnly, RaftSpec):
    """MODULE FlexibleRaft (FlexibleRaft.tla): size-threshold quorums, no pendingResponse."""
    module = "FlexibleRaft"
    variables = ("messages", "acked", "electionCtr", "restartCtr", "currentTerm",
                 "state", "votedFor", "log", "commitIndex", "votesGranted",
                 "nextIndex", "matchIndex")

    def setup(self, consts):
        self.ElectionQuorumSize = int(consts["ElectionQuorumSize"])
        self.ReplicationQuorumSize = int(consts["ReplicationQuorumSize"])

    def init_states(self):
        for s in RaftSpec.init_states(self):
            del s["pendingResponse"]
            yield s

    def Restart(self, s, i):
        # FlexibleRaft.tla:200-208
        if not self._guard("Restart", s, (i,), lambda: s["restartCtr"] < self.MaxRestarts):
            return
        N = self.N
        t = dict(s)
        t["state"] = fset(s["state"], i, FOLLOWER)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset())
        t["nextIndex"] = fset(s["nextIndex"], i, tuple(1 for _ in range(N)))
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(0 for _ in range(N)))
        t["commitIndex"] = fset(s["commitIndex"], i, 0)
        t["restartCtr"] = s["restartCtr"] + 1
        yield t

    def AppendEntries(self, s, i, j):
        # FlexibleRaft.tla:236-256 (no pendingResponse gate; once-only Send)
        if i == j or s["state"][i] != LEADER:
            return
        log_i = s["log"][i]
        nxt = s["nextIndex"][i][j]
        prevLogIndex = nxt - 1
        prevLogTerm = seq_get(log_i, prevLogIndex).term if prevLogIndex > 0 else 0
        lastEntry = min(len(log_i), nxt)
        entries = tuple(seq_get(log_i, k) for k in range(nxt, lastEntry + 1))
        if not self.ae_gate(s, i, lastEntry):
            return
        m = Rec(mtype=AEREQ, mterm=s["currentTerm"][i], mprevLogIndex=prevLogIndex,
                mprevLogTerm=prevLogTerm, mentries=entries,
                mcommitIndex=min(s["commitIndex"][i], lastEntry), msource=i, mdest=j)
        msgs = self.Send(s["messages"], m)
        if msgs is None:
            return
        t = dict(s)
        t["messages"] = msgs
        yield t

    def ae_gate(self, s, i, lastEntry):
        return True

    def BecomeLeader(self, s, i):
        # FlexibleRaft.tla:260-269: Cardinality(votesGranted[i]) >= ElectionQuorumSize
        if not self._guard("BecomeLeader", s, (i,), lambda: s["state"][i] == CANDIDATE and
                           len(s["votesGranted"][i]) >= self.ElectionQuorumSize):
            return
        N = self.N
        t = dict(s)
        t["state"] = fset(s["state"], i, LEADER)
        t["nextIndex"] = fset(s["nextIndex"], i, tuple(len(s["log"][i]) + 1 for _ in range(N)))
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(0 for _ in range(N)))
        yield t

    def agree_ok(self, s, i, index):
        # FlexibleRaft.tla:296: Cardinality(Agree(index)) >= ReplicationQuorumSize
        return len(self.agree_set(s, i, index)) >= self.ReplicationQuorumSize

    def after_aeresp(self, s, t, i, j):
        pass  # no pendingResponse (FlexibleRaft.tla:455-469)


class RaftFsyncSpec(_SendOnceOnly, RaftSpec):
    """MODULE RaftFsync (RaftFsync.tla): fsyncIndex + three fsync policy flags."""
    module = "RaftFsync"
    variables = ("messages", "acked", "electionCtr", "restartCtr", "currentTerm",
                 "state", "votedFor", "log", "commitIndex", "fsyncIndex",
                 "votesGranted", "nextIndex", "matchIndex")

    def setup(self, consts):
        self.LeaderFsyncBeforeAppendEntries = bool(consts["LeaderFsyncBeforeAppendEntries"])
        self.LeaderFsyncBeforeIncludeInQuorum = bool(consts["LeaderFsyncBeforeIncludeInQuorum"])
        self.FollowerFsyncBeforeReply = bool(consts["FollowerFsyncBeforeReply"])

    def init_states(self):
        for s in RaftSpec.init_states(self):
            del s["pendingResponse"]
            s["fsyncIndex"] = tuple(0 for _ in range(self.N))  # RaftFsync.tla:184
            yield s

    def Restart(self, s, i):
        # RaftFsync.tla:203-218
        if not self._guard("Restart", s, (i,), lambda: s["restartCtr"] < self.MaxRestarts):
            return
        N = self.N
        t = dict(s)
        t["state"] = fset(s["state"], i, FOLLOWER)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset())
        t["nextIndex"] = fset(s["nextIndex"], i, tuple(1 for _ in range(N)))
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(0 for _ in range(N)))
        t["commitIndex"] = fset(s["commitIndex"], i, 0)
        t["restartCtr"] = s["restartCtr"] + 1
        lg, f = s["log"][i], s["fsyncIndex"][i]
        if f == 0:
            nl = ()
        elif len(lg) > 0 and len(lg) > f:
            nl = tuple(seq_get(lg, k) for k in range(1, f + 1))  # SubSeq(@, 1, fsyncIndex[i])
        else:
            nl = lg
        t["log"] = fset(s["log"], i, nl)
        yield t

    def Timeout(self, s, i):
        # RaftFsync.tla:222-230
        if not self._guard("Timeout", s, (i,), lambda: s["electionCtr"] < self.MaxElections and
                           s["state"][i] in (FOLLOWER, CANDIDATE)):
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, CANDIDATE)
        t["currentTerm"] = fset(s["currentTerm"], i, s["currentTerm"][i] + 1)
        t["votedFor"] = fset(s["votedFor"], i, i)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset([i]))
        t["electionCtr"] = s["electionCtr"] + 1
        yield t

    def RequestVoteIJ(self, s, i, j):
        # RaftFsync.tla:234-243
        if not self._guard("RequestVote", s, (i, j), lambda: s["state"][i] == CANDIDATE and i != j):
            return
        m = Rec(mtype=RVREQ, mterm=s["currentTerm"][i], mlastLogTerm=self.LastTerm(s["log"][i]),
                mlastLogIndex=len(s["log"][i]), msource=i, mdest=j)
        msgs = self.Send(s["messages"], m)
        if msgs is None:
            return
        t = dict(s)
        t["messages"] = msgs
        yield t

    AppendEntries = FlexibleRaftSpec.AppendEntries

    def ae_gate(self, s, i, lastEntry):
        # RaftFsync.tla:261-263
        if self.LeaderFsyncBeforeAppendEntries:
            return s["fsyncIndex"][i] >= lastEntry
        return True

    def BecomeLeader(self, s, i):
        # RaftFsync.tla:276-285
        if not self._guard("BecomeLeader", s, (i,), lambda: s["state"][i] == CANDIDATE and
                           self.IsQuorum(s["votesGranted"][i])):
            return
        N = self.N
        t = dict(s)
        t["state"] = fset(s["state"], i, LEADER)
        t["nextIndex"] = fset(s["nextIndex"], i, tuple(len(s["log"][i]) + 1 for _ in range(N)))
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(0 for _ in range(N)))
        yield t

    def agree_set(self, s, i, index):
        # RaftFsync.tla:313-315
        ks = frozenset(k for k in self.Server if s["matchIndex"][i][k] >= index)
        if self.LeaderFsyncBeforeIncludeInQuorum and index > s["fsyncIndex"][i]:
            return ks
        return frozenset([i]) | ks

    def AdvanceFsyncIndex(self, s, i):
        # RaftFsync.tla:339-343
        if not s["fsyncIndex"][i] < len(s["log"][i]):
            return
        t = dict(s)
        t["fsyncIndex"] = fset(s["fsyncIndex"], i, s["fsyncIndex"][i] + 1)
        yield t

    def after_accept(self, s, t, i, nl):
        # RaftFsync.tla:468-470
        if self.FollowerFsyncBeforeReply:
            t["fsyncIndex"] = fset(s["fsyncIndex"], i, len(nl))

    def after_aeresp(self, s, t, i, j):
        pass

    def default_actions(self):
        """Next (RaftFsync.tla:522-536) split into TLC actions, in TLC order."""
        A = []
        n, vn = self.server_names, self.value_names
        for i in self.Server:
            A.append(("Restart(%s)" % n[i], lambda s, i=i: self.Restart(s, i)))
        for i in self.Server:
            A.append(("Timeout(%s)" % n[i], lambda s, i=i: self.Timeout(s, i)))
        for i, j in self.pairs():
            A.append(("RequestVote(%s,%s)" % (n[i], n[j]),
                      lambda s, i=i, j=j: self.RequestVoteIJ(s, i, j)))
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
        for i in self.Server:
            A.append(("AdvanceFsyncIndex(%s)" % n[i], lambda s, i=i: self.AdvanceFsyncIndex(s, i)))
        A.append(("UpdateTerm", self.UpdateTerm))
        A.append(("HandleRequestVoteRequest", self.HandleRequestVoteRequest))
        A.append(("HandleRequestVoteResponse", self.HandleRequestVoteResponse))
        A.append(("RejectAppendEntriesRequest", self.RejectAppendEntriesRequest))
        A.append(("AcceptAppendEntriesRequest", self.AcceptAppendEntriesRequest))
        A.append(("HandleAppendEntriesResponse", self.HandleAppendEntriesResponse))
        return A


# ---------------------------------------------------------------- PullRaft
LNREQ, PEREQ, PERESP = "LeaderNotifyRequest", "PullEntriesRequest", "PullEntriesResponse"


class PullRaftSpec(RaftSpec):
    """MODULE PullRaft (PullRaft.tla): followers pull entries from the leader."""
    module = "PullRaft"
    variables = ("messages", "acked", "electionCtr", "restartCtr", "currentTerm",
                 "state", "leader", "log", "commitIndex", "votesGranted", "matchIndex")
    # view == <<messages, serverVars, candidateVars, leaderVars, logVars, acked>> (PullRaft.tla:123)
    hidden_vars = ("electionCtr", "restartCtr")

    def init_states(self):
        # PullRaft.tla:231-250
        N = self.N
        yield dict(
            messages=(),
            acked=tuple(NIL for _ in self.Value),
            electionCtr=0, restartCtr=0,
            currentTerm=tuple(1 for _ in range(N)),
            state=tuple(FOLLOWER for _ in range(N)),
            leader=tuple(NIL for _ in range(N)),
            log=tuple(() for _ in range(N)),
            commitIndex=tuple(0 for _ in range(N)),
            votesGranted=tuple(frozenset() for _ in range(N)),
            matchIndex=tuple(tuple(0 for _ in range(N)) for _ in range(N)),
        )

    def Send(self, msgs, m):
        # PullRaft.tla:137-139
        return self._SendOnce(msgs, m)

    def Reply(self, msgs, response, request):
        # PullRaft.tla:158-161
        d = dict(msgs)
        if not d[request] > 0:
            return None
        if response in d:
            return None
        d[request] -= 1
        d[response] = 1
        return freeze_msgs(d)

    # PullRaft.tla:180-182 NeedsTruncation is defined but never used.
    def PTruncateLog(self, s, i, m):
        # PullRaft.tla:185-188
        idx = m.mlastCommonEntry.index
        if idx == 0:
            return ()
        return tuple(seq_get(s["log"][i], k) for k in range(1, idx + 1))

    def ValidPullPosition(self, s, i, m):
        # PullRaft.tla:192-196
        if m.mlastLogIndex == 0:
            return True
        return (m.mlastLogIndex > 0 and m.mlastLogIndex <= len(s["log"][i]) and
                m.mlastLogTerm == seq_get(s["log"][i], m.mlastLogIndex).term)

    @staticmethod
    def CompareEntries(index1, term1, index2, term2):
        # PullRaft.tla:203-207
        if term1 > term2:
            return 1
        if term1 == term2 and index1 > index2:
            return 1
        if term1 == term2 and index1 == index2:
            return 0
        return -1

    def LastCommonEntry(self, s, i, lastIndex, lastTerm):
        # PullRaft.tla:211-226
        lg = s["log"][i]
        if lg == ():
            return Rec(index=0, term=0)
        ok = [idx for idx in range(1, len(lg) + 1)
              if self.CompareEntries(idx, seq_get(lg, idx).term, lastIndex, lastTerm) <= 0]
        if not ok:
            return Rec(index=0, term=0)
        index = max(ok)  # the unique CHOOSE witness: no larger qualifying index2
        return Rec(index=index, term=seq_get(lg, index).term)

    def Restart(self, s, i):
        # PullRaft.tla:258-265
        if not self._guard("Restart", s, (i,), lambda: s["restartCtr"] < self.MaxRestarts):
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, FOLLOWER)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset())
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(0 for _ in range(self.N)))
        t["commitIndex"] = fset(s["commitIndex"], i, 0)
        t["restartCtr"] = s["restartCtr"] + 1
        yield t

    def UpdateTerm(self, s):
        # PullRaft.tla:269-276
        for m, _ in s["messages"]:
            d = m.mdest
            if m.mterm > s["currentTerm"][d]:
                t = dict(s)
                t["currentTerm"] = fset(s["currentTerm"], d, m.mterm)
                t["state"] = fset(s["state"], d, FOLLOWER)
                t["leader"] = fset(s["leader"], d, NIL)
                yield t

    def RequestVote(self, s, i):
        # PullRaft.tla:283-298
        if not self._guard("RequestVote", s, (i,), lambda: s["electionCtr"] < self.MaxElections and
                           s["state"][i] in (FOLLOWER, CANDIDATE)):
            return
        term = s["currentTerm"][i] + 1
        ms = [Rec(mtype=RVREQ, mterm=term, mlastLogTerm=self.LastTerm(s["log"][i]),
                  mlastLogIndex=len(s["log"][i]), msource=i, mdest=j)
              for j in self.Server if j != i]
        msgs = RaftSpec.SendMultipleOnce(s["messages"], ms)
        if msgs is None:
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, CANDIDATE)
        t["currentTerm"] = fset(s["currentTerm"], i, term)
        t["leader"] = fset(s["leader"], i, i)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset([i]))
        t["electionCtr"] = s["electionCtr"] + 1
        t["messages"] = msgs
        yield t

    def HandleRequestVoteRequest(self, s):
        # PullRaft.tla:306-330
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, RVREQ, LEQ):
                continue
            i, j = m.mdest, m.msource
            lt = self.LastTerm(s["log"][i])
            logOk = (m.mlastLogTerm > lt or
                     (m.mlastLogTerm == lt and m.mlastLogIndex >= len(s["log"][i])))
            grant = (m.mterm == s["currentTerm"][i] and logOk and s["leader"][i] in (NIL, j))
            if not m.mterm <= s["currentTerm"][i]:
                continue
            resp = Rec(mtype=RVRESP, mterm=s["currentTerm"][i], mvoteGranted=grant,
                       msource=i, mdest=j)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t = dict(s)
            if grant:
                t["leader"] = fset(s["leader"], i, j)
            t["messages"] = msgs
            yield t

    # HandleRequestVoteResponse: PullRaft.tla:335-350 is textually Raft's.

    def BecomeLeader(self, s, i):
        # PullRaft.tla:354-366
        if not self._guard("BecomeLeader", s, (i,), lambda: s["state"][i] == CANDIDATE and
                           self.IsQuorum(s["votesGranted"][i])):
            return
        ms = [Rec(mtype=LNREQ, mterm=s["currentTerm"][i], msource=i, mdest=j)
              for j in self.Server if j not in s["votesGranted"][i]]
        msgs = RaftSpec.SendMultipleOnce(s["messages"], ms)
        if msgs is None:
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, LEADER)
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(0 for _ in range(self.N)))
        t["messages"] = msgs
        yield t

    # ClientRequest: PullRaft.tla:370-379 is textually Raft's.

    def LearnOfLeader(self, s):
        # PullRaft.tla:383-391
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, LNREQ, EQUAL):
                continue
            i, j = m.mdest, m.msource
            msgs = self.Discard(s["messages"], m)
            if msgs is None:
                continue
            t = dict(s)
            t["leader"] = fset(s["leader"], i, j)
            t["messages"] = msgs
            yield t

    def SendPullEntriesRequest(self, s, i, j):
        # PullRaft.tla:396-411
        if i == j or s["state"][i] != FOLLOWER or s["leader"][i] != j:
            return
        lastLogIndex = len(s["log"][i])
        lastLogTerm = seq_get(s["log"][i], lastLogIndex).term if lastLogIndex > 0 else 0
        m = Rec(mtype=PEREQ, mterm=s["currentTerm"][i], mlastLogIndex=lastLogIndex,
                mlastLogTerm=lastLogTerm, msource=i, mdest=j)
        msgs = self.Send(s["messages"], m)
        if msgs is None:
            return
        t = dict(s)
        t["messages"] = msgs
        yield t

    def RejectPullEntriesRequest(self, s):
        # PullRaft.tla:418-436
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, PEREQ, EQUAL):
                continue
            i, j = m.mdest, m.msource
            if s["state"][i] != LEADER:
                continue
            if self.ValidPullPosition(s, i, m):
                continue
            resp = Rec(mtype=PERESP, mterm=s["currentTerm"][i], msuccess=False,
                       mlastCommonEntry=self.LastCommonEntry(s, i, m.mlastLogIndex, m.mlastLogTerm),
                       msource=i, mdest=j)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t = dict(s)
            t["messages"] = msgs
            yield t

    def NewCommitIndex(self, s, i, iMatchIndex):
        # PullRaft.tla:446-458
        lg = s["log"][i]

        def agree(index):
            return frozenset([i]) | frozenset(k for k in self.Server if iMatchIndex[k] >= index)

        agreeIndexes = [index for index in range(1, len(lg) + 1) if self.IsQuorum(agree(index))]
        if agreeIndexes and seq_get(lg, max(agreeIndexes)).term == s["currentTerm"][i]:
            return max(agreeIndexes)
        return s["commitIndex"][i]

    def AcceptPullEntriesRequest(self, s):
        # PullRaft.tla:460-488
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, PEREQ, EQUAL):
                continue
            i, j = m.mdest, m.msource
            index = m.mlastLogIndex + 1
            if s["state"][i] != LEADER:
                continue
            if not self.ValidPullPosition(s, i, m):
                continue
            if not index <= len(s["log"][i]):
                continue
            newMatchIndex = fset(s["matchIndex"][i], j, m.mlastLogIndex)
            newCommitIndex = self.NewCommitIndex(s, i, newMatchIndex)
            lg = s["log"][i]
            committed = {seq_get(lg, ind).value
                         for ind in range(s["commitIndex"][i] + 1, newCommitIndex + 1)}
            resp = Rec(mtype=PERESP, mterm=s["currentTerm"][i], msuccess=True,
                       mentries=(seq_get(lg, index),), mcommitIndex=min(newCommitIndex, index),
                       msource=i, mdest=j)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t = dict(s)
            t["matchIndex"] = fset(s["matchIndex"], i, newMatchIndex)
            t["commitIndex"] = fset(s["commitIndex"], i, newCommitIndex)
            t["acked"] = tuple((v in committed) if s["acked"][v] is False else s["acked"][v]
                               for v in self.Value)
            t["messages"] = msgs
            yield t

    def HandleSuccessPullEntriesResponse(self, s):
        # PullRaft.tla:493-503 (appends without a position check; preserved)
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, PERESP, EQUAL):
                continue
            i = m.mdest
            if not m.msuccess:
                continue
            msgs = self.Discard(s["messages"], m)
            if msgs is None:
                continue
            t = dict(s)
            t["commitIndex"] = fset(s["commitIndex"], i, m.mcommitIndex)
            t["log"] = fset(s["log"], i, s["log"][i] + (seq_get(m.mentries, 1),))
            t["messages"] = msgs
            yield t

    def HandleFailPullEntriesResponse(self, s):
        # PullRaft.tla:510-520
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, PERESP, EQUAL):
                continue
            i = m.mdest
            if m.msuccess:
                continue
            nl = self.PTruncateLog(s, i, m)
            msgs = self.Discard(s["messages"], m)
            if msgs is None:
                continue
            t = dict(s)
            t["log"] = fset(s["log"], i, nl)
            t["messages"] = msgs
            yield t

    def default_actions(self):
        """Next (PullRaft.tla:542-558) split into TLC actions, in TLC order."""
        A = []
        n, vn = self.server_names, self.value_names
        for i in self.Server:
            A.append(("Restart(%s)" % n[i], lambda s, i=i: self.Restart(s, i)))
        A.append(("UpdateTerm", self.UpdateTerm))
        for i in self.Server:
            A.append(("RequestVote(%s)" % n[i], lambda s, i=i: self.RequestVote(s, i)))
        A.append(("HandleRequestVoteRequest", self.HandleRequestVoteRequest))
        A.append(("HandleRequestVoteResponse", self.HandleRequestVoteResponse))
        for i in self.Server:
            A.append(("BecomeLeader(%s)" % n[i], lambda s, i=i: self.BecomeLeader(s, i)))
        for v in self.Value:
            for i in self.Server:
                A.append(("ClientRequest(%s,%s)" % (n[i], vn[v]),
                          lambda s, i=i, v=v: self.ClientRequest(s, i, v)))
        A.append(("RejectPullEntriesRequest", self.RejectPullEntriesRequest))
        A.append(("AcceptPullEntriesRequest", self.AcceptPullEntriesRequest))
        A.append(("LearnOfLeader", self.LearnOfLeader))
        for i, j in self.pairs():
            A.append(("SendPullEntriesRequest(%s,%s)" % (n[i], n[j]),
                      lambda s, i=i, j=j: self.SendPullEntriesRequest(s, i, j)))
        A.append(("HandleSuccessPullEntriesResponse", self.HandleSuccessPullEntriesResponse))
        A.append(("HandleFailPullEntriesResponse", self.HandleFailPullEntriesResponse))
        return A

    def permute_value(self, var, val, p):
        if var == "messages":
            out = []
            for m, c in val:
                out.append((m.replace(msource=p[m.msource], mdest=p[m.mdest]), c))
            out.sort()
            return tuple(out)
        if var == "acked":
            return val
        return RaftSpec.permute_value(self, var, val, p)


# -------------------------------------------------------- PullRaftVariant2
class PullRaftVariant2Spec(PullRaftSpec):
    """MODULE PullRaftVariant2 (pull-raft/PullRaftVariant2.tla): PullRaft, but a
    follower pulls only after a LeaderNotifyRequest names the leader; votedFor
    is a variable again, candidates record each voter's last log entry
    (votesLastEntry) and the leader's notification carries the last common
    entry, which the follower truncates to (:12-26 of the notes)."""
    module = "PullRaftVariant2"
    # declaration order of VARIABLES (PullRaftVariant2.tla:56-106)
    variables = ("messages", "acked", "electionCtr", "restartCtr", "currentTerm",
                 "state", "leader", "votedFor", "log", "commitIndex", "votesGranted",
                 "votesLastEntry", "matchIndex")
    # view == <<messages, serverVars, candidateVars, leaderVars, logVars>> (:114): acked is hidden
    hidden_vars = ("acked", "electionCtr", "restartCtr")

    def init_states(self):
        # PullRaftVariant2.tla:222-243
        N = self.N
        for s in PullRaftSpec.init_states(self):
            s["votedFor"] = tuple(NIL for _ in range(N))
            s["votesLastEntry"] = tuple(tuple(NIL for _ in range(N)) for _ in range(N))
            yield s

    def Restart(self, s, i):
        # PullRaftVariant2.tla:251-260
        if not self._guard("Restart", s, (i,), lambda: s["restartCtr"] < self.MaxRestarts):
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, FOLLOWER)
        t["leader"] = fset(s["leader"], i, NIL)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset())
        t["votesLastEntry"] = fset(s["votesLastEntry"], i, tuple(NIL for _ in range(self.N)))
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(0 for _ in range(self.N)))
        t["commitIndex"] = fset(s["commitIndex"], i, 0)
        t["restartCtr"] = s["restartCtr"] + 1
        yield t

    def UpdateTerm(self, s):
        # PullRaftVariant2.tla:264-272
        for m, _ in s["messages"]:
            d = m.mdest
            if m.mterm > s["currentTerm"][d]:
                t = dict(s)
                t["currentTerm"] = fset(s["currentTerm"], d, m.mterm)
                t["state"] = fset(s["state"], d, FOLLOWER)
                t["votedFor"] = fset(s["votedFor"], d, NIL)
                t["leader"] = fset(s["leader"], d, NIL)
                yield t

    def RequestVote(self, s, i):
        # PullRaftVariant2.tla:279-295
        if not self._guard("RequestVote", s, (i,), lambda: s["electionCtr"] < self.MaxElections and
                           s["state"][i] in (FOLLOWER, CANDIDATE)):
            return
        term = s["currentTerm"][i] + 1
        ms = [Rec(mtype=RVREQ, mterm=term, mlastLogTerm=self.LastTerm(s["log"][i]),
                  mlastLogIndex=len(s["log"][i]), msource=i, mdest=j)
              for j in self.Server if j != i]
        msgs = RaftSpec.SendMultipleOnce(s["messages"], ms)
        if msgs is None:
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, CANDIDATE)
        t["currentTerm"] = fset(s["currentTerm"], i, term)
        t["votedFor"] = fset(s["votedFor"], i, i)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset([i]))
        t["leader"] = fset(s["leader"], i, NIL)
        t["electionCtr"] = s["electionCtr"] + 1
        t["messages"] = msgs
        yield t

    def HandleRequestVoteRequest(self, s):
        # PullRaftVariant2.tla:303-326: grant on votedFor; the response carries the voter's last entry
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, RVREQ, LEQ):
                continue
            i, j = m.mdest, m.msource
            lt = self.LastTerm(s["log"][i])
            logOk = (m.mlastLogTerm > lt or
                     (m.mlastLogTerm == lt and m.mlastLogIndex >= len(s["log"][i])))
            grant = (m.mterm == s["currentTerm"][i] and logOk and s["votedFor"][i] in (NIL, j))
            if not m.mterm <= s["currentTerm"][i]:
                continue
            resp = Rec(mtype=RVRESP, mterm=s["currentTerm"][i], mvoteGranted=grant,
                       mlastLogIndex=len(s["log"][i]), mlastLogTerm=lt, msource=i, mdest=j)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t = dict(s)
            if grant:
                t["votedFor"] = fset(s["votedFor"], i, j)
            t["messages"] = msgs
            yield t

    def HandleRequestVoteResponse(self, s):
        # PullRaftVariant2.tla:331-349
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
                t["votesLastEntry"] = fset2(s["votesLastEntry"], i, j,
                                            Rec(index=m.mlastLogIndex, term=m.mlastLogTerm))
            t["messages"] = msgs
            yield t

    def BecomeLeader(self, s, i):
        # PullRaftVariant2.tla:361-379: notify every other server, with the last
        # common entry for the voters whose last entry is known
        if not self._guard("BecomeLeader", s, (i,), lambda: s["state"][i] == CANDIDATE and
                           self.IsQuorum(s["votesGranted"][i])):
            return
        ms = []
        for j in self.Server:
            if j == i:
                continue
            vle = s["votesLastEntry"][i][j]
            lce = NIL if vle == NIL else self.LastCommonEntry(s, i, vle.index, vle.term)
            ms.append(Rec(mtype=LNREQ, mterm=s["currentTerm"][i], mlastCommonEntry=lce,
                          msource=i, mdest=j))
        msgs = RaftSpec.SendMultipleOnce(s["messages"], ms)
        if msgs is None:
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, LEADER)
        t["leader"] = fset(s["leader"], i, i)
        t["matchIndex"] = fset(s["matchIndex"], i, tuple(0 for _ in range(self.N)))
        t["messages"] = msgs
        yield t

    def NeedsTruncation(self, s, i, m):
        # PullRaftVariant2.tla:171-173
        return m.mlastCommonEntry != NIL and len(s["log"][i]) >= m.mlastCommonEntry.index

    def LearnOfLeader(self, s):
        # PullRaftVariant2.tla:398-410 (the LET's `index == m.mlastLogIndex` is never used)
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, LNREQ, EQUAL):
                continue
            i, j = m.mdest, m.msource
            msgs = self.Discard(s["messages"], m)
            if msgs is None:
                continue
            t = dict(s)
            if self.NeedsTruncation(s, i, m):
                t["log"] = fset(s["log"], i, self.PTruncateLog(s, i, m))
            t["leader"] = fset(s["leader"], i, j)
            t["messages"] = msgs
            yield t

    def default_actions(self):
        """Next (PullRaftVariant2.tla:560-576): PullRaft's disjuncts in the same order."""
        return PullRaftSpec.default_actions(self)

    def permute_value(self, var, val, p):
        # canonical forms only need an injective, totally ordered encoding:
        # Nil and records are mapped to comparable keys
        N = self.N
        inv = [0] * N
        for a, b in enumerate(p):
            inv[b] = a
        if var == "messages":
            out = [(tlc_key(m.replace(msource=p[m.msource], mdest=p[m.mdest])), c) for m, c in val]
            out.sort()
            return tuple(out)
        if var == "votesLastEntry":
            def k(x):
                return (0,) if x == NIL else (1, x.index, x.term)
            return tuple(tuple(k(val[inv[a]][inv[b]]) for b in range(N)) for a in range(N))
        return RaftSpec.permute_value(self, var, val, p)
