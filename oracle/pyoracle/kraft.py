"""Literal restatement of /root/reference/specifications/pull-raft/KRaft.tla.

TEST INFRASTRUCTURE ONLY (the checker the HIP path is compared against; the
product path never imports it).  Every operator cites the TLA+ lines it
restates.  Encoding as in raft.py: servers are indices 0..N-1 in model-value
name order, values 0..V-1, the model value Nil is NIL (-1) where a server is
expected (votedFor, leader, mleader), records are `Rec`, sequences tuples.
The other model values (server states, message types, fetch results and
errors) are their names as strings, so TLC's by-name order of model values is
Python's string order; `merror` holds "Nil" (a model value compared with the
error names), `pendingFetch[i]` is NIL or the FetchRequest record.
"""
import itertools

from .tlc import NIL, Rec, seq_get, fset, fset2, freeze_msgs, msg_in, permutations, tlc_key

FOLLOWER, CANDIDATE, LEADER = "Follower", "Candidate", "Leader"
UNATTACHED, VOTED, ILLEGAL = "Unattached", "Voted", "IllegalState"
RVREQ, RVRESP = "RequestVoteRequest", "RequestVoteResponse"
BQREQ, BQRESP = "BeginQuorumRequest", "BeginQuorumResponse"
FREQ, FRESP = "FetchRequest", "FetchResponse"
OK, NOTOK, DIVERGING = "Ok", "NotOk", "Diverging"
FENCED, NOTLEADER, UNKNOWNLEADER = "FencedLeaderEpoch", "NotLeader", "UnknownLeader"
NILE = "Nil"  # the model value Nil where an error is expected (merror)


class KRaftSpec:
    """MODULE KRaft (KRaft.tla:1-959) bound to a cfg (KRaft.cfg:5-50)."""
    module = "KRaft"
    # declaration order of VARIABLES (KRaft.tla:100-144)
    variables = ("messages", "acked", "electionCtr", "restartCtr", "currentEpoch",
                 "state", "votedFor", "leader", "pendingFetch", "log", "highWatermark",
                 "votesGranted", "endOffset")
    # view == <<messages, serverVars, candidateVars, leaderVars, logVars, acked>> (KRaft.tla:154)
    hidden_vars = ("electionCtr", "restartCtr")

    def __init__(self, consts, invariants=("LeaderHasAllAckedValues", "NoLogDivergence",
                                           "NeverTwoLeadersInSameEpoch", "NoIllegalState")):
        self.server_names = sorted(str(x) for x in consts["Server"])
        self.value_names = sorted(str(x) for x in consts["Value"])
        self.N = len(self.server_names)
        self.V = len(self.value_names)
        self.Server = range(self.N)
        self.Value = range(self.V)
        self.MaxElections = int(consts["MaxElections"])
        self.MaxRestarts = int(consts["MaxRestarts"])
        self.perms = permutations(self.N)
        table = {"LeaderHasAllAckedValues": self.LeaderHasAllAckedValues,
                 "NoLogDivergence": self.NoLogDivergence,
                 "NeverTwoLeadersInSameEpoch": self.NeverTwoLeadersInSameEpoch,
                 "NoIllegalState": self.NoIllegalState,
                 "CommittedEntriesReachMajority": self.CommittedEntriesReachMajority}
        self.invariants = [(n, table[n]) for n in invariants]

    # ---------------------------------------------------------------- helpers
    def IsQuorum(self, s):
        # Quorum == {i \in SUBSET(Server) : Cardinality(i) * 2 > Cardinality(Server)}  (:162)
        return len(s) * 2 > self.N

    @staticmethod
    def LastEpoch(xlog):
        # :165
        return 0 if len(xlog) == 0 else seq_get(xlog, len(xlog)).epoch

    @staticmethod
    def _SendNoRestriction(msgs, m):
        # :169-173
        d = dict(msgs)
        d[m] = d.get(m, 0) + 1
        return freeze_msgs(d)

    @staticmethod
    def _SendOnce(msgs, m):
        # :178-180; None = disabled
        if msg_in(msgs, m):
            return None
        d = dict(msgs)
        d[m] = 1
        return freeze_msgs(d)

    def Send(self, msgs, m):
        # :190-194
        if m.mtype in (RVREQ, BQREQ):
            return self._SendOnce(msgs, m)
        return self._SendNoRestriction(msgs, m)

    @staticmethod
    def SendMultipleOnce(msgs, ms):
        # :199-201
        for m in ms:
            if msg_in(msgs, m):
                return None
        d = dict(msgs)
        for m in ms:
            d[m] = 1
        return freeze_msgs(d)

    @staticmethod
    def Discard(msgs, m):
        # :210-213
        d = dict(msgs)
        if m not in d or not d[m] > 0:
            return None
        d[m] -= 1
        return freeze_msgs(d)

    @staticmethod
    def Reply(msgs, response, request):
        # :220-227: a FetchResponse must be new; other responses increment
        d = dict(msgs)
        if not d[request] > 0:
            return None
        if response in d:
            if response.mtype == FRESP:
                return None
            d[request] -= 1
            d[response] += 1
        else:
            d[request] -= 1
            d[response] = 1
        return freeze_msgs(d)

    @staticmethod
    def ReceivableMessage(s, m, count, mtype, equal_epoch):
        # :230-235
        if not count > 0 or m.mtype != mtype:
            return False
        return (not equal_epoch) or m.mepoch == s["currentEpoch"][m.mdest]

    @staticmethod
    def CompareEntries(offset1, epoch1, offset2, epoch2):
        # :247-251
        if epoch1 > epoch2:
            return 1
        if epoch1 == epoch2 and offset1 > offset2:
            return 1
        if epoch1 == epoch2 and offset1 == offset2:
            return 0
        return -1

    def HighestCommonOffset(self, s, i, endOffsetForEpoch, epoch):
        # :255-273 (CASE arms in order; the CHOOSE picks the unique highest offset)
        lg = s["log"][i]
        if lg == ():
            return (0, 0)
        offs = [o for o in range(1, len(lg) + 1)
                if self.CompareEntries(o, lg[o - 1].epoch, endOffsetForEpoch, epoch) <= 0]
        if not offs:
            return (0, 0)
        o = max(offs)
        return (o, lg[o - 1].epoch)

    def TruncateLog(self, s, i, m):
        # :276-282
        o, _ = self.HighestCommonOffset(s, i, m.mdivergingEndOffset, m.mdivergingEpoch)
        return () if o == 0 else tuple(s["log"][i][:o])

    @staticmethod
    def EndOffsetForEpoch(s, i, lastFetchedEpoch):
        # :285-301
        lg = s["log"][i]
        if lg == ():
            return (0, 0)
        offs = [o for o in range(1, len(lg) + 1) if lg[o - 1].epoch <= lastFetchedEpoch]
        if not offs:
            return (0, 0)
        o = max(offs)
        return (o, lg[o - 1].epoch)

    def ValidFetchPosition(self, s, i, m):
        # :305-310
        if m.mfetchOffset == 0 and m.mlastFetchedEpoch == 0:
            return True
        off, ep = self.EndOffsetForEpoch(s, i, m.mlastFetchedEpoch)
        return m.mfetchOffset <= off and m.mlastFetchedEpoch == ep

    @staticmethod
    def HasConsistentLeader(s, i, leaderId, epoch):
        # :316-327
        if leaderId == i:
            return s["state"][i] == LEADER
        return (epoch != s["currentEpoch"][i] or leaderId == NIL or s["leader"][i] == NIL or
                s["leader"][i] == leaderId)

    # transition records as (state, epoch, leader) triples (:329-349)
    ILLEGAL_T = (ILLEGAL, 0, NIL)

    @staticmethod
    def NoTransition(s, i):
        return (s["state"][i], s["currentEpoch"][i], s["leader"][i])

    def TransitionToVoted(self, s, i, epoch, state0):
        # :335-339
        if state0[1] == epoch and state0[0] != UNATTACHED:
            return self.ILLEGAL_T
        return (VOTED, epoch, NIL)

    @staticmethod
    def TransitionToUnattached(epoch):
        # :341-342
        return (UNATTACHED, epoch, NIL)

    def TransitionToFollower(self, s, i, leaderId, epoch):
        # :344-349
        if s["currentEpoch"][i] == epoch and s["state"][i] in (FOLLOWER, LEADER):
            return self.ILLEGAL_T
        return (FOLLOWER, epoch, leaderId)

    def MaybeTransition(self, s, i, leaderId, epoch):
        # :351-367
        if not self.HasConsistentLeader(s, i, leaderId, epoch):
            return self.ILLEGAL_T
        if epoch > s["currentEpoch"][i]:
            if leaderId == NIL:
                return self.TransitionToUnattached(epoch)
            return self.TransitionToFollower(s, i, leaderId, epoch)
        if leaderId != NIL and s["leader"][i] == NIL:
            return self.TransitionToFollower(s, i, leaderId, epoch)
        return self.NoTransition(s, i)

    def MaybeHandleCommonResponse(self, s, i, leaderId, epoch, errors):
        # :369-392 -> ((state, epoch, leader), handled)
        cur = s["currentEpoch"][i]
        if epoch < cur:
            return (s["state"][i], cur, s["leader"][i]), True
        if epoch > cur or errors != NILE:
            return self.MaybeTransition(s, i, leaderId, epoch), True
        if epoch == cur and leaderId != NIL and s["leader"][i] == NIL:
            return (FOLLOWER, cur, leaderId), True
        return (s["state"][i], cur, s["leader"][i]), False

    @staticmethod
    def apply_transition(s, t, i, ns):
        t["state"] = fset(s["state"], i, ns[0])
        t["currentEpoch"] = fset(s["currentEpoch"], i, ns[1])
        t["leader"] = fset(s["leader"], i, ns[2])

    # ------------------------------------------------------------------- Init
    def init_states(self):
        # :397-415
        N = self.N
        yield dict(
            messages=(),
            acked=tuple(NIL for _ in self.Value),
            electionCtr=0,
            restartCtr=0,
            currentEpoch=tuple(1 for _ in range(N)),
            state=tuple(UNATTACHED for _ in range(N)),
            votedFor=tuple(NIL for _ in range(N)),
            leader=tuple(NIL for _ in range(N)),
            pendingFetch=tuple(NIL for _ in range(N)),
            log=tuple(() for _ in range(N)),
            highWatermark=tuple(0 for _ in range(N)),
            votesGranted=tuple(frozenset() for _ in range(N)),
            endOffset=tuple(tuple(0 for _ in range(N)) for _ in range(N)),
        )

    # ---------------------------------------------------------------- actions
    def Restart(self, s, i):
        # :423-432
        if not s["restartCtr"] < self.MaxRestarts:
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, FOLLOWER)
        t["leader"] = fset(s["leader"], i, NIL)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset())
        t["endOffset"] = fset(s["endOffset"], i, tuple(0 for _ in range(self.N)))
        t["highWatermark"] = fset(s["highWatermark"], i, 0)
        t["pendingFetch"] = fset(s["pendingFetch"], i, NIL)
        t["restartCtr"] = s["restartCtr"] + 1
        yield t

    def RequestVote(self, s, i):
        # :439-456
        if not s["electionCtr"] < self.MaxElections:
            return
        if s["state"][i] not in (FOLLOWER, CANDIDATE, UNATTACHED):
            return
        epoch = s["currentEpoch"][i] + 1
        ms = [Rec(mtype=RVREQ, mepoch=epoch, mlastLogEpoch=self.LastEpoch(s["log"][i]),
                  mlastLogOffset=len(s["log"][i]), msource=i, mdest=j)
              for j in self.Server if j != i]
        msgs = self.SendMultipleOnce(s["messages"], ms)
        if msgs is None:
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, CANDIDATE)
        t["currentEpoch"] = fset(s["currentEpoch"], i, epoch)
        t["leader"] = fset(s["leader"], i, NIL)
        t["votedFor"] = fset(s["votedFor"], i, i)
        t["votesGranted"] = fset(s["votesGranted"], i, frozenset([i]))
        t["pendingFetch"] = fset(s["pendingFetch"], i, NIL)
        t["electionCtr"] = s["electionCtr"] + 1
        t["messages"] = msgs
        yield t

    def HandleRequestVoteRequest(self, s):
        # :464-513
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, RVREQ, False):
                continue
            i, j = m.mdest, m.msource
            cur = s["currentEpoch"][i]
            error = FENCED if m.mepoch < cur else NILE
            state0 = self.TransitionToUnattached(m.mepoch) if m.mepoch > cur else self.NoTransition(s, i)
            logOk = self.CompareEntries(m.mlastLogOffset, m.mlastLogEpoch, len(s["log"][i]),
                                        self.LastEpoch(s["log"][i])) >= 0
            grant = ((state0[0] == UNATTACHED or (state0[0] == VOTED and s["votedFor"][i] == j)) and logOk)
            final = (self.TransitionToVoted(s, i, m.mepoch, state0)
                     if grant and state0[0] == UNATTACHED else state0)
            t = dict(s)
            if error == NILE:
                self.apply_transition(s, t, i, final)
                if grant:
                    t["votedFor"] = fset(s["votedFor"], i, j)
                if t["state"] != s["state"]:
                    t["pendingFetch"] = fset(s["pendingFetch"], i, NIL)
                resp = Rec(mtype=RVRESP, mepoch=m.mepoch, mleader=final[2], mvoteGranted=grant,
                           merror=NILE, msource=i, mdest=j)
            else:
                resp = Rec(mtype=RVRESP, mepoch=cur, mleader=s["leader"][i], mvoteGranted=False,
                           merror=error, msource=i, mdest=j)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t["messages"] = msgs
            yield t

    def HandleRequestVoteResponse(self, s):
        # :519-541
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, RVRESP, False):
                continue
            i, j = m.mdest, m.msource
            ns, handled = self.MaybeHandleCommonResponse(s, i, m.mleader, m.mepoch, m.merror)
            t = dict(s)
            if handled:
                self.apply_transition(s, t, i, ns)
            else:
                if s["state"][i] != CANDIDATE:
                    continue
                if m.mvoteGranted:
                    t["votesGranted"] = fset(s["votesGranted"], i, s["votesGranted"][i] | {j})
            msgs = self.Discard(s["messages"], m)
            if msgs is None:
                continue
            t["messages"] = msgs
            yield t

    def BecomeLeader(self, s, i):
        # :546-558
        if s["state"][i] != CANDIDATE or not self.IsQuorum(s["votesGranted"][i]):
            return
        ms = [Rec(mtype=BQREQ, mepoch=s["currentEpoch"][i], msource=i, mdest=j)
              for j in self.Server if j != i]
        msgs = self.SendMultipleOnce(s["messages"], ms)
        if msgs is None:
            return
        t = dict(s)
        t["state"] = fset(s["state"], i, LEADER)
        t["leader"] = fset(s["leader"], i, i)
        t["endOffset"] = fset(s["endOffset"], i, tuple(0 for _ in range(self.N)))
        t["messages"] = msgs
        yield t

    def HandleBeginQuorumRequest(self, s):
        # :563-590
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, BQREQ, False):
                continue
            i, j = m.mdest, m.msource
            cur = s["currentEpoch"][i]
            t = dict(s)
            if not m.mepoch < cur:
                ns = self.MaybeTransition(s, i, m.msource, m.mepoch)
                self.apply_transition(s, t, i, ns)
                t["pendingFetch"] = fset(s["pendingFetch"], i, NIL)
                resp = Rec(mtype=BQRESP, mepoch=m.mepoch, msource=i, mdest=j, merror=NILE)
            else:
                resp = Rec(mtype=BQRESP, mepoch=cur, msource=i, mdest=j, merror=FENCED)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t["messages"] = msgs
            yield t

    def ClientRequest(self, s, i, v):
        # :594-603
        if s["state"][i] != LEADER or s["acked"][v] != NIL:
            return
        t = dict(s)
        t["log"] = fset(s["log"], i, s["log"][i] + (Rec(epoch=s["currentEpoch"][i], value=v),))
        t["acked"] = fset(s["acked"], v, False)
        yield t

    def SendFetchRequest(self, s, i, j):
        # :607-624
        if i == j or s["state"][i] != FOLLOWER or s["leader"][i] != j or s["pendingFetch"][i] != NIL:
            return
        lg = s["log"][i]
        fetch = Rec(mtype=FREQ, mepoch=s["currentEpoch"][i], mfetchOffset=len(lg),
                    mlastFetchedEpoch=lg[-1].epoch if lg else 0, msource=i, mdest=j)
        t = dict(s)
        t["pendingFetch"] = fset(s["pendingFetch"], i, fetch)
        t["messages"] = self.Send(s["messages"], fetch)
        yield t

    def RejectFetchRequest(self, s):
        # :631-651
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, FREQ, False):
                continue
            i, j = m.mdest, m.msource
            cur = s["currentEpoch"][i]
            if s["state"][i] != LEADER:
                error = NOTLEADER
            elif m.mepoch < cur:
                error = FENCED
            elif m.mepoch > cur:
                error = UNKNOWNLEADER
            else:
                continue
            resp = Rec(mtype=FRESP, mresult=NOTOK, merror=error, mleader=s["leader"][i], mepoch=cur,
                       mhwm=s["highWatermark"][i], msource=i, mdest=j, correlation=m)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t = dict(s)
            t["messages"] = msgs
            yield t

    def DivergingFetchRequest(self, s):
        # :658-679
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, FREQ, True):
                continue
            i, j = m.mdest, m.msource
            if s["state"][i] != LEADER or self.ValidFetchPosition(s, i, m):
                continue
            off, ep = self.EndOffsetForEpoch(s, i, m.mlastFetchedEpoch)
            resp = Rec(mtype=FRESP, mepoch=s["currentEpoch"][i], mresult=DIVERGING, merror=NILE,
                       mdivergingEpoch=ep, mdivergingEndOffset=off, mleader=s["leader"][i],
                       mhwm=s["highWatermark"][i], msource=i, mdest=j, correlation=m)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t = dict(s)
            t["messages"] = msgs
            yield t

    def NewHighwaterMark(self, s, i, newEndOffset):
        # :689-701
        lg = s["log"][i]
        agree = [o for o in range(1, len(lg) + 1)
                 if self.IsQuorum({i} | {k for k in self.Server if newEndOffset[k] >= o})]
        if agree and seq_get(lg, max(agree)).epoch == s["currentEpoch"][i]:
            return max(agree)
        return s["highWatermark"][i]

    def AcceptFetchRequest(self, s):
        # :703-736
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, FREQ, True):
                continue
            i, j = m.mdest, m.msource
            if s["state"][i] != LEADER or not self.ValidFetchPosition(s, i, m):
                continue
            lg = s["log"][i]
            offset = m.mfetchOffset + 1
            entries = () if offset > len(lg) else (seq_get(lg, offset),)
            newEnd = fset(s["endOffset"][i], j, m.mfetchOffset)
            newHwm = self.NewHighwaterMark(s, i, newEnd)
            committed = {seq_get(lg, k).value for k in range(s["highWatermark"][i] + 1, newHwm + 1)}
            resp = Rec(mtype=FRESP, mepoch=s["currentEpoch"][i], mleader=s["leader"][i], mresult=OK,
                       merror=NILE, mentries=entries, mhwm=min(newHwm, offset), msource=i, mdest=j,
                       correlation=m)
            msgs = self.Reply(s["messages"], resp, m)
            if msgs is None:
                continue
            t = dict(s)
            t["endOffset"] = fset(s["endOffset"], i, newEnd)
            t["highWatermark"] = fset(s["highWatermark"], i, newHwm)
            t["acked"] = tuple((v in committed) if s["acked"][v] is False else s["acked"][v]
                               for v in self.Value)
            t["messages"] = msgs
            yield t

    def _fetch_response(self, s, want_handled, result):
        for m, c in s["messages"]:
            if not self.ReceivableMessage(s, m, c, FRESP, False):
                continue
            i = m.mdest
            ns, handled = self.MaybeHandleCommonResponse(s, i, m.mleader, m.mepoch, m.merror)
            if handled != want_handled or s["pendingFetch"][i] != m.correlation:
                continue
            if result is not None and m.mresult != result:
                continue
            yield m, i, ns

    def HandleSuccessFetchResponse(self, s):
        # :742-757
        for m, i, _ in self._fetch_response(s, False, OK):
            msgs = self.Discard(s["messages"], m)
            if msgs is None:
                continue
            t = dict(s)
            t["highWatermark"] = fset(s["highWatermark"], i, m.mhwm)
            if len(m.mentries) > 0:
                t["log"] = fset(s["log"], i, s["log"][i] + (seq_get(m.mentries, 1),))
            t["pendingFetch"] = fset(s["pendingFetch"], i, NIL)
            t["messages"] = msgs
            yield t

    def HandleDivergingFetchResponse(self, s):
        # :766-780
        for m, i, _ in self._fetch_response(s, False, DIVERGING):
            msgs = self.Discard(s["messages"], m)
            if msgs is None:
                continue
            t = dict(s)
            t["log"] = fset(s["log"], i, self.TruncateLog(s, i, m))
            t["pendingFetch"] = fset(s["pendingFetch"], i, NIL)
            t["messages"] = msgs
            yield t

    def HandleErrorFetchResponse(self, s):
        # :786-801
        for m, i, ns in self._fetch_response(s, True, None):
            msgs = self.Discard(s["messages"], m)
            if msgs is None:
                continue
            t = dict(s)
            self.apply_transition(s, t, i, ns)
            t["pendingFetch"] = fset(s["pendingFetch"], i, NIL)
            t["messages"] = msgs
            yield t

    # ------------------------------------------------------------------- Next
    def pairs(self):
        # \E i, j \in Server : the first bound variable varies fastest (TLC)
        return [(i, j) for j in self.Server for i in self.Server]

    def actions(self):
        """Next (KRaft.tla:823-840) split into TLC actions, in TLC order."""
        A = []
        n, vn = self.server_names, self.value_names
        for i in self.Server:
            A.append(("Restart(%s)" % n[i], lambda s, i=i: self.Restart(s, i)))
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
        A.append(("RejectFetchRequest", self.RejectFetchRequest))
        A.append(("DivergingFetchRequest", self.DivergingFetchRequest))
        A.append(("AcceptFetchRequest", self.AcceptFetchRequest))
        A.append(("HandleBeginQuorumRequest", self.HandleBeginQuorumRequest))
        for i, j in self.pairs():
            A.append(("SendFetchRequest(%s,%s)" % (n[i], n[j]),
                      lambda s, i=i, j=j: self.SendFetchRequest(s, i, j)))
        A.append(("HandleSuccessFetchResponse", self.HandleSuccessFetchResponse))
        A.append(("HandleDivergingFetchResponse", self.HandleDivergingFetchResponse))
        A.append(("HandleErrorFetchResponse", self.HandleErrorFetchResponse))
        return A

    # ------------------------------------------------------------- invariants
    def NoIllegalState(self, s):
        # :887-889
        return not any(st == ILLEGAL for st in s["state"])

    def NoLogDivergence(self, s):
        # :894-907; \A s1, s2 enumerated with s1 fastest
        hw, lg = s["highWatermark"], s["log"]
        for s2 in self.Server:
            for s1 in self.Server:
                if s1 == s2:
                    continue
                c = hw[s1] if hw[s1] < hw[s2] else hw[s2]
                if c > 0:
                    for offset in range(1, c + 1):
                        if seq_get(lg[s1], offset) != seq_get(lg[s2], offset):
                            return False
        return True

    def NeverTwoLeadersInSameEpoch(self, s):
        # :916-921
        ld, ep = s["leader"], s["currentEpoch"]
        for i in self.Server:
            for j in self.Server:
                if ld[i] != NIL and ld[j] != NIL and ld[i] != ld[j] and ep[i] == ep[j]:
                    return False
        return True

    def LeaderHasAllAckedValues(self, s):
        # :925-941
        for v in self.Value:
            if s["acked"][v] is True:
                for i in self.Server:
                    if (s["state"][i] == LEADER and
                            not any(l != i and s["currentEpoch"][l] > s["currentEpoch"][i]
                                    for l in self.Server) and
                            not any(e.value == v for e in s["log"][i])):
                        return False
        return True

    def CommittedEntriesReachMajority(self, s):
        # :946-957 (not enabled by the shipped cfg)
        lead = [i for i in self.Server if s["state"][i] == LEADER and s["highWatermark"][i] > 0]
        if not lead:
            return True
        size = self.N // 2 + 1
        for i in lead:
            h = s["highWatermark"][i]
            for q in itertools.combinations(self.Server, size):
                if i not in q:
                    continue
                if all(len(s["log"][j]) >= h and seq_get(s["log"][j], h) == seq_get(s["log"][i], h)
                       for j in q):
                    return True
        return False

    # ----------------------------------------------------- VIEW and SYMMETRY
    def view_vars(self):
        return [v for v in self.variables if v not in self.hidden_vars]

    def permute_value(self, var, val, p):
        """Apply server permutation p (old index -> new index) to one variable,
        as a totally ordered key (canonical forms need injectivity only)."""
        N = self.N
        inv = [0] * N
        for a, b in enumerate(p):
            inv[b] = a

        def srv(x):
            return x if x == NIL else p[x]

        def prec(r):  # a FetchRequest (pendingFetch, correlation)
            return r.replace(msource=p[r.msource], mdest=p[r.mdest])

        if var == "messages":
            out = []
            for m, c in val:
                kw = dict(msource=p[m.msource], mdest=p[m.mdest])
                if m.mtype == RVRESP or m.mtype == FRESP:
                    kw["mleader"] = srv(m.mleader)
                if m.mtype == FRESP:
                    kw["correlation"] = prec(m.correlation)
                out.append((tlc_key(m.replace(**kw)), c))
            out.sort()
            return tuple(out)
        if var == "pendingFetch":
            return tuple((0,) if val[inv[k]] == NIL else (1, tlc_key(prec(val[inv[k]])))
                         for k in range(N))
        if var in ("votedFor", "leader"):
            return tuple(srv(val[inv[k]]) for k in range(N))
        if var == "votesGranted":
            return tuple(tuple(sorted(p[x] for x in val[inv[k]])) for k in range(N))
        if var == "endOffset":
            return tuple(tuple(val[inv[k]][inv[q]] for q in range(N)) for k in range(N))
        if var in ("currentEpoch", "state", "log", "highWatermark"):
            return tuple(val[inv[k]] for k in range(N))
        return val  # acked

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
