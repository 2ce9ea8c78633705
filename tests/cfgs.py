"""cfg texts for the parity cases (TLC .cfg syntax, same grammar as the reference cfgs)."""

FSYNC_FLAGS = dict(LeaderFsyncBeforeAppendEntries=False, LeaderFsyncBeforeIncludeInQuorum=True,
                   FollowerFsyncBeforeReply=True)


def cfg_text(module, n=3, v=1, E=2, R=0, inv=("LeaderHasAllAckedValues", "NoLogDivergence"),
             symmetry=True, **extra):
    lines = ["CONSTANTS"]
    lines += ["    n%d = n%d" % (i, i) for i in range(1, n + 1)]
    lines += ["    v%d = v%d" % (i, i) for i in range(1, v + 1)]
    lines.append("    Server = {%s}" % ", ".join("n%d" % i for i in range(1, n + 1)))
    lines.append("    Value = {%s}" % ", ".join("v%d" % i for i in range(1, v + 1)))
    for k in ("Follower", "Candidate", "Leader", "Nil", "EqualTerm", "LessOrEqualTerm"):
        lines.append("    %s = %s" % (k, k))
    lines.append("    MaxElections = %d" % E)
    lines.append("    MaxRestarts = %d" % R)
    if module == "RaftFsync":
        for k, val in dict(FSYNC_FLAGS, **extra).items():
            lines.append("    %s = %s" % (k, "TRUE" if val else "FALSE"))
    elif module == "FlexibleRaft":
        lines.append("    ElectionQuorumSize = %d" % extra.get("ElectionQuorumSize", n // 2 + 1))
        lines.append("    ReplicationQuorumSize = %d" % extra.get("ReplicationQuorumSize", n // 2 + 1))
    lines += ["INIT Init", "NEXT Next", "VIEW view"]
    if symmetry:
        lines.append("SYMMETRY symmServers")
    lines.append("INVARIANT")
    lines += list(inv)
    return "\n".join(lines) + "\n"


# (name, module, kwargs): small parity cases (oracle seconds), covering every spec
SMALL = [
    ("raft_n3v1e1", "Raft", dict(n=3, v=1, E=1)),
    ("raft_n2v1e2", "Raft", dict(n=2, v=1, E=2)),
    ("raft_n3v1e1r1", "Raft", dict(n=3, v=1, E=1, R=1)),
    ("raft_n2v2e2", "Raft", dict(n=2, v=2, E=2)),
    ("pull_n3v1e1", "PullRaft", dict(n=3, v=1, E=1)),
    ("pull_n3v2e1", "PullRaft", dict(n=3, v=2, E=1)),
    ("pull_n2v1e2r1", "PullRaft", dict(n=2, v=1, E=2, R=1)),
    ("fsync_n3v1e1", "RaftFsync", dict(n=3, v=1, E=1)),
    ("fsync_n2v1e2r1", "RaftFsync", dict(n=2, v=1, E=2, R=1)),
    ("flex_n3v1e1", "FlexibleRaft", dict(n=3, v=1, E=1, ElectionQuorumSize=2, ReplicationQuorumSize=2)),
    ("flex_n2v1e2", "FlexibleRaft", dict(n=2, v=1, E=2, ElectionQuorumSize=2, ReplicationQuorumSize=1)),
]

# medium cases: C oracle only (too slow for the literal Python oracle)
MEDIUM = [
    ("flex_n4v1e1", "FlexibleRaft", dict(n=4, v=1, E=1, ElectionQuorumSize=3, ReplicationQuorumSize=2)),
    ("pull_n3v1e2r1", "PullRaft", dict(n=3, v=1, E=2, R=1)),
    ("fsync_n3v1e2_unsafe", "RaftFsync", dict(n=3, v=1, E=2, R=1, FollowerFsyncBeforeReply=False)),
    ("raft_n4v1e1", "Raft", dict(n=4, v=1, E=1)),
]

# 5-server cases (the N=5 kernels: 120-permutation symmetry).  Exhaustive runs
# take the C oracle minutes to hours, so these are pinned level by level up to
# the first level at which the oracle has found >= max_distinct states
# (truncated at a level boundary; the GPU runs the same number of levels).
# (name, module, kwargs, C oracle max_distinct, Python oracle max_states)
N5 = [
    ("flex_n5v1e1_eq3rq3", "FlexibleRaft", dict(n=5, v=1, E=1, ElectionQuorumSize=3, ReplicationQuorumSize=3),
     400000, 3000),
    ("flex_n5v1e1_eq3rq4", "FlexibleRaft", dict(n=5, v=1, E=1, ElectionQuorumSize=3, ReplicationQuorumSize=4),
     400000, 3000),
    ("flex_n5v1e1_eq2rq4", "FlexibleRaft", dict(n=5, v=1, E=1, ElectionQuorumSize=2, ReplicationQuorumSize=4),
     400000, 3000),
    # FlexibleRaft.cfg's constants (BASELINE config 3), first levels
    ("flex_n5v2e2_cfg", "FlexibleRaft", dict(n=5, v=2, E=2, ElectionQuorumSize=3, ReplicationQuorumSize=4),
     1000000, 3000),
    ("raft_n5v1e1", "Raft", dict(n=5, v=1, E=1), 400000, 3000),
    ("pull_n5v1e1", "PullRaft", dict(n=5, v=1, E=1), 400000, 3000),
    ("fsync_n5v1e1r1", "RaftFsync", dict(n=5, v=1, E=1, R=1), 400000, 3000),
]
# 5 servers, election quorums of 2 (two disjoint quorums elect two leaders of one term)
N5_UNSAFE = [
    ("flex_n5v1e2_eq2rq2_unsafe", "FlexibleRaft", dict(n=5, v=1, E=2, ElectionQuorumSize=2, ReplicationQuorumSize=2)),
]

# known-unsafe configs (violations reachable): Flexible
# with quorums of 1 (FlexibleRaft.tla:16-24 lists the valid pairs; these are not)
UNSAFE = [
    ("flex_n3v1e2_q1", "FlexibleRaft", dict(n=3, v=1, E=2, ElectionQuorumSize=1, ReplicationQuorumSize=1)),
    ("flex_n3v2e2_eq1", "FlexibleRaft", dict(n=3, v=2, E=2, ElectionQuorumSize=1, ReplicationQuorumSize=2)),
]

# TLC-order first-wins sensitivity (SURVEY.md §7 hard part 1): configs with
# same-level hidden-variable collisions (VIEW drops acked/electionCtr/restartCtr
# which gate actions).  For the first three, letting the LAST successor in TLC
# order win (the C oracle's --reverse-order probe) changes the counts, so only
# the first-in-TLC-order winner reproduces them.
ORDER = [
    ("fsync_n2v1e3_order", "RaftFsync", dict(n=2, v=1, E=3, R=0)),
    ("raft_n2v2e2r2_order", "Raft", dict(n=2, v=2, E=2, R=2)),
    ("fsync_n2v1e3r1_order", "RaftFsync", dict(n=2, v=1, E=3, R=1)),
    ("fsync_n2v2e1r1_hidden", "RaftFsync", dict(n=2, v=2, E=1, R=1)),
    ("fsync_n2v2e2r1_hidden", "RaftFsync", dict(n=2, v=2, E=2, R=1)),
]

# PullRaftVariant2 (pull-raft/PullRaftVariant2.tla): followers
# pull only after LeaderNotify, which carries the last common entry.
# (name, kwargs): both oracles (small) / C oracle (medium) / 5-server prefix
VARIANT2_SMALL = [
    ("pull2_n2v1e1", dict(n=2, v=1, E=1)),
    ("pull2_n3v1e1", dict(n=3, v=1, E=1)),
    ("pull2_n2v1e2r1", dict(n=2, v=1, E=2, R=1)),
    ("pull2_n3v2e1", dict(n=3, v=2, E=1)),
    ("pull2_n4v1e1", dict(n=4, v=1, E=1)),
    # two elections: truncation on LeaderNotify and HandleFailPullEntriesResponse
    ("pull2_n3v1e2", dict(n=3, v=1, E=2)),
]
VARIANT2_MEDIUM = [
    ("pull2_n3v1e2r1", dict(n=3, v=1, E=2, R=1)),
]
VARIANT2_N5 = [
    ("pull2_n5v1e1", dict(n=5, v=1, E=1), 400000, 3000),
]


def kraft_cfg_text(n=3, v=1, E=2, R=0, inv=("LeaderHasAllAckedValues", "NoLogDivergence",
                                            "NeverTwoLeadersInSameEpoch", "NoIllegalState")):
    """A cfg in KRaft.cfg's shape (pull-raft/KRaft.cfg:5-50): its model values
    and invariants, with the given bounds."""
    lines = ["CONSTANTS"]
    lines += ["    n%d = n%d" % (i, i) for i in range(1, n + 1)]
    lines += ["    v%d = v%d" % (i, i) for i in range(1, v + 1)]
    lines.append("    Server = {%s}" % ", ".join("n%d" % i for i in range(1, n + 1)))
    lines.append("    Value = {%s}" % ", ".join("v%d" % i for i in range(1, v + 1)))
    for k in ("Follower", "Candidate", "Leader", "Unattached", "Voted", "Nil", "RequestVoteRequest",
              "RequestVoteResponse", "BeginQuorumRequest", "BeginQuorumResponse", "EndQuorumRequest",
              "FetchRequest", "FetchResponse", "Ok", "NotOk", "Diverging", "FencedLeaderEpoch", "NotLeader",
              "UnknownLeader", "IllegalState", "EqualEpoch", "AnyEpoch"):
        lines.append("    %s = %s" % (k, k))
    lines.append("    MaxElections = %d" % E)
    lines.append("    MaxRestarts = %d" % R)
    lines += ["INIT Init", "NEXT Next", "VIEW view", "SYMMETRY symmServers", "INVARIANT"]
    lines += list(inv)
    return "\n".join(lines) + "\n"


# KRaft (pull-raft/KRaft.tla): (name, kwargs); the Python
# oracle (oracle/pyoracle/kraft.py) pins them
KRAFT = [
    ("kraft_n2v1e1", dict(n=2, v=1, E=1)),
    ("kraft_n2v1e2", dict(n=2, v=1, E=2)),
    ("kraft_n3v1e1", dict(n=3, v=1, E=1)),
    ("kraft_n2v2e2", dict(n=2, v=2, E=2)),
    ("kraft_n2v1e2r1", dict(n=2, v=1, E=2, R=1)),
    ("kraft_n3v1e1r1", dict(n=3, v=1, E=1, R=1)),
    ("kraft_n2v2e1r1", dict(n=2, v=2, E=1, R=1)),
    ("kraft_n3v2e1", dict(n=3, v=2, E=1)),
]


# BASELINE configs 2 and 5 at their scaled bounds (configs/Raft_n3v2e3.cfg,
# configs/RaftFsync_n3v2e3r1.cfg): exhausting them is beyond one GPU, so they
# are pinned level by level up to the first level boundary at which the C
# oracle has found >= max_distinct states; the Python oracle reproduces a
# shorter prefix.  (name, module, cfg path, C max_distinct, Python max_states)
LADDERS = [
    ("raft_n3v2e3_cfg2", "Raft", "configs/Raft_n3v2e3.cfg", 20000000, 20000),
    ("fsync_n3v2e3r1_cfg5", "RaftFsync", "configs/RaftFsync_n3v2e3r1.cfg", 20000000, 20000),
    # the exhaustible rungs below them (the bench workload and config 5's
    # largest exhausted rung), pinned by the oracles on their first levels
    ("raft_n3v2e2_bench", "Raft", "configs/Raft_n3v2e2.cfg", 20000000, 20000),
    ("fsync_n3v1e2r1_rung", "RaftFsync", "configs/RaftFsync_n3v1e2r1.cfg", 20000000, 20000),
    # BASELINE config 3 verbatim (FlexibleRaft.cfg: N=5, EQ=3, RQ=4, V=2, E=2)
    ("flex_cfg3", "FlexibleRaft", "configs/FlexibleRaft.cfg", 10000000, 3000),
]

# FlexibleRaft's Restart (FlexibleRaft.tla:200-208) with MaxRestarts >= 1:
# (name, kwargs, C max_distinct or 0 = exhaustive, Python max_states or 0 = exhaustive)
FLEX_RESTART = [
    ("flex_n3v1e1r1", dict(n=3, v=1, E=1, R=1, ElectionQuorumSize=2, ReplicationQuorumSize=2), 0, 0),
    ("flex_n2v1e2r1", dict(n=2, v=1, E=2, R=1, ElectionQuorumSize=2, ReplicationQuorumSize=1), 0, 0),
    ("flex_n3v1e2r1", dict(n=3, v=1, E=2, R=1, ElectionQuorumSize=2, ReplicationQuorumSize=2), 5000000, 30000),
    ("flex_n3v2e2r1_eq1", dict(n=3, v=2, E=2, R=1, ElectionQuorumSize=1, ReplicationQuorumSize=2), 0, 0),
    ("flex_n5v1e1r1_eq3rq4", dict(n=5, v=1, E=1, R=1, ElectionQuorumSize=3, ReplicationQuorumSize=4), 400000, 3000),
]

# The classic Raft safety properties as opt-in invariants (ElectionSafety,
# LogMatching, LeaderCompleteness, StateMachineSafety; INTEGRATION.md gives
# their TLA+): (name, module, kwargs, invariants in cfg order).  Safe configs
# must satisfy them (same counts as with the shipped invariants); the
# non-intersecting Flexible quorums break ElectionSafety.
CLASSIC = ("ElectionSafety", "LogMatching", "LeaderCompleteness", "StateMachineSafety")
SHIPPED_INV = ("LeaderHasAllAckedValues", "NoLogDivergence")
EXTRAS = [
    ("raft_n3v1e1_classic", "Raft", dict(n=3, v=1, E=1), SHIPPED_INV + CLASSIC),
    ("raft_n2v2e2_classic", "Raft", dict(n=2, v=2, E=2), SHIPPED_INV + CLASSIC),
    ("raft_n3v1e1r1_classic", "Raft", dict(n=3, v=1, E=1, R=1), CLASSIC),
    ("pull_n3v2e1_classic", "PullRaft", dict(n=3, v=2, E=1), SHIPPED_INV + CLASSIC),
    ("pull_n2v1e2r1_classic", "PullRaft", dict(n=2, v=1, E=2, R=1), CLASSIC),
    ("fsync_n3v1e1_classic", "RaftFsync", dict(n=3, v=1, E=1), SHIPPED_INV + CLASSIC),
    ("fsync_n2v1e2r1_classic", "RaftFsync", dict(n=2, v=1, E=2, R=1), CLASSIC),
    ("flex_n3v1e1_classic", "FlexibleRaft", dict(n=3, v=1, E=1, ElectionQuorumSize=2, ReplicationQuorumSize=2),
     SHIPPED_INV + CLASSIC),
    ("pull2_n3v1e1_classic", "PullRaftVariant2", dict(n=3, v=1, E=1), CLASSIC),
    # FollowerFsyncBeforeReply = FALSE with a restart: acknowledged entries can be lost
    ("fsync_n2v1e2r1_nofsync_classic", "RaftFsync", dict(n=2, v=1, E=2, R=1, FollowerFsyncBeforeReply=False), CLASSIC),
    # quorums of 1 (FlexibleRaft.tla:16-24 lists the valid pairs): two leaders of one term
    ("flex_n3v1e2_q1_classic", "FlexibleRaft", dict(n=3, v=1, E=2, ElectionQuorumSize=1, ReplicationQuorumSize=1),
     CLASSIC),
    ("flex_n3v1e2_q1_lm", "FlexibleRaft", dict(n=3, v=1, E=2, ElectionQuorumSize=1, ReplicationQuorumSize=1),
     ("LogMatching", "LeaderCompleteness", "StateMachineSafety")),
]

# The TLA+ front end (raft-tlaplus_amd/csrc/rmc_tla.cpp):
# modules whose Next differs from the reference's -- reordered, reduced, or
# with the network actions Raft.tla:540-541 leaves commented out -- lowered
# onto the action library.  (name, module, kwargs, Next as operator names,
# max_depth: 0 = exhaustive; DuplicateMessage makes the state space infinite,
# "There is no state-space control for this action", Raft.tla:509-511).
NEXT_RAFT = ("Restart", "RequestVote", "BecomeLeader", "ClientRequest", "AdvanceCommitIndex", "AppendEntries",
             "UpdateTerm", "HandleRequestVoteRequest", "HandleRequestVoteResponse", "RejectAppendEntriesRequest",
             "AcceptAppendEntriesRequest", "HandleAppendEntriesResponse")
NEXT_FSYNC = ("Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest", "AdvanceCommitIndex",
              "AppendEntries", "AdvanceFsyncIndex", "UpdateTerm", "HandleRequestVoteRequest",
              "HandleRequestVoteResponse", "RejectAppendEntriesRequest", "AcceptAppendEntriesRequest",
              "HandleAppendEntriesResponse")
NEXT_PULL = ("Restart", "UpdateTerm", "RequestVote", "HandleRequestVoteRequest", "HandleRequestVoteResponse",
             "BecomeLeader", "ClientRequest", "RejectPullEntriesRequest", "AcceptPullEntriesRequest",
             "LearnOfLeader", "SendPullEntriesRequest", "HandleSuccessPullEntriesResponse",
             "HandleFailPullEntriesResponse")
FRONTEND = [
    ("raft_dup_n3v1e2", "Raft", dict(n=3, v=1, E=2), NEXT_RAFT + ("DuplicateMessage",), 8),
    ("raft_dupdrop_n3v1e1", "Raft", dict(n=3, v=1, E=1), NEXT_RAFT + ("DuplicateMessage", "DropMessage"), 8),
    ("raft_drop_n3v1e1", "Raft", dict(n=3, v=1, E=1), NEXT_RAFT + ("DropMessage",), 0),
    ("raft_reversed_n3v1e1", "Raft", dict(n=3, v=1, E=1), tuple(reversed(NEXT_RAFT)), 0),
    # reversed Next with same-level hidden-variable collisions: TLC's winner order changes
    ("raft_reversed_n2v2e2r1", "Raft", dict(n=2, v=2, E=2, R=1), tuple(reversed(NEXT_RAFT)), 0),
    ("raft_no_restart_drop_n2v1e2", "Raft", dict(n=2, v=1, E=2, R=1),
     tuple(d for d in NEXT_RAFT if d != "Restart") + ("DropMessage",), 0),
    ("raft_no_hrvresp_n3v1e1", "Raft", dict(n=3, v=1, E=1), tuple(d for d in NEXT_RAFT if d != "HandleRequestVoteResponse"), 0),
    ("flex_dup_n3v1e1", "FlexibleRaft", dict(n=3, v=1, E=1, ElectionQuorumSize=2, ReplicationQuorumSize=2),
     ("DuplicateMessage",) + NEXT_RAFT, 7),
    ("fsync_dropdup_n2v1e1r1", "RaftFsync", dict(n=2, v=1, E=1, R=1), NEXT_FSYNC + ("DropMessage", "DuplicateMessage"), 8),
    ("pull_dup_n3v1e1", "PullRaft", dict(n=3, v=1, E=1), NEXT_PULL + ("DuplicateMessage",), 8),
    ("pull2_drop_reversed_n3v1e1", "PullRaftVariant2", dict(n=3, v=1, E=1), tuple(reversed(NEXT_PULL)) + ("DropMessage",), 0),
]


# (name, module, kwargs, [(action, params, TLA+ guard)], max_depth): Next with
# actions behind a guard other than the reference's -- what a module whose
# action keeps the reference's effect but states another guard lowers to
# through the TLA+ front end (rmc_guard.cpp; rmc_model_set_guard is the same
# table).  The Python side of each guard is make_golden.GUARD_PY[name].
GUARDS = [
    # Raft.tla:242-257 RequestVote with `electionCtr <= MaxElections`: one more election
    ("raft_rv_le_n2v1e1", "Raft", dict(n=2, v=1, E=1),
     [("RequestVote", "i", "electionCtr <= MaxElections /\\ state[i] \\in {Follower, Candidate}")], 0),
    # Raft.tla:289-300 BecomeLeader that wants every vote
    ("raft_bl_all_n3v1e1", "Raft", dict(n=3, v=1, E=1),
     [("BecomeLeader", "i", "state[i] = Candidate /\\ votesGranted[i] = Server")], 0),
    # Raft.tla:226-235 Restart only of a non-leader
    ("raft_restart_nonleader_n2v1e2r1", "Raft", dict(n=2, v=1, E=2, R=1),
     [("Restart", "i", "restartCtr < MaxRestarts /\\ state[i] /= Leader")], 0),
    # Raft.tla:304-313 ClientRequest only while the leader has no entry of its own term
    ("raft_client_lastterm_n2v2e2", "Raft", dict(n=2, v=2, E=2),
     [("ClientRequest", "i, v",
       "/\\ state[i] = Leader\n    /\\ acked[v] = Nil\n    /\\ LastTerm(log[i]) < currentTerm[i]")], 0),
    # quantifiers, IF/LET and a set filter, two guards at once
    ("raft_quant_n2v1e2", "Raft", dict(n=2, v=1, E=2),
     [("BecomeLeader", "i",
       "state[i] = Candidate /\\ votesGranted[i] \\in Quorum /\\ \\A j \\in Server : currentTerm[j] <= currentTerm[i]"),
      ("RequestVote", "i",
       "LET busy == \\E j \\in Server : state[j] = Leader IN "
       "electionCtr < MaxElections /\\ state[i] \\in {Follower, Candidate} /\\ "
       "IF busy THEN Cardinality({j \\in Server : currentTerm[j] > currentTerm[i]}) > 0 ELSE TRUE")], 0),
    # FlexibleRaft.tla BecomeLeader at a fixed election quorum of 3 of 3
    ("flex_bl_card_n3v1e1", "FlexibleRaft", dict(n=3, v=1, E=1, ElectionQuorumSize=2, ReplicationQuorumSize=2),
     [("BecomeLeader", "i", "state[i] = Candidate /\\ Cardinality(votesGranted[i]) >= 3")], 0),
    # RaftFsync.tla Timeout only of a follower, RequestVote(i, j) only to a server at a term <= i's
    ("fsync_timeout_rvij_n2v1e2r1", "RaftFsync", dict(n=2, v=1, E=2, R=1),
     [("Timeout", "i", "electionCtr < MaxElections /\\ state[i] = Follower"),
      ("RequestVote", "i, j", "state[i] = Candidate /\\ i /= j /\\ currentTerm[j] <= currentTerm[i]")], 0),
    # PullRaft.tla:283-298 RequestVote only with no known leader
    ("pull_rv_noleader_n2v1e2r1", "PullRaft", dict(n=2, v=1, E=2, R=1),
     [("RequestVote", "i", "electionCtr < MaxElections /\\ state[i] \\in {Follower, Candidate} /\\ leader[i] = Nil")],
     0),
    # PullRaftVariant2 Restart gated on an empty log
    ("pull2_restart_emptylog_n2v1e2r1", "PullRaftVariant2", dict(n=2, v=1, E=2, R=1),
     [("Restart", "i", "restartCtr < MaxRestarts /\\ Len(log[i]) = 0")], 0),
]


# (name, module, kwargs, Next (names), [(action, form, params, TLA+ body)],
# max_depth): actions the TLA+ front end compiles whole -- guard AND effect
# (rmc_guard.cpp compile_effect) -- given as TLA+ text (rmc_model_define_action
# is the table a module with such a Next disjunct lowers to).  The Python side
# of each action is make_golden._effect_py()[name].
_RV_BODY = """/\\ electionCtr < MaxElections
    /\\ state[i] \\in {Follower, Candidate}
    /\\ state' = [state EXCEPT ![i] = Candidate]
    /\\ currentTerm' = [currentTerm EXCEPT ![i] = currentTerm[i] + 1]
    /\\ votedFor' = [votedFor EXCEPT ![i] = Nil]
    /\\ votesGranted' = [votesGranted EXCEPT ![i] = {}]
    /\\ electionCtr' = electionCtr + 1
    /\\ %s({[mtype |-> RequestVoteRequest, mterm |-> currentTerm[i] + 1, mlastLogTerm |-> LastTerm(log[i]),
          mlastLogIndex |-> Len(log[i]), msource |-> i, mdest |-> j] : j \\in Server \\ {i}})
    /\\ UNCHANGED <<acked, leaderVars, logVars, restartCtr>>"""
EFFECTS = [
    # Raft.tla:242-257 RequestVote whose candidate does not vote for itself
    ("raft_rv_noself_n3v1e2", "Raft", dict(n=3, v=1, E=2),
     ("Restart", "RequestVoteNoSelf") + NEXT_RAFT[2:],
     [("RequestVoteNoSelf", "i", "i", _RV_BODY % "SendMultipleOnce")], 0),
    # RequestVote that moves two terms on but asks for votes at the next term, with @ in the EXCEPTs
    ("raft_rv_term2_n2v1e2", "Raft", dict(n=2, v=1, E=2),
     ("Restart", "RequestVoteTwo") + NEXT_RAFT[2:],
     [("RequestVoteTwo", "i", "i", """/\\ electionCtr < MaxElections
    /\\ state[i] \\in {Follower, Candidate}
    /\\ state' = [state EXCEPT ![i] = Candidate]
    /\\ currentTerm' = [currentTerm EXCEPT ![i] = @ + 2]
    /\\ votedFor' = [votedFor EXCEPT ![i] = i]
    /\\ votesGranted' = [votesGranted EXCEPT ![i] = {i}]
    /\\ electionCtr' = electionCtr + 1
    /\\ SendMultipleOnce({[mtype |-> RequestVoteRequest, mterm |-> currentTerm[i] + 1, mlastLogTerm |-> LastTerm(log[i]),
          mlastLogIndex |-> Len(log[i]), msource |-> i, mdest |-> j] : j \\in Server \\ {i}})
    /\\ UNCHANGED <<acked, leaderVars, logVars, restartCtr>>""")], 0),
    # Raft.tla:304-313 ClientRequest that acks the value at once: LeaderHasAllAckedValues breaks
    ("raft_client_eager_n3v1e2", "Raft", dict(n=3, v=1, E=2),
     NEXT_RAFT[:3] + ("ClientRequestEager",) + NEXT_RAFT[4:],
     [("ClientRequestEager", "iv", "i, v", """/\\ state[i] = Leader
    /\\ acked[v] = Nil
    /\\ log' = [log EXCEPT ![i] = Append(@, [term |-> currentTerm[i], value |-> v])]
    /\\ acked' = [acked EXCEPT ![v] = TRUE]
    /\\ UNCHANGED <<messages, serverVars, candidateVars, leaderVars, commitIndex, electionCtr, restartCtr>>""")], 0),
    # Raft.tla:226-235 Restart that keeps the leader's rows and its commitIndex at 0
    ("raft_restart_keep_n2v1e2r1", "Raft", dict(n=2, v=1, E=2, R=1),
     ("RestartKeep",) + NEXT_RAFT[1:],
     [("RestartKeep", "i", "i", """/\\ restartCtr < MaxRestarts
    /\\ state' = [state EXCEPT ![i] = Follower]
    /\\ votesGranted' = [votesGranted EXCEPT ![i] = {}]
    /\\ commitIndex' = [commitIndex EXCEPT ![i] = 0]
    /\\ restartCtr' = restartCtr + 1
    /\\ UNCHANGED <<messages, currentTerm, votedFor, leaderVars, log, acked, electionCtr>>""")], 0),
    # Raft: a candidate re-sends its vote request (Send: _SendNoRestriction, count + 1); depth-bounded
    # below the 3-bit message count's cap (7)
    ("raft_resend_rv_n2v1e1", "Raft", dict(n=2, v=1, E=1),
     NEXT_RAFT + ("ResendVote",),
     [("ResendVote", "ij", "i, j", """/\\ state[i] = Candidate
    /\\ i /= j
    /\\ Send([mtype |-> RequestVoteRequest, mterm |-> currentTerm[i], mlastLogTerm |-> LastTerm(log[i]),
             mlastLogIndex |-> Len(log[i]), msource |-> i, mdest |-> j])
    /\\ UNCHANGED <<serverVars, candidateVars, leaderVars, logVars, auxVars>>""")], 8),
    # RaftFsync.tla:234-243 RequestVote(i, j) that claims an empty log
    ("fsync_rvij_empty_n2v1e2r1", "RaftFsync", dict(n=2, v=1, E=2, R=1),
     NEXT_FSYNC[:2] + ("RequestVoteEmpty",) + NEXT_FSYNC[3:],
     [("RequestVoteEmpty", "ij", "i, j", """/\\ state[i] = Candidate
    /\\ i # j
    /\\ Send([mtype |-> RequestVoteRequest, mterm |-> currentTerm[i], mlastLogTerm |-> 0,
             mlastLogIndex |-> 0, msource |-> i, mdest |-> j])
    /\\ UNCHANGED <<serverVars, candidateVars, leaderVars, logVars, auxVars>>""")], 0),
    # Raft.tla:226-235 Restart counting two restarts (its leader rows reset as the reference's)
    ("raft_restart_two_n2v1e2r3", "Raft", dict(n=2, v=1, E=2, R=3),
     ("RestartTwo",) + NEXT_RAFT[1:],
     [("RestartTwo", "i", "i", """/\\ restartCtr < MaxRestarts
    /\\ state'           = [state EXCEPT ![i] = Follower]
    /\\ votesGranted'    = [votesGranted EXCEPT ![i] = {}]
    /\\ nextIndex'       = [nextIndex EXCEPT ![i] = [j \\in Server |-> 1]]
    /\\ matchIndex'      = [matchIndex EXCEPT ![i] = [j \\in Server |-> 0]]
    /\\ pendingResponse' = [pendingResponse EXCEPT ![i] = [j \\in Server |-> FALSE]]
    /\\ commitIndex'     = [commitIndex EXCEPT ![i] = 0]
    /\\ restartCtr'      = restartCtr + 2
    /\\ UNCHANGED <<messages, currentTerm, votedFor, log, acked, electionCtr>>""")], 0),
    # Raft.tla:289-300 BecomeLeader that starts every follower's nextIndex at 1 and marks its own
    # pendingResponse[i][i]
    ("raft_bl_next1_n2v1e2", "Raft", dict(n=2, v=1, E=2),
     NEXT_RAFT[:2] + ("BecomeLeaderNext1",) + NEXT_RAFT[3:],
     [("BecomeLeaderNext1", "i", "i", """/\\ state[i] = Candidate
    /\\ votesGranted[i] \\in Quorum
    /\\ state'      = [state EXCEPT ![i] = Leader]
    /\\ nextIndex'  = [nextIndex EXCEPT ![i] = [j \\in Server |-> 1]]
    /\\ matchIndex' = [matchIndex EXCEPT ![i] = [j \\in Server |-> IF j = i THEN Len(log[i]) ELSE 0]]
    /\\ pendingResponse' = [pendingResponse EXCEPT ![i][i] = TRUE]
    /\\ UNCHANGED <<messages, currentTerm, votedFor, candidateVars, auxVars, logVars>>""")], 0),
    # FlexibleRaft.tla:215-230 RequestVote without the self vote (SendMultiple)
    ("flex_rv_noself_n3v1e1", "FlexibleRaft", dict(n=3, v=1, E=1, ElectionQuorumSize=2, ReplicationQuorumSize=2),
     ("Restart", "RequestVoteNoSelf") + NEXT_RAFT[2:],
     [("RequestVoteNoSelf", "i", "i", _RV_BODY % "SendMultiple")], 0),
]


# (name, module, kwargs, Next (names), [(action, "m", "m", TLA+ body)], max_depth):
# message handlers the TLA+ front end compiles whole (rmc_guard.cpp
# compile_handler) -- the body of \E m \in DOMAIN messages : body, given as TLA+
# text (rmc_model_define_action form "m" is the table a module whose Next has
# such a bare action lowers to).  The Python side of each is
# make_golden._handler_py()[name].
def _nx(base, old, new):
    return tuple(new if d == old else d for d in base)


_HRVRESP = """/\\ ReceivableMessage(m, RequestVoteResponse, EqualTerm)
    /\\ LET i == m.mdest
           j == m.msource
       IN
          /\\ \\/ /\\ m.mvoteGranted
                /\\ votesGranted' = [votesGranted EXCEPT ![i] = votesGranted[i] \\cup {j}]
             \\/ /\\ ~m.mvoteGranted
                /\\ UNCHANGED <<votesGranted>>
          /\\ Discard(m)
          /\\ UNCHANGED <<serverVars, votedFor, leaderVars, logVars, auxVars>>"""
_HRVRESP_ALL = """/\\ ReceivableMessage(m, RequestVoteResponse, EqualTerm)
    /\\ LET i == m.mdest
           j == m.msource
       IN
          /\\ votesGranted' = [votesGranted EXCEPT ![i] = votesGranted[i] \\cup {j}]
          /\\ Discard(m)
          /\\ UNCHANGED <<serverVars, votedFor, leaderVars, logVars, auxVars>>"""
_HRVREQ_NOLOG = """/\\ ReceivableMessage(m, RequestVoteRequest, LessOrEqualTerm)
    /\\ LET i     == m.mdest
           j     == m.msource
           grant == /\\ m.mterm = currentTerm[i]
                    /\\ votedFor[i] \\in {Nil, j}
        IN /\\ m.mterm <= currentTerm[i]
           /\\ \\/ grant  /\\ votedFor' = [votedFor EXCEPT ![i] = j]
              \\/ ~grant /\\ UNCHANGED votedFor
           /\\ Reply([mtype        |-> RequestVoteResponse,
                     mterm        |-> currentTerm[i],
                     mvoteGranted |-> grant,
                     msource      |-> i,
                     mdest        |-> j],
                     m)
           /\\ UNCHANGED <<state, currentTerm, candidateVars, leaderVars, logVars, auxVars>>"""
_REJAE = """/\\ ReceivableMessage(m, AppendEntriesRequest, LessOrEqualTerm)
    /\\ LET i     == m.mdest
           j     == m.msource
           logOk == \\/ m.mprevLogIndex = 0
                    \\/ /\\ m.mprevLogIndex > 0
                       /\\ m.mprevLogIndex <= Len(log[i])
                       /\\ m.mprevLogTerm = log[i][m.mprevLogIndex].term
       IN  /\\ %s
           /\\ Reply([mtype           |-> AppendEntriesResponse,
                     mterm           |-> currentTerm[i],
                     msuccess        |-> FALSE,
                     mmatchIndex     |-> 0,
                     msource         |-> i,
                     mdest           |-> j],
                     m)
           /\\ UNCHANGED <<state, candidateVars, leaderVars, serverVars, logVars, auxVars>>"""
_REJAE_REF = _REJAE % """\\/ m.mterm < currentTerm[i]
              \\/ /\\ m.mterm = currentTerm[i]
                 /\\ state[i] = Follower
                 /\\ \\lnot logOk"""
_REJAE_LENIDX = (_REJAE % """\/ m.mterm < currentTerm[i]
              \/ /\ m.mterm = currentTerm[i]
                 /\ state[i] = Follower
                 /\ \lnot logOk""").replace("mmatchIndex     |-> 0", "mmatchIndex     |-> Len(log[i])")
_UPDATETERM_STAY = """/\\ m.mterm > currentTerm[m.mdest]
    /\\ currentTerm'    = [currentTerm EXCEPT ![m.mdest] = m.mterm]
    /\\ votedFor'       = [votedFor    EXCEPT ![m.mdest] = Nil]
    /\\ UNCHANGED <<messages, state, candidateVars, leaderVars, logVars, auxVars>>"""
_HAERESP = """/\\ ReceivableMessage(m, AppendEntriesResponse, EqualTerm)
    /\\ LET i     == m.mdest
           j     == m.msource
       IN
          /\\ \\/ /\\ m.msuccess \\* successful
                /\\ nextIndex'  = [nextIndex  EXCEPT ![i][j] = %s]
                /\\ matchIndex' = [matchIndex EXCEPT ![i][j] = m.mmatchIndex]
             \\/ /\\ \\lnot m.msuccess \\* not successful
                /\\ nextIndex' = [nextIndex EXCEPT ![i][j] =
                                     Max({nextIndex[i][j] - %d, 1})]
                /\\ UNCHANGED <<matchIndex>>%s
          /\\ Discard(m)
          /\\ UNCHANGED <<serverVars, candidateVars, logVars, auxVars>>"""
_PEND = """
          /\\ pendingResponse' = [pendingResponse EXCEPT ![i][j] = FALSE]"""
HANDLERS = [
    # Raft.tla:386-401 HandleRequestVoteResponse written out: compiled, it checks the built-in space
    ("raft_hrvresp_text_n3v1e1", "Raft", dict(n=3, v=1, E=1),
     _nx(NEXT_RAFT, "HandleRequestVoteResponse", "HRVRespText"), [("HRVRespText", "m", "m", _HRVRESP)], 0),
    # ... tallying every response as a vote (the mvoteGranted test dropped)
    ("raft_hrvresp_all_n2v1e2", "Raft", dict(n=2, v=1, E=2),
     _nx(NEXT_RAFT, "HandleRequestVoteResponse", "HRVRespAll"), [("HRVRespAll", "m", "m", _HRVRESP_ALL)], 0),
    # Raft.tla:360-381 HandleRequestVoteRequest without the log comparison (logOk dropped)
    ("raft_hrvreq_nolog_n2v1e2", "Raft", dict(n=2, v=1, E=2),
     _nx(NEXT_RAFT, "HandleRequestVoteRequest", "HRVReqNoLog"), [("HRVReqNoLog", "m", "m", _HRVREQ_NOLOG)], 0),
    # Raft.tla:412-430 RejectAppendEntriesRequest written out (LogOk inlined)
    ("raft_rejae_text_n2v2e2", "Raft", dict(n=2, v=2, E=2),
     _nx(NEXT_RAFT, "RejectAppendEntriesRequest", "RejAEText"), [("RejAEText", "m", "m", _REJAE_REF)], 0),
    # ... whose rejection carries the follower's log length as mmatchIndex
    ("raft_rejae_lenidx_n2v2e2", "Raft", dict(n=2, v=2, E=2),
     _nx(NEXT_RAFT, "RejectAppendEntriesRequest", "RejAELen"), [("RejAELen", "m", "m", _REJAE_LENIDX)], 0),
    # Raft.tla:348-355 UpdateTerm that does not step down to Follower
    ("raft_updateterm_stay_n2v1e2", "Raft", dict(n=2, v=1, E=2),
     _nx(NEXT_RAFT, "UpdateTerm", "UpdateTermStay"), [("UpdateTermStay", "m", "m", _UPDATETERM_STAY)], 0),
    # two compiled handlers at once, one of them with its reference text
    ("raft_two_handlers_n2v1e2r1", "Raft", dict(n=2, v=1, E=2, R=1),
     _nx(_nx(NEXT_RAFT, "HandleRequestVoteResponse", "HRVRespAll"), "RejectAppendEntriesRequest", "RejAEText"),
     [("HRVRespAll", "m", "m", _HRVRESP_ALL), ("RejAEText", "m", "m", _REJAE_REF)], 0),
    # FlexibleRaft (Reply refuses a response already in DOMAIN) and RaftFsync
    ("flex_hrvresp_all_n2v1e2", "FlexibleRaft", dict(n=2, v=1, E=2, ElectionQuorumSize=2, ReplicationQuorumSize=1),
     _nx(NEXT_RAFT, "HandleRequestVoteResponse", "HRVRespAll"), [("HRVRespAll", "m", "m", _HRVRESP_ALL)], 0),
    ("fsync_rejae_text_n2v1e2r1", "RaftFsync", dict(n=2, v=1, E=2, R=1),
     _nx(NEXT_FSYNC, "RejectAppendEntriesRequest", "RejAEText"), [("RejAEText", "m", "m", _REJAE_REF)], 0),
    ("fsync_hrvreq_nolog_n2v1e2r1", "RaftFsync", dict(n=2, v=1, E=2, R=1),
     _nx(NEXT_FSYNC, "HandleRequestVoteRequest", "HRVReqNoLog"), [("HRVReqNoLog", "m", "m", _HRVREQ_NOLOG)], 0),
    # Raft.tla:490-505 HandleAppendEntriesResponse written out (Max, rows at [i][j] = [mdest][msource])
    ("raft_haeresp_text_n3v1e1", "Raft", dict(n=3, v=1, E=1),
     _nx(NEXT_RAFT, "HandleAppendEntriesResponse", "HAERespText"),
     [("HAERespText", "m", "m", _HAERESP % ("m.mmatchIndex + 1", 1, _PEND))], 0),
    # ... re-sending the last acknowledged entry: nextIndex = Max({mmatchIndex, 1}) on success, and
    # backing off by two on a rejection
    ("raft_haeresp_resend_n2v2e2", "Raft", dict(n=2, v=2, E=2),
     _nx(NEXT_RAFT, "HandleAppendEntriesResponse", "HAERespResend"),
     [("HAERespResend", "m", "m", _HAERESP % ("Max({m.mmatchIndex, 1})", 2, _PEND))], 0),
    # RaftFsync.tla:486-500 (no pendingResponse) written out
    ("fsync_haeresp_text_n2v1e2r1", "RaftFsync", dict(n=2, v=1, E=2, R=1),
     _nx(NEXT_FSYNC, "HandleAppendEntriesResponse", "HAERespText"),
     [("HAERespText", "m", "m", _HAERESP % ("m.mmatchIndex + 1", 1, ""))], 0),
]
