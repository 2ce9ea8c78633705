"""Generate raft-tlaplus_amd/csrc/rmc_tla_known.inc: the closure hashes of the
reference modules' definitions that the TLA+ front end (rmc_tla.cpp) matches
a module's Init / Next disjuncts / VIEW / SYMMETRY / INVARIANTs against.

Runs in the build container only (it reads /root/reference); the output holds
hashes and names, no spec text.  The table maps each lowered definition of
each spec family to its library action (rmc_spec.h ActId + binding form),
invariant id or role:

    python tools/gen_tla_known.py     # after building librmc.so once
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/specifications"
OUT = os.path.join(ROOT, "raft-tlaplus_amd", "csrc", "rmc_tla_known.inc")

# module -> (spec kind, file)
MODULES = [("Raft", "RAFT", "standard-raft/Raft.tla"),
           ("FlexibleRaft", "FLEX", "flexible-raft/FlexibleRaft.tla"),
           ("RaftFsync", "FSYNC", "raft-and-fsync/RaftFsync.tla"),
           ("PullRaft", "PULL", "pull-raft/PullRaft.tla"),
           ("PullRaftVariant2", "PULL2", "pull-raft/PullRaftVariant2.tla"),
           ("KRaft", "KRAFT", "pull-raft/KRaft.tla")]

NETWORK = {"DuplicateMessage": ("A_DUP", "K_M"), "DropMessage": ("A_DROP", "K_M")}
RAFT_ACTIONS = {"Restart": ("A_RESTART", "K_I"), "RequestVote": ("A_REQUESTVOTE", "K_I"),
                "BecomeLeader": ("A_BECOMELEADER", "K_I"), "ClientRequest": ("A_CLIENT", "K_IV"),
                "AdvanceCommitIndex": ("A_ADVCOMMIT", "K_I"), "AppendEntries": ("A_APPENDENTRIES", "K_IJ"),
                "UpdateTerm": ("A_UPDATETERM", "K_MSG"), "HandleRequestVoteRequest": ("A_HRVREQ", "K_MSG"),
                "HandleRequestVoteResponse": ("A_HRVRESP", "K_MSG"),
                "RejectAppendEntriesRequest": ("A_REJAE", "K_MSG"),
                "AcceptAppendEntriesRequest": ("A_ACCAE", "K_MSG"),
                "HandleAppendEntriesResponse": ("A_HAERESP", "K_MSG")}
FSYNC_ACTIONS = dict(RAFT_ACTIONS, Timeout=("A_TIMEOUT", "K_I"), RequestVote=("A_RVIJ", "K_IJ"),
                     AdvanceFsyncIndex=("A_ADVFSYNC", "K_I"))
PULL_ACTIONS = {"Restart": ("A_RESTART", "K_I"), "UpdateTerm": ("A_UPDATETERM", "K_MSG"),
                "RequestVote": ("A_REQUESTVOTE", "K_I"), "HandleRequestVoteRequest": ("A_HRVREQ", "K_MSG"),
                "HandleRequestVoteResponse": ("A_HRVRESP", "K_MSG"), "BecomeLeader": ("A_BECOMELEADER", "K_I"),
                "ClientRequest": ("A_CLIENT", "K_IV"), "RejectPullEntriesRequest": ("A_REJPULL", "K_MSG"),
                "AcceptPullEntriesRequest": ("A_ACCPULL", "K_MSG"), "LearnOfLeader": ("A_LEARN", "K_MSG"),
                "SendPullEntriesRequest": ("A_SENDPULL", "K_IJ"),
                "HandleSuccessPullEntriesResponse": ("A_HSUCC", "K_MSG"),
                "HandleFailPullEntriesResponse": ("A_HFAIL", "K_MSG")}
KRAFT_ACTIONS = {"Restart": ("A_RESTART", "K_I"), "RequestVote": ("A_REQUESTVOTE", "K_I"),
                 "HandleRequestVoteRequest": ("A_HRVREQ", "K_MSG"),
                 "HandleRequestVoteResponse": ("A_HRVRESP", "K_MSG"), "BecomeLeader": ("A_BECOMELEADER", "K_I"),
                 "ClientRequest": ("A_CLIENT", "K_IV"), "RejectFetchRequest": ("A_KREJFETCH", "K_MSG"),
                 "DivergingFetchRequest": ("A_KDIVFETCH", "K_MSG"), "AcceptFetchRequest": ("A_KACCFETCH", "K_MSG"),
                 "HandleBeginQuorumRequest": ("A_KHBQ", "K_MSG"), "SendFetchRequest": ("A_KSENDFETCH", "K_IJ"),
                 "HandleSuccessFetchResponse": ("A_KHSUCC", "K_MSG"),
                 "HandleDivergingFetchResponse": ("A_KHDIV", "K_MSG"),
                 "HandleErrorFetchResponse": ("A_KHERR", "K_MSG")}
ACTIONS = {"Raft": RAFT_ACTIONS, "FlexibleRaft": RAFT_ACTIONS, "RaftFsync": FSYNC_ACTIONS, "PullRaft": PULL_ACTIONS,
           "PullRaftVariant2": PULL_ACTIONS, "KRaft": KRAFT_ACTIONS}
# invariant ids of rmc::Model::inv (rmc_spec.h)
INVARIANTS = {"LeaderHasAllAckedValues": 0, "NoLogDivergence": 1, "CommittedEntriesReachMajority": 2,
              "NeverTwoLeadersInSameEpoch": 3, "NoIllegalState": 4}


# Actions whose guard the front end may replace (rmc_guard.cpp): their library
# functions check exactly the reference's effect-free conjuncts and run the
# rest unguarded when a compiled guard stands in (rmc_spec.h `ug`).
GUARDED = {"Restart", "RequestVote", "Timeout", "BecomeLeader", "ClientRequest"}


# The bag helpers the effect compiler implements (by their reference semantics):
# 0 = a set of records, all new, each sent once (Raft.tla:153-155 SendMultipleOnce,
# FlexibleRaft.tla:131-133 SendMultiple); 1 = one record, new, sent once
# (Raft.tla:136-138 _SendOnce, FlexibleRaft.tla:127-129 / RaftFsync.tla:131-134
# Send); 2 = one non-empty-AppendEntries record, count + 1 (Raft.tla:129-132
# _SendNoRestriction, and Raft.tla:145-149 Send for every record but an empty
# AppendEntriesRequest)
HELPERS = {"RAFT": {"SendMultipleOnce": 0, "_SendOnce": 1, "Send": 2, "_SendNoRestriction": 2},
           "FLEX": {"SendMultiple": 0, "Send": 1},
           "FSYNC": {"Send": 1}}
# ... and the bag helpers a compiled message handler may call (rmc_guard.cpp
# compile_handler): 3 = Discard(m) (Raft.tla:164-167), 4 = Reply(response,
# request) (Raft.tla:170-176; FlexibleRaft.tla:148-151 and RaftFsync.tla:149-152
# refuse a response already in DOMAIN -- rmc_spec.h op_reply)
for _k in HELPERS:
    HELPERS[_k].update(Discard=3, Reply=4)


def hashes(lib, text):
    buf = ctypes.create_string_buffer(1 << 20)
    n = lib.rmc_tla_hashes(text.encode(), buf, len(buf))
    if n < 0:
        raise SystemExit(buf.value.decode())
    out, vars_h, effects = {}, None, {}
    for line in buf.value.decode().splitlines():
        if line.startswith("#vars "):
            vars_h = line.split()[1]
        elif line.startswith("effect:"):
            name, h = line[len("effect:"):].split()
            effects[name] = h
        elif not line.startswith("#"):
            name, h = line.split()
            out[name] = h
    return out, vars_h, effects


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "raft-tlaplus_amd", "build", "librmc.so"))
    rows = ["// Generated by tools/gen_tla_known.py from the reference modules (closure hashes only, no spec text).",
            "// {spec, role, id, binding form, closure hash, reference definition}"]
    for module, kind, rel in MODULES:
        h, vh, eff = hashes(lib, open(os.path.join(REF, rel)).read())
        rows.append("// %s (specifications/%s)" % (module, rel))
        rows.append("{%s, R_VARS, 0, 0, 0x%sULL, \"VARIABLES\"}," % (kind, vh))
        rows.append("{%s, R_INIT, 0, 0, 0x%sULL, \"Init\"}," % (kind, h["Init"]))
        rows.append("{%s, R_VIEW, 0, 0, 0x%sULL, \"view\"}," % (kind, h["view"]))
        rows.append("{%s, R_SYMM, 0, 0, 0x%sULL, \"symmServers\"}," % (kind, h["symmServers"]))
        acts = dict(ACTIONS[module], **NETWORK)
        for name, (act, form) in acts.items():
            if name not in h:
                if name in NETWORK:
                    continue
                raise SystemExit("%s: no hash for %s" % (module, name))
            rows.append("{%s, R_ACTION, %s, %s, 0x%sULL, \"%s\"}," % (kind, act, form, h[name], name))
            if name in GUARDED and name in eff and kind != "KRAFT":
                rows.append("{%s, R_EFFECT, %s, %s, 0x%sULL, \"%s\"}," % (kind, act, form, eff[name], name))
        # bag helpers an action compiled whole may call (rmc_guard.cpp compile_effect)
        for name, cls in HELPERS.get(kind, {}).items():
            rows.append("{%s, R_HELPER, %d, 0, 0x%sULL, \"%s\"}," % (kind, cls, h[name], name))
        for name, iid in INVARIANTS.items():
            if name in h:
                rows.append("{%s, R_INV, %d, 0, 0x%sULL, \"%s\"}," % (kind, iid, h[name], name))
    open(OUT, "w").write("\n".join(rows) + "\n")
    print("wrote", OUT, len(rows), "lines")


if __name__ == "__main__":
    sys.exit(main())
