"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of kikimo/tla-raft's hot path.

This module is the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker; the
product path (``tla-raft_amd/``) never imports, links or executes anything under
``oracle/``.

What it restates
----------------
* ``Raft.tla`` (``/root/reference/Raft.tla``, cited as ``tla:N``): Init (tla:93-105),
  the 11 disjuncts of Next in their textual order (tla:416-430), the helpers
  MajoritySize / SendMsg / Min / Max / Median / LogMatch (tla:41-49, 70-75, 271-273),
  the invariant LeaderHasAllCommittedEntries (tla:491-499) and the debug invariants
  (tla:434-487), the symmetry set (tla:21) and the VIEW (tla:38).
* ``Raft.cfg`` (cfg:1-34) and ``myrun.sh`` (run:3): TLC breadth-first search with
  ``-deadlock``, first-discovery-wins under SYMMETRY+VIEW, invariants checked on
  Init and on every newly discovered state.

TLC semantics (tla2tools.jar is not shipped by the reference, gitignore:3) are
restated from TLC's published design with ``-workers 1`` discovery order:
FIFO queue, successors of a state enumerated server-major (s1 < s2 < ...), then the
11 disjuncts in textual order, then each ``\\E`` witness in TLC's normalised value
order (records compare by field count, then (sorted field name, value) pairs;
tuples by length then elements; model values by name; FALSE < TRUE).

Parity status: **unpinned** by the reference -- the reference ships no TLC, no
logs and no expected counts (gitignore:1, BASELINE.json "published": {}).  This
oracle is pinned only by the hand-derived known answers of SURVEY.md Appendix C
(checked in tests/test_oracle.py) and by agreement with the independent C
restatement in ``oracle/raft_oracle.c``.

Representation
--------------
Servers are 0..n-1 (s1..sn), values 0..V-1 (v1..vV), ``None`` is -1.  Roles:
Follower 0, Candidate 1, Leader 2.  A message *is* its TLC order key, so Python's
tuple order on messages equals TLC's enumeration order of ``msgs``:

* VoteResp   (4 fields dst,src,term,type)                    -> (4, dst, src, term)
* VoteReq    (6 fields dst,lastLogIndex,lastLogTerm,src,term,type)
                                                            -> (6, dst, 0, lli, llt, src, term)
* AppendResp (6 fields dst,prevLogIndex,src,succ,term,type) -> (6, dst, 1, pli, src, succ, term)
* AppendReq  (8 fields dst,entries,leaderCommit,prevLogIndex,prevLogTerm,src,term,type)
                                                            -> (8, dst, entries, lc, pli, plt, src, term)

("lastLogIndex" < "prevLogIndex" as strings, so a VoteReq precedes an AppendResp
to the same dst; entries is () or ((term, val),), and () precedes any 1-tuple.)
"""
from __future__ import annotations

import itertools
from collections import deque
from dataclasses import dataclass, field
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

NONE = -1
FOLLOWER, CANDIDATE, LEADER = 0, 1, 2
ROLE_NAMES = ("Follower", "Candidate", "Leader")

# Action indices in Next's textual order (tla:418-430).
ACTIONS = (
    "BecomeCandidate",      # tla:107
    "UpdateTerm",           # tla:175
    "ResponseVote",         # tla:132
    "BecomeLeader",         # tla:157
    "ClientReq",            # tla:233
    "LeaderAppendEntry",    # tla:242
    "FollowerAcceptEntry",  # tla:275
    "FollowerRejectEntry",  # tla:302
    "HandleAppendResp",     # tla:374
    "LeaderCanCommit",      # tla:398
    "Restart",              # tla:409
    "FollowerAppendEntry",  # tla:323 (A_FAPP, the tla:425 variant)
    "BecomeFollower",       # tla:226 (A_BF, the tla:420 variant)
)
A_BC, A_UT, A_RV, A_BL, A_CR, A_LAE, A_FAE, A_FRE, A_HAR, A_LCC, A_RS = range(11)
A_FAPP = 11  # FollowerAppendEntry (tla:323), in Next only in the tla:425 variant
A_BF = 12    # BecomeFollower (tla:226), in Next only in the tla:420 variant (right after UpdateTerm)

INVARIANTS = ("Inv", "LeaderHasAllCommittedEntries", "NoSplitVote", "RaftCanCommt",
              "FollowerCanCommit", "CommitAll", "NoAllCommit", "ExistLeaderAndCandidate")


# --------------------------------------------------------------------------- messages
def vote_req(src, dst, term, lli, llt):
    return (6, dst, 0, lli, llt, src, term)


def vote_resp(src, dst, term):
    return (4, dst, src, term)


def append_req(src, dst, term, pli, plt, entries, lc):
    return (8, dst, entries, lc, pli, plt, src, term)


def append_resp(src, dst, term, pli, succ):
    return (6, dst, 1, pli, src, 1 if succ else 0, term)


def mtype(m) -> str:
    if m[0] == 4:
        return "VoteResp"
    if m[0] == 8:
        return "AppendReq"
    return "VoteReq" if m[2] == 0 else "AppendResp"


def mdst(m):
    return m[1]


def msrc(m):
    t = mtype(m)
    if t == "VoteResp":
        return m[2]
    if t == "VoteReq":
        return m[5]
    if t == "AppendResp":
        return m[4]
    return m[6]


def mterm(m):
    return m[-1] if mtype(m) != "VoteResp" else m[3]


def mfields(m) -> dict:
    """Record fields of message m (for printing / fixtures)."""
    t = mtype(m)
    if t == "VoteResp":
        return dict(type=t, src=m[2], dst=m[1], term=m[3])
    if t == "VoteReq":
        return dict(type=t, src=m[5], dst=m[1], term=m[6], lastLogIndex=m[3], lastLogTerm=m[4])
    if t == "AppendResp":
        return dict(type=t, src=m[4], dst=m[1], term=m[6], prevLogIndex=m[3], succ=bool(m[5]))
    return dict(type=t, src=m[6], dst=m[1], term=m[7], prevLogIndex=m[4], prevLogTerm=m[5],
                entries=[list(e) for e in m[2]], leaderCommit=m[3])


def permute_msg(m, pi):
    t = mtype(m)
    if t == "VoteResp":
        return (4, pi[m[1]], pi[m[2]], m[3])
    if t == "VoteReq":
        return (6, pi[m[1]], 0, m[3], m[4], pi[m[5]], m[6])
    if t == "AppendResp":
        return (6, pi[m[1]], 1, m[3], pi[m[4]], m[5], m[6])
    return (8, pi[m[1]], m[2], m[3], m[4], m[5], pi[m[6]], m[7])


# --------------------------------------------------------------------------- state
@dataclass(frozen=True)
class State:
    """The 12 variables in declaration order (tla:26,29,34)."""
    votedFor: tuple
    currentTerm: tuple
    logs: tuple          # tuple per server of tuple of (term, val)
    matchIndex: tuple    # [s][t]
    nextIndex: tuple     # [s][t]
    commitIndex: tuple
    msgs: frozenset
    role: tuple
    electionCount: int
    restartCount: int
    pendingResponse: tuple  # [s][p] bool
    valSent: tuple       # per value: NONE or 0 (FALSE)

    def view(self):
        """view == <<votedFor, currentTerm, logs, matchIndex, nextIndex, commitIndex, msgs, role>> (tla:38)."""
        return (self.votedFor, self.currentTerm, self.logs, self.matchIndex, self.nextIndex,
                self.commitIndex, tuple(sorted(self.msgs)), self.role)


@dataclass(frozen=True)
class Config:
    n: int = 3                 # |Servers|  (cfg:18)
    V: int = 2                 # |Vals|     (cfg:21)
    max_election: int = 3      # MaxElection (cfg:4)
    max_restart: int = 3       # MaxRestart  (cfg:3)
    invariants: Tuple[str, ...] = ("Inv",)   # cfg:33-34
    check_deadlock: bool = False             # myrun.sh passes -deadlock (run:3)
    seeded: bool = False       # RaftSeeded: Median threshold Cardinality(Servers)
    follower_append_entry: bool = False  # variant: tla:425's `\/ FollowerAppendEntry(s)` uncommented
    become_follower: bool = False  # variant: tla:420's `\/ BecomeFollower(s)` uncommented
    # test-only variants (tools/make_seeded_spec.py) that make TLC's two error kinds reachable in a BFS:
    split_brain: bool = False  # RaftSplitBrain: BecomeLeader's quorum (tla:164) is 1 -- two leaders of
    #                            one term, so UpdateTerm's Assert (tla:185) fails
    commit_past_log: bool = False  # RaftCommitPastLog: FollowerAcceptEntry's newCommitIndex (tla:294) is
    #                            Max(commitIndex, leaderCommit) -- commitIndex past the log, so Inv's
    #                            logs[p][index] (tla:499) is out of domain
    symmetry: bool = True      # SYMMETRY symmServers (cfg:24)
    view: bool = True          # VIEW view (cfg:26)

    @property
    def majority(self) -> int:
        # MajoritySize == Cardinality(Servers) \div 2 + 1   (tla:41)
        return self.n // 2 + 1


def init_state(cfg: Config) -> State:
    """Init (tla:93-105)."""
    n = cfg.n
    return State(
        votedFor=(NONE,) * n,
        currentTerm=(0,) * n,
        logs=(((0, NONE),),) * n,
        matchIndex=((1,) * n,) * n,
        nextIndex=((2,) * n,) * n,
        commitIndex=(1,) * n,
        msgs=frozenset(),
        role=(FOLLOWER,) * n,
        electionCount=0,
        restartCount=0,
        pendingResponse=((False,) * n,) * n,
        valSent=(NONE,) * cfg.V,
    )


def _set(t: tuple, i, v) -> tuple:
    lst = list(t)
    lst[i] = v
    return tuple(lst)


def _set2(t: tuple, i, j, v) -> tuple:
    return _set(t, i, _set(t[i], j, v))


class AssertionFailure(Exception):
    """TLC Assert(FALSE, "split brain") raised while expanding a state (tla:185)."""


class EvalError(Exception):
    """TLC evaluation error (e.g. tuple index out of domain in Inv, tla:499)."""


def median(cfg: Config, F: Sequence[int]) -> int:
    """Median(F) (tla:70-75): the smallest F[s] with |{p : F[p] <= F[s]}| >= threshold.

    The seeded variant uses Cardinality(Servers) as the threshold.
    """
    k = cfg.n if cfg.seeded else cfg.majority
    mset = [s for s in range(len(F)) if sum(1 for p in range(len(F)) if F[p] <= F[s]) >= k]
    return min(F[s] for s in mset)


# --------------------------------------------------------------------------- actions
# Each generator yields (witness, successor) in TLC enumeration order.

def become_candidate(cfg, st: State, s):
    """BecomeCandidate(s) (tla:107-130)."""
    if not (st.electionCount < cfg.max_election):
        return
    if st.role[s] not in (FOLLOWER, CANDIDATE):
        return
    lli = len(st.logs[s])
    llt = st.logs[s][lli - 1][0]
    term = st.currentTerm[s] + 1
    reqs = {vote_req(s, p, term, lli, llt) for p in range(cfg.n) if p != s}
    yield 0, State(
        votedFor=_set(st.votedFor, s, s),
        currentTerm=_set(st.currentTerm, s, term),
        logs=st.logs, matchIndex=st.matchIndex, nextIndex=st.nextIndex,
        commitIndex=st.commitIndex,
        msgs=st.msgs | reqs,
        role=_set(st.role, s, CANDIDATE),
        electionCount=st.electionCount + 1,
        restartCount=st.restartCount, pendingResponse=st.pendingResponse, valSent=st.valSent)


def update_term(cfg, st: State, s, msgs_sorted):
    """UpdateTerm(s) (tla:175-188); the Assert (tla:185) precedes the role guard."""
    for w, m in enumerate(msgs_sorted):
        if mdst(m) != s:
            continue
        if mterm(m) > st.currentTerm[s]:
            yield w, State(
                votedFor=_set(st.votedFor, s, NONE),
                currentTerm=_set(st.currentTerm, s, mterm(m)),
                logs=st.logs, matchIndex=st.matchIndex, nextIndex=st.nextIndex,
                commitIndex=st.commitIndex, msgs=st.msgs,
                role=_set(st.role, s, FOLLOWER),
                electionCount=st.electionCount, restartCount=st.restartCount,
                pendingResponse=st.pendingResponse, valSent=st.valSent)
        elif mterm(m) == st.currentTerm[s] and mtype(m) == "AppendReq":
            if st.role[s] == LEADER:
                raise AssertionFailure("split brain")
            if st.role[s] == CANDIDATE:
                yield w, State(
                    votedFor=st.votedFor, currentTerm=st.currentTerm, logs=st.logs,
                    matchIndex=st.matchIndex, nextIndex=st.nextIndex,
                    commitIndex=st.commitIndex, msgs=st.msgs,
                    role=_set(st.role, s, FOLLOWER),
                    electionCount=st.electionCount, restartCount=st.restartCount,
                    pendingResponse=st.pendingResponse, valSent=st.valSent)


def become_follower(cfg, st: State, s, msgs_sorted):
    r"""BecomeFollower(s) (tla:226-229) = FollowerUpdateTerm(s) (tla:191-197) \/ CandidateToFollower(s)
    (tla:200-212) \/ LeaderToFollower(s) (tla:215-223).  role[s] enables exactly one of the three,
    each an \E m \in msgs; no Assert here (the candidate's AppendReq case just steps down)."""
    r, ct = st.role[s], st.currentTerm[s]

    def succ(term, role, voted):
        return State(votedFor=_set(st.votedFor, s, voted), currentTerm=_set(st.currentTerm, s, term),
                     logs=st.logs, matchIndex=st.matchIndex, nextIndex=st.nextIndex,
                     commitIndex=st.commitIndex, msgs=st.msgs, role=_set(st.role, s, role),
                     electionCount=st.electionCount, restartCount=st.restartCount,
                     pendingResponse=st.pendingResponse, valSent=st.valSent)
    for w, m in enumerate(msgs_sorted):
        if mdst(m) != s:
            continue
        mt = mterm(m)
        if r == FOLLOWER:
            if mt > ct:  # FollowerUpdateTerm: votedFor and role unchanged
                yield w, succ(mt, FOLLOWER, st.votedFor[s])
        elif r == CANDIDATE:
            if mt > ct:
                yield w, succ(mt, FOLLOWER, NONE)
            elif mt == ct and mtype(m) == "AppendReq":
                yield w, succ(ct, FOLLOWER, st.votedFor[s])
        elif mt > ct:  # LeaderToFollower
            yield w, succ(mt, FOLLOWER, NONE)


def response_vote(cfg, st: State, s, msgs_sorted):
    """ResponseVote(s) (tla:132-155)."""
    if st.role[s] != FOLLOWER:
        return
    for w, m in enumerate(msgs_sorted):
        if mdst(m) != s or mtype(m) != "VoteReq" or mterm(m) != st.currentTerm[s]:
            continue
        f = mfields(m)
        if not (st.votedFor[s] == NONE or st.votedFor[s] == f["src"]):
            continue
        lli = len(st.logs[s])
        llt = st.logs[s][lli - 1][0]
        if not (f["lastLogTerm"] > llt or (f["lastLogTerm"] == llt and f["lastLogIndex"] >= lli)):
            continue
        grant = vote_resp(s, f["src"], f["term"])
        if grant in st.msgs:
            continue
        yield w, State(
            votedFor=_set(st.votedFor, s, f["src"]),
            currentTerm=st.currentTerm, logs=st.logs, matchIndex=st.matchIndex,
            nextIndex=st.nextIndex, commitIndex=st.commitIndex,
            msgs=st.msgs | {grant}, role=st.role,
            electionCount=st.electionCount, restartCount=st.restartCount,
            pendingResponse=st.pendingResponse, valSent=st.valSent)


def become_leader(cfg, st: State, s):
    """BecomeLeader(s) (tla:157-173)."""
    if st.role[s] != CANDIDATE:
        return
    resps = sum(1 for m in st.msgs
                if mdst(m) == s and mterm(m) == st.currentTerm[s] and mtype(m) == "VoteResp")
    if not (resps + 1 >= (1 if cfg.split_brain else cfg.majority)):
        return
    L = len(st.logs[s])
    yield 0, State(
        votedFor=st.votedFor, currentTerm=st.currentTerm, logs=st.logs,
        matchIndex=_set(st.matchIndex, s, tuple(1 if u != s else L for u in range(cfg.n))),
        nextIndex=_set(st.nextIndex, s, (L + 1,) * cfg.n),
        commitIndex=st.commitIndex, msgs=st.msgs,
        role=_set(st.role, s, LEADER),
        electionCount=st.electionCount, restartCount=st.restartCount,
        pendingResponse=_set(st.pendingResponse, s, (False,) * cfg.n),
        valSent=st.valSent)


def client_req(cfg, st: State, s):
    """ClientReq(s) (tla:233-240)."""
    if st.role[s] != LEADER:
        return
    for v in range(cfg.V):
        if st.valSent[v] != NONE:
            continue
        L = len(st.logs[s])
        yield v, State(
            votedFor=st.votedFor, currentTerm=st.currentTerm,
            logs=_set(st.logs, s, st.logs[s] + ((st.currentTerm[s], v),)),
            matchIndex=_set2(st.matchIndex, s, s, L + 1),
            nextIndex=st.nextIndex, commitIndex=st.commitIndex, msgs=st.msgs, role=st.role,
            electionCount=st.electionCount, restartCount=st.restartCount,
            pendingResponse=st.pendingResponse, valSent=_set(st.valSent, v, 0))


def leader_append_entry(cfg, st: State, s):
    """LeaderAppendEntry(s) (tla:242-269)."""
    if st.role[s] != LEADER:
        return
    log = st.logs[s]
    L = len(log)
    for dst in range(cfg.n):
        if dst == s:
            continue
        ni = st.nextIndex[s][dst]
        if not (ni <= L + 1):
            continue
        if st.pendingResponse[s][dst]:
            continue
        pli = ni - 1
        plt = log[pli - 1][0]
        entries = (log[ni - 1],) if ni <= L else ()
        m = append_req(s, dst, st.currentTerm[s], pli, plt, entries, st.commitIndex[s])
        if m in st.msgs:
            continue
        yield dst, State(
            votedFor=st.votedFor, currentTerm=st.currentTerm, logs=st.logs,
            matchIndex=st.matchIndex, nextIndex=st.nextIndex, commitIndex=st.commitIndex,
            msgs=st.msgs | {m}, role=st.role,
            electionCount=st.electionCount, restartCount=st.restartCount,
            pendingResponse=_set2(st.pendingResponse, s, dst, True), valSent=st.valSent)


def log_match(st: State, s, f) -> bool:
    """LogMatch(s, m) (tla:271-273), short-circuit conjunction."""
    log = st.logs[s]
    return f["prevLogIndex"] <= len(log) and f["prevLogTerm"] == log[f["prevLogIndex"] - 1][0]


def follower_accept_entry(cfg, st: State, s, msgs_sorted):
    """FollowerAcceptEntry(s) (tla:275-300); no \\notin guard on the response."""
    if st.role[s] != FOLLOWER:
        return
    for w, m in enumerate(msgs_sorted):
        if mdst(m) != s or mterm(m) != st.currentTerm[s] or mtype(m) != "AppendReq":
            continue
        f = mfields(m)
        if not log_match(st, s, f):
            continue
        ent = m[2]
        log = st.logs[s]
        resp = append_resp(s, f["src"], f["term"], f["prevLogIndex"] + len(ent), True)
        new_log = log[:f["prevLogIndex"]] + ent
        append_new = len(new_log) > len(log)
        truncated = len(new_log) <= len(log) and new_log != log[:len(new_log)]
        new_ci = max(st.commitIndex[s], f["leaderCommit"] if cfg.commit_past_log
                     else min(f["leaderCommit"], len(new_log)))
        updated = new_log if (truncated or append_new) else log
        yield w, State(
            votedFor=st.votedFor, currentTerm=st.currentTerm,
            logs=_set(st.logs, s, updated),
            matchIndex=st.matchIndex, nextIndex=st.nextIndex,
            commitIndex=_set(st.commitIndex, s, new_ci),
            msgs=st.msgs | {resp}, role=st.role,
            electionCount=st.electionCount, restartCount=st.restartCount,
            pendingResponse=st.pendingResponse, valSent=st.valSent)


# how often FollowerAppendEntry reached its closing UNCHANGED (tla:371): the variant test uses it
# to show the check is exercised, not vacuous
FAPP_STATS = {"reached_unchanged": 0, "enabled": 0}


def follower_append_entry(cfg, st: State, s, msgs_sorted):
    """FollowerAppendEntry(s) (tla:323-371), commented out of Next at tla:425.

    Restated as TLC evaluates the conjunction left to right: each IF/ELSE branch assigns
    commitIndex' (IF only), logs' and msgs' (SendMsg, tla:77-78), and the action's last
    top-level conjunct, tla:371's UNCHANGED << votedFor, currentTerm, msgs, matchIndex,
    nextIndex, commitIndex, logs, ... >>, then *tests* msgs' = msgs, commitIndex' =
    commitIndex and logs' = logs.  The ELSE branch requires resp \notin msgs (so msgs'
    differs); the IF branch requires resp \notin msgs or a larger commitIndex (so msgs' or
    commitIndex' differs): the action is never enabled, and the variant's state graph is
    Raft.tla's."""
    if st.role[s] != FOLLOWER:
        return
    for w, m in enumerate(msgs_sorted):
        if mdst(m) != s or mterm(m) != st.currentTerm[s] or mtype(m) != "AppendReq":
            continue
        f = mfields(m)
        log, ci = st.logs[s], st.commitIndex[s]
        if log_match(st, s, f):
            ent = m[2]
            resp = append_resp(s, f["src"], f["term"], f["prevLogIndex"] + len(ent), True)
            new_log = log[:f["prevLogIndex"]] + ent
            new_ci = max(ci, min(f["leaderCommit"], len(new_log)))
            if not (resp not in st.msgs or new_ci > ci):
                continue
            append_new = len(new_log) > len(log)
            truncated = len(new_log) <= len(log) and new_log != log[:len(new_log)]
            logs2, ci2 = (new_log if (append_new or truncated) else log), new_ci
        else:
            resp = append_resp(s, f["src"], f["term"], f["prevLogIndex"] - 1, False)
            if resp in st.msgs:
                continue
            logs2, ci2 = log, ci
        msgs2 = st.msgs | {resp}
        FAPP_STATS["reached_unchanged"] += 1
        if msgs2 != st.msgs or ci2 != ci or logs2 != log:  # tla:371
            continue
        FAPP_STATS["enabled"] += 1
        yield w, st


def follower_reject_entry(cfg, st: State, s, msgs_sorted):
    """FollowerRejectEntry(s) (tla:302-321)."""
    if st.role[s] != FOLLOWER:
        return
    for w, m in enumerate(msgs_sorted):
        if mdst(m) != s or mterm(m) != st.currentTerm[s] or mtype(m) != "AppendReq":
            continue
        f = mfields(m)
        if log_match(st, s, f):
            continue
        resp = append_resp(s, f["src"], f["term"], f["prevLogIndex"], False)
        if resp in st.msgs:
            continue
        yield w, State(
            votedFor=st.votedFor, currentTerm=st.currentTerm, logs=st.logs,
            matchIndex=st.matchIndex, nextIndex=st.nextIndex, commitIndex=st.commitIndex,
            msgs=st.msgs | {resp}, role=st.role,
            electionCount=st.electionCount, restartCount=st.restartCount,
            pendingResponse=st.pendingResponse, valSent=st.valSent)


def handle_append_resp(cfg, st: State, s, msgs_sorted):
    """HandleAppendResp(s) (tla:374-396)."""
    if st.role[s] != LEADER:
        return
    for w, m in enumerate(msgs_sorted):
        if mtype(m) != "AppendResp" or mdst(m) != s or mterm(m) != st.currentTerm[s]:
            continue
        f = mfields(m)
        src = f["src"]
        if not st.pendingResponse[s][src]:
            continue
        if f["succ"]:
            if not (st.matchIndex[s][src] < f["prevLogIndex"]):
                continue
            yield w, State(
                votedFor=st.votedFor, currentTerm=st.currentTerm, logs=st.logs,
                matchIndex=_set2(st.matchIndex, s, src, f["prevLogIndex"]),
                nextIndex=_set2(st.nextIndex, s, src, f["prevLogIndex"] + 1),
                commitIndex=st.commitIndex, msgs=st.msgs, role=st.role,
                electionCount=st.electionCount, restartCount=st.restartCount,
                pendingResponse=_set2(st.pendingResponse, s, src, False), valSent=st.valSent)
        else:
            if not (f["prevLogIndex"] + 1 == st.nextIndex[s][src]):
                continue
            if not (f["prevLogIndex"] > st.matchIndex[s][src]):
                continue
            yield w, State(
                votedFor=st.votedFor, currentTerm=st.currentTerm, logs=st.logs,
                matchIndex=st.matchIndex,
                nextIndex=_set2(st.nextIndex, s, src, f["prevLogIndex"]),
                commitIndex=st.commitIndex, msgs=st.msgs, role=st.role,
                electionCount=st.electionCount, restartCount=st.restartCount,
                pendingResponse=_set2(st.pendingResponse, s, src, False), valSent=st.valSent)


def leader_can_commit(cfg, st: State, s):
    """LeaderCanCommit(s) (tla:398-407)."""
    if st.role[s] != LEADER:
        return
    med = median(cfg, st.matchIndex[s])
    if not (med > st.commitIndex[s]):
        return
    yield 0, State(
        votedFor=st.votedFor, currentTerm=st.currentTerm, logs=st.logs,
        matchIndex=st.matchIndex, nextIndex=st.nextIndex,
        commitIndex=_set(st.commitIndex, s, med), msgs=st.msgs, role=st.role,
        electionCount=st.electionCount, restartCount=st.restartCount,
        pendingResponse=st.pendingResponse, valSent=st.valSent)


def restart(cfg, st: State, s):
    """Restart(s) (tla:409-414)."""
    if st.role[s] != LEADER or not (st.restartCount < cfg.max_restart):
        return
    yield 0, State(
        votedFor=st.votedFor, currentTerm=st.currentTerm, logs=st.logs,
        matchIndex=st.matchIndex, nextIndex=st.nextIndex, commitIndex=st.commitIndex,
        msgs=st.msgs, role=_set(st.role, s, FOLLOWER),
        electionCount=st.electionCount, restartCount=st.restartCount + 1,
        pendingResponse=st.pendingResponse, valSent=st.valSent)


def successor_batches(cfg: Config, st: State):
    """Next (tla:416-430) in TLC enumeration order, one batch per sub-action.

    Yields (server, action, [(witness, successor), ...]) for the n*11 sub-actions
    in order (server-major, then the disjuncts of Next in textual order).  The
    witness is the index into sorted(msgs) for message actions, the value index for
    ClientReq, the destination server for LeaderAppendEntry and 0 otherwise.
    TLC's getNextStates evaluates a whole sub-action before any of its successors
    is fingerprinted, so an Assert inside UpdateTerm(s) (tla:185) raises
    AssertionFailure before that sub-action's batch is yielded.
    """
    msgs_sorted = sorted(st.msgs)
    for s in range(cfg.n):
        gens = (
            (A_BC, lambda: become_candidate(cfg, st, s)),
            (A_UT, lambda: update_term(cfg, st, s, msgs_sorted)),
            # variant only (tla:420)
            (A_BF, lambda: become_follower(cfg, st, s, msgs_sorted)),
            (A_RV, lambda: response_vote(cfg, st, s, msgs_sorted)),
            (A_BL, lambda: become_leader(cfg, st, s)),
            (A_CR, lambda: client_req(cfg, st, s)),
            (A_LAE, lambda: leader_append_entry(cfg, st, s)),
            # variant only (tla:425); never enabled, so its key index (A_FAPP) never appears
            (A_FAPP, lambda: follower_append_entry(cfg, st, s, msgs_sorted)),
            (A_FAE, lambda: follower_accept_entry(cfg, st, s, msgs_sorted)),
            (A_FRE, lambda: follower_reject_entry(cfg, st, s, msgs_sorted)),
            (A_HAR, lambda: handle_append_resp(cfg, st, s, msgs_sorted)),
            (A_LCC, lambda: leader_can_commit(cfg, st, s)),
            (A_RS, lambda: restart(cfg, st, s)),
        )
        for a, mk in gens:
            if (a == A_FAPP and not cfg.follower_append_entry) or (a == A_BF and not cfg.become_follower):
                continue
            yield s, a, list(mk())


def successors(cfg: Config, st: State) -> List[Tuple[Tuple[int, int, int], State]]:
    """All successors of st as ((server, action, witness), state), keys increasing."""
    out = []
    for s, a, batch in successor_batches(cfg, st):
        out.extend(((s, a, w), t) for w, t in batch)
    return out


# --------------------------------------------------------------------------- invariants
def inv_leader_has_all_committed(cfg: Config, st: State) -> bool:
    """LeaderHasAllCommittedEntries (tla:491-499) with TLC's left-to-right short-circuit.

    Raises EvalError where TLC would hit ``logs[p][index]`` out of domain (tla:499).
    """
    n = cfg.n
    if not any(st.role[p] == LEADER for p in range(n)):
        return True
    for l in range(n):
        if st.role[l] != LEADER:
            continue
        found_bad = False
        for p in range(n):
            if p == l:
                continue
            if not (st.currentTerm[p] <= st.currentTerm[l]):
                continue
            ll = len(st.logs[l])
            if st.commitIndex[p] > ll:
                found_bad = True
                break
            # commitIndex[p] <= Len(logs[l])
            bad = False
            for index in range(1, st.commitIndex[p] + 1):
                if index > len(st.logs[p]):
                    raise EvalError(f"logs[{p}][{index}] out of domain")
                if st.logs[p][index - 1] != st.logs[l][index - 1]:
                    bad = True
                    break
            if bad:
                found_bad = True
                break
        if not found_bad:
            return True
    return False


def inv_no_split_vote(cfg, st):
    """NoSplitVote (tla:444-448)."""
    n = cfg.n
    return not any(a != b and st.currentTerm[a] == st.currentTerm[b] and
                   st.role[a] == LEADER and st.role[b] == LEADER
                   for a in range(n) for b in range(n))


def inv_raft_can_commit(cfg, st):
    """RaftCanCommt (tla:434)."""
    return any(st.commitIndex[s] > 1 for s in range(cfg.n))


def inv_follower_can_commit(cfg, st):
    """FollowerCanCommit (tla:436-439)."""
    return any(st.role[s] == FOLLOWER and st.commitIndex[s] > 1 for s in range(cfg.n))


def inv_commit_all(cfg, st):
    """CommitAll (tla:442)."""
    return all(st.commitIndex[s] == 3 for s in range(cfg.n))


def inv_exist_leader_and_candidate(cfg, st):
    """ExistLeaderAndCandidate (tla:483-487)."""
    n = cfg.n
    return any(a != b and st.role[a] == LEADER and st.role[b] == CANDIDATE
               for a in range(n) for b in range(n))


def inv_no_all_commit(cfg, st):
    """NoAllCommit (tla:451-481)."""
    n = cfg.n
    for s1, s2, s3 in itertools.product(range(n), repeat=3):
        if not (s1 != s2 and s2 != s3 and st.role[s1] == LEADER and st.role[s2] == FOLLOWER
                and st.role[s3] == FOLLOWER and st.currentTerm[s1] == st.currentTerm[s3]
                and st.commitIndex[s1] == 2 and st.commitIndex[s2] == 2
                and st.commitIndex[s3] == 1 and st.matchIndex[s1][s2] == 2
                and st.matchIndex[s1][s3] == 2):
            continue
        fs = [mfields(m) for m in st.msgs]
        c1 = any(f["dst"] == s3 and f["src"] == s1 and f["term"] == st.currentTerm[s3]
                 and f["type"] == "AppendReq" and f["prevLogIndex"] == 1 for f in fs)
        c2 = any(f["dst"] == s1 and f["src"] == s3 and f["term"] == st.currentTerm[s3]
                 and f["type"] == "AppendResp" and f["prevLogIndex"] == 1 and f["succ"] for f in fs)
        c3 = any(f["dst"] == s3 and f["src"] == s1 and f["type"] == "AppendReq"
                 and f["prevLogIndex"] == 2 for f in fs)
        if c1 and c2 and c3:
            return True
    return False


INV_FUNCS = {
    "Inv": inv_leader_has_all_committed,   # Inv == LeaderHasAllCommittedEntries (tla:502-503)
    "LeaderHasAllCommittedEntries": inv_leader_has_all_committed,
    "NoSplitVote": inv_no_split_vote,
    "RaftCanCommt": inv_raft_can_commit,
    "FollowerCanCommit": inv_follower_can_commit,
    "CommitAll": inv_commit_all,
    "NoAllCommit": inv_no_all_commit,
    "ExistLeaderAndCandidate": inv_exist_leader_and_candidate,
}


# --------------------------------------------------------------------------- symmetry
def permute_view(view, pi):
    """Apply server permutation pi (old index -> new index) to a view tuple (tla:21,38).

    Vals are not permuted (cfg:28 is commented out)."""
    votedFor, currentTerm, logs, matchIndex, nextIndex, commitIndex, msgs, role = view
    n = len(votedFor)
    inv = [0] * n
    for i in range(n):
        inv[pi[i]] = i
    return (
        tuple(NONE if votedFor[inv[k]] == NONE else pi[votedFor[inv[k]]] for k in range(n)),
        tuple(currentTerm[inv[k]] for k in range(n)),
        tuple(logs[inv[k]] for k in range(n)),
        tuple(tuple(matchIndex[inv[k]][inv[l]] for l in range(n)) for k in range(n)),
        tuple(tuple(nextIndex[inv[k]][inv[l]] for l in range(n)) for k in range(n)),
        tuple(commitIndex[inv[k]] for k in range(n)),
        tuple(sorted(permute_msg(m, pi) for m in msgs)),
        tuple(role[inv[k]] for k in range(n)),
    )


def canonical(cfg: Config, st: State):
    """Distinct-state identity: the orbit of view (tla:38) under Permutations(Servers).

    TLC fingerprints VIEW(min_pi pi(state)); since the view is exactly the first 8
    declared variables (tla:26,29) the fingerprint classes are the view orbits for
    any total order.  We use Python's tuple order.
    """
    if cfg.view:
        v = st.view()
    else:
        v = st.view() + (st.electionCount, st.restartCount, st.pendingResponse, st.valSent)
    if not cfg.symmetry:
        return v
    if not cfg.view:
        raise NotImplementedError("symmetry without view")
    return min(permute_view(v, pi) for pi in itertools.permutations(range(cfg.n)))


# --------------------------------------------------------------------------- BFS (TLC)
@dataclass
class Result:
    verdict: str                       # "ok" | "invariant" | "assert" | "eval_error" | "deadlock"
    generated: int
    distinct: int
    depth: int
    levels: List[int] = field(default_factory=list)          # distinct states per level
    generated_per_level: List[int] = field(default_factory=list)  # successors generated by expanding level L
    violated: Optional[str] = None
    trace: Optional[List[Tuple[Optional[Tuple[int, int, int]], State]]] = None
    queue_left: int = 0
    states: Optional[List[State]] = None   # every distinct state in discovery order (keep_states=True)
    state_levels: Optional[List[int]] = None


def bfs(cfg: Config, max_states: Optional[int] = None, order: str = "tlc", seed: int = 0,
        keep_states: bool = False) -> Result:
    """TLC breadth-first search with -workers 1 discovery order (first-wins per fingerprint).

    ``order="shuffle"`` permutes the successors of every state with a fixed seed: the
    order-sensitivity probe of SURVEY App. D.2.
    """
    import random
    rng = random.Random(seed)
    inv_names = list(cfg.invariants)
    s0 = init_state(cfg)
    seen: Dict[object, int] = {}
    # per state: (parent id, key, state)
    parent: List[int] = []
    keys: List[Optional[Tuple[int, int, int]]] = []
    states: List[State] = []
    levels_of: List[int] = []

    def trace_of(i):
        out = []
        while i >= 0:
            out.append((keys[i], states[i]))
            i = parent[i]
        return list(reversed(out))

    generated = 1  # TLC counts the initial state as generated
    seen[canonical(cfg, s0)] = 0
    parent.append(-1)
    keys.append(None)
    states.append(s0)
    levels_of.append(1)
    levels = [1]
    gen_per_level: List[int] = []

    def check(i) -> Optional[str]:
        for name in inv_names:
            if not INV_FUNCS[name](cfg, states[i]):
                return name
        return None

    try:
        bad = check(0)
    except EvalError:
        return Result("eval_error", generated, 1, 1, levels, gen_per_level, trace=trace_of(0))
    if bad:
        return Result("invariant", generated, 1, 1, levels, gen_per_level, violated=bad,
                      trace=trace_of(0))

    queue = deque([0])
    cur_level = 1
    while queue:
        i = queue.popleft()
        lvl = levels_of[i]
        if lvl != cur_level:
            cur_level = lvl
        while len(gen_per_level) < lvl:
            gen_per_level.append(0)
        st = states[i]
        if order == "shuffle":
            try:
                succ = successors(cfg, st)
            except AssertionFailure:
                return Result("assert", generated, len(states), max(levels_of), levels,
                              gen_per_level, trace=trace_of(i), queue_left=len(queue))
            rng.shuffle(succ)
            batches = [succ]
        else:
            batches = None
        n_succ = 0
        it = iter(batches) if batches is not None else (
            [((s, a, w), t) for w, t in b] for s, a, b in successor_batches(cfg, st))
        while True:
            try:
                batch = next(it)
            except StopIteration:
                break
            except AssertionFailure:
                return Result("assert", generated, len(states), max(levels_of), levels,
                              gen_per_level, trace=trace_of(i), queue_left=len(queue))
            # TLC adds a sub-action's whole batch to "states generated" before
            # fingerprinting any of it.
            generated += len(batch)
            gen_per_level[lvl - 1] += len(batch)
            n_succ += len(batch)
            for key, t in batch:
                c = canonical(cfg, t)
                if c in seen:
                    continue
                j = len(states)
                seen[c] = j
                parent.append(i)
                keys.append(key)
                states.append(t)
                levels_of.append(lvl + 1)
                if len(levels) < lvl + 1:
                    levels.append(0)
                levels[lvl] += 1
                try:
                    bad = check(j)
                except EvalError:
                    return Result("eval_error", generated, len(states), lvl + 1, levels,
                                  gen_per_level, trace=trace_of(j), queue_left=len(queue))
                if bad:
                    return Result("invariant", generated, len(states), lvl + 1, levels,
                                  gen_per_level, violated=bad, trace=trace_of(j),
                                  queue_left=len(queue))
                queue.append(j)
                if max_states is not None and len(states) >= max_states:
                    raise RuntimeError(f"state budget {max_states} exceeded")
        if n_succ == 0 and cfg.check_deadlock:
            return Result("deadlock", generated, len(states), max(levels_of), levels,
                          gen_per_level, trace=trace_of(i), queue_left=len(queue))
    r = Result("ok", generated, len(states), len(levels), levels, gen_per_level)
    if keep_states:
        r.states, r.state_levels = states, levels_of
    return r


# --------------------------------------------------------------------------- fixtures
def state_to_json(st: State) -> dict:
    return dict(
        votedFor=list(st.votedFor), currentTerm=list(st.currentTerm),
        logs=[[list(e) for e in log] for log in st.logs],
        matchIndex=[list(r) for r in st.matchIndex], nextIndex=[list(r) for r in st.nextIndex],
        commitIndex=list(st.commitIndex),
        msgs=[mfields(m) for m in sorted(st.msgs)],
        role=list(st.role), electionCount=st.electionCount, restartCount=st.restartCount,
        pendingResponse=[[bool(x) for x in r] for r in st.pendingResponse],
        valSent=list(st.valSent))


def msg_from_json(f: dict):
    t = f["type"]
    if t == "VoteResp":
        return vote_resp(f["src"], f["dst"], f["term"])
    if t == "VoteReq":
        return vote_req(f["src"], f["dst"], f["term"], f["lastLogIndex"], f["lastLogTerm"])
    if t == "AppendResp":
        return append_resp(f["src"], f["dst"], f["term"], f["prevLogIndex"], f["succ"])
    return append_req(f["src"], f["dst"], f["term"], f["prevLogIndex"], f["prevLogTerm"],
                      tuple(tuple(e) for e in f["entries"]), f["leaderCommit"])


def state_from_json(d: dict) -> State:
    return State(
        votedFor=tuple(d["votedFor"]), currentTerm=tuple(d["currentTerm"]),
        logs=tuple(tuple(tuple(e) for e in log) for log in d["logs"]),
        matchIndex=tuple(tuple(r) for r in d["matchIndex"]),
        nextIndex=tuple(tuple(r) for r in d["nextIndex"]),
        commitIndex=tuple(d["commitIndex"]),
        msgs=frozenset(msg_from_json(f) for f in d["msgs"]),
        role=tuple(d["role"]), electionCount=d["electionCount"], restartCount=d["restartCount"],
        pendingResponse=tuple(tuple(bool(x) for x in r) for r in d["pendingResponse"]),
        valSent=tuple(d["valSent"]))


if __name__ == "__main__":  # pragma: no cover - manual exploration helper
    import argparse
    import time
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3)
    ap.add_argument("--V", type=int, default=1)
    ap.add_argument("--E", type=int, default=2)
    ap.add_argument("--R", type=int, default=3)
    ap.add_argument("--seeded", action="store_true")
    ap.add_argument("--shuffle", action="store_true")
    a = ap.parse_args()
    c = Config(n=a.n, V=a.V, max_election=a.E, max_restart=a.R, seeded=a.seeded)
    t0 = time.time()
    r = bfs(c, order="shuffle" if a.shuffle else "tlc")
    dt = time.time() - t0
    print(f"verdict={r.verdict} violated={r.violated} generated={r.generated} distinct={r.distinct} "
          f"depth={r.depth} time={dt:.1f}s ({r.distinct / max(dt, 1e-9):.0f} states/s)")
    print("levels", r.levels)
    print("gen/level", r.generated_per_level)
    if r.trace:
        print("trace length", len(r.trace))
