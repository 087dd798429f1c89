#!/usr/bin/env python3
"""Derive RaftSeeded.tla (the seeded-violation variant, SURVEY.md App. B / BASELINE config 5)
from a user-supplied Raft.tla.

The variant changes exactly two things in kikimo/tla-raft's Raft.tla:
  * the module name (line 1), so TLC accepts the file name RaftSeeded.tla;
  * Median's threshold (Raft.tla:72) ``>= MajoritySize`` -> ``>= Cardinality(Servers)``,
    i.e. a leader may commit an entry that only it holds (for 3 servers this is the
    commented ``pos == Len(mlist) \\div 2`` mistake of Raft.tla:65-66).

Usage: make_seeded_spec.py /path/to/Raft.tla > RaftSeeded.tla
The launcher recognises the output by content hash (rmc_cfg.cpp).

Two further test-only variants (--split-brain / --commit-past-log) make TLC's other two error kinds
reachable in a breadth-first search -- the shipped specs reach neither -- so their precedence in a
BFS and TLC's counters at them are tested end to end (both oracles implement them):

  RaftSplitBrain     BecomeLeader's guard (Raft.tla:164) ``Cardinality(resps) + 1 >= 1``: two
                     candidates of one term both lead, and the AppendReq one sends the other fails
                     UpdateTerm's Assert (Raft.tla:185).
  RaftCommitPastLog  FollowerAcceptEntry's newCommitIndex (Raft.tla:294) ``Max(commitIndex[s],
                     m.leaderCommit)``: a follower's commitIndex passes its log, and Inv's
                     ``logs[p][index]`` (Raft.tla:499) is applied out of its domain.

Usage: make_seeded_spec.py [--split-brain | --commit-past-log] /path/to/Raft.tla > RaftSeeded.tla
"""
import sys

MEDIAN_OLD = "Cardinality({ p \\in DOMAIN F : F[p] <= F[s] }) >= MajoritySize }"
MEDIAN_NEW = "Cardinality({ p \\in DOMAIN F : F[p] <= F[s] }) >= Cardinality(Servers) }"


QUORUM_OLD = "/\\ Cardinality(resps) + 1 >= MajoritySize"
QUORUM_NEW = "/\\ Cardinality(resps) + 1 >= 1"
COMMIT_OLD = "newCommitIndex == Max(commitIndex[s], Min(m.leaderCommit, Len(newLog)))"
COMMIT_NEW = "newCommitIndex == Max(commitIndex[s], m.leaderCommit)"


def _variant(text: str, module: str, old: str, new: str, count: int) -> str:
    text = text.replace("\r\n", "\n")
    if text.count(old) != count or " MODULE Raft " not in text.splitlines()[0]:
        raise SystemExit("input is not kikimo/tla-raft's Raft.tla")
    lines = text.split("\n")
    lines[0] = lines[0].replace(" MODULE Raft ", f" MODULE {module} ", 1)
    return "\n".join(lines).replace(old, new, 1)  # (the first: FollowerAcceptEntry's, tla:294)


def split_brain(text: str) -> str:
    return _variant(text, "RaftSplitBrain", QUORUM_OLD, QUORUM_NEW, 1)


def commit_past_log(text: str) -> str:
    return _variant(text, "RaftCommitPastLog", COMMIT_OLD, COMMIT_NEW, 2)


def seeded(text: str) -> str:
    text = text.replace("\r\n", "\n")
    if text.count(MEDIAN_OLD) != 1 or " MODULE Raft " not in text.splitlines()[0]:
        raise SystemExit("input is not kikimo/tla-raft's Raft.tla")
    lines = text.split("\n")
    lines[0] = lines[0].replace(" MODULE Raft ", " MODULE RaftSeeded ", 1)
    return "\n".join(lines).replace(MEDIAN_OLD, MEDIAN_NEW)


if __name__ == "__main__":
    path = [a for a in sys.argv[1:] if not a.startswith("--")][0]
    text = open(path, encoding="utf-8").read()
    if "--split-brain" in sys.argv[1:]:
        sys.stdout.write(split_brain(text))
    elif "--commit-past-log" in sys.argv[1:]:
        sys.stdout.write(commit_past_log(text))
    else:
        sys.stdout.write(seeded(text))
