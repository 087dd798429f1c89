#!/usr/bin/env python3
"""Derive the Next variants of kikimo/tla-raft's Raft.tla: one of Next's
commented-out disjuncts uncommented, the edit a maintainer would make in place.  Module name and
everything else unchanged.

  (default)          `\\* \\/ FollowerAppendEntry(s)` (Raft.tla:425)
  --become-follower  `\\* \\/ BecomeFollower(s)` (Raft.tla:420): FollowerUpdateTerm /
                     CandidateToFollower / LeaderToFollower (tla:190-229) join Next right after
                     UpdateTerm; the launcher runs it as RMC_SPEC_BECOME_FOLLOWER

As TLC evaluates it the action is never enabled (its closing UNCHANGED, Raft.tla:371, tests
msgs' = msgs after its own SendMsg; oracle/raft_ref.py:follower_append_entry), so the variant's
state graph is Raft.tla's: the launcher recognises this text by content hash (rmc_cfg.cpp) and
runs the Raft.tla model on it.

Usage: make_variant_spec.py [--become-follower] /path/to/Raft.tla > Raft.tla
"""
import sys

OLD = "    \\* \\/ FollowerAppendEntry(s)\n"
NEW = "    \\/ FollowerAppendEntry(s)\n"
OLD_BF = "    \\* \\/ BecomeFollower(s)           \n"
NEW_BF = "    \\/ BecomeFollower(s)           \n"


def _uncomment(text: str, old: str, new: str) -> str:
    text = text.replace("\r\n", "\n")
    if text.count(old) != 1 or " MODULE Raft " not in text.splitlines()[0]:
        raise SystemExit("input is not kikimo/tla-raft's Raft.tla")
    return text.replace(old, new)


def follower_append_entry(text: str) -> str:
    return _uncomment(text, OLD, NEW)


def become_follower(text: str) -> str:
    return _uncomment(text, OLD_BF, NEW_BF)


if __name__ == "__main__":
    bf = "--become-follower" in sys.argv[1:]
    path = [a for a in sys.argv[1:] if not a.startswith("--")][0]
    text = open(path, encoding="utf-8").read()
    sys.stdout.write(become_follower(text) if bf else follower_append_entry(text))
