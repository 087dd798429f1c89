#!/usr/bin/env python3
"""Derive the FollowerAppendEntry variant of kikimo/tla-raft's Raft.tla:
Next's commented-out disjunct `\\* \\/ FollowerAppendEntry(s)` (Raft.tla:425) uncommented, the
edit a maintainer would make in place.  Module name and everything else unchanged.

As TLC evaluates it the action is never enabled (its closing UNCHANGED, Raft.tla:371, tests
msgs' = msgs after its own SendMsg; oracle/raft_ref.py:follower_append_entry), so the variant's
state graph is Raft.tla's: the launcher recognises this text by content hash (rmc_cfg.cpp) and
runs the Raft.tla model on it.

Usage: make_variant_spec.py /path/to/Raft.tla > Raft.tla
"""
import sys

OLD = "    \\* \\/ FollowerAppendEntry(s)\n"
NEW = "    \\/ FollowerAppendEntry(s)\n"


def follower_append_entry(text: str) -> str:
    text = text.replace("\r\n", "\n")
    if text.count(OLD) != 1 or " MODULE Raft " not in text.splitlines()[0]:
        raise SystemExit("input is not kikimo/tla-raft's Raft.tla")
    return text.replace(OLD, NEW)


if __name__ == "__main__":
    sys.stdout.write(follower_append_entry(open(sys.argv[1], encoding="utf-8").read()))
