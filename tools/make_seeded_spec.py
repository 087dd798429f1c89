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
"""
import sys

MEDIAN_OLD = "Cardinality({ p \\in DOMAIN F : F[p] <= F[s] }) >= MajoritySize }"
MEDIAN_NEW = "Cardinality({ p \\in DOMAIN F : F[p] <= F[s] }) >= Cardinality(Servers) }"


def seeded(text: str) -> str:
    text = text.replace("\r\n", "\n")
    if text.count(MEDIAN_OLD) != 1 or " MODULE Raft " not in text.splitlines()[0]:
        raise SystemExit("input is not kikimo/tla-raft's Raft.tla")
    lines = text.split("\n")
    lines[0] = lines[0].replace(" MODULE Raft ", " MODULE RaftSeeded ", 1)
    return "\n".join(lines).replace(MEDIAN_OLD, MEDIAN_NEW)


if __name__ == "__main__":
    sys.stdout.write(seeded(open(sys.argv[1], encoding="utf-8").read()))
