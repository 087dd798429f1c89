#!/bin/bash
# Drop-in for kikimo/tla-raft's myrun.sh (myrun.sh:3): same flags, same inputs
# (Raft.tla, Raft.cfg in the current directory), TLC-style output teed to raft.log --
# the state space is explored on the MI355X by librmc instead of TLC.
DIR=$(cd "$(dirname "$0")" && pwd)
"$DIR/build/raftmc" -deadlock -workers 4 -config Raft.cfg Raft.tla $@ 2>&1 | tee raft.log
