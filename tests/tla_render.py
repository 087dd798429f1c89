"""TLA+ value syntax for oracle states (test helper): how TLC prints a behavior's states.

Written for the tests from TLC's printing conventions, independently of the
launcher's printer (tla-raft_amd/launcher/raftmc.cpp): functions over Servers as
``(s1 :> x @@ s2 :> y)``, records with their fields in name order ``[f |-> v, ...]``, sequences
``<< ... >>``, sets ``{ ... }`` in TLC's value order (the fixtures already list msgs in it),
booleans TRUE/FALSE, model values by name."""

ROLE = ["Follower", "Candidate", "Leader"]


def render_state(st, servers, vals):
    n = len(st["currentTerm"])

    def sv(i):
        return "None" if i < 0 else servers[i]

    def fn(xs):
        return "(" + " @@ ".join(f"{servers[i]} :> {xs[i]}" for i in range(n)) + ")"

    def entry(t, v):
        return f"[term |-> {t}, val |-> {'None' if v < 0 else vals[v]}]"

    def rec(fields):
        return "[" + ", ".join(f"{k} |-> {v}" for k, v in sorted(fields.items())) + "]"

    def msg(m):
        f = {"dst": sv(m["dst"]), "src": sv(m["src"]), "term": m["term"], "type": m["type"]}
        if m["type"] == "VoteReq":
            f.update(lastLogIndex=m["lastLogIndex"], lastLogTerm=m["lastLogTerm"])
        elif m["type"] == "AppendResp":
            f.update(prevLogIndex=m["prevLogIndex"], succ="TRUE" if m["succ"] else "FALSE")
        elif m["type"] == "AppendReq":
            e = m["entries"]
            f.update(prevLogIndex=m["prevLogIndex"], prevLogTerm=m["prevLogTerm"], leaderCommit=m["leaderCommit"],
                     entries="<<" + (entry(e[0][0], e[0][1]) if e else "") + ">>")
        return rec(f)

    logs = ["<<" + ", ".join(entry(t, v) for t, v in log) + ">>" for log in st["logs"]]
    mat = lambda M, b=False: fn([fn([("TRUE" if x else "FALSE") if b else x for x in row]) for row in M])
    vs = "(" + " @@ ".join(f"{vals[v]} :> {'None' if x < 0 else 'FALSE'}" for v, x in enumerate(st["valSent"])) + ")"
    return [
        "/\\ votedFor = " + fn([sv(x) for x in st["votedFor"]]),
        "/\\ currentTerm = " + fn(st["currentTerm"]),
        "/\\ logs = " + fn(logs),
        "/\\ matchIndex = " + mat(st["matchIndex"]),
        "/\\ nextIndex = " + mat(st["nextIndex"]),
        "/\\ commitIndex = " + fn(st["commitIndex"]),
        "/\\ msgs = {" + ", ".join(msg(m) for m in st["msgs"]) + "}",
        "/\\ role = " + fn([ROLE[r] for r in st["role"]]),
        "/\\ electionCount = " + str(st["electionCount"]),
        "/\\ restartCount = " + str(st["restartCount"]),
        "/\\ pendingResponse = " + mat(st["pendingResponse"], True),
        "/\\ valSent = " + vs,
    ]
