// rmc_cfg.cpp -- TLC model-config parser (the subset Raft.cfg uses) and spec identification.
//
// Replaces, for this one spec, TLC's ModelConfig (Raft.cfg:1-34) and SANY (Raft.tla):
// the transition relation is compiled ahead of time, so Raft.tla is only identified
// by content (FNV-1a 64 of the text with CRLF normalised) -- the shipped Raft.tla or
// the seeded variant produced by tools/make_seeded_spec.py.  Pure CPU code.
#include "rmc_cfg.h"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>

namespace rmc {

static const uint64_t FNV_RAFT = 0x0a385fb43445e617ULL;         // kikimo/tla-raft Raft.tla
static const uint64_t FNV_RAFT_SEEDED = 0xc2b84ca613379636ULL;  // tools/make_seeded_spec.py output
// Raft.tla with Next's `\/ FollowerAppendEntry(s)` uncommented (tla:425; tools/make_variant_spec.py).
// The action is never enabled as TLC evaluates it (its closing UNCHANGED, tla:371, tests msgs' =
// msgs after its own SendMsg; oracle/raft_ref.py:follower_append_entry), so this text runs the
// Raft.tla model unchanged.
static const uint64_t FNV_RAFT_FAPP = 0x1319b28a1b001651ULL;
// Raft.tla with Next's `\/ BecomeFollower(s)` uncommented (tla:420; tools/make_variant_spec.py
// --become-follower): RMC_SPEC_BECOME_FOLLOWER.
static const uint64_t FNV_RAFT_BF = 0xc3850410336560ebULL;
// test variants (tools/make_seeded_spec.py --split-brain / --commit-past-log): the Assert (tla:185) and
// the evaluation error (tla:499) reachable in a BFS
static const uint64_t FNV_RAFT_SPLIT_BRAIN = 0x3dd92c869822b066ULL;
static const uint64_t FNV_RAFT_COMMIT_PAST_LOG = 0x1d4d6d5e2014bcc5ULL;

uint64_t fnv1a_spec(const std::string &text) {
    uint64_t h = 0xcbf29ce484222325ULL;
    for (size_t i = 0; i < text.size(); i++) {
        if (text[i] == '\r' && i + 1 < text.size() && text[i + 1] == '\n') continue;
        h ^= (unsigned char)text[i];
        h *= 0x100000001b3ULL;
    }
    return h;
}

namespace {

struct Tok {
    enum Kind { ID, NUM, SYM, END } kind;
    std::string s;
    int line;
};

std::vector<Tok> lex(const std::string &t, std::string &err) {
    std::vector<Tok> out;
    int line = 1;
    size_t i = 0;
    while (i < t.size()) {
        char c = t[i];
        if (c == '\n') { line++; i++; continue; }
        if (isspace((unsigned char)c)) { i++; continue; }
        if (c == '\\' && i + 1 < t.size() && t[i + 1] == '*') {  // \* line comment
            while (i < t.size() && t[i] != '\n') i++;
            continue;
        }
        if (c == '(' && i + 1 < t.size() && t[i + 1] == '*') {  // (* block comment *)
            int depth = 0;
            while (i + 1 < t.size()) {
                if (t[i] == '(' && t[i + 1] == '*') { depth++; i += 2; continue; }
                if (t[i] == '*' && t[i + 1] == ')') { depth--; i += 2; if (!depth) break; continue; }
                if (t[i] == '\n') line++;
                i++;
            }
            continue;
        }
        if (isalpha((unsigned char)c) || c == '_') {
            size_t j = i;
            while (j < t.size() && (isalnum((unsigned char)t[j]) || t[j] == '_')) j++;
            out.push_back({Tok::ID, t.substr(i, j - i), line});
            i = j;
            continue;
        }
        if (isdigit((unsigned char)c) || (c == '-' && i + 1 < t.size() && isdigit((unsigned char)t[i + 1]))) {
            size_t j = i + 1;
            while (j < t.size() && isdigit((unsigned char)t[j])) j++;
            out.push_back({Tok::NUM, t.substr(i, j - i), line});
            i = j;
            continue;
        }
        if (c == '<' && i + 1 < t.size() && t[i + 1] == '-') { out.push_back({Tok::SYM, "<-", line}); i += 2; continue; }
        if (c == '"') {
            size_t j = i + 1;
            while (j < t.size() && t[j] != '"') j++;
            out.push_back({Tok::ID, t.substr(i, j + 1 - i), line});
            i = j + 1;
            continue;
        }
        if (strchr("={},", c)) { out.push_back({Tok::SYM, std::string(1, c), line}); i++; continue; }
        err = "cfg line " + std::to_string(line) + ": unexpected character '" + std::string(1, c) + "'";
        return {};
    }
    out.push_back({Tok::END, "", line});
    return out;
}

bool is_keyword(const std::string &s) {
    static const char *kw[] = {"CONSTANT", "CONSTANTS", "INIT", "NEXT", "SPECIFICATION", "INVARIANT", "INVARIANTS",
                               "PROPERTY", "PROPERTIES", "SYMMETRY", "VIEW", "CONSTRAINT", "CONSTRAINTS",
                               "ACTION_CONSTRAINT", "ACTION_CONSTRAINTS", "CHECK_DEADLOCK", "ALIAS", "POSTCONDITION"};
    for (const char *k : kw)
        if (s == k) return true;
    return false;
}

struct Value {
    enum Kind { INT, MODEL, SET, OTHER } kind = OTHER;
    long iv = 0;
    std::string name;
    std::vector<std::string> elems;
};

}  // namespace

// Invariant names of Raft.tla that are compiled (tla:434-503).
static const std::pair<const char *, uint32_t> kInvNames[] = {
    {"Inv", RMC_INV_LEADER_HAS_ALL_COMMITTED},
    {"LeaderHasAllCommittedEntries", RMC_INV_LEADER_HAS_ALL_COMMITTED},
    {"NoSplitVote", RMC_INV_NO_SPLIT_VOTE},
    {"RaftCanCommt", RMC_INV_RAFT_CAN_COMMIT},
    {"FollowerCanCommit", RMC_INV_FOLLOWER_CAN_COMMIT},
    {"CommitAll", RMC_INV_COMMIT_ALL},
    {"NoAllCommit", RMC_INV_NO_ALL_COMMIT},
    {"ExistLeaderAndCandidate", RMC_INV_EXIST_LEADER_AND_CANDIDATE},
};

bool parse_model(const std::string &cfg_text, const char *tla_text, ParsedModel *pm, std::string &err) {
    *pm = ParsedModel();
    std::vector<Tok> tk = lex(cfg_text, err);
    if (tk.empty()) return false;
    std::map<std::string, Value> consts;
    std::string section;
    bool have_init = false, have_next = false;
    size_t i = 0;
    auto fail = [&](const Tok &t, const std::string &m) {
        err = "cfg line " + std::to_string(t.line) + ": " + m;
        return false;
    };
    while (tk[i].kind != Tok::END) {
        const Tok &t = tk[i];
        if (t.kind == Tok::ID && is_keyword(t.s)) {
            section = t.s;
            i++;
            if (section == "CHECK_DEADLOCK") {
                if (tk[i].kind != Tok::ID || (tk[i].s != "TRUE" && tk[i].s != "FALSE"))
                    return fail(tk[i], "CHECK_DEADLOCK expects TRUE or FALSE");
                pm->check_deadlock_cfg = tk[i].s == "TRUE" ? 1 : 0;
                i++;
            }
            continue;
        }
        if (section == "CONSTANT" || section == "CONSTANTS") {
            if (t.kind != Tok::ID) return fail(t, "expected a constant name");
            const std::string name = t.s;
            i++;
            if (tk[i].kind == Tok::SYM && tk[i].s == "<-")
                return fail(tk[i], "constant substitution (<-) is not supported for " + name);
            if (!(tk[i].kind == Tok::SYM && tk[i].s == "=")) return fail(tk[i], "expected '=' after " + name);
            i++;
            Value v;
            const Tok &x = tk[i];
            if (x.kind == Tok::NUM) {
                v.kind = Value::INT;
                v.iv = strtol(x.s.c_str(), nullptr, 10);
                i++;
            } else if (x.kind == Tok::ID) {
                v.kind = (x.s == "TRUE" || x.s == "FALSE" || x.s[0] == '"') ? Value::OTHER : Value::MODEL;
                v.name = x.s;
                i++;
            } else if (x.kind == Tok::SYM && x.s == "{") {
                v.kind = Value::SET;
                i++;
                while (!(tk[i].kind == Tok::SYM && tk[i].s == "}")) {
                    if (tk[i].kind != Tok::ID) return fail(tk[i], "only sets of model values are supported");
                    v.elems.push_back(tk[i].s);
                    i++;
                    if (tk[i].kind == Tok::SYM && tk[i].s == ",") i++;
                    else if (!(tk[i].kind == Tok::SYM && tk[i].s == "}")) return fail(tk[i], "expected ',' or '}'");
                }
                i++;
            } else {
                return fail(x, "unsupported value for constant " + name);
            }
            consts[name] = v;
            continue;
        }
        if (t.kind != Tok::ID) return fail(t, "unexpected token '" + t.s + "'");
        if (section == "INIT") { if (t.s != "Init") return fail(t, "INIT must be Init (Raft.tla:93)"); have_init = true; }
        else if (section == "NEXT") { if (t.s != "Next") return fail(t, "NEXT must be Next (Raft.tla:416)"); have_next = true; }
        else if (section == "SPECIFICATION") return fail(t, "SPECIFICATION is not supported; use INIT/NEXT");
        else if (section == "SYMMETRY") {
            if (t.s != "symmServers") return fail(t, "only SYMMETRY symmServers (Raft.tla:21) is supported");
            pm->symmetry = true;
        } else if (section == "VIEW") {
            if (t.s != "view") return fail(t, "only VIEW view (Raft.tla:38) is supported");
            pm->view = true;
        } else if (section == "INVARIANT" || section == "INVARIANTS") {
            uint32_t bit = 0;
            for (const auto &p : kInvNames)
                if (t.s == p.first) bit = p.second;
            if (!bit) return fail(t, "invariant " + t.s + " is not compiled");
            if (!(pm->cfg.invariants & bit)) {
                // TLC checks the invariants in the order the cfg lists them: id + 1 per nibble
                int id = 0;
                while (!((bit >> id) & 1u)) id++;
                pm->cfg.invariant_order |= (uint32_t)(id + 1) << (4 * pm->invariant_names.size());
                pm->invariant_names.push_back(t.s);
            }
            pm->cfg.invariants |= bit;
        } else {
            return fail(t, section.empty() ? "text before the first section" : section + " is not supported");
        }
        i++;
    }
    if (!have_init || !have_next) { err = "cfg must name INIT Init and NEXT Next (Raft.cfg:30-31)"; return false; }
    if (!pm->view) { err = "cfg must select VIEW view (Raft.cfg:26): only the VIEW configuration is compiled"; return false; }
    auto need_int = [&](const char *n, int32_t *dst, int lo, int hi) {
        auto it = consts.find(n);
        if (it == consts.end() || it->second.kind != Value::INT) { err = std::string("CONSTANT ") + n + " must be an integer"; return false; }
        if (it->second.iv < lo || it->second.iv > hi) {
            err = std::string("CONSTANT ") + n + " = " + std::to_string(it->second.iv) + " is outside " +
                  std::to_string(lo) + ".." + std::to_string(hi);
            return false;
        }
        *dst = (int32_t)it->second.iv;
        return true;
    };
    if (!need_int("MaxElection", &pm->cfg.max_election, 0, 7)) return false;
    if (!need_int("MaxRestart", &pm->cfg.max_restart, 0, 15)) return false;
    for (const char *mv : {"Follower", "Candidate", "Leader", "None", "VoteReq", "VoteResp", "AppendReq", "AppendResp"}) {
        auto it = consts.find(mv);
        if (it == consts.end() || it->second.kind != Value::MODEL) {
            err = std::string("CONSTANT ") + mv + " must be a model value (e.g. " + mv + " = " + mv + ")";
            return false;
        }
    }
    auto need_set = [&](const char *n, std::vector<std::string> *names, int lo, int hi) {
        auto it = consts.find(n);
        if (it == consts.end() || it->second.kind != Value::SET) { err = std::string("CONSTANT ") + n + " must be a set of model values"; return false; }
        std::vector<std::string> e = it->second.elems;
        std::sort(e.begin(), e.end());  // TLC orders model values by name
        if (std::adjacent_find(e.begin(), e.end()) != e.end()) { err = std::string(n) + " lists a value twice"; return false; }
        if ((int)e.size() < lo || (int)e.size() > hi) {
            err = std::string("|") + n + "| = " + std::to_string(e.size()) + " is outside " + std::to_string(lo) + ".." + std::to_string(hi);
            return false;
        }
        *names = e;
        return true;
    };
    if (!need_set("Servers", &pm->servers, 1, 5)) return false;  // ASSUME Servers # {} (tla:19)
    if (!need_set("Vals", &pm->vals, 0, 3)) return false;
    pm->cfg.n_servers = (int32_t)pm->servers.size();
    pm->cfg.n_vals = (int32_t)pm->vals.size();
    pm->cfg.no_symmetry = pm->symmetry ? 0 : 1;
    pm->cfg.world_size = 1;
    pm->cfg.device = -1;
    for (const auto &kv : consts) {  // TLC accepts assignments to undeclared names (MaxTerm, s4, s5: Raft.cfg:2,16-17)
        static const char *known[] = {"MaxElection", "MaxRestart", "Servers", "Vals", "Follower", "Candidate", "Leader",
                                      "None", "VoteReq", "VoteResp", "AppendReq", "AppendResp"};
        bool k = false;
        for (const char *n : known) k |= kv.first == n;
        // s1 = s1, v1 = v1 (Raft.cfg:7-20): the model values Servers / Vals are built from
        k |= kv.second.kind == Value::MODEL &&
             (std::count(pm->servers.begin(), pm->servers.end(), kv.first) ||
              std::count(pm->vals.begin(), pm->vals.end(), kv.first));
        if (!k) pm->ignored_constants.push_back(kv.first);
    }
    if (tla_text) {
        const uint64_t h = fnv1a_spec(tla_text);
        if (h == FNV_RAFT || h == FNV_RAFT_FAPP) { pm->cfg.spec_variant = RMC_SPEC_RAFT; pm->module = "Raft"; }
        else if (h == FNV_RAFT_SEEDED) { pm->cfg.spec_variant = RMC_SPEC_SEEDED; pm->module = "RaftSeeded"; }
        else if (h == FNV_RAFT_BF) { pm->cfg.spec_variant = RMC_SPEC_BECOME_FOLLOWER; pm->module = "Raft"; }
        else if (h == FNV_RAFT_SPLIT_BRAIN) { pm->cfg.spec_variant = RMC_SPEC_SPLIT_BRAIN; pm->module = "RaftSplitBrain"; }
        else if (h == FNV_RAFT_COMMIT_PAST_LOG) {
            pm->cfg.spec_variant = RMC_SPEC_COMMIT_PAST_LOG;
            pm->module = "RaftCommitPastLog";
        }
        else {
            char buf[64];
            snprintf(buf, sizeof buf, "%016llx", (unsigned long long)h);
            err = std::string("the .tla file is not kikimo/tla-raft's Raft.tla nor one of its variants (fnv1a64 ") +
                  buf + "): only those specs are compiled into this checker";
            return false;
        }
    }
    return true;
}

}  // namespace rmc

extern "C" int rmc_parse_config(const char *cfg_text, const char *tla_text, rmc_config *out, char *err, size_t cap) {
    if (!cfg_text || !out) return RMC_E_ARG;
    rmc::ParsedModel pm;
    std::string e;
    const int32_t keep_variant = out->spec_variant;
    if (!rmc::parse_model(cfg_text, tla_text, &pm, e)) {
        if (err && cap) { strncpy(err, e.c_str(), cap - 1); err[cap - 1] = 0; }
        return RMC_E_PARSE;
    }
    *out = pm.cfg;
    if (!tla_text) out->spec_variant = keep_variant;
    if (err && cap) err[0] = 0;
    return RMC_OK;
}
