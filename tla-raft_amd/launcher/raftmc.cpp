// raftmc -- TLC-compatible command line over librmc (the drop-in for myrun.sh:3).
//
//   raftmc [-deadlock] [-workers N] [-config Raft.cfg] [-device D] [-gpus N] [-msgcap C] [-seenlog2 K] Raft.tla
//
// Accepts the flags myrun.sh passes to TLC (myrun.sh:3), reads the same Raft.tla /
// Raft.cfg, and prints TLC's result lines (states generated, distinct states, depth,
// the counterexample) so that parsers of raft.log keep working.  GPU-specific lines
// are printed after TLC's block.  Exit codes follow TLC's (0 ok, 11 deadlock,
// 12 safety violation, 14 Assert, 75 evaluation error, 150/151 spec/config errors).
#include <fcntl.h>
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <filesystem>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "rmc.h"
#include "rmc_cfg.h"

namespace {

// rmc_trace_step.action ids (Raft.tla's Next disjuncts; 11 never appears, 12 only in the tla:420 variant)
const char *kActionNames[13] = {"BecomeCandidate", "UpdateTerm", "ResponseVote", "BecomeLeader",
                                "ClientReq", "LeaderAppendEntry", "FollowerAcceptEntry", "FollowerRejectEntry",
                                "HandleAppendResp", "LeaderCanCommit", "Restart", "FollowerAppendEntry",
                                "BecomeFollower"};
const char *kInvNames[7] = {"Inv", "NoSplitVote", "RaftCanCommt", "FollowerCanCommit", "CommitAll", "NoAllCommit",
                            "ExistLeaderAndCandidate"};

std::string now_str() {
    char buf[64];
    std::time_t t = std::time(nullptr);
    std::strftime(buf, sizeof buf, "%Y-%m-%d %H:%M:%S", std::localtime(&t));
    return buf;
}

// TLC's metadir name: states/YY-MM-DD-HH-MM-SS
std::string stamp_str() {
    char buf[64];
    std::time_t t = std::time(nullptr);
    std::strftime(buf, sizeof buf, "%y-%m-%d-%H-%M-%S", std::localtime(&t));
    return buf;
}

bool read_file(const std::string &path, std::string *out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    *out = ss.str();
    return true;
}

// Source range of each action definition body in the spec text: TLC prints
// "<Name line L, col C to line L2, col C2 of module M>" for trace steps.
struct Loc {
    int l0 = 0, c0 = 0, l1 = 0, c1 = 0;
};

// BecomeFollower (tla:226) is a disjunction of three actions; TLC names a step by the one taken,
// which role[s] of the step's first state decides
const char *kBfNames[3] = {"FollowerUpdateTerm", "CandidateToFollower", "LeaderToFollower"};

std::vector<Loc> action_locations(const std::string &tla, const std::vector<std::string> &names) {
    std::vector<std::string> lines;
    std::stringstream ss(tla);
    std::string ln;
    while (std::getline(ss, ln)) {
        if (!ln.empty() && ln.back() == '\r') ln.pop_back();
        lines.push_back(ln);
    }
    std::vector<Loc> locs(names.size());
    for (size_t a = 0; a < names.size(); a++) {
        const std::string head = names[a] + "(s) ==";
        for (size_t i = 0; i < lines.size(); i++) {
            if (lines[i].compare(0, head.size(), head) != 0) continue;
            // body starts at the first non-blank character after "=="
            size_t li = i, col = head.size();
            while (li < lines.size()) {
                while (col < lines[li].size() && isspace((unsigned char)lines[li][col])) col++;
                if (col < lines[li].size()) break;
                li++;
                col = 0;
            }
            Loc L;
            L.l0 = (int)li + 1;
            L.c0 = (int)col + 1;
            // body ends at the last token before the next column-1 line: blank lines, comment-only
            // lines (tla:173 "\* /\ Print(...)" after BecomeLeader's last conjunct) and a line's
            // trailing "\*" comment are not part of the expression
            auto code_end = [&](size_t k) -> long {  // last code column (0-based) of line k, -1 if none
                const std::string &s = lines[k];
                size_t cut = s.find("\\*");
                long e = (long)std::min(cut, s.size()) - 1;
                while (e >= 0 && isspace((unsigned char)s[e])) e--;
                return e;
            };
            size_t j = li + 1;
            while (j < lines.size() && (lines[j].empty() || isspace((unsigned char)lines[j][0]))) j++;
            size_t e = j - 1;
            while (e > li && code_end(e) < 0) e--;
            L.l1 = (int)e + 1;
            L.c1 = (int)code_end(e) + 1;
            locs[a] = L;
            break;
        }
    }
    return locs;
}

struct Printer {
    const rmc::ParsedModel &pm;
    int n, V;
    std::string sv(int i) const { return i < 0 ? "None" : pm.servers[i]; }
    std::string fn_servers(const std::vector<std::string> &vals) const {
        std::string s = "(";
        for (int i = 0; i < n; i++) s += (i ? " @@ " : "") + pm.servers[i] + " :> " + vals[i];
        return s + ")";
    }
    std::string entry(int t, int v) const {
        return "[term |-> " + std::to_string(t) + ", val |-> " + (v < 0 ? std::string("None") : pm.vals[v]) + "]";
    }
    std::string state(const int32_t *u) const {
        int k = 0;
        std::vector<std::string> vf, ct, role, ci, logs;
        for (int i = 0; i < n; i++) vf.push_back(sv(u[k++]));
        for (int i = 0; i < n; i++) ct.push_back(std::to_string(u[k++]));
        static const char *rn[3] = {"Follower", "Candidate", "Leader"};
        for (int i = 0; i < n; i++) role.push_back(rn[u[k++]]);
        for (int i = 0; i < n; i++) ci.push_back(std::to_string(u[k++]));
        std::vector<int> ll;
        for (int i = 0; i < n; i++) ll.push_back(u[k++]);
        for (int i = 0; i < n; i++) {
            std::string s = "<<";
            for (int x = 1; x <= V + 1; x++) {
                int t = u[k], v = u[k + 1];
                k += 2;
                if (x <= ll[i]) s += (x > 1 ? ", " : "") + entry(t, v);
            }
            logs.push_back(s + ">>");
        }
        auto matrix = [&](bool boolean) {
            std::vector<std::string> rows;
            for (int i = 0; i < n; i++) {
                std::vector<std::string> r;
                for (int j = 0; j < n; j++) {
                    int v = u[k++];
                    r.push_back(boolean ? (v ? "TRUE" : "FALSE") : std::to_string(v));
                }
                rows.push_back(fn_servers(r));
            }
            return fn_servers(rows);
        };
        std::string mi = matrix(false), ni = matrix(false), pend = matrix(true);
        int ec = u[k++], rc = u[k++];
        std::string vs = "(";
        for (int v = 0; v < V; v++) vs += (v ? " @@ " : "") + pm.vals[v] + " :> " + (u[k++] < 0 ? "None" : "FALSE");
        vs += ")";
        if (V == 0) vs = "<<>>";
        int nm = u[k++];
        std::string msgs = "{";
        static const char *tn[4] = {"VoteReq", "VoteResp", "AppendReq", "AppendResp"};
        for (int q = 0; q < nm; q++, k += 8) {
            const int32_t *m = u + k;
            std::string r;
            switch (m[0]) {
            case 0:
                r = "[dst |-> " + sv(m[2]) + ", lastLogIndex |-> " + std::to_string(m[4]) + ", lastLogTerm |-> " +
                    std::to_string(m[5]) + ", src |-> " + sv(m[1]) + ", term |-> " + std::to_string(m[3]) +
                    ", type |-> VoteReq]";
                break;
            case 1:
                r = "[dst |-> " + sv(m[2]) + ", src |-> " + sv(m[1]) + ", term |-> " + std::to_string(m[3]) +
                    ", type |-> VoteResp]";
                break;
            case 2:
                r = "[dst |-> " + sv(m[2]) + ", entries |-> <<" + (m[7] < 0 ? "" : entry(m[7] / 8, m[7] % 8)) +
                    ">>, leaderCommit |-> " + std::to_string(m[6]) + ", prevLogIndex |-> " + std::to_string(m[4]) +
                    ", prevLogTerm |-> " + std::to_string(m[5]) + ", src |-> " + sv(m[1]) + ", term |-> " +
                    std::to_string(m[3]) + ", type |-> AppendReq]";
                break;
            default:
                r = "[dst |-> " + sv(m[2]) + ", prevLogIndex |-> " + std::to_string(m[4]) + ", src |-> " + sv(m[1]) +
                    ", succ |-> " + (m[5] ? "TRUE" : "FALSE") + ", term |-> " + std::to_string(m[3]) +
                    ", type |-> AppendResp]";
            }
            (void)tn;
            msgs += (q ? ",\n   " : "") + r;
        }
        msgs += "}";
        std::string o;
        o += "/\\ votedFor = " + fn_servers(vf) + "\n";
        o += "/\\ currentTerm = " + fn_servers(ct) + "\n";
        o += "/\\ logs = " + fn_servers(logs) + "\n";
        o += "/\\ matchIndex = " + mi + "\n";
        o += "/\\ nextIndex = " + ni + "\n";
        o += "/\\ commitIndex = " + fn_servers(ci) + "\n";
        o += "/\\ msgs = " + msgs + "\n";
        o += "/\\ role = " + fn_servers(role) + "\n";
        o += "/\\ electionCount = " + std::to_string(ec) + "\n";
        o += "/\\ restartCount = " + std::to_string(rc) + "\n";
        o += "/\\ pendingResponse = " + pend + "\n";
        o += "/\\ valSent = " + vs + "\n";
        return o;
    }
};

int usage(const char *msg) {
    std::fprintf(stderr, "raftmc: %s\nusage: raftmc [-deadlock] [-workers N] [-config FILE.cfg] [-device D] "
                         "[-gpus N [-onerank] [-shardmin K]] [-msgcap C] [-seenlog2 K] [-checkpoint MIN] [-metadir DIR] "
                         "[-recover DIR] FILE.tla\n", msg);
    return 150;
}

bool io_all(int fd, void *buf, size_t n, bool wr) {
    char *p = static_cast<char *>(buf);
    while (n) {
        const ssize_t k = wr ? ::write(fd, p, n) : ::read(fd, p, n);
        if (k <= 0) return false;
        p += k;
        n -= (size_t)k;
    }
    return true;
}

// -gpus N: one rank process per GPU, forked before anything touches a GPU.  Rank 0
// creates the RCCL unique id (its bootstrap root lives in that process) and sends it up a pipe;
// this process hands it down to ranks 1 .. N-1.  Rank r runs the checker on device base + r with
// world_size N (-onerank: one rank, world_size 1 with the id -- the sharded protocol through a
// one-rank communicator); only rank 0 writes TLC's output, the others' stdout goes to /dev/null.
// Returns rank 0's exit code.  A rank that dies, or ends with an error while rank 0 still runs,
// takes the others down (they would wait in a collective); after rank 0 ends the others get 60 s.
int run_ranks(int N, bool onerank, const rmc_config &base, const std::function<int(const rmc_config &)> &body) {
    std::fflush(stdout);
    std::fflush(stderr);
    int up[2];
    if (::pipe(up) != 0) { std::printf("Error: pipe failed\n"); return 75; }
    std::vector<pid_t> pid(N, -1);
    std::vector<int> down(N, -1);
    for (int r = 0; r < N; r++) {
        int p[2];
        if (::pipe(p) != 0) { std::printf("Error: pipe failed\n"); return 75; }
        const pid_t k = ::fork();
        if (k < 0) { std::printf("Error: fork failed\n"); return 75; }
        if (k == 0) {  // rank r
            ::close(p[1]);
            ::close(up[0]);
            if (r != 0) ::close(up[1]);  // (only rank 0 writes up: the others must not hold it open)
            for (int q = 0; q < r; q++) ::close(down[q]);
            // RCCL's own messages (its version line, warnings) go to stderr: stdout is TLC's
            ::setenv("NCCL_DEBUG_FILE", "/dev/stderr", 0);
            unsigned char id[128];
            if (r == 0) {
                const int rc = rmc_comm_unique_id(id);
                if (rc != RMC_OK) {
                    std::printf("Error: could not start the GPU model checker (RCCL unique id: code %d)\n", rc);
                    std::fflush(stdout);
                    std::_Exit(75);
                }
                if (!io_all(up[1], id, sizeof id, true)) std::_Exit(75);
            } else if (!io_all(p[0], id, sizeof id, false)) {
                std::_Exit(75);  // rank 0 could not start: nothing to join
            }
            if (r == 0) ::close(up[1]);
            ::close(p[0]);
            if (r != 0) {
                const int dn = ::open("/dev/null", O_WRONLY);
                if (dn >= 0) ::dup2(dn, 1);
            }
            rmc_config c = base;
            c.rank = onerank ? 0 : r;
            c.world_size = onerank ? 1 : N;
            c.comm_unique_id = id;
            c.device = (base.device >= 0 ? base.device : 0) + r;
            const int code = body(c);
            std::fflush(stdout);
            std::fflush(stderr);
            std::_Exit(code);
        }
        ::close(p[0]);
        down[r] = p[1];
        pid[r] = k;
    }
    ::close(up[1]);
    unsigned char id[128];
    const bool have = io_all(up[0], id, sizeof id, false);
    ::close(up[0]);
    for (int r = 1; r < N; r++) {
        if (have) io_all(down[r], id, sizeof id, true);
        ::close(down[r]);
    }
    ::close(down[0]);
    int code0 = 75, alive = N;
    bool rank0_done = false;
    auto kill_all = [&] {
        for (int r = 0; r < N; r++)
            if (pid[r] > 0) ::kill(pid[r], SIGKILL);
    };
    auto t_done = std::chrono::steady_clock::now();
    while (alive) {
        int st = 0;
        const pid_t w = ::waitpid(-1, &st, rank0_done ? WNOHANG : 0);
        if (w < 0) break;
        if (w == 0) {  // rank 0 has ended; the others finish their last collectives or are stopped
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t_done).count() > 60.0) kill_all();
            ::usleep(100000);
            continue;
        }
        const int r = (int)(std::find(pid.begin(), pid.end(), w) - pid.begin());
        if (r >= N) continue;
        pid[r] = -1;
        alive--;
        const bool clean = WIFEXITED(st);
        const int code = clean ? WEXITSTATUS(st) : 75;
        if (r == 0) {
            code0 = code;
            rank0_done = true;
            t_done = std::chrono::steady_clock::now();
        } else if (!clean || (!rank0_done && code != 0 && code != 11 && code != 12 && code != 14)) {
            std::fprintf(stderr, "raftmc: rank %d ended (%s %d); stopping the other ranks\n", r,
                         clean ? "exit" : "signal", clean ? code : WTERMSIG(st));
            kill_all();
        }
    }
    return code0;
}

// The process that prints TLC's output is not the one whose exit frees the run's memory: run_detached
// forks one worker before anything touches a GPU; the worker prints everything, then closes its
// stdout / stderr (tee's pipe, myrun.sh:3) and reports its exit code up a pipe before it exits.  The
// kernel's teardown of the worker (~110 GB of host trace and the device memory after a Raft.cfg
// exhaustion: ~4 s) then runs after this process has returned TLC's exit code,
// so the shell returns as the "Finished" line prints.
// The worker frees the device memory itself (rmc_release_device) before it reports, so a GPU job started
// right after the shell returns finds the device free; only the host trace's teardown overlaps it.
int g_report_fd = -1;

void report(int code) {  // (a no-op in the one-process mode)
    std::fflush(stdout);
    std::fflush(stderr);
    if (g_report_fd < 0) return;
    ::close(1);  // (exit tears memory down before it closes files: tee would wait for the teardown)
    ::close(2);
    unsigned char c = (unsigned char)code;
    io_all(g_report_fd, &c, 1, true);
    ::close(g_report_fd);
    g_report_fd = -1;
}

[[noreturn]] void report_and_exit(int code) {
    report(code);
    std::_Exit(code);
}

int run_detached(const rmc_config &cfg, const std::function<int(const rmc_config &)> &body) {
    std::fflush(stdout);
    std::fflush(stderr);
    int pp[2];
    if (::pipe(pp) != 0) return body(cfg);
    const pid_t k = ::fork();
    if (k < 0) {
        ::close(pp[0]);
        ::close(pp[1]);
        return body(cfg);  // no worker: run here
    }
    if (k == 0) {
        ::close(pp[0]);
        g_report_fd = pp[1];
        report_and_exit(body(cfg));
    }
    ::close(pp[1]);
    unsigned char c = 0;
    const bool got = io_all(pp[0], &c, 1, false);
    ::close(pp[0]);
    if (got) return c;  // the worker's teardown goes on without us
    int st = 0;  // the worker ended without reporting (a crash): its status
    if (::waitpid(k, &st, 0) < 0) return 75;
    return WIFEXITED(st) ? WEXITSTATUS(st) : 75;
}

}  // namespace

// RMC_LAUNCHER_TIMES=1: seconds since process start at each phase, on stderr (stdout stays TLC's)
static const auto g_t_start = std::chrono::steady_clock::now();
static void phase_time(const char *what) {
    static const bool on = std::getenv("RMC_LAUNCHER_TIMES") && std::string(std::getenv("RMC_LAUNCHER_TIMES")) == "1";
    if (on)
        std::fprintf(stderr, "raftmc: %s at %.3f s\n", what,
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - g_t_start).count());
}

int main(int argc, char **argv) {
    std::string tla_path, cfg_path;
    int check_deadlock = 1, device = -1, msgcap = 0, seenlog2 = 0, workers = 1, gpus = 1;
    bool onerank = false;                // -gpus 1 through a one-rank RCCL communicator (tests)
    unsigned long long shardmin = 0;     // -gpus: levels below this many states run replicated (0 = 2^20)
    bool print_locations = false;       // print each action's source range and exit (no GPU needed)
    double progress_s = 60.0;           // TLC reports Progress once a minute (and at the end)
    double ckpt_minutes = 30.0;         // TLC -checkpoint: minutes between checkpoints (0 = never)
    std::string metadir, recover_dir;   // TLC -metadir / -recover: where checkpoints go / come from
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto need = [&](const char *f) -> const char * {
            if (i + 1 >= argc) { std::fprintf(stderr, "raftmc: %s needs an argument\n", f); std::exit(150); }
            return argv[++i];
        };
        if (a == "-deadlock") check_deadlock = 0;  // TLC: -deadlock turns deadlock checking OFF
        else if (a == "-workers") workers = std::atoi(need("-workers"));  // CPU threads in TLC; the GPU path ignores it
        else if (a == "-config") cfg_path = need("-config");
        else if (a == "-device") device = std::atoi(need("-device"));
        else if (a == "-gpus") gpus = std::atoi(need("-gpus"));
        else if (a == "-onerank") onerank = true;
        else if (a == "-shardmin") shardmin = std::strtoull(need("-shardmin"), nullptr, 10);
        else if (a == "-msgcap") msgcap = std::atoi(need("-msgcap"));
        else if (a == "-seenlog2") seenlog2 = std::atoi(need("-seenlog2"));
        else if (a == "-checkpoint") ckpt_minutes = std::atof(need("-checkpoint"));
        else if (a == "-metadir") metadir = need("-metadir");
        else if (a == "-recover") recover_dir = need("-recover");
        else if (a == "-progress") progress_s = std::atof(need("-progress"));
        else if (a == "-print-locations") print_locations = true;
        else if (a.size() > 4 && a.compare(a.size() - 4, 4, ".tla") == 0) tla_path = a;
        else if (a[0] != '-' && tla_path.empty()) tla_path = a + ".tla";
        else return usage(("unsupported option " + a).c_str());
    }
    if (tla_path.empty()) return usage("missing spec file");
    if (gpus < 1 || gpus > 64) return usage("-gpus must be 1..64");
    if (cfg_path.empty()) cfg_path = tla_path.substr(0, tla_path.size() - 4) + ".cfg";
    std::string tla, cfgtxt;
    const bool skip_spec = std::getenv("RMC_SKIP_SPEC_CHECK") && std::string(std::getenv("RMC_SKIP_SPEC_CHECK")) == "1";
    if (!read_file(tla_path, &tla)) {
        if (!skip_spec) { std::fprintf(stderr, "Error: cannot read %s\n", tla_path.c_str()); return 150; }
        tla.clear();
    }
    if (print_locations) {
        // the "<Action line L, col C to line L', col C' of module M>" ranges the trace headers use
        std::vector<std::string> names(kActionNames, kActionNames + 13);
        names.insert(names.end(), kBfNames, kBfNames + 3);
        std::vector<Loc> locs = action_locations(tla, names);
        for (size_t a = 0; a < names.size(); a++)
            std::printf("%s %d %d %d %d\n", names[a].c_str(), locs[a].l0, locs[a].c0, locs[a].l1, locs[a].c1);
        return 0;
    }
    if (!read_file(cfg_path, &cfgtxt)) { std::fprintf(stderr, "Error: cannot read %s\n", cfg_path.c_str()); return 151; }
    rmc::ParsedModel pm;
    std::string err;
    if (!rmc::parse_model(cfgtxt, skip_spec ? nullptr : tla.c_str(), &pm, err)) {
        std::fprintf(stdout, "Error: %s\n", err.c_str());
        return err.rfind("cfg", 0) == 0 || err.rfind("CONSTANT", 0) == 0 ? 151 : 150;
    }
    if (skip_spec) {
        const std::string base = tla_path.substr(tla_path.find_last_of('/') + 1);
        if (base == "RaftSeeded.tla") { pm.cfg.spec_variant = RMC_SPEC_SEEDED; pm.module = "RaftSeeded"; }
        if (base == "RaftSplitBrain.tla") { pm.cfg.spec_variant = RMC_SPEC_SPLIT_BRAIN; pm.module = "RaftSplitBrain"; }
        if (base == "RaftCommitPastLog.tla") { pm.cfg.spec_variant = RMC_SPEC_COMMIT_PAST_LOG; pm.module = "RaftCommitPastLog"; }
    }
    if (pm.check_deadlock_cfg >= 0 && check_deadlock) check_deadlock = pm.check_deadlock_cfg;
    rmc_config cfg = pm.cfg;
    cfg.check_deadlock = check_deadlock;
    cfg.device = device;
    cfg.msg_cap = msgcap;
    cfg.seen_log2 = seenlog2;
    cfg.shard_min_states = shardmin;

    std::printf("raftmc (MI355X-native model checker for kikimo/tla-raft) -- TLC-compatible output\n");
    std::printf("Running breadth-first search Model-Checking on %d GPU%s (TLC -workers %d order: 1).\n", gpus,
                gpus > 1 ? "s" : "", workers);
    std::printf("Parsing file %s\n", tla_path.c_str());
    std::printf("Semantic processing of module %s\n", pm.module.c_str());
    for (const auto &c : pm.ignored_constants) std::printf("(ignoring assignment to undeclared constant %s)\n", c.c_str());
    std::printf("Starting... (%s)\n", now_str().c_str());
    auto check = [&](const rmc_config &cfg) -> int {
    const auto t0 = std::chrono::steady_clock::now();
    void *ctx = nullptr;
    phase_time("create");
    // a rank's communicator set-up prints RCCL's banner on stdout: send it to stderr (stdout is TLC's)
    const int saved_out = cfg.comm_unique_id ? ::dup(1) : -1;
    if (saved_out >= 0) {
        std::fflush(stdout);
        ::dup2(2, 1);
    }
    int rc = rmc_create(&cfg, &ctx);
    if (saved_out >= 0) {
        std::fflush(stdout);
        ::dup2(saved_out, 1);
        ::close(saved_out);
    }
    phase_time("created");
    if (rc != RMC_OK) { std::printf("Error: could not start the GPU model checker (code %d)\n", rc); return 75; }
    rmc_level_stats st;
    if (!recover_dir.empty()) {
        // TLC -recover: carry on from the checkpoint in that directory (rmc_resume)
        const std::string f = recover_dir + "/raftmc.ckpt";
        std::printf("Starting recovery from checkpoint %s\n", recover_dir.c_str());
        rc = rmc_resume(ctx, f.c_str());
        if (rc < 0) { std::printf("Error: %s\n", rmc_last_error(ctx)); rmc_destroy(ctx); return 75; }
        rmc_result r0;
        rmc_get_result(ctx, &r0);
        std::printf("Recovery completed. %llu states examined. %llu states on queue.\n",
                    (unsigned long long)r0.distinct, (unsigned long long)r0.queue);
        if (metadir.empty()) metadir = recover_dir;
        rc = r0.status;
    } else {
        std::printf("Computing initial states...\n");
        rc = rmc_init(ctx, &st);
        if (rc < 0) { std::printf("Error: %s\n", rmc_last_error(ctx)); rmc_destroy(ctx); return 75; }
        std::printf("Finished computing initial states: 1 distinct state generated at %s.\n", now_str().c_str());
    }
    if (metadir.empty()) metadir = "states/" + stamp_str();
    auto last_ckpt = std::chrono::steady_clock::now();
    double gpu_seconds = 0;
    std::vector<rmc_level_stats> lv(65);
    // TLC prints Progress at start, then once per reporting interval, then at the end of the search
    auto progress = [&](const rmc_level_stats &q) {
        const double el = std::max(1e-9, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        std::printf("Progress(%d) at %s: %llu states generated (%.0f s/min), %llu distinct states found (%.0f ds/min), "
                    "%llu states left on queue.\n",
                    q.level + 1, now_str().c_str(), (unsigned long long)q.total_generated,
                    q.total_generated / el * 60.0, (unsigned long long)q.total_distinct,
                    q.total_distinct / el * 60.0, (unsigned long long)q.queue);
        std::fflush(stdout);
    };
    auto last_progress = std::chrono::steady_clock::now();
    bool reported = false, have_last = false;
    int printed_level = -1;  // the level of the last Progress line
    rmc_level_stats last{};
    while (rc == RMC_OK) {
        uint32_t nl = 0;
        rc = rmc_steps(ctx, lv.data(), (uint32_t)lv.size(), &nl);
        if (rc < 0) break;
        for (uint32_t i = 0; i < nl; i++) gpu_seconds += lv[i].seconds;
        if (nl == 0) continue;
        last = lv[nl - 1];
        have_last = true;
        const auto now = std::chrono::steady_clock::now();
        if (!reported || std::chrono::duration<double>(now - last_progress).count() >= progress_s) {
            progress(last);
            reported = true;
            printed_level = last.level;
            last_progress = now;
        }
        const double since = std::chrono::duration<double>(std::chrono::steady_clock::now() - last_ckpt).count();
        if (rc == RMC_OK && ckpt_minutes > 0 && since >= ckpt_minutes * 60.0) {
            // TLC -checkpoint: the run so far, between two levels (rmc_checkpoint)
            std::printf("Checkpointing of run %s\n", metadir.c_str());
            std::error_code ec;
            std::filesystem::create_directories(metadir, ec);  // TLC's states/ metadir (no shell)
            if (ec) std::fprintf(stderr, "raftmc: cannot create %s: %s\n", metadir.c_str(), ec.message().c_str());
            const std::string f = metadir + "/raftmc.ckpt";
            if (rmc_checkpoint(ctx, f.c_str()) < 0) std::printf("Warning: checkpoint failed: %s\n", rmc_last_error(ctx));
            else std::printf("Checkpointing completed at (%s)\n", now_str().c_str());
            last_ckpt = std::chrono::steady_clock::now();
        }
    }
    if (rc < 0) {
        std::printf("Error: %s\n", rmc_last_error(ctx));
        rmc_destroy(ctx);
        return 75;
    }
    if (have_last && last.level != printed_level) progress(last);  // the closing report (once)
    rmc_result res;
    rmc_get_result(ctx, &res);
    int exit_code = 0;
    if (res.status == RMC_DONE) {
        std::printf("Model checking completed. No error has been found.\n");
    } else {
        if (res.status == RMC_VIOLATION) {
            // the name the cfg used for the violated invariant (Inv and LeaderHasAllCommittedEntries share bit 0)
            std::string name = kInvNames[res.violated];
            for (const std::string &n : pm.invariant_names)
                if ((res.violated == 0 && (n == "Inv" || n == "LeaderHasAllCommittedEntries")) || n == kInvNames[res.violated])
                    name = n;
            std::printf("Error: Invariant %s is violated.\n", name.c_str());
            exit_code = 12;
        } else if (res.status == RMC_ASSERT) {
            std::printf("Error: The first argument of Assert evaluated to FALSE; the second argument was:\n\"split brain\"\n");
            exit_code = 14;
        } else if (res.status == RMC_EVAL_ERROR) {
            std::printf("Error: Evaluating invariant %s failed.\nAttempted to apply a tuple to an index out of its domain "
                        "(logs[p][index], %s.tla line 499).\n", kInvNames[res.violated], pm.module.c_str());
            exit_code = 75;
        } else if (res.status == RMC_DEADLOCK) {
            std::printf("Error: Deadlock reached.\n");
            exit_code = 11;
        }
        std::printf("Error: The behavior up to this point is:\n");
        std::vector<std::string> names(kActionNames, kActionNames + 13);
        names.insert(names.end(), kBfNames, kBfNames + 3);  // 13..15
        std::vector<Loc> locs = action_locations(tla, names);
        Printer pr{pm, cfg.n_servers, cfg.n_vals};
        std::vector<int32_t> buf(RMC_UNPACKED_INTS(5, 3, 256));
        std::vector<int32_t> prev_role(cfg.n_servers, 0);
        for (uint32_t i = 0; i < res.trace_len; i++) {
            int32_t a, s, w;
            int nints = rmc_trace_state(ctx, i, buf.data(), buf.size(), &a, &s, &w);
            if (nints < 0) break;
            if (a < 0) std::printf("State %u: <Initial predicate>\n", i + 1);
            else {
                const int an = (a == 12 && s >= 0 && s < cfg.n_servers) ? 13 + prev_role[s] : a;  // role: 0 F, 1 C, 2 L
                const Loc &L = locs[an];
                if (L.l0)
                    std::printf("State %u: <%s line %d, col %d to line %d, col %d of module %s>\n", i + 1,
                                names[an].c_str(), L.l0, L.c0, L.l1, L.c1, pm.module.c_str());
                else
                    std::printf("State %u: <%s(%s)>\n", i + 1, names[an].c_str(), pm.servers[s].c_str());
            }
            for (int q = 0; q < cfg.n_servers; q++) prev_role[q] = buf[2 * cfg.n_servers + q];  // unpacked: vf, ct, role
            std::printf("%s\n", pr.state(buf.data()).c_str());
        }
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("%llu states generated, %llu distinct states found, %llu states left on queue.\n",
                (unsigned long long)res.generated, (unsigned long long)res.distinct, (unsigned long long)res.queue);
    if (res.status == RMC_DONE)
        std::printf("The depth of the complete state graph search is %d.\n", res.depth);
    std::printf("Finished in %.2fs at (%s)\n", el, now_str().c_str());
    std::printf("GPU: %.0f distinct states/s over %.3f s of BFS levels (MI355X, %d device%s).\n",
                gpu_seconds > 0 ? res.distinct / gpu_seconds : 0.0, gpu_seconds, cfg.world_size > 1 ? cfg.world_size : 1,
                cfg.world_size > 1 ? "s" : "");
    // The process ends here: by default the device and host memory (~250 GB and ~110 GB of
    // trace at Raft.cfg) go back with the process instead of through rmc_destroy, whose frees took
    // ~16 s after a Raft.cfg exhaustion (RMC_FAST_EXIT=0 destroys the context first).
    std::fflush(stdout);
    std::fflush(stderr);
    const char *fe = std::getenv("RMC_FAST_EXIT");
    if (!(fe && std::string(fe) == "0")) {
        if (g_report_fd >= 0) {  // detached worker: the device goes back before the caller has its code
            phase_time("release device");
            rmc_release_device(ctx);
            phase_time("device released");
            report(exit_code);
        }
        std::_Exit(exit_code);
    }
    phase_time("destroy");
    rmc_destroy(ctx);
    phase_time("destroyed");
    return exit_code;
    };
    if (gpus > 1 || onerank) return run_ranks(gpus, onerank, cfg, check);
    const char *det = std::getenv("RMC_DETACH");  // RMC_DETACH=0: one process, exit after the teardown
    if (det && std::string(det) == "0") return check(cfg);
    return run_detached(cfg, check);
}
