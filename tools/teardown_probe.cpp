// Where a large run's teardown goes (myrun.sh: ~12 s between "Finished" and the shell prompt after a
// Raft.cfg exhaustion): free of pinned host blocks (the trace: ~110 GB in 32 MB hipHostMalloc
// blocks), of pageable host memory (4 KB pages or transparent huge pages) and of device memory.
// usage: teardown_probe MODE GB   MODE = pinned | pageable | thp | device, each timed alloc+touch
// and free; MODE-exit: the same allocation left to process exit (time it from the shell).
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    std::string mode = argv[1];
    const bool leave = mode.size() > 5 && mode.substr(mode.size() - 5) == "-exit";
    if (leave) mode = mode.substr(0, mode.size() - 5);
    const size_t gb = strtoull(argv[2], nullptr, 10), bytes = gb << 30, blk = 32ull << 20;
    double t0 = now();
    if (mode == "pinned") {
        std::vector<void *> v;
        for (size_t done = 0; done < bytes; done += blk) {
            void *p = nullptr;
            if (hipHostMalloc(&p, blk, hipHostMallocDefault) != hipSuccess) { fprintf(stderr, "hipHostMalloc failed\n"); return 1; }
            memset(p, 1, blk);
            v.push_back(p);
        }
        double t1 = now();
        printf("pinned %zu GB: alloc+touch %.2f s\n", gb, t1 - t0);
        fflush(stdout);
        if (leave) return 0;
        for (void *p : v) (void)hipHostFree(p);
        printf("pinned %zu GB: free %.2f s\n", gb, now() - t1);
    } else if (mode == "pageable" || mode == "thp") {
        void *p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) return 1;
        if (mode == "thp") madvise(p, bytes, MADV_HUGEPAGE);
        memset(p, 1, bytes);
        double t1 = now();
        printf("%s %zu GB: alloc+touch %.2f s\n", mode.c_str(), gb, t1 - t0);
        fflush(stdout);
        if (leave) return 0;
        munmap(p, bytes);
        printf("%s %zu GB: free %.2f s\n", mode.c_str(), gb, now() - t1);
    } else if (mode == "device") {
        std::vector<void *> v;
        const size_t dblk = 16ull << 30;
        for (size_t done = 0; done < bytes; done += dblk) {
            void *p = nullptr;
            if (hipMalloc(&p, dblk) != hipSuccess) { fprintf(stderr, "hipMalloc failed\n"); return 1; }
            (void)hipMemset(p, 1, dblk);
            v.push_back(p);
        }
        (void)hipDeviceSynchronize();
        double t1 = now();
        printf("device %zu GB: alloc+touch %.2f s\n", gb, t1 - t0);
        fflush(stdout);
        if (leave) return 0;
        for (void *p : v) (void)hipFree(p);
        (void)hipDeviceSynchronize();
        printf("device %zu GB: free %.2f s\n", gb, now() - t1);
    }
    return 0;
}
