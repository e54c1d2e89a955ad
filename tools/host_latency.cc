// Small synchronous HOST allreduce latency through the C ABI, no Python in
// the loop: forks `world` ranks (before any HIP call) on GPU 0, each times
// RdcAllreduce on a pageable buffer; rank 0 prints medians (microseconds).
//   g++ -O2 -std=c++17 -Iinclude -o tools/host_latency tools/host_latency.cc -Lrdc_amd -lrdc_amd \
//       -Wl,-rpath,'$ORIGIN/../rdc_amd' -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -L/opt/rocm/lib -lamdhip64
//   tools/host_latency [world] [iters] [bytes,bytes,...]
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "rdc_amd.h"

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

static std::vector<size_t> g_sizes = {4, 4096, 16384, 65536};

static int run(int rank, int world, int port, int iters) {
    std::string a0 = "RDC_RANK=" + std::to_string(rank), a1 = "RDC_WORLD_SIZE=" + std::to_string(world),
                a2 = "RDC_TRACKER_PORT=" + std::to_string(port), a3 = "RDC_TRACKER_URI=127.0.0.1";
    char* argv[4] = {&a0[0], &a1[0], &a2[0], &a3[0]};
    if (RdcInit(4, argv) != 0) return 1;
    if (rank == 0) fprintf(stderr, "[host_latency] world %d initialised\n", world);
    std::vector<float> buf(16384);
    // pointer classification alone
    std::vector<double> tattr;
    for (int i = 0; i < 2000; ++i) {
        hipPointerAttribute_t at;
        auto t0 = std::chrono::steady_clock::now();
        if (hipPointerGetAttributes(&at, buf.data()) != hipSuccess) (void)hipGetLastError();
        tattr.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::string out = "{\"world\": " + std::to_string(world) + ", \"iters\": " + std::to_string(iters) +
                      ", \"ptr_attr_us\": " + std::to_string(median(tattr));
    int bad = 0;
    for (size_t bytes : g_sizes) {
        const size_t count = bytes / 4;
        std::vector<double> t;
        for (int i = 0; i < iters + 100; ++i) {
            for (size_t j = 0; j < count; ++j) buf[j] = (float)(rank + 1 + (j % 7));
            RdcBarrier();
            auto t0 = std::chrono::steady_clock::now();
            if (RdcAllreduce(buf.data(), count, 6, 2, nullptr, nullptr) != 0) return 2;
            auto t1 = std::chrono::steady_clock::now();
            if (i >= 100) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            for (size_t j = 0; j < count; ++j)
                if (buf[j] != (float)(world * (world + 1) / 2 + world * (j % 7))) ++bad;
        }
        // back-to-back (no barrier between calls): the steady-state rate
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < iters; ++i)
            if (RdcAllreduce(buf.data(), count, 6, 0, nullptr, nullptr) != 0) return 3;
        const double b2b = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
        if (rank == 0) fprintf(stderr, "[host_latency] world %d bytes %zu done\n", world, bytes);
        out += ", \"" + std::to_string(bytes) + "\": {\"after_barrier_us\": " + std::to_string(median(t)) +
               ", \"back_to_back_us\": " + std::to_string(b2b) + "}";
    }
    out += ", \"bad\": " + std::to_string(bad) + "}";
    if (rank == 0) printf("%s\n", out.c_str());
    RdcFinalize();
    return bad ? 4 : 0;
}

int main(int argc, char** argv) {
    const int world = argc > 1 ? atoi(argv[1]) : 2;
    const int iters = argc > 2 ? atoi(argv[2]) : 2000;
    if (argc > 3) {  // comma-separated byte sizes
        g_sizes.clear();
        for (char* t = strtok(argv[3], ","); t; t = strtok(nullptr, ",")) g_sizes.push_back((size_t)atol(t));
    }
    const int port = 20000 + (int)(getpid() % 20000);
    std::vector<pid_t> kids;
    for (int r = 1; r < world; ++r) {
        pid_t p = fork();
        if (p == 0) _exit(run(r, world, port, iters));
        kids.push_back(p);
    }
    int rc = run(0, world, port, iters);
    for (pid_t p : kids) {
        int st = 0;
        waitpid(p, &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = rc ? rc : 10;
    }
    return rc;
}
