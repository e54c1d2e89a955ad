// Timing of the custom-reducer allreduce (include/rdc.h
// ICommunicator::Allreduce(Buffer, ReduceFunction); the reference's
// communicator.h:92-93 with a user reducer, called per received chunk) on a
// HOST buffer, one process per rank.
//
//   custom_reducer_bench <MiB> <iters> [key=val ...]   (RDC_RANK / rdc_world_size / tracker keys)
//
// Prints one JSON line per rank: median / min ms per call and the process's
// peak resident set (the host memory the path holds), and checks the result
// (every rank's value is r + 1 at every element -> sum n(n+1)/2, exact).
#include <stdio.h>
#include <stdlib.h>
#include <sys/resource.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "rdc.h"

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s <MiB> <iters> [key=val ...]\n", argv[0]);
        return 2;
    }
    const size_t mib = (size_t)atol(argv[1]);
    const int iters = atoi(argv[2]);
    rdc::Init(argc - 3, argv + 3);
    const int r = rdc::GetRank(), n = rdc::GetWorldSize();
    const size_t N = mib * (1u << 20) / 4;
    std::vector<float> f(N);
    rdc::comm::ICommunicator* c = rdc::GetCommunicator();
    std::vector<double> ms;
    for (int it = 0; it < iters + 1; ++it) {
        std::fill(f.begin(), f.end(), (float)(r + 1));
        rdc::Buffer b(f.data(), N * 4);
        b.set_item_size(4);
        rdc::Barrier();
        const auto t0 = std::chrono::steady_clock::now();
        c->Allreduce(b, [](rdc::Buffer src, rdc::Buffer dst) {
            float* d = dst.As<float>();
            const float* s = src.As<float>();
            for (uint64_t i = 0; i < dst.Count(); ++i) d[i] += s[i];
        });
        const double el = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (it > 0) ms.push_back(el);  // the first call is a warm-up (engines, slots)
        const float want = (float)(n * (n + 1) / 2);
        for (size_t i = 0; i < N; i += 4099)
            if (f[i] != want) {
                fprintf(stderr, "rank %d: wrong result at %zu: %f\n", r, i, f[i]);
                return 1;
            }
    }
    std::sort(ms.begin(), ms.end());
    struct rusage ru;
    getrusage(RUSAGE_SELF, &ru);
    printf("{\"rank\": %d, \"n\": %d, \"MiB\": %zu, \"iters\": %d, \"median_ms\": %.3f, \"min_ms\": %.3f, "
           "\"max_rss_MiB\": %.1f}\n",
           r, n, mib, iters, ms[ms.size() / 2], ms[0], ru.ru_maxrss / 1024.0);
    rdc::Finalize();
    return 0;
}
