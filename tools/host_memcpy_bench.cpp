// Host memcpy bandwidth on the GPU box (no GPU involved): S bytes from a
// touched pageable buffer into another, split over T threads, plain memcpy
// vs streaming stores (rdc_copypool.h StreamCopy), best of 5.  The host
// path's copy into pinned slots is this copy.
//   g++ -O2 -std=c++17 -pthread -I rdc_amd/csrc tools/host_memcpy_bench.cpp -o tools/host_memcpy_bench
//   tools/host_memcpy_bench [bytes]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <thread>
#include <vector>

#include "rdc_copypool.h"

static double now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char** argv) {
    const size_t S = argc > 1 ? strtoull(argv[1], 0, 0) : (256ull << 20);
    char* src = static_cast<char*>(aligned_alloc(4096, S));
    char* dst = static_cast<char*>(aligned_alloc(4096, S));
    memset(src, 1, S);
    memset(dst, 2, S);
    printf("{\"bytes\": %zu", S);
    for (int nt = 0; nt < 2; ++nt)
        for (int T : {1, 2, 4, 8, 16}) {
            double best = 1e30;
            for (int r = 0; r < 5; ++r) {
                const double t0 = now();
                std::vector<std::thread> th;
                const size_t per = (S / T + 4095) & ~(size_t)4095;
                for (int i = 0; i < T; ++i)
                    th.emplace_back([&, i] {
                        const size_t lo = (size_t)i * per;
                        if (lo >= S) return;
                        const size_t n = std::min(per, S - lo);
                        if (nt) rdc_amd::StreamCopy(dst + lo, src + lo, n);
                        else memcpy(dst + lo, src + lo, n);
                    });
                for (auto& t : th) t.join();
                const double t = now() - t0;
                if (t < best) best = t;
            }
            printf(", \"%s_t%d_GBps\": %.1f", nt ? "stream" : "memcpy", T, S / best / 1e9);
        }
    printf("}\n");
    return 0;
}
