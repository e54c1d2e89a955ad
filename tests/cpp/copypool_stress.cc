// Stress of rdc_amd::CopyPool (rdc_amd/csrc/rdc_copypool.h): many short
// Run() calls back to back, each job a lambda on the caller's stack that is
// destroyed as soon as Run returns, so a pool thread that woke late and ran
// an item with a stale job would touch a dead frame (the crash this test was
// written for).  Every item of every call must run exactly once.
//   g++ -O2 -std=c++17 -pthread -I rdc_amd/csrc tests/cpp/copypool_stress.cc
#include <atomic>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rdc_copypool.h"

int main(int argc, char** argv) {
    const int calls = argc > 1 ? atoi(argv[1]) : 200000;
    rdc_amd::CopyPool pool(3);
    long bad = 0;
    for (int c = 0; c < calls; ++c) {
        const int n = 2 + (c % 2);
        std::vector<int> hits(n, 0);
        // the job lives on the heap and is freed as soon as Run returns: a
        // pool thread running an item with a stale job pointer touches freed
        // memory (AddressSanitizer reports it; on the stack the next call's
        // job would sit at the same address and hide it)
        auto* job = new std::function<void(int)>([&hits](int i) { hits[i] += 1; });
        pool.Run(n, *job);
        delete job;
        for (int i = 0; i < n; ++i)
            if (hits[i] != 1) ++bad;
    }
    printf("{\"calls\": %d, \"bad\": %ld}\n", calls, bad);
    return bad ? 1 : 0;
}
