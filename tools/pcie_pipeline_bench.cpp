// The host-buffer allreduce's PCIe pipeline WITHOUT the allreduce
// (rdc_host.cpp): per piece, the caller memcpys the piece from a pageable
// buffer into one of 3 pinned slots (4 threads), H2D on one stream; a drain
// thread waits for the piece and copies it back into the pageable buffer with
// a pageable D2H on a second stream.  What the link and the host give one
// process — and, started together (a shared start time), two processes on the
// same GPU, as the n = 2 rehearsal runs.
//
//   hipcc -O2 --offload-arch=gfx950 tools/pcie_pipeline_bench.cpp -o tools/pcie_pipeline_bench
//   tools/pcie_pipeline_bench <bytes> <piece bytes> <iters> [start_at_epoch_ms]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../rdc_amd/csrc/rdc_copypool.h"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static double now_ms() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}
static double epoch_ms() {
    timespec t;
    clock_gettime(CLOCK_REALTIME, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

// the host path's own copy pool (3 threads + the caller), same split
static rdc_amd::CopyPool g_pool(3);
static void par_copy(char* dst, const char* src, size_t bytes) {
    const int parts = (int)std::min<size_t>(16, bytes / (256 << 10));
    const size_t per = (bytes / (size_t)parts + 4095) & ~(size_t)4095;
    g_pool.Run(parts, [&](int i) {
        const size_t lo = (size_t)i * per;
        if (lo < bytes) memcpy(dst + lo, src + lo, std::min(per, bytes - lo));
    });
}

int main(int argc, char** argv) {
    const size_t S = argc > 1 ? strtoull(argv[1], nullptr, 0) : (64u << 20);
    const size_t P = argc > 2 ? strtoull(argv[2], nullptr, 0) : (8u << 20);
    const int iters = argc > 3 ? atoi(argv[3]) : 10;
    const double start_at = argc > 4 ? atof(argv[4]) : 0;
    const int K = (int)((S + P - 1) / P);
    const int kSlots = 3;
    std::vector<char> user(S, 1);
    char* dev = nullptr;
    CK(hipMalloc(&dev, S));
    char* slot[kSlots];
    hipEvent_t in_done[kSlots];
    for (int i = 0; i < kSlots; ++i) {
        CK(hipHostMalloc(reinterpret_cast<void**>(&slot[i]), P, hipHostMallocDefault));
        CK(hipEventCreateWithFlags(&in_done[i], hipEventDisableTiming));
    }
    std::vector<hipEvent_t> ready((size_t)K);
    for (auto& ev : ready) CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipStream_t h2d, d2h;
    CK(hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking));
    auto one_call = [&] {
        std::atomic<int> posted{0};
        std::thread drain([&] {
            for (int k = 0; k < K; ++k) {
                while (posted.load() <= k) std::this_thread::yield();
                CK(hipEventSynchronize(ready[(size_t)k]));
                const size_t len = std::min(P, S - (size_t)k * P);
                CK(hipMemcpyAsync(user.data() + (size_t)k * P, dev + (size_t)k * P, len, hipMemcpyDeviceToHost, d2h));
                CK(hipStreamSynchronize(d2h));
            }
        });
        for (int k = 0; k < K; ++k) {
            const int s = k % kSlots;
            const size_t len = std::min(P, S - (size_t)k * P);
            if (k >= kSlots) CK(hipEventSynchronize(in_done[s]));
            par_copy(slot[s], user.data() + (size_t)k * P, len);
            CK(hipMemcpyAsync(dev + (size_t)k * P, slot[s], len, hipMemcpyHostToDevice, h2d));
            CK(hipEventRecord(in_done[s], h2d));
            CK(hipEventRecord(ready[(size_t)k], h2d));
            posted.store(k + 1);
        }
        drain.join();
    };
    one_call();  // warm-up
    if (start_at > 0)
        while (epoch_ms() < start_at) std::this_thread::sleep_for(std::chrono::microseconds(100));
    std::vector<double> ms;
    for (int i = 0; i < iters; ++i) {
        const double t0 = now_ms();
        one_call();
        ms.push_back(now_ms() - t0);
    }
    std::sort(ms.begin(), ms.end());
    printf("{\"bytes\": %zu, \"piece\": %zu, \"iters\": %d, \"median_ms\": %.3f, \"min_ms\": %.3f, "
           "\"GBps_each_way\": %.1f}\n",
           S, P, iters, ms[ms.size() / 2], ms[0], S / (ms[ms.size() / 2] * 1e-3) / 1e9);
    return 0;
}
