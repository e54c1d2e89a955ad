// Host<->device copy options for the host-resident allreduce path (rdc's
// buffers begin and end in host memory).  Times, for one pageable buffer of
// S bytes: pageable hipMemcpyAsync H2D / D2H; hipHostRegister + async copies
// + hipHostUnregister (per call); copies from an already registered buffer;
// hipHostMalloc'd buffers.
//   hipcc -O2 tools/host_copy_bench.cpp -o /tmp/host_copy_bench && /tmp/host_copy_bench [bytes]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <thread>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));       \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

static double now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char** argv) {
    const size_t S = argc > 1 ? strtoull(argv[1], 0, 0) : (256ull << 20);
    char* h = (char*)aligned_alloc(4096, S);
    memset(h, 1, S);
    char* d;
    CK(hipMalloc(&d, S));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto rate = [&](const char* what, double t) { printf("%-44s %8.3f ms  %6.1f GB/s\n", what, t * 1e3, S / t / 1e9); };
    for (int rep = 0; rep < 2; ++rep) {
        double t0 = now();
        CK(hipMemcpyAsync(d, h, S, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        rate("pageable H2D", now() - t0);
        t0 = now();
        CK(hipMemcpyAsync(h, d, S, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        rate("pageable D2H", now() - t0);
        t0 = now();
        CK(hipHostRegister(h, S, hipHostRegisterDefault));
        const double treg = now() - t0;
        rate("hipHostRegister", treg);
        t0 = now();
        CK(hipMemcpyAsync(d, h, S, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        rate("registered H2D", now() - t0);
        t0 = now();
        CK(hipMemcpyAsync(h, d, S, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        rate("registered D2H", now() - t0);
        t0 = now();
        CK(hipMemcpyAsync(d, h, S / 2, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(h + S / 2, d + S / 2, S / 2, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        rate("registered H2D+D2H half each, one stream", now() - t0);
        t0 = now();
        CK(hipHostUnregister(h));
        rate("hipHostUnregister", now() - t0);
    }
    char* p;
    CK(hipHostMalloc(&p, S, hipHostMallocDefault));
    memset(p, 2, S);
    double t0 = now();
    CK(hipMemcpyAsync(d, p, S, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    rate("hipHostMalloc H2D", now() - t0);
    t0 = now();
    CK(hipMemcpyAsync(p, d, S, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    rate("hipHostMalloc D2H", now() - t0);
    t0 = now();
    memcpy(p, h, S);
    rate("host memcpy pageable -> pinned (1 thread)", now() - t0);
    for (int T : {2, 4, 8}) {
        t0 = now();
        std::vector<std::thread> th;
        for (int i = 0; i < T; ++i)
            th.emplace_back([&, i] { memcpy(p + S / T * i, h + S / T * i, S / T); });
        for (auto& x : th) x.join();
        char what[64];
        snprintf(what, sizeof(what), "host memcpy pageable -> pinned (%d threads)", T);
        rate(what, now() - t0);
    }
    {   // full duplex: pinned H2D and D2H of S each, concurrently on two streams
        char* p2;
        char* d2;
        CK(hipHostMalloc(&p2, S, hipHostMallocDefault));
        CK(hipMalloc(&d2, S));
        hipStream_t s2;
        CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        for (int rep = 0; rep < 2; ++rep) {
            t0 = now();
            CK(hipMemcpyAsync(d, p, S, hipMemcpyHostToDevice, s));
            CK(hipMemcpyAsync(p2, d2, S, hipMemcpyDeviceToHost, s2));
            CK(hipStreamSynchronize(s));
            CK(hipStreamSynchronize(s2));
            rate("pinned H2D || D2H, 2 streams (S each way)", now() - t0);
            t0 = now();
            CK(hipMemcpyAsync(d, p, S, hipMemcpyHostToDevice, s));
            CK(hipMemcpyAsync(h, d2, S, hipMemcpyDeviceToHost, s2));  // pageable D2H
            CK(hipStreamSynchronize(s));
            CK(hipStreamSynchronize(s2));
            rate("pinned H2D || pageable D2H (S each way)", now() - t0);
        }
        CK(hipHostFree(p2));
        CK(hipFree(d2));
    }
    CK(hipHostFree(p));
    CK(hipFree(d));
    free(h);
    return 0;
}
