// Raw PCIe capacity of this GPU's link as the host path uses it: DMA only,
// no host memcpy.  Times S bytes
//   h2d    : pinned -> device, one stream
//   d2h    : device -> pinned, one stream
//   d2h_pg : device -> pageable (what the pipeline's drain does)
//   duplex : h2d and d2h at once on two streams (pinned both ways)
//   duplex_pg: h2d (pinned) and d2h (pageable) at once
// Optional argv[2] = start time (ms since the epoch, CLOCK_REALTIME) so two
// processes can start together on the same GPU (the n = 2 rehearsal's sharing).
//   hipcc -O2 tools/pcie_duplex.cpp -o tools/pcie_duplex && tools/pcie_duplex [bytes] [start_ms]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static double now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char** argv) {
    const size_t S = argc > 1 ? strtoull(argv[1], 0, 0) : (256ull << 20);
    const long long start_ms = argc > 2 ? atoll(argv[2]) : 0;
    char *hin, *hout, *dev_in, *dev_out;
    CK(hipHostMalloc(reinterpret_cast<void**>(&hin), S, hipHostMallocDefault));
    CK(hipHostMalloc(reinterpret_cast<void**>(&hout), S, hipHostMallocDefault));
    char* pg = static_cast<char*>(aligned_alloc(4096, S));
    memset(hin, 1, S);
    memset(hout, 2, S);
    memset(pg, 3, S);
    CK(hipMalloc(&dev_in, S));
    CK(hipMalloc(&dev_out, S));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    // warm-up (first-touch mappings, pageable pinning paths)
    CK(hipMemcpyAsync(dev_in, hin, S, hipMemcpyHostToDevice, a));
    CK(hipMemcpyAsync(hout, dev_out, S, hipMemcpyDeviceToHost, b));
    CK(hipMemcpyAsync(pg, dev_out, S, hipMemcpyDeviceToHost, b));
    CK(hipDeviceSynchronize());
    if (start_ms > 0) {
        for (;;) {
            timespec t;
            clock_gettime(CLOCK_REALTIME, &t);
            const long long ms = (long long)t.tv_sec * 1000 + t.tv_nsec / 1000000;
            if (ms >= start_ms) break;
            usleep(200);
        }
    }
    const int reps = 5;
    auto run = [&](int mode) {
        double best = 1e30;
        for (int r = 0; r < reps; ++r) {
            const double t0 = now();
            if (mode == 0 || mode == 3 || mode == 4) CK(hipMemcpyAsync(dev_in, hin, S, hipMemcpyHostToDevice, a));
            if (mode == 1 || mode == 3) CK(hipMemcpyAsync(hout, dev_out, S, hipMemcpyDeviceToHost, b));
            if (mode == 2 || mode == 4) CK(hipMemcpyAsync(pg, dev_out, S, hipMemcpyDeviceToHost, b));
            CK(hipStreamSynchronize(a));
            CK(hipStreamSynchronize(b));
            const double t = now() - t0;
            if (t < best) best = t;
        }
        return best;
    };
    const char* names[] = {"h2d", "d2h", "d2h_pg", "duplex", "duplex_pg"};
    printf("{\"bytes\": %zu", S);
    for (int m = 0; m < 5; ++m) {
        const double t = run(m);
        const double moved = (m >= 3 ? 2.0 : 1.0) * (double)S;
        printf(", \"%s_ms\": %.3f, \"%s_GBps\": %.1f", names[m], t * 1e3, names[m], moved / t / 1e9);
    }
    printf("}\n");
    return 0;
}
