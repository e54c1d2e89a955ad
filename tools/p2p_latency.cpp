// Point-to-point engine latency without Python: a 2-rank single-process group
// on GPU 0 (RdcCommInitAll), rank 0 -> rank 1 transfers of device buffers
// through the C ABI, one at a time (post send + recv, wait both).
// g++ -O2 -Iinclude tools/p2p_latency.cpp -Lrdc_amd -lrdc_amd -Wl,-rpath,$PWD/rdc_amd -o tools/p2p_latency
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>

#include "rdc_amd.h"

int main(int argc, char** argv) {
    void* comms[2];
    int devs[2] = {0, 0};
    if (RdcCommInitAll(comms, 2, devs, 16 << 20)) {
        printf("init: %s\n", RdcGetLastError());
        return 1;
    }
    const size_t sizes[] = {4, 4096, 65536, 1 << 20, 4 << 20, 64 << 20};
    for (size_t S : sizes) {
        void *x, *y;
        if (hipMalloc(&x, S) || hipMalloc(&y, S)) return 1;
        hipMemset(x, 1, S);
        hipDeviceSynchronize();
        const int iters = S >= (64 << 20) ? 20 : 500;
        double tot = 0, best = 1e9;
        for (int i = 0; i < iters + 20; ++i) {
            auto t0 = std::chrono::steady_clock::now();
            void *ws, *wr;
            if (RdcCommIRecv(&wr, comms[1], y, S, 0, nullptr) || RdcCommISend(&ws, comms[0], x, S, 1, nullptr)) {
                printf("post: %s\n", RdcGetLastError());
                return 1;
            }
            if (RdcWorkCompletionWait(ws) || RdcWorkCompletionWait(wr)) {
                printf("wait: %s\n", RdcGetLastError());
                return 1;
            }
            RdcDelWorkCompletion(ws);
            RdcDelWorkCompletion(wr);
            const double dt = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            if (i >= 20) {
                tot += dt;
                if (dt < best) best = dt;
            }
        }
        printf("p2p %10zu B: mean %8.2f us  best %8.2f us  %.2f GB/s\n", S, tot / iters, best, S / (tot / iters) / 1e3);
        hipFree(x);
        hipFree(y);
    }
    RdcCommDestroy(comms[0]);
    RdcCommDestroy(comms[1]);
    return 0;
}
