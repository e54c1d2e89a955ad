// Write-counter calibration for stores into ANOTHER process's uncached
// scratch through a HIP IPC mapping (what the collectives' scatter / gather
// pushes do), beside stores into the writer's own uncached memory.
//   hipcc --offload-arch=gfx950 -O3 -o tools/uc_ipc_pmc tools/uc_ipc_pmc.hip
//   tools/uc_ipc_pmc owner DIR &                      # exports 256 MiB, waits for DIR/done
//   rocprofv3 --pmc WRITE_SIZE -d OUT -o run --output-format csv -- tools/uc_ipc_pmc writer DIR
//   tools/uc_ipc_pmc busy SECONDS        # an unprofiled process storing into its own memory meanwhile
// Kernels: k_ipc_store (256 MiB into the owner's memory), k_local_store (256 MiB local).
// TCC counters are device-wide: with `busy` running, the profiled dispatches
// also count its stores.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

__global__ __launch_bounds__(256) void k_ipc_store(v4u* d, uint64_t nvec) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * 256)
        __builtin_nontemporal_store(v4u{(uint32_t)i, 7u, 8u, 9u}, d + i);
}
__global__ __launch_bounds__(256) void k_local_store(v4u* d, uint64_t nvec) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * 256)
        __builtin_nontemporal_store(v4u{(uint32_t)i, 7u, 8u, 9u}, d + i);
}

static const uint64_t kBytes = 256ull << 20;

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s owner|writer DIR\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1], dir = argv[2];
    if (mode == "busy") {  // store into own uncached memory for `dir` seconds
        void* p = nullptr;
        CK(hipExtMallocWithFlags(&p, kBytes, hipDeviceMallocUncached));
        const double secs = atof(dir.c_str());
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0));
        int launches = 0;
        for (float el = 0; el < secs * 1000; ++launches) {
            for (int k = 0; k < 20; ++k) {
                hipLaunchKernelGGL(k_local_store, dim3(1024), dim3(256), 0, 0, (v4u*)p, kBytes / 16);
                CK(hipGetLastError());
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&el, e0, e1));
        }
        float el = 0;
        CK(hipEventElapsedTime(&el, e0, e1));
        printf("{\"busy_launches\": %d, \"busy_GBps\": %.1f}\n", launches * 20,
               (double)launches * 20 * kBytes / (el * 1e-3) / 1e9);
        CK(hipFree(p));
        return 0;
    }
    const std::string hfile = dir + "/handle", dfile = dir + "/done";
    if (mode == "owner") {
        void* p = nullptr;
        CK(hipExtMallocWithFlags(&p, kBytes, hipDeviceMallocUncached));
        CK(hipMemset(p, 0, kBytes));
        CK(hipDeviceSynchronize());
        hipIpcMemHandle_t h;
        CK(hipIpcGetMemHandle(&h, p));
        const std::string tmp = hfile + ".tmp";
        FILE* f = fopen(tmp.c_str(), "wb");
        if (!f || fwrite(&h, sizeof h, 1, f) != 1) return 3;
        fclose(f);
        rename(tmp.c_str(), hfile.c_str());
        for (int i = 0; i < 6000 && access(dfile.c_str(), F_OK) != 0; ++i) usleep(10000);  // <= 60 s
        uint32_t probe[4] = {0, 0, 0, 0};
        CK(hipMemcpy(probe, static_cast<char*>(p) + 16 * 12345, 16, hipMemcpyDeviceToHost));
        printf("{\"owner_check\": %s}\n", probe[0] == 12345 && probe[1] == 7 ? "true" : "false");
        CK(hipFree(p));
        return 0;
    }
    for (int i = 0; i < 6000 && access(hfile.c_str(), F_OK) != 0; ++i) usleep(10000);
    hipIpcMemHandle_t h;
    FILE* f = fopen(hfile.c_str(), "rb");
    if (!f || fread(&h, sizeof h, 1, f) != 1) return 4;
    fclose(f);
    void* remote = nullptr;
    CK(hipIpcOpenMemHandle(&remote, h, hipIpcMemLazyEnablePeerAccess));
    void* local = nullptr;
    CK(hipExtMallocWithFlags(&local, kBytes, hipDeviceMallocUncached));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t nvec = kBytes / 16;
    for (int rep = 0; rep < 2; ++rep) {
        float a = 0, b = 0;
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_ipc_store, dim3(1024), dim3(256), 0, 0, (v4u*)remote, nvec);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&a, e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_local_store, dim3(1024), dim3(256), 0, 0, (v4u*)local, nvec);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&b, e0, e1));
        printf("{\"rep\": %d, \"bytes\": %llu, \"ipc_ms\": %.4f, \"local_ms\": %.4f}\n", rep,
               (unsigned long long)kBytes, a, b);
    }
    CK(hipIpcCloseMemHandle(remote));
    CK(hipFree(local));
    FILE* d = fopen(dfile.c_str(), "w");
    if (d) fclose(d);
    return 0;
}
