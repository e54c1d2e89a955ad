// PCIe rates of KERNEL accesses to registered host memory vs the DMA engines
// (hipMemcpyAsync), one process, one GPU: is a zero-copy allreduce of a
// registered host buffer (the kernel reading its input from and writing its
// result to host memory, no device image) PCIe-bound at the link rate?
//   hipcc --offload-arch=gfx950 -O3 -o tools/zc_bw tools/zc_bw.hip && tools/zc_bw [MiB]
// Prints one JSON line per (variant, grid): GB/s of host bytes moved.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

// mode 0: dev = host (read host), 1: host = dev (write host), 2: host += dev (read + write host)
template <int MODE>
__global__ __launch_bounds__(256) void k_zc(v4u* __restrict__ host, v4u* __restrict__ dev, uint64_t nvec) {
    constexpr int U = 4;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        v4u a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (MODE != 1) a[u] = __builtin_nontemporal_load(host + i + u * stride);
            if (MODE != 0) b[u] = __builtin_nontemporal_load(dev + i + u * stride);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (MODE == 0) __builtin_nontemporal_store(a[u], dev + i + u * stride);
            if (MODE == 1) __builtin_nontemporal_store(b[u], host + i + u * stride);
            if (MODE == 2) __builtin_nontemporal_store(a[u] + b[u], host + i + u * stride);
        }
    }
    for (; i < nvec; i += stride) {
        if (MODE == 0) dev[i] = host[i];
        if (MODE == 1) host[i] = dev[i];
        if (MODE == 2) host[i] = host[i] + dev[i];
    }
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 256;
    const size_t bytes = mib << 20;
    void* h = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (h == MAP_FAILED) return 1;
    memset(h, 1, bytes);
    CHECK(hipHostRegister(h, bytes, hipHostRegisterMapped));
    void* hd = nullptr;
    CHECK(hipHostGetDevicePointer(&hd, h, 0));
    void* d = nullptr;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMemset(d, 0, bytes));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const uint64_t nvec = bytes / 16;
    auto timeit = [&](auto&& fn, int reps) {
        fn();
        CHECK(hipStreamSynchronize(s));
        CHECK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; ++r) fn();
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        return ms / reps;
    };
    const char* names[3] = {"kernel_read_host", "kernel_write_host", "kernel_rw_host"};
    for (int grid : {64, 128, 256, 512, 1024, 2048}) {
        for (int mode = 0; mode < 3; ++mode) {
            float ms = timeit([&] {
                if (mode == 0) hipLaunchKernelGGL(k_zc<0>, dim3(grid), dim3(256), 0, s, (v4u*)hd, (v4u*)d, nvec);
                if (mode == 1) hipLaunchKernelGGL(k_zc<1>, dim3(grid), dim3(256), 0, s, (v4u*)hd, (v4u*)d, nvec);
                if (mode == 2) hipLaunchKernelGGL(k_zc<2>, dim3(grid), dim3(256), 0, s, (v4u*)hd, (v4u*)d, nvec);
            }, 5);
            const double moved = mode == 2 ? 2.0 * bytes : (double)bytes;
            printf("{\"variant\": \"%s\", \"grid\": %d, \"MiB\": %zu, \"ms\": %.3f, \"GBps_host_bytes\": %.1f}\n",
                   names[mode], grid, mib, ms, moved / (ms * 1e-3) / 1e9);
        }
    }
    float h2d = timeit([&] { CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s)); }, 5);
    float d2h = timeit([&] { CHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s)); }, 5);
    printf("{\"variant\": \"dma_h2d\", \"MiB\": %zu, \"ms\": %.3f, \"GBps_host_bytes\": %.1f}\n", mib, h2d,
           bytes / (h2d * 1e-3) / 1e9);
    printf("{\"variant\": \"dma_d2h\", \"MiB\": %zu, \"ms\": %.3f, \"GBps_host_bytes\": %.1f}\n", mib, d2h,
           bytes / (d2h * 1e-3) / 1e9);
    CHECK(hipHostUnregister(h));
    munmap(h, bytes);
    return 0;
}
