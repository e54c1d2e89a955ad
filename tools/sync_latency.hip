// Host round-trip latency of a tiny launch on MI355X: what a small
// host-buffer collective pays per call besides the collective itself.
//   a) kernel + hipStreamSynchronize
//   b) kernel + hipStreamWriteValue32 into pinned memory + host spin on it
//   c) kernel whose last store goes to pinned memory (system scope) + host spin
// hipcc --offload-arch=gfx950 -O2 tools/sync_latency.hip -o tools/sync_latency
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>

__global__ void k_touch(uint32_t* dev, uint32_t* host_flag, uint32_t v) {
    if (threadIdx.x == 0) {
        dev[0] = v;
        if (host_flag) __hip_atomic_store(host_flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t* dev;
    CK(hipMalloc(&dev, 64));
    uint32_t* flag;
    CK(hipHostMalloc(&flag, 64, hipHostMallocCoherent));
    *flag = 0;
    uint32_t* flag_dev;
    CK(hipHostGetDevicePointer((void**)&flag_dev, flag, 0));
    const int iters = 2000;
    auto now = [] { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    for (int mode = 0; mode < 3; ++mode) {
        uint32_t v = 0;
        double best = 1e9, tot = 0;
        for (int i = 0; i < iters + 100; ++i) {
            ++v;
            const double t0 = now();
            if (mode == 0) {
                hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, dev, (uint32_t*)nullptr, v);
                CK(hipStreamSynchronize(s));
            } else if (mode == 1) {
                hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, dev, (uint32_t*)nullptr, v);
                CK(hipStreamWriteValue32(s, flag_dev, v, 0));
                while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) __builtin_ia32_pause();
            } else {
                hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, dev, flag_dev, v);
                while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) __builtin_ia32_pause();
            }
            const double dt = now() - t0;
            if (i >= 100) {
                tot += dt;
                if (dt < best) best = dt;
            }
        }
        CK(hipStreamSynchronize(s));
        static const char* names[] = {"kernel + hipStreamSynchronize", "kernel + hipStreamWriteValue32 + spin",
                                      "kernel (pinned system-scope store) + spin"};
        printf("%-45s mean %.2f us  best %.2f us\n", names[mode], tot / iters, best);
    }
    return 0;
}
