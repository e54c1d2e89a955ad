// Calibration for the HBM write counters on the collectives' uncached
// (MTYPE UC) scratch: one launch of 16-B-per-lane streaming stores over
// 256 MiB of (a) hipExtMallocWithFlags(hipDeviceMallocUncached) memory and
// (b) ordinary hipMalloc memory, as separate kernels so rocprofv3 --pmc
// attributes each.  Known byte count: 256 MiB per launch.
//   hipcc --offload-arch=gfx950 -O3 -o tools/uc_write_pmc tools/uc_write_pmc.hip
//   rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d DIR -o run --output-format csv -- tools/uc_write_pmc
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

__global__ __launch_bounds__(256) void k_store_uncached(v4u* d, uint64_t nvec) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * 256)
        __builtin_nontemporal_store(v4u{(uint32_t)i, 1u, 2u, 3u}, d + i);
}
__global__ __launch_bounds__(256) void k_store_normal(v4u* d, uint64_t nvec) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * 256)
        __builtin_nontemporal_store(v4u{(uint32_t)i, 1u, 2u, 3u}, d + i);
}

int main() {
    const uint64_t bytes = 256ull << 20, nvec = bytes / 16;
    v4u *uc = nullptr, *nm = nullptr;
    CK(hipExtMallocWithFlags((void**)&uc, bytes, hipDeviceMallocUncached));
    CK(hipMalloc((void**)&nm, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep) {
        float ms_uc = 0, ms_nm = 0;
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_store_uncached, dim3(1024), dim3(256), 0, 0, uc, nvec);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_uc, e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_store_normal, dim3(1024), dim3(256), 0, 0, nm, nvec);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_nm, e0, e1));
        printf("{\"rep\": %d, \"bytes\": %llu, \"uncached_ms\": %.4f, \"normal_ms\": %.4f}\n", rep,
               (unsigned long long)bytes, ms_uc, ms_nm);
    }
    CK(hipFree(uc));
    CK(hipFree(nm));
    return 0;
}
