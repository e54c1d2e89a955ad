// Variant sweep for the 1-GPU reduce kernel (dst += src, fp32, 1 GiB):
// load/store cache policy, unroll depth, grid size, grid-stride vs
// block-contiguous walk.  Prints one line per variant: ms and GB/s (3*S).
//   hipcc --offload-arch=gfx950 -O3 -I rdc_amd/csrc tools/bench_reduce.hip -o /tmp/bench_reduce
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "rdc_device.h"

using namespace rdc_amd;

template <bool NTL, bool NTS>
__device__ __forceinline__ v4u LD(const v4u* p) {
    if (NTL) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NTS>
__device__ __forceinline__ void ST(v4u* p, v4u v) {
    if (NTS) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// grid-stride, U independent 16-B positions per lane per iteration
template <int U, bool NTL, bool NTS, int B>
__global__ __launch_bounds__(B) void k_gs(v4u* __restrict__ d, const v4u* __restrict__ s, uint64_t nvec) {
    const uint64_t stride = (uint64_t)gridDim.x * B;
    uint64_t i = (uint64_t)blockIdx.x * B + threadIdx.x;
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        v4u a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = LD<NTL, NTS>(d + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = LD<NTL, NTS>(s + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) ST<NTS>(d + i + u * stride, reduce16<RDC_OP_SUM, float>(a[u], b[u]));
    }
    for (; i < nvec; i += stride) ST<NTS>(d + i, reduce16<RDC_OP_SUM, float>(LD<NTL, NTS>(d + i), LD<NTL, NTS>(s + i)));
}

// block-contiguous: block b owns [b*per, (b+1)*per), walks it U*B vectors at a time
template <int U, bool NTL, bool NTS, int B>
__global__ __launch_bounds__(B) void k_bc(v4u* __restrict__ d, const v4u* __restrict__ s, uint64_t nvec) {
    const uint64_t per = (nvec + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per;
    uint64_t hi = lo + per;
    if (hi > nvec) hi = nvec;
    uint64_t i = lo + threadIdx.x;
    for (; i + (U - 1) * B < hi; i += U * B) {
        v4u a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = LD<NTL, NTS>(d + i + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = LD<NTL, NTS>(s + i + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) ST<NTS>(d + i + u * B, reduce16<RDC_OP_SUM, float>(a[u], b[u]));
    }
    for (; i < hi; i += B) ST<NTS>(d + i, reduce16<RDC_OP_SUM, float>(LD<NTL, NTS>(d + i), LD<NTL, NTS>(s + i)));
}

// block-contiguous, software pipelined: next iteration's loads issued before
// this iteration's stores
template <int U, int B>
__global__ __launch_bounds__(B) void k_bcp(v4u* __restrict__ d, const v4u* __restrict__ s, uint64_t nvec) {
    const uint64_t per = ((nvec + gridDim.x - 1) / gridDim.x + U * B - 1) / (U * B) * (U * B);
    const uint64_t lo = (uint64_t)blockIdx.x * per;
    uint64_t hi = lo + per;
    if (hi > nvec) hi = nvec;
    if (lo >= hi) return;
    uint64_t i = lo + threadIdx.x;
    v4u a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t j = i + u * B;
        if (j < hi) { a[u] = LD<true, true>(d + j); b[u] = LD<true, true>(s + j); }
    }
    for (; i < hi; i += U * B) {
        v4u na[U], nb[U];
        const uint64_t ni = i + U * B;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = ni + u * B;
            if (j < hi) { na[u] = LD<true, true>(d + j); nb[u] = LD<true, true>(s + j); }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + u * B;
            if (j < hi) ST<true>(d + j, reduce16<RDC_OP_SUM, float>(a[u], b[u]));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) { a[u] = na[u]; b[u] = nb[u]; }
    }
}

// wave-contiguous: each wave owns a contiguous span, U x 1 KiB per step
template <int U, int B>
__global__ __launch_bounds__(B) void k_wc(v4u* __restrict__ d, const v4u* __restrict__ s, uint64_t nvec) {
    const int waves = gridDim.x * (B / 64);
    const int w = blockIdx.x * (B / 64) + threadIdx.x / 64;
    const int lane = threadIdx.x & 63;
    const uint64_t per = (nvec + waves - 1) / waves;
    const uint64_t lo = (uint64_t)w * per;
    uint64_t hi = lo + per;
    if (hi > nvec) hi = nvec;
    uint64_t i = lo + lane;
    for (; i + (U - 1) * 64 < hi; i += U * 64) {
        v4u a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = LD<true, true>(d + i + u * 64);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = LD<true, true>(s + i + u * 64);
#pragma unroll
        for (int u = 0; u < U; ++u) ST<true>(d + i + u * 64, reduce16<RDC_OP_SUM, float>(a[u], b[u]));
    }
    for (; i < hi; i += 64) ST<true>(d + i, reduce16<RDC_OP_SUM, float>(LD<true, true>(d + i), LD<true, true>(s + i)));
}

// grid-stride with an XCD-aware block order: hardware dispatches block b to
// XCD b % 8, so logical block = (b % 8) * (G / 8) + b / 8 gives every XCD one
// contiguous eighth of each sweep window (G a multiple of 8)
template <int U, int B>
__global__ __launch_bounds__(B) void k_gsx(v4u* __restrict__ d, const v4u* __restrict__ s, uint64_t nvec) {
    const unsigned G = gridDim.x;
    const unsigned lb = (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8;
    const uint64_t stride = (uint64_t)G * B;
    uint64_t i = (uint64_t)lb * B + threadIdx.x;
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        v4u a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = LD<true, true>(d + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = LD<true, true>(s + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) ST<true>(d + i + u * stride, reduce16<RDC_OP_SUM, float>(a[u], b[u]));
    }
    for (; i < nvec; i += stride) ST<true>(d + i, reduce16<RDC_OP_SUM, float>(LD<true, true>(d + i), LD<true, true>(s + i)));
}

// grid-stride, loads interleaved d0 s0 d1 s1 (same bytes in flight as k_gs)
template <int U, int B>
__global__ __launch_bounds__(B) void k_gsi(v4u* __restrict__ d, const v4u* __restrict__ s, uint64_t nvec) {
    const uint64_t stride = (uint64_t)gridDim.x * B;
    uint64_t i = (uint64_t)blockIdx.x * B + threadIdx.x;
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        v4u a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u] = LD<true, true>(d + i + u * stride);
            b[u] = LD<true, true>(s + i + u * stride);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) ST<true>(d + i + u * stride, reduce16<RDC_OP_SUM, float>(a[u], b[u]));
    }
    for (; i < nvec; i += stride) ST<true>(d + i, reduce16<RDC_OP_SUM, float>(LD<true, true>(d + i), LD<true, true>(s + i)));
}

// grid-stride, software-pipelined: the next window's loads are issued before
// this window's stores (2 x U x 32 B in flight per lane)
template <int U, int B>
__global__ __launch_bounds__(B) void k_gsp(v4u* __restrict__ d, const v4u* __restrict__ s, uint64_t nvec) {
    const uint64_t stride = (uint64_t)gridDim.x * B;
    uint64_t i = (uint64_t)blockIdx.x * B + threadIdx.x;
    const uint64_t full = nvec / (U * stride) * (U * stride);  // whole windows
    v4u a[U], b[U];
    if (i < full) {
#pragma unroll
        for (int u = 0; u < U; ++u) { a[u] = LD<true, true>(d + i + u * stride); b[u] = LD<true, true>(s + i + u * stride); }
    }
    for (; i < full; i += U * stride) {
        v4u na[U], nb[U];
        const uint64_t ni = i + U * stride;
        const bool more = ni < full;
        if (more) {
#pragma unroll
            for (int u = 0; u < U; ++u) { na[u] = LD<true, true>(d + ni + u * stride); nb[u] = LD<true, true>(s + ni + u * stride); }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) ST<true>(d + i + u * stride, reduce16<RDC_OP_SUM, float>(a[u], b[u]));
        if (more) {
#pragma unroll
            for (int u = 0; u < U; ++u) { a[u] = na[u]; b[u] = nb[u]; }
        }
    }
    for (i = full + (uint64_t)blockIdx.x * B + threadIdx.x; i < nvec; i += stride)
        ST<true>(d + i, reduce16<RDC_OP_SUM, float>(LD<true, true>(d + i), LD<true, true>(s + i)));
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

typedef void (*KFn)(v4u*, const v4u*, uint64_t);

// splitmix64 bits mapped to floats in [-1, 1) (a bounded Sum stays finite)
__global__ void k_fill_random(v4u* p, uint64_t nvec, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * blockDim.x) {
        v4u v;
        for (int k = 0; k < 4; ++k) {
            uint64_t z = (seed << 40) ^ (4 * i + k);
            z += 0x9E3779B97F4A7C15ull;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            v[k] = __float_as_uint((float)((z >> 40) * (1.0 / 16777216.0)) * 2.0f - 1.0f);
        }
        p[i] = v;
    }
}

struct Variant {
    const char* name;
    KFn fn;
    int block;
};

int main(int argc, char** argv) {
    const size_t S = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 30);
    const uint64_t nvec = S / 16;
    v4u *d, *s;
    CK(hipMalloc(&d, S));
    CK(hipMalloc(&s, S));
    CK(hipMemset(d, 0, S));
    CK(hipMemset(s, 0, S));
    if (getenv("SWEEP_RANDOM")) {  // full-entropy floats instead of zeros (the bench's data)
        hipLaunchKernelGGL(k_fill_random, dim3(1024), dim3(256), 0, 0, d, nvec, 1ull);
        hipLaunchKernelGGL(k_fill_random, dim3(1024), dim3(256), 0, 0, const_cast<v4u*>(s), nvec, 2ull);
        CK(hipDeviceSynchronize());
    }
    const bool quick = getenv("SWEEP_QUICK") != nullptr;
    std::vector<Variant> qv = {
        {"gs U2 nt/nt B256", (KFn)k_gs<2, true, true, 256>, 256},
        {"gsx U2 B256 (XCD order)", (KFn)k_gsx<2, 256>, 256},
        {"gsx U4 B256 (XCD order)", (KFn)k_gsx<4, 256>, 256},
        {"gsi U2 B256 (interleaved)", (KFn)k_gsi<2, 256>, 256},
        {"gsp U1 B256 (pipelined)", (KFn)k_gsp<1, 256>, 256},
        {"gsp U2 B256 (pipelined)", (KFn)k_gsp<2, 256>, 256},
        {"gs U1 nt/nt B512", (KFn)k_gs<1, true, true, 512>, 512},
        {"gsx U1 B512 (XCD order)", (KFn)k_gsx<1, 512>, 512},
    };
    std::vector<Variant> vs = {
        {"bc U4 nt/nt B256", (KFn)k_bc<4, true, true, 256>, 256},
        {"bc U4 nt/nt B1024", (KFn)k_bc<4, true, true, 1024>, 1024},
        {"gs U1 nt/nt B256", (KFn)k_gs<1, true, true, 256>, 256},
        {"gs U2 nt/nt B256", (KFn)k_gs<2, true, true, 256>, 256},
        {"gs U4 nt/nt B256", (KFn)k_gs<4, true, true, 256>, 256},
        {"gs U2 nt/nt B512", (KFn)k_gs<2, true, true, 512>, 512},
        {"gs U2 nt/nt B1024", (KFn)k_gs<2, true, true, 1024>, 1024},
        {"gs U4 nt/nt B1024", (KFn)k_gs<4, true, true, 1024>, 1024},
        {"gs U2 plain B256", (KFn)k_gs<2, false, false, 256>, 256},
    };
    if (quick) vs = qv;
    const int grids[] = {128, 256, 384, 512, 768, 1024};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep)
    for (auto& v : vs) {
        for (int g : grids) {
            if (quick && g != 256 && g != 512) continue;
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(v.fn, dim3(g), dim3(v.block), 0, 0, d, s, nvec);
            CK(hipDeviceSynchronize());
            const int it = 30;
            CK(hipEventRecord(e0));
            for (int k = 0; k < it; ++k) hipLaunchKernelGGL(v.fn, dim3(g), dim3(v.block), 0, 0, d, s, nvec);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= it;
            printf("%-24s grid %6d : %.4f ms  %.1f GB/s (3S)\n", v.name, g, ms, 3.0 * S / (ms * 1e-3) / 1e9);
        }
    }
    // copy reference: hipMemcpy D2D (2S traffic)
    for (int w = 0; w < 3; ++w) CK(hipMemcpy(d, s, S, hipMemcpyDeviceToDevice));
    CK(hipEventRecord(e0));
    for (int k = 0; k < 20; ++k) CK(hipMemcpyAsync(d, s, S, hipMemcpyDeviceToDevice, 0));
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 20;
    printf("%-24s          : %.4f ms  %.1f GB/s (2S)\n", "hipMemcpy D2D", ms, 2.0 * S / (ms * 1e-3) / 1e9);
    return 0;
}
