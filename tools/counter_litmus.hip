// Launch-counter litmus: the collectives' launch_begin / launch_done protocol
// (rdc_kernels_impl.h) in isolation.  Every block of launch k reads the
// device launch counter at its start (relaxed agent-scope load, thread 0),
// the launch's last block (relaxed agent-scope atomicAdd arrival count, reset
// by the last) stores k into it (relaxed agent-scope store).  The host issues
// K launches back to back on one stream, passing k; a block that reads
// anything but k - 1 counts a mismatch (and records the first one).
//
// Variants (argv): grid, launches, streams (round-robin launches over S
// streams of this process chained by events: a queue change between
// consecutive launches, as when a process has more streams than hardware
// queues), memory (0 hipMalloc as the product, 1 uncached), busy (also keep
// a spinning kernel resident on another stream so the queues time-slice).
//   hipcc --offload-arch=gfx950 -O3 -o tools/counter_litmus tools/counter_litmus.hip
//   tools/counter_litmus [GRID] [LAUNCHES] [STREAMS] [MEM] [BUSY_MS]
// Run several processes at once (GPU_MAX_HW_QUEUES=3 each) to rehearse the
// 5 ranks x 3 queues configuration of round 4's lost hand-off.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

struct Out {
    unsigned long long mismatches;
    unsigned long long first_k, first_seen, first_block;
};

// words: [16] arrivals, [32..33] launch counter (the product's err_ layout)
__global__ __launch_bounds__(256) void k_counter(uint32_t* words, uint64_t k, Out* out) {
    __shared__ uint64_t s_done;
    if (threadIdx.x == 0) {
        s_done = __hip_atomic_load(reinterpret_cast<uint64_t*>(words + 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const uint64_t done = s_done;
    if (threadIdx.x == 0 && done + 1 != k) {
        if (atomicAdd(&out->mismatches, 1ull) == 0) {
            out->first_k = k;
            out->first_seen = done;
            out->first_block = blockIdx.x;
        }
    }
    // a little work so blocks overlap across XCDs
    uint32_t acc = threadIdx.x;
    for (int i = 0; i < 64; ++i) acc = acc * 1664525u + 1013904223u;
    if (acc == 0x12345678u) out->first_block = ~0ull;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const bool last = gridDim.x == 1 || atomicAdd(words + 16, 1u) == gridDim.x - 1;
        if (last) {
            if (gridDim.x > 1) __hip_atomic_store(words + 16, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(reinterpret_cast<uint64_t*>(words + 32), k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// keeps some CUs and a queue busy for `ticks` (100 MHz wall clock)
__global__ void k_busy(uint64_t ticks, uint32_t* sink) {
    const uint64_t end = wall_clock64() + ticks;
    uint32_t x = threadIdx.x;
    while (wall_clock64() < end) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) *sink = x;
}

int main(int argc, char** argv) {
    const int grid = argc > 1 ? atoi(argv[1]) : 256;
    const int launches = argc > 2 ? atoi(argv[2]) : 20000;
    const int nstreams = argc > 3 ? atoi(argv[3]) : 1;
    const int mem = argc > 4 ? atoi(argv[4]) : 0;
    const int busy_ms = argc > 5 ? atoi(argv[5]) : 0;
    uint32_t* words = nullptr;
    if (mem == 0) CK(hipMalloc(&words, 512));
    else CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&words), 512, hipDeviceMallocUncached));
    CK(hipMemset(words, 0, 512));
    Out* out = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&out), sizeof(Out), hipHostMallocCoherent));
    *out = Out{0, 0, 0, 0};
    std::vector<hipStream_t> st((size_t)nstreams);
    std::vector<hipEvent_t> ev((size_t)nstreams);
    for (int i = 0; i < nstreams; ++i) {
        CK(hipStreamCreate(&st[(size_t)i]));
        CK(hipEventCreateWithFlags(&ev[(size_t)i], hipEventDisableTiming));
    }
    hipStream_t bs = nullptr;
    uint32_t* sink = nullptr;
    if (busy_ms > 0) {
        CK(hipStreamCreate(&bs));
        CK(hipMalloc(&sink, 4));
    }
    CK(hipDeviceSynchronize());
    int prev = -1;
    for (int k = 1; k <= launches; ++k) {
        if (busy_ms > 0 && k % 500 == 1)
            hipLaunchKernelGGL(k_busy, dim3(32), dim3(64), 0, bs, (uint64_t)busy_ms * 100000ull, sink);
        const int s = (k - 1) % nstreams;
        if (prev >= 0 && prev != s) CK(hipStreamWaitEvent(st[(size_t)s], ev[(size_t)prev], 0));
        hipLaunchKernelGGL(k_counter, dim3(grid), dim3(256), 0, st[(size_t)s], words, (uint64_t)k, out);
        if (nstreams > 1) CK(hipEventRecord(ev[(size_t)s], st[(size_t)s]));
        prev = s;
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    uint64_t ctr = 0;
    CK(hipMemcpy(&ctr, words + 32, 8, hipMemcpyDeviceToHost));
    printf("{\"grid\": %d, \"launches\": %d, \"streams\": %d, \"memory\": \"%s\", \"busy_ms\": %d, \"final_counter\": %llu, "
           "\"mismatched_blocks\": %llu, \"first\": [%llu, %llu, %llu]}\n",
           grid, launches, nstreams, mem ? "uncached" : "hipMalloc", busy_ms, (unsigned long long)ctr, out->mismatches,
           out->first_k, out->first_seen, out->first_block);
    return out->mismatches ? 1 : 0;
}
