// PCIe signalling floor for the small-allreduce service (rdc_service.h): a
// resident block polls a word in pinned host memory and answers; the host
// times post -> answer.  Variants: bare signal; plus a read + write of
// `bytes` of the mailbox; host memcpy into / out of the mailbox pages.
//   hipcc --offload-arch=gfx950 -O3 -o tools/pcie_pingpong tools/pcie_pingpong.hip
//   tools/pcie_pingpong [iters]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

struct Box {
    alignas(64) uint64_t req;
    alignas(64) uint32_t done;
    alignas(64) uint32_t stop;
    alignas(256) char data[64 << 10];
};

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_pong(Box* box, char* scratch, int sleep) {
    __shared__ uint64_t s_q;
    __shared__ int s_go;
    uint32_t next = 1;
    for (;;) {
        if (threadIdx.x == 0) {
            int go = 0;
            uint64_t q = 0;
            for (;;) {
                q = __hip_atomic_load(&box->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if ((uint32_t)(q >> 32) == next) {
                    go = 1;
                    break;
                }
                if (__hip_atomic_load(&box->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
                if (sleep) __builtin_amdgcn_s_sleep(1);
            }
            s_go = go;
            s_q = q;
        }
        __syncthreads();
        if (!s_go) break;
        const uint64_t bytes = s_q & 0xffffffffu;
        const uint64_t nvec = bytes >> 4;
        for (uint64_t i = threadIdx.x; i < nvec; i += 256)
            reinterpret_cast<v4u*>(scratch)[i] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(box->data) + i);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (uint64_t i = threadIdx.x; i < nvec; i += 256) {
            v4u v = reinterpret_cast<const v4u*>(scratch)[i];
            v.x += 1;
            reinterpret_cast<v4u*>(box->data)[i] = v;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(&box->done, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ++next;
        __syncthreads();
    }
}

static double median(std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    const unsigned flags_list[2] = {hipHostMallocUncached | hipHostMallocMapped, hipHostMallocCoherent | hipHostMallocMapped};
    const char* names[2] = {"uncached", "coherent"};
    char* scratch;
    CK(hipMalloc(&scratch, 64 << 10));
    printf("{");
    for (int f = 0; f < 2; ++f) {
        Box* box;
        CK(hipHostMalloc((void**)&box, sizeof(Box), flags_list[f]));
        memset(box, 0, sizeof(Box));
        Box* dbox;
        CK(hipHostGetDevicePointer((void**)&dbox, box, 0));
        std::vector<char> host(64 << 10, 1);
        // host memcpy cost into / out of the pages
        for (int sz : {4096, 65536}) {
            std::vector<double> tin, tout;
            for (int i = 0; i < 2000; ++i) {
                auto t0 = std::chrono::steady_clock::now();
                memcpy(box->data, host.data(), sz);
                auto t1 = std::chrono::steady_clock::now();
                memcpy(host.data(), box->data, sz);
                auto t2 = std::chrono::steady_clock::now();
                tin.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
                tout.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
            }
            printf("\"%s_memcpy_in_%d_us\": %.3f, \"%s_memcpy_out_%d_us\": %.3f, ", names[f], sz, median(tin), names[f],
                   sz, median(tout));
        }
        for (int sleep = 0; sleep < 2; ++sleep) {
            hipStream_t s;
            CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            box->req = 0;
            box->done = 0;
            box->stop = 0;
            hipLaunchKernelGGL(k_pong, dim3(1), dim3(256), 0, s, dbox, scratch, sleep);
            CK(hipGetLastError());
            uint32_t seq = 0;
            for (int sz : {0, 4096, 65536}) {
                std::vector<double> t;
                for (int i = 0; i < iters; ++i) {
                    ++seq;
                    auto t0 = std::chrono::steady_clock::now();
                    __atomic_store_n(&box->req, ((uint64_t)seq << 32) | (uint64_t)sz, __ATOMIC_SEQ_CST);
                    while (__atomic_load_n(&box->done, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
                    auto t1 = std::chrono::steady_clock::now();
                    t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
                }
                printf("\"%s_sleep%d_pingpong_%d_us\": %.3f, ", names[f], sleep, sz, median(t));
            }
            __atomic_store_n(&box->stop, 1u, __ATOMIC_SEQ_CST);
            CK(hipStreamSynchronize(s));
            CK(hipStreamDestroy(s));
        }
        CK(hipHostFree(box));
    }
    printf("\"iters\": %d}\n", iters);
    return 0;
}
