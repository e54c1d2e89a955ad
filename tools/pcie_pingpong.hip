// PCIe signalling floor for the small-allreduce service (rdc_service.h): a
// resident block polls a request word and answers; the host times post ->
// answer (median microseconds).  Every answer is verified.
//   mode "host":  request word + input in uncached pinned host memory (the
//                 GPU polls and reads them over PCIe), result written to it
//   mode "dev":   request word + input written by the CPU into device memory
//                 (host-visible device allocation, if the runtime gives one),
//                 the GPU polls its own HBM; result to uncached host memory
// per size: `rw` = read input + write result; `r` = read only; `w` = write only.
//   hipcc --offload-arch=gfx950 -O3 -o tools/pcie_pingpong tools/pcie_pingpong.hip
//   tools/pcie_pingpong [iters]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

constexpr int kMax = 64 << 10;
struct Req {
    alignas(64) uint64_t req;  // (seq << 32) | flags << 24 | bytes; flags: 1 read, 2 write
    alignas(64) uint32_t stop;
    alignas(256) char data[kMax];
};
struct Resp {
    alignas(64) uint32_t done;
    alignas(256) char data[kMax];
};

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int BS>
__global__ __launch_bounds__(BS) void k_pong(Req* rq, Resp* rs, char* scratch) {
    __shared__ uint64_t s_q;
    __shared__ int s_go;
    uint32_t next = 1;
    for (;;) {
        if (threadIdx.x == 0) {
            int go = 0;
            uint64_t q = 0;
            for (;;) {
                q = __hip_atomic_load(&rq->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if ((uint32_t)(q >> 32) == next) {
                    go = 1;
                    break;
                }
                if (__hip_atomic_load(&rq->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
                __builtin_amdgcn_s_sleep(1);
            }
            s_go = go;
            s_q = q;
        }
        __syncthreads();
        if (!s_go) break;
        const uint64_t bytes = s_q & 0xffffffu;
        const int fl = (int)((s_q >> 24) & 0xff);
        const uint64_t nvec = bytes >> 4;
        constexpr int U = 4;
        if (fl & 1) {  // input: all loads of a thread in flight together
            for (uint64_t i = threadIdx.x; i < nvec; i += U * BS) {
                v4u v[U];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (i + u * BS < nvec) v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(rq->data) + i + u * BS);
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (i + u * BS < nvec) reinterpret_cast<v4u*>(scratch)[i + u * BS] = v[u];
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (fl & 2) {
            for (uint64_t i = threadIdx.x; i < nvec; i += BS) {
                v4u v = (fl & 1) ? reinterpret_cast<const v4u*>(scratch)[i] : v4u{(uint32_t)i, next, 0u, 0u};
                v.w = next;
                reinterpret_cast<v4u*>(rs->data)[i] = v;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (threadIdx.x == 0) __hip_atomic_store(&rs->done, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ++next;
        __syncthreads();
    }
}

static double median(std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 10000;
    char* scratch;
    CK(hipMalloc(&scratch, kMax));
    std::string out = "{";
    auto add = [&](const std::string& k, double v) {
        char b[64];
        snprintf(b, sizeof b, "%.3f", v);
        out += "\"" + k + "\": " + b + ", ";
    };
    // result mailbox: uncached pinned host memory
    Resp* rs;
    CK(hipHostMalloc((void**)&rs, sizeof(Resp), hipHostMallocUncached | hipHostMallocMapped));
    memset(rs, 0, sizeof(Resp));
    Resp* drs;
    CK(hipHostGetDevicePointer((void**)&drs, rs, 0));
    for (int mode = 0; mode < 2; ++mode) {
        Req* hrq = nullptr;  // CPU address
        Req* drq = nullptr;  // GPU address
        if (mode == 0) {
            CK(hipHostMalloc((void**)&hrq, sizeof(Req), hipHostMallocUncached | hipHostMallocMapped));
            CK(hipHostGetDevicePointer((void**)&drq, hrq, 0));
        } else {
            // device memory the CPU can store into (large BAR): try the
            // fine-grained / uncached device allocations and keep the first
            // one that reports a host address
            const unsigned fl[2] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained};
            for (int k = 0; k < 2 && !hrq; ++k) {
                void* p = nullptr;
                if (hipExtMallocWithFlags(&p, sizeof(Req), fl[k]) != hipSuccess) {
                    (void)hipGetLastError();
                    continue;
                }
                hipPointerAttribute_t a;
                memset(&a, 0, sizeof a);
                if (hipPointerGetAttributes(&a, p) == hipSuccess && a.hostPointer) {
                    hrq = (Req*)a.hostPointer;
                    drq = (Req*)p;
                    add(std::string("dev_alloc_flag"), (double)fl[k]);
                } else {
                    (void)hipGetLastError();
                    (void)hipFree(p);
                }
            }
            if (!hrq) {
                out += "\"dev\": \"no host-visible device memory\", ";
                continue;
            }
        }
        const char* mname = mode == 0 ? "host" : "dev";
        memset(hrq, 0, sizeof(Req));
        std::vector<char> src(kMax), dst(kMax);
        for (int i = 0; i < kMax; ++i) src[i] = (char)(i * 7 + 1);
        for (int bs : {256, 1024}) {
            hrq->req = 0;
            hrq->stop = 0;
            rs->done = 0;
            hipStream_t s;
            CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            if (bs == 256)
                hipLaunchKernelGGL(k_pong<256>, dim3(1), dim3(256), 0, s, drq, drs, scratch);
            else
                hipLaunchKernelGGL(k_pong<1024>, dim3(1), dim3(1024), 0, s, drq, drs, scratch);
            CK(hipGetLastError());
            uint32_t seq = 0;
            long bad = 0;
            for (int sz : {0, 16, 4096, 16384, 65536}) {
                for (int fl : {3, 1, 2}) {
                    if (sz == 0 && fl != 3) continue;
                    std::vector<double> t;
                    for (int i = 0; i < iters; ++i) {
                        ++seq;
                        auto t0 = std::chrono::steady_clock::now();
                        if (fl & 1) memcpy(hrq->data, src.data(), sz);
                        __atomic_store_n(&hrq->req, ((uint64_t)seq << 32) | ((uint64_t)fl << 24) | (uint64_t)sz,
                                         __ATOMIC_SEQ_CST);
                        while (__atomic_load_n(&rs->done, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
                        if (fl & 2) memcpy(dst.data(), rs->data, sz);
                        auto t1 = std::chrono::steady_clock::now();
                        t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
                        if (fl == 3 && i % 97 == 0) {  // the answer is the input with word 3 of each 16 B = seq
                            for (int v = 0; v < sz / 16; ++v) {
                                uint32_t w[4], x[4];
                                memcpy(w, dst.data() + 16 * v, 16);
                                memcpy(x, src.data() + 16 * v, 16);
                                if (w[0] != x[0] || w[1] != x[1] || w[2] != x[2] || w[3] != seq) ++bad;
                            }
                        }
                    }
                    const char* fn = fl == 3 ? "rw" : fl == 1 ? "r" : "w";
                    add(std::string(mname) + "_bs" + std::to_string(bs) + "_" + fn + "_" + std::to_string(sz), median(t));
                }
            }
            add(std::string(mname) + "_bs" + std::to_string(bs) + "_bad", (double)bad);
            __atomic_store_n(&hrq->stop, 1u, __ATOMIC_SEQ_CST);
            CK(hipStreamSynchronize(s));
            CK(hipStreamDestroy(s));
        }
        if (mode == 0) CK(hipHostFree(hrq));
        else CK(hipFree(drq));
    }
    out += "\"iters\": " + std::to_string(iters) + "}";
    printf("%s\n", out.c_str());
    return 0;
}
