// Host <-> resident-block round trip for the small-allreduce service's
// mailbox (rdc_service.h), by where the request word lives:
//   host:  pinned host memory (hipHostMallocUncached; the current mailbox):
//          the block polls it over PCIe (a read round trip per poll)
//   vram:  device memory the CPU writes through the BAR (HSA pool allocation
//          of the GPU's coarse-grained pool, CPU given access): the block
//          polls local HBM; the CPU's store is a posted PCIe write
// The block answers into a pinned host word the CPU spins on (a posted write
// the other way).  Median / p10 / p90 microseconds over N round trips.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mailbox_rtt tools/mailbox_rtt.hip -lhsa-runtime64
//   tools/mailbox_rtt [N]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
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

__global__ void k_echo(const uint32_t* req, uint32_t* resp, int n) {
    if (threadIdx.x != 0) return;
    const uint64_t deadline0 = wall_clock64() + 300000000ull;  // 3 s
    for (int k = 1; k <= n; ++k) {
        while (__hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != (uint32_t)k) {
            if (wall_clock64() > deadline0) return;
        }
        __hip_atomic_store(resp, (uint32_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// payload round trip: the request is B bytes as LL words {4 payload bytes,
// k} (2B bytes) in the mailbox; the block (256 threads) polls the words until
// every one carries k, writes B result bytes to the host, drains, then `done`
__global__ __launch_bounds__(256) void k_echo_ll(const uint64_t* ll, uint32_t* out, uint32_t* done, int nwords, int n) {
    const uint64_t deadline0 = wall_clock64() + 300000000ull;  // 3 s
    __shared__ int s_ok;
    for (int k = 1; k <= n; ++k) {
        while (true) {
            bool mine = true;
            for (int w = threadIdx.x; w < nwords; w += 256)
                mine = mine && (uint32_t)(__hip_atomic_load(ll + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >> 32) == (uint32_t)k;
            if (__syncthreads_and(mine)) break;
            if (wall_clock64() > deadline0) return;
        }
        for (int w = threadIdx.x; w < nwords; w += 256)
            out[w] = (uint32_t)__hip_atomic_load(ll + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1u;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(done, (uint32_t)k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    (void)s_ok;
}

static void run_ll(const char* name, uint64_t* ll_host_view, uint64_t* ll_dev_view, uint32_t* out, uint32_t* done,
                   int bytes, int n) {
    const int nwords = bytes / 4;
    *done = 0;
    for (int w = 0; w < nwords; ++w) ll_host_view[w] = 0;
    __builtin_ia32_sfence();
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(k_echo_ll, dim3(1), dim3(256), 0, s, ll_dev_view, out, done, nwords, n);
    CK(hipGetLastError());
    std::vector<double> t;
    volatile uint32_t* d = done;
    for (int k = 1; k <= n; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        const uint64_t tag = (uint64_t)k << 32;
        for (int w = 0; w < nwords; ++w) __atomic_store_n(ll_host_view + w, tag | (uint32_t)w, __ATOMIC_RELAXED);
        __builtin_ia32_sfence();
        const auto tl = t0 + std::chrono::seconds(4);
        bool lost = false;
        while (*d != (uint32_t)k)
            if (std::chrono::steady_clock::now() > tl) {
                lost = true;
                break;
            }
        if (lost) {
            CK(hipStreamSynchronize(s));
            printf("{\"mailbox\": \"%s LL %d B\", \"error\": \"request %d lost\"}\n", name, bytes, k);
            return;
        }
        t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CK(hipStreamSynchronize(s));
    std::vector<double> w(t.begin() + n / 10, t.end());
    std::sort(w.begin(), w.end());
    printf("{\"mailbox\": \"%s LL %d B\", \"round_trips\": %zu, \"median_us\": %.3f, \"p10_us\": %.3f, \"p90_us\": %.3f}\n",
           name, bytes, w.size(), w[w.size() / 2], w[w.size() / 10], w[w.size() * 9 / 10]);
    fflush(stdout);
}

struct Ctx {
    hsa_agent_t gpu{}, cpu{};
    hsa_amd_memory_pool_t pool{};
    bool have_pool = false;
};
static hsa_status_t find_agents(hsa_agent_t a, void* d) {
    Ctx* c = static_cast<Ctx*>(d);
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && c->gpu.handle == 0) c->gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && c->cpu.handle == 0) c->cpu = a;
    return HSA_STATUS_SUCCESS;
}
static uint32_t g_want_flag = HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED;
static hsa_status_t find_pool(hsa_amd_memory_pool_t p, void* d) {
    Ctx* c = static_cast<Ctx*>(d);
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if (seg == HSA_AMD_SEGMENT_GLOBAL && !c->have_pool && (flags & g_want_flag)) {
        c->pool = p;
        c->have_pool = true;
    }
    return HSA_STATUS_SUCCESS;
}

static void run(const char* name, uint32_t* req_host_view, uint32_t* req_dev_view, uint32_t* resp, int n) {
    *resp = 0;
    __atomic_store_n(req_host_view, 0u, __ATOMIC_SEQ_CST);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(k_echo, dim3(1), dim3(64), 0, s, req_dev_view, resp, n);
    CK(hipGetLastError());
    std::vector<double> t;
    t.reserve(n);
    volatile uint32_t* r = resp;
    for (int k = 1; k <= n; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(req_host_view, (uint32_t)k, __ATOMIC_RELEASE);
        __builtin_ia32_sfence();  // a BAR mapping may be write-combining: push the store out now
        const auto tl = t0 + std::chrono::seconds(4);
        bool lost = false;
        while (*r != (uint32_t)k) {
            if (std::chrono::steady_clock::now() > tl) {
                lost = true;
                break;
            }
        }
        if (lost) {
            CK(hipStreamSynchronize(s));  // the block gives up after 3 s
            std::sort(t.begin(), t.end());
            printf("{\"mailbox\": \"%s\", \"error\": \"request %d never seen by the block\", \"median_us_before\": %.3f}\n",
                   name, k, t.empty() ? 0.0 : t[t.size() / 2]);
            fflush(stdout);
            return;
        }
        t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CK(hipStreamSynchronize(s));
    std::vector<double> w(t.begin() + n / 10, t.end());  // drop warm-up
    std::sort(w.begin(), w.end());
    printf("{\"mailbox\": \"%s\", \"round_trips\": %zu, \"median_us\": %.3f, \"p10_us\": %.3f, \"p90_us\": %.3f}\n", name,
           w.size(), w[w.size() / 2], w[w.size() / 10], w[w.size() * 9 / 10]);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 20000;
    CK(hipSetDevice(0));
    uint32_t* resp = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&resp), 4096, hipHostMallocUncached));
    // 1) host-memory request word (current design)
    uint32_t* req = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&req), 4096, hipHostMallocUncached));
    run("host", req, req, resp, n);
    uint64_t* llh = nullptr;
    uint32_t* outh = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&llh), 1 << 16, hipHostMallocUncached));
    CK(hipHostMalloc(reinterpret_cast<void**>(&outh), 1 << 16, hipHostMallocUncached));
    for (int b : {4, 1024, 4096}) run_ll("host", llh, llh, outh, resp, b, n / 4);
    // 2) VRAM request word, written by the CPU through the BAR: the GPU's
    //    fine-grained pool, then its coarse-grained one
    for (int variant = 0; variant < 4; ++variant) {
        const int fine = variant & 1, uc = variant >> 1;
        const char* names[] = {"vram coarse-grained", "vram fine-grained", "vram coarse-grained uncached",
                               "vram fine-grained uncached"};
        const char* name = names[variant];
        Ctx c;
        g_want_flag = fine ? HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED : HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED;
        hsa_iterate_agents(find_agents, &c);
        hsa_amd_agent_iterate_memory_pools(c.gpu, find_pool, &c);
        void* v = nullptr;
        if (!c.have_pool || hsa_amd_memory_pool_allocate(c.pool, 4096, uc ? HSA_AMD_MEMORY_POOL_UNCACHED_FLAG : 0, &v) != HSA_STATUS_SUCCESS) {
            printf("{\"mailbox\": \"%s\", \"error\": \"no pool\"}\n", name);
            continue;
        }
        hsa_agent_t both[2] = {c.gpu, c.cpu};
        const hsa_status_t st = hsa_amd_agents_allow_access(2, both, nullptr, v);
        if (st != HSA_STATUS_SUCCESS) {
            printf("{\"mailbox\": \"%s\", \"error\": \"allow_access %d\"}\n", name, (int)st);
            continue;
        }
        run(name, static_cast<uint32_t*>(v), static_cast<uint32_t*>(v), resp, n);
        if (uc && fine) {
            void* lv = nullptr;
            if (hsa_amd_memory_pool_allocate(c.pool, 1 << 16, HSA_AMD_MEMORY_POOL_UNCACHED_FLAG, &lv) == HSA_STATUS_SUCCESS &&
                hsa_amd_agents_allow_access(2, both, nullptr, lv) == HSA_STATUS_SUCCESS)
                for (int b : {4, 1024, 4096})
                    run_ll(name, static_cast<uint64_t*>(lv), static_cast<uint64_t*>(lv), outh, resp, b, n / 4);
        }
    }
    return 0;
}
