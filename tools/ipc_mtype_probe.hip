// What cache treatment do the L2s give a HIP IPC import?  (VERDICT r5 item 3:
// the 5 x 3 lost hand-off, where every device read kind on one XCD returned
// the old flag while the host read the new one.)
//
// The owner allocates one region of each memory kind the library uses
// (hipMalloc, hipExtMallocWithFlags Uncached = the scratch and flags, Fine-
// grained); the peer imports all three with hipIpcOpenMemHandle.  Both
// processes then run the same kernels on every region, one after the other
// (stages in POSIX shared memory), each kernel instantiated per (memory kind,
// side) so a per-dispatch counter run names what each access was:
//
//   mode "mtype" (run each process under rocprofv3 --pmc):
//     k_read<M,S>   256 workgroups read the region twice with plain loads
//     k_store<M,S>  one workgroup stores it once (system-scope stores)
//     k_atomic<M,S> one workgroup adds 0 to every dword (system scope)
//   TCP_TCC_{UC,NC,RW,CC}_{READ,WRITE,ATOMIC}_REQ_sum name the MTYPE the L2
//   saw per request; TCC_HIT_sum / TCC_MISS_sum show whether the second read
//   pass hits.
//
//   mode "alias" (no profiler): can an L2 serve a line that memory no longer
//   holds?  Per trial: the writer side stores `old` (one workgroup, system
//   scope, drained), the toucher side reads the region with plain loads on
//   every XCD, the writer stores `new`, then BOTH sides read it on every XCD
//   with four load kinds (plain, sc0 sc1, nt, atomic add 0) and count lanes
//   that still see `old`.  Roles: owner writes / peer touches, and peer
//   writes (through its import, as the collectives' producers do) / peer
//   touches.
//
// Kinds 3 and 4 (round 6, after the first run found hipDeviceMallocUncached
// to be MTYPE CC): the GPU's coarse / fine-grained HSA pool allocated with
// HSA_AMD_MEMORY_POOL_UNCACHED_FLAG, shared with hsa_amd_ipc_memory_create /
// _attach (HIP's IPC does not know HSA allocations).
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/ipc_mtype_probe tools/ipc_mtype_probe.hip -lrt -lhsa-runtime64
//   tools/ipc_mtype_probe owner NAME MODE & tools/ipc_mtype_probe peer NAME MODE
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <string>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr size_t kRegion = 1 << 20;   // bytes per region (mtype reads)
constexpr size_t kAlias = 64 << 10;   // bytes per region the alias trials use
constexpr int kKinds = 5;
static const char* kMemName[kKinds] = {"hipMalloc", "uncached", "finegrained", "hsa coarse UNCACHED_FLAG",
                                       "hsa fine UNCACHED_FLAG"};
static const char* kLoadName[4] = {"plain", "sc0 sc1", "nt", "atomic add 0"};

struct Ctl {
    int stage_o, stage_p;
    hipIpcMemHandle_t h[kKinds];
    hsa_amd_ipc_memory_t hh[kKinds];
};

struct Stale {
    unsigned long long lanes[4];  // per load kind: lanes reading `old`
    unsigned long long reads[4];
    unsigned int xcc_mask[4];     // XCDs on which a stale read happened
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
    const uint64_t b = (uint64_t)(uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, 0xffffffffu, 0x00020000);
}

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf; }

// ---------------------------------------------------------------- mtype ----
template <int M, int S>
__global__ __launch_bounds__(256) void k_read(const char* r, unsigned* sink) {
    uint32_t acc = 0;
    for (int pass = 0; pass < 2; ++pass)
        for (uint32_t off = (blockIdx.x * 256u + threadIdx.x) * 16u; off < kRegion; off += gridDim.x * 256u * 16u) {
            const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(r), off, 0, 0);
            acc += v.x ^ v.w;
        }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int M, int S>
__global__ __launch_bounds__(256) void k_store(char* r, uint32_t v) {
    for (uint32_t off = threadIdx.x * 16u; off < (uint32_t)kAlias; off += 256u * 16u)
        __builtin_amdgcn_raw_buffer_store_b128(v4u{v, v, v, v}, rsrc(r), off, 0, 17);
}

template <int M, int S>
__global__ __launch_bounds__(256) void k_atomic(char* r, unsigned* sink) {
    uint32_t acc = 0;
    for (uint32_t i = threadIdx.x; i < kAlias / 4; i += 256)
        acc += __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(r) + i, 0u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM);
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int M, int S>
static void run_kind(char* const* reg, unsigned* sink) {
    hipLaunchKernelGGL((k_read<M, S>), dim3(256), dim3(256), 0, 0, reg[M], sink);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL((k_store<M, S>), dim3(1), dim3(256), 0, 0, reg[M], 7u);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL((k_atomic<M, S>), dim3(1), dim3(256), 0, 0, reg[M], sink);
    CK(hipDeviceSynchronize());
}

template <int S>
static void run_mtype(char* const* reg, unsigned* sink) {
    run_kind<0, S>(reg, sink);
    run_kind<1, S>(reg, sink);
    run_kind<2, S>(reg, sink);
    if (reg[3]) run_kind<3, S>(reg, sink);
    if (reg[4]) run_kind<4, S>(reg, sink);
}

// the visible GPU's HSA agent and its coarse (fine = false) or fine-grained global pool
struct HsaPick {
    hsa_agent_t gpu{};
    bool have_gpu = false, fine = false, have_pool = false;
    hsa_amd_memory_pool_t pool{};
};
static hsa_status_t pick_gpu(hsa_agent_t a, void* d) {
    HsaPick* p = static_cast<HsaPick*>(d);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU &&
        !p->have_gpu) {
        p->gpu = a;
        p->have_gpu = true;
    }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t pick_pool(hsa_amd_memory_pool_t pool, void* d) {
    HsaPick* p = static_cast<HsaPick*>(d);
    hsa_amd_segment_t seg;
    uint32_t flags = 0;
    if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    const uint32_t want = p->fine ? HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED
                                  : HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED;
    if (seg == HSA_AMD_SEGMENT_GLOBAL && (flags & want) && !p->have_pool) {
        p->pool = pool;
        p->have_pool = true;
    }
    return HSA_STATUS_SUCCESS;
}
static HsaPick hsa_pick(bool fine) {
    HsaPick p;
    p.fine = fine;
    hsa_init();
    hsa_iterate_agents(pick_gpu, &p);
    if (p.have_gpu) hsa_amd_agent_iterate_memory_pools(p.gpu, pick_pool, &p);
    return p;
}

// ---------------------------------------------------------------- alias ----
__global__ __launch_bounds__(256) void k_set(char* r, uint32_t v) {
    for (uint32_t off = threadIdx.x * 16u; off < (uint32_t)kAlias; off += 256u * 16u)
        __builtin_amdgcn_raw_buffer_store_b128(v4u{v, v, v, v}, rsrc(r), off, 0, 17);  // sc0 sc1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ __launch_bounds__(256) void k_touch(const char* r, unsigned* sink) {
    uint32_t acc = 0;
    for (uint32_t off = threadIdx.x * 16u; off < (uint32_t)kAlias; off += 256u * 16u) {
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(r), off, 0, 0);
        acc += v.x;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// every workgroup reads the whole region with load kind K
template <int K>
__global__ __launch_bounds__(256) void k_check(char* r, uint32_t old_v, Stale* st) {
    unsigned long long s = 0, n = 0;
    for (uint32_t off = threadIdx.x * 16u; off < (uint32_t)kAlias; off += 256u * 16u) {
        uint32_t x;
        if constexpr (K == 0) x = ((v4u)__builtin_amdgcn_raw_buffer_load_b128(rsrc(r), off, 0, 0)).x;
        else if constexpr (K == 1) x = ((v4u)__builtin_amdgcn_raw_buffer_load_b128(rsrc(r), off, 0, 17)).x;
        else if constexpr (K == 2) x = ((v4u)__builtin_amdgcn_raw_buffer_load_b128(rsrc(r), off, 0, 2)).x;
        else
            x = __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(r + off), 0u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
        s += x == old_v;
        ++n;
    }
    if (s) {
        atomicAdd(&st->lanes[K], s);
        atomicOr(&st->xcc_mask[K], 1u << xcc_id());
    }
    atomicAdd(&st->reads[K], n);
}

static void check_all(char* r, uint32_t old_v, Stale* st) {
    hipLaunchKernelGGL(k_check<0>, dim3(256), dim3(256), 0, 0, r, old_v, st);
    hipLaunchKernelGGL(k_check<1>, dim3(256), dim3(256), 0, 0, r, old_v, st);
    hipLaunchKernelGGL(k_check<2>, dim3(256), dim3(256), 0, 0, r, old_v, st);
    hipLaunchKernelGGL(k_check<3>, dim3(256), dim3(256), 0, 0, r, old_v, st);
    CK(hipDeviceSynchronize());
}

// ----------------------------------------------------------------- host ----
static Ctl* open_ctl(const std::string& name, bool create) {
    const std::string path = "/rdc_mtype_" + name;
    int fd = -1;
    for (int t = 0; t < 400 && fd < 0; ++t) {
        fd = shm_open(path.c_str(), create ? (O_CREAT | O_RDWR) : O_RDWR, 0600);
        if (fd < 0) usleep(25000);
    }
    if (fd < 0 || (create && ftruncate(fd, sizeof(Ctl)) != 0)) {
        perror("shm");
        exit(1);
    }
    void* m = mmap(nullptr, sizeof(Ctl), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) exit(1);
    if (create) memset(m, 0, sizeof(Ctl));
    return static_cast<Ctl*>(m);
}

static void wait_stage(int* field, int want) {
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(field, __ATOMIC_ACQUIRE) < want) {
        usleep(100);
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 60) {
            fprintf(stderr, "timed out waiting for stage %d\n", want);
            exit(3);
        }
    }
}

static void stage(int* field, int v) { __atomic_store_n(field, v, __ATOMIC_RELEASE); }

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s owner|peer NAME mtype|alias [TRIALS]\n", argv[0]);
        return 2;
    }
    const std::string role = argv[1], name = argv[2], mode = argv[3];
    const int trials = argc > 4 ? atoi(argv[4]) : 50;
    const bool owner = role == "owner";
    Ctl* ctl = open_ctl(name, owner);
    char* reg[kKinds] = {};
    unsigned* sink = nullptr;
    CK(hipMalloc(&sink, 64));
    Stale* st = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&st), sizeof(Stale) * kKinds * 2, hipHostMallocCoherent));
    memset(st, 0, sizeof(Stale) * kKinds * 2);
    int s = 0;  // stage counter, the same sequence in both processes
    if (owner) {
        for (int m = 0; m < kKinds; ++m) {
            void* p = nullptr;
            if (m >= 3) {
                HsaPick hp = hsa_pick(m == 4);
                if (!hp.have_pool ||
                    hsa_amd_memory_pool_allocate(hp.pool, kRegion, HSA_AMD_MEMORY_POOL_UNCACHED_FLAG, &p) !=
                        HSA_STATUS_SUCCESS ||
                    hsa_amd_ipc_memory_create(p, kRegion, &ctl->hh[m]) != HSA_STATUS_SUCCESS) {
                    fprintf(stderr, "kind %d: HSA allocation / IPC export failed\n", m);
                    exit(1);
                }
                CK(hipMemset(p, 0, kRegion));
                reg[m] = static_cast<char*>(p);
                continue;
            }
            if (m == 0) CK(hipMalloc(&p, kRegion));
            else CK(hipExtMallocWithFlags(&p, kRegion, m == 1 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
            CK(hipMemset(p, 0, kRegion));
            reg[m] = static_cast<char*>(p);
            CK(hipIpcGetMemHandle(&ctl->h[m], p));
        }
        CK(hipDeviceSynchronize());
        stage(&ctl->stage_o, ++s);
    } else {
        wait_stage(&ctl->stage_o, ++s);
        for (int m = 0; m < kKinds; ++m) {
            if (m >= 3) {
                HsaPick hp = hsa_pick(false);
                void* q = nullptr;
                if (!hp.have_gpu || hsa_amd_ipc_memory_attach(&ctl->hh[m], kRegion, 1, &hp.gpu, &q) != HSA_STATUS_SUCCESS) {
                    fprintf(stderr, "kind %d: HSA IPC attach failed\n", m);
                    exit(1);
                }
                reg[m] = static_cast<char*>(q);
                continue;
            }
            CK(hipIpcOpenMemHandle(reinterpret_cast<void**>(&reg[m]), ctl->h[m], hipIpcMemLazyEnablePeerAccess));
        }
    }
    if (mode == "mtype") {
        // owner's kernels, then the peer's (never both at once: the counters are device-wide)
        if (owner) {
            run_mtype<0>(reg, sink);
            stage(&ctl->stage_o, ++s);
            wait_stage(&ctl->stage_p, s);
        } else {
            wait_stage(&ctl->stage_o, ++s);
            run_mtype<1>(reg, sink);
            stage(&ctl->stage_p, s);
        }
        printf("{\"role\": \"%s\", \"mode\": \"mtype\", \"regions\": [\"%p\", \"%p\", \"%p\", \"%p\", \"%p\"]}\n",
               role.c_str(), reg[0], reg[1], reg[2], reg[3], reg[4]);
    } else {
        // variant 0: owner writes, peer touches; variant 1: peer writes (import), peer touches
        for (int var = 0; var < 2; ++var)
            for (int m = 0; m < kKinds; ++m) {
                memset(st, 0, sizeof(Stale) * kKinds * 2);
                for (int t = 0; t < trials; ++t) {
                    const uint32_t oldv = 0x1000u + 2u * (uint32_t)t + (uint32_t)var * 0x100000u, newv = oldv + 1u;
                    const bool i_write = (var == 0) == owner;
                    // 1. writer stores old   2. peer touches   3. writer stores new   4. owner checks   5. peer checks
                    if (i_write) {
                        hipLaunchKernelGGL(k_set, dim3(1), dim3(256), 0, 0, reg[m], oldv);
                        CK(hipDeviceSynchronize());
                    }
                    if (owner) stage(&ctl->stage_o, ++s); else { stage(&ctl->stage_p, ++s); }
                    wait_stage(owner ? &ctl->stage_p : &ctl->stage_o, s);
                    if (!owner) {
                        hipLaunchKernelGGL(k_touch, dim3(256), dim3(256), 0, 0, reg[m], sink);
                        CK(hipDeviceSynchronize());
                    }
                    if (owner) stage(&ctl->stage_o, ++s); else { stage(&ctl->stage_p, ++s); }
                    wait_stage(owner ? &ctl->stage_p : &ctl->stage_o, s);
                    if (i_write) {
                        hipLaunchKernelGGL(k_set, dim3(1), dim3(256), 0, 0, reg[m], newv);
                        CK(hipDeviceSynchronize());
                    }
                    if (owner) stage(&ctl->stage_o, ++s); else { stage(&ctl->stage_p, ++s); }
                    wait_stage(owner ? &ctl->stage_p : &ctl->stage_o, s);
                    if (owner) check_all(reg[m], oldv, &st[0]);
                    if (owner) stage(&ctl->stage_o, ++s); else { stage(&ctl->stage_p, ++s); }
                    wait_stage(owner ? &ctl->stage_p : &ctl->stage_o, s);
                    if (!owner) check_all(reg[m], oldv, &st[1]);
                    if (owner) stage(&ctl->stage_o, ++s); else { stage(&ctl->stage_p, ++s); }
                    wait_stage(owner ? &ctl->stage_p : &ctl->stage_o, s);
                }
                const Stale& me = st[owner ? 0 : 1];
                for (int k = 0; k < 4; ++k)
                    printf("{\"mode\": \"alias\", \"writer\": \"%s\", \"toucher\": \"peer\", \"memory\": \"%s\", "
                           "\"reader\": \"%s\", \"load\": \"%s\", \"trials\": %d, \"reads\": %llu, "
                           "\"stale_lanes\": %llu, \"stale_xcc_mask\": %u}\n",
                           var == 0 ? "owner" : "peer (import)", kMemName[m], owner ? "owner" : "peer (import)",
                           kLoadName[k], trials, me.reads[k], me.lanes[k], me.xcc_mask[k]);
                fflush(stdout);
            }
    }
    if (!owner)
        for (int m = 0; m < kKinds; ++m) {
            if (m >= 3) hsa_amd_ipc_memory_detach(reg[m]);
            else CK(hipIpcCloseMemHandle(reg[m]));
        }
    else {
        stage(&ctl->stage_o, 1 << 30);
        shm_unlink(("/rdc_mtype_" + name).c_str());
    }
    return 0;
}
