// Hand-off litmus for the collectives' flag/payload protocol on gfx950: can
// a consumer read a STALE payload (or keep polling a stale flag) after a
// producer on another CU / XCD published it the way rdc_device.h does?
//
// Per pair p (reader block, writer block: consecutive blocks, which dispatch
// deals to different XCDs; each block records its XCC_ID) and iteration i:
//   reader: load the 1 KiB payload X_p with the load kind under test AND a
//           plain load (so whatever cache those loads fill holds i-1), then
//           ack_p = i (relaxed system-scope store);
//   writer: poll ack_p == i, store X_p = i with `buffer_store_dwordx4 sc0 sc1`
//           (the product's st16_wt), every lane `s_waitcnt vmcnt(0)`, wave
//           barrier, lane 0: flag_p = i (relaxed system-scope 64-bit store);
//   reader: poll flag_p >= i (relaxed system-scope 64-bit loads, the
//           product's block_wait), then load X_p with the kind under test and
//           count the 16-B lanes that do not hold i.
// Load kinds: 0 plain buffer load, 1 nt, 2 sc1, 3 sc0 sc1, 4 global nt
// (__builtin_nontemporal_load: the product's ld16_nt), 5 global plain.
// Memory kinds: 0 hipMalloc, 1 hipExtMallocWithFlags(Uncached) (the product's
// scratch and flags), 2 hipExtMallocWithFlags(Finegrained).
// Every wait is bounded (10 ms per iteration, 20 s for the first): a lost
// flag is counted as a timeout and both blocks of the pair stop.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/handoff_litmus tools/handoff_litmus.hip
//   tools/handoff_litmus local [ITERS]           # every (memory, load) pair, one process
//   tools/handoff_litmus owner DIR MEM LOAD &    # IPC: readers here, on this process's memory
//   tools/handoff_litmus writer DIR              #      writers here, through the IPC import
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

constexpr int kPairs = 64;
constexpr int kLine = 1024;  // payload bytes per pair (64 lanes x 16 B)
// layout of one region: [kPairs] payloads, then flag[kPairs], ack[kPairs] (one 128-B line each)
constexpr size_t kFlagOff = (size_t)kPairs * kLine;
constexpr size_t kAckOff = kFlagOff + (size_t)kPairs * 128;
constexpr size_t kRegion = kAckOff + (size_t)kPairs * 128;

struct Result {
    unsigned long long stale;     // 16-B lanes read with an old value
    unsigned long long timeouts;  // waits that gave up
    unsigned long long iters;     // iterations completed (reader side)
    unsigned int xcc[2 * kPairs];
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
    const uint64_t b = (uint64_t)(uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, 0xffffffffu, 0x00020000);
}

template <int LOAD>
__device__ __forceinline__ v4u load_kind(const char* x, uint32_t off) {
    if constexpr (LOAD == 0) return __builtin_amdgcn_raw_buffer_load_b128(rsrc(x), off, 0, 0);
    else if constexpr (LOAD == 1) return __builtin_amdgcn_raw_buffer_load_b128(rsrc(x), off, 0, 2);
    else if constexpr (LOAD == 2) return __builtin_amdgcn_raw_buffer_load_b128(rsrc(x), off, 0, 16);
    else if constexpr (LOAD == 3) return __builtin_amdgcn_raw_buffer_load_b128(rsrc(x), off, 0, 17);
    else if constexpr (LOAD == 4) return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(x + off));
    else return *reinterpret_cast<const volatile v4u*>(x + off);
}

__device__ __forceinline__ uint64_t ld_sys64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys64(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ unsigned xcc_id() {
    // s_getreg_b32 HW_REG_XCC_ID (id 20), bits [3:0]
    return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf;
}

// wave-uniform wait for *p >= want; false on timeout
__device__ __forceinline__ bool wait_ge(const uint64_t* p, uint64_t want, uint64_t ticks) {
    const uint64_t deadline = wall_clock64() + ticks;
    while (true) {
        const uint64_t v = ld_sys64(p);
        if (__builtin_amdgcn_readfirstlane((uint32_t)(v >= want))) return true;
        if (wall_clock64() > deadline) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}

// role bits: 1 reader, 2 writer.  Blocks 2p (reader) and 2p+1 (writer).
template <int LOAD>
__global__ __launch_bounds__(64) void k_litmus(char* region, int iters, int roles, Result* res) {
    const int pair = blockIdx.x >> 1;
    const bool reader = (blockIdx.x & 1) == 0;
    const unsigned lane = threadIdx.x;
    char* x = region + (size_t)pair * kLine;
    uint64_t* flag = reinterpret_cast<uint64_t*>(region + kFlagOff + (size_t)pair * 128);
    uint64_t* ack = reinterpret_cast<uint64_t*>(region + kAckOff + (size_t)pair * 128);
    if (lane == 0) res->xcc[blockIdx.x] = xcc_id();
    unsigned long long stale = 0, timeouts = 0, done = 0;
    if (reader && (roles & 1)) {
        uint32_t sink = 0;
        for (int i = 1; i <= iters; ++i) {
            const v4u a = load_kind<LOAD>(x, lane * 16);
            const v4u b = load_kind<5>(x, lane * 16);
            sink += a.x + b.y;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) st_sys64(ack, (uint64_t)i);
            if (!wait_ge(flag, (uint64_t)i, i == 1 ? 2000000000ull : 1000000ull)) {
                ++timeouts;
                break;
            }
            const v4u v = load_kind<LOAD>(x, lane * 16);
            const uint32_t w = (uint32_t)i;
            stale += (v.x != w || v.y != w || v.z != w || v.w != w) ? 1 : 0;
            ++done;
        }
        if (sink == 0xdeadbeefu) stale += 1000000;  // keeps the pre-touch loads live
        atomicAdd(&res->stale, stale);
        if (lane == 0) {
            atomicAdd(&res->timeouts, timeouts);
            atomicAdd(&res->iters, done);
        }
    } else if (!reader && (roles & 2)) {
        const __amdgpu_buffer_rsrc_t r = rsrc(x);
        for (int i = 1; i <= iters; ++i) {
            if (!wait_ge(ack, (uint64_t)i, i == 1 ? 2000000000ull : 1000000ull)) {
                if (lane == 0) atomicAdd(&res->timeouts, 1ull);
                break;
            }
            const uint32_t w = (uint32_t)i;
            __builtin_amdgcn_raw_buffer_store_b128(v4u{w, w, w, w}, r, lane * 16, 0, 17);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) st_sys64(flag, (uint64_t)i);
        }
    }
}

typedef void (*KFn)(char*, int, int, Result*);
static KFn kernel_for(int load) {
    switch (load) {
        case 0: return k_litmus<0>;
        case 1: return k_litmus<1>;
        case 2: return k_litmus<2>;
        case 3: return k_litmus<3>;
        case 4: return k_litmus<4>;
        default: return k_litmus<5>;
    }
}
static const char* kLoadName[] = {"buffer plain", "buffer nt", "buffer sc1", "buffer sc0 sc1", "global nt", "global plain"};
static const char* kMemName[] = {"hipMalloc", "uncached", "finegrained"};

static char* alloc_kind(int mem) {
    void* p = nullptr;
    if (mem == 0) CK(hipMalloc(&p, kRegion));
    else CK(hipExtMallocWithFlags(&p, kRegion, mem == 1 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
    CK(hipMemset(p, 0, kRegion));
    CK(hipDeviceSynchronize());
    return static_cast<char*>(p);
}

static void report(const char* mode, int mem, int load, const Result& r, int iters) {
    int cross = 0;
    for (int p = 0; p < kPairs; ++p) cross += r.xcc[2 * p] != r.xcc[2 * p + 1];
    printf("{\"mode\": \"%s\", \"memory\": \"%s\", \"load\": \"%s\", \"pairs\": %d, \"cross_xcd_pairs\": %d, "
           "\"iters\": %d, \"reads\": %llu, \"stale_lanes\": %llu, \"timeouts\": %llu}\n",
           mode, kMemName[mem], kLoadName[load], kPairs, cross, iters, r.iters, r.stale, r.timeouts);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "local";
    Result* res = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&res), sizeof(Result), hipHostMallocCoherent));
    if (mode == "local") {
        const int iters = argc > 2 ? atoi(argv[2]) : 2000;
        for (int mem = 0; mem < 3; ++mem) {
            for (int load = 0; load < 6; ++load) {
                char* reg = alloc_kind(mem);
                memset(res, 0, sizeof(Result));
                hipLaunchKernelGGL(kernel_for(load), dim3(2 * kPairs), dim3(64), 0, 0, reg, iters, 3, res);
                CK(hipGetLastError());
                CK(hipDeviceSynchronize());
                report("local", mem, load, *res, iters);
                CK(hipFree(reg));
            }
        }
        return 0;
    }
    if (argc < 3) {
        fprintf(stderr, "usage: %s local [ITERS] | owner DIR MEM LOAD [ITERS] | writer DIR\n", argv[0]);
        return 2;
    }
    const std::string dir = argv[2];
    if (mode == "owner") {
        const int mem = atoi(argv[3]), load = atoi(argv[4]);
        const int iters = argc > 5 ? atoi(argv[5]) : 2000;
        char* reg = alloc_kind(mem);
        hipIpcMemHandle_t h;
        CK(hipIpcGetMemHandle(&h, reg));
        FILE* f = fopen((dir + "/handle.tmp").c_str(), "wb");
        fwrite(&h, sizeof(h), 1, f);
        fwrite(&iters, sizeof(iters), 1, f);
        fclose(f);
        rename((dir + "/handle.tmp").c_str(), (dir + "/handle").c_str());
        memset(res, 0, sizeof(Result));
        hipLaunchKernelGGL(kernel_for(load), dim3(2 * kPairs), dim3(64), 0, 0, reg, iters, 1, res);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        report("ipc owner reads", mem, load, *res, iters);
        FILE* d = fopen((dir + "/done").c_str(), "w");
        fclose(d);
        return 0;
    }
    if (mode == "writer") {
        hipIpcMemHandle_t h;
        int iters = 0;
        FILE* f = nullptr;
        for (int t = 0; t < 600 && !(f = fopen((dir + "/handle").c_str(), "rb")); ++t) usleep(50000);
        if (!f) {
            fprintf(stderr, "no handle\n");
            return 1;
        }
        if (fread(&h, sizeof(h), 1, f) != 1 || fread(&iters, sizeof(iters), 1, f) != 1) return 1;
        fclose(f);
        void* reg = nullptr;
        CK(hipIpcOpenMemHandle(&reg, h, hipIpcMemLazyEnablePeerAccess));
        memset(res, 0, sizeof(Result));
        hipLaunchKernelGGL(kernel_for(5), dim3(2 * kPairs), dim3(64), 0, 0, static_cast<char*>(reg), iters, 2, res);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        printf("{\"mode\": \"ipc writer\", \"timeouts\": %llu}\n", res->timeouts);
        CK(hipIpcCloseMemHandle(reg));
        return 0;
    }
    return 2;
}
