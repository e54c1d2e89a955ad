// Rotating-writer hand-off litmus (round 5): the writer of a
// flag / payload moves from XCD to XCD between hand-offs, as the block that
// owns tile t does between launches when dispatch places the grid
// differently (e.g. under queue time-slicing).  Question: after a write-
// through (sc0 sc1) store from XCD b, can a reader on XCD a still see the
// value an earlier store from XCD a left there?
//
// P pairs (P = 9, coprime with the 8 XCDs); pair p has a payload X_p (1 KiB),
// a flag F_p and an ack A_p, each in lines of its own.  Writer blocks
// b = k * P + p (k = 0..7) sit on 8 different XCDs; at iteration i only
// writer k = i % 8 of pair p acts: wait A_p >= i, store X_p = i (sc0 sc1,
// 16 B lanes), s_waitcnt vmcnt(0), F_p = i (relaxed system-scope store).
// Reader block p: poll F_p >= i (relaxed system-scope 64-bit loads), read X_p
// (load kind under test), count lanes != i, then A_p = i + 1.
// Every wait is bounded (10 ms per iteration): a flag never seen counts as a
// timeout and records what the reader saw.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/rotate_litmus tools/rotate_litmus.hip
//   tools/rotate_litmus local MEM LOAD [ITERS]        # one process, one allocation
//   tools/rotate_litmus owner DIR MEM LOAD [ITERS] &  # IPC: readers on this process's memory
//   tools/rotate_litmus writer DIR                    #      writers through the import
// MEM: 0 hipMalloc, 1 uncached (the collectives' scratch), 2 fine-grained.
// LOAD: 0 plain, 1 nt, 3 sc0 sc1 (buffer loads).
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

constexpr int kP = 9;
constexpr size_t kLine = 1024;
constexpr size_t kFlagOff = kP * kLine;
constexpr size_t kAckOff = kFlagOff + kP * 256;
constexpr size_t kRegion = kAckOff + kP * 256;

struct Result {
    unsigned long long stale, timeouts, iters;
    unsigned long long first_iter, first_seen;
    unsigned int xcc[8 * kP + kP];
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
    else return __builtin_amdgcn_raw_buffer_load_b128(rsrc(x), off, 0, 17);
}
__device__ __forceinline__ uint64_t ld_sys64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys64(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf; }

// wave-uniform wait for *p >= want; returns the last value seen; *ok = matched
__device__ __forceinline__ uint64_t wait_ge(const uint64_t* p, uint64_t want, uint64_t ticks, bool* ok) {
    const uint64_t deadline = wall_clock64() + ticks;
    uint64_t v = 0;
    while (true) {
        v = ld_sys64(p);
        if (__builtin_amdgcn_readfirstlane((uint32_t)(v >= want))) {
            *ok = true;
            return v;
        }
        if (wall_clock64() > deadline) {
            *ok = false;
            return v;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// blocks [0, P): readers (roles & 1); [P, P + 8P): writers (roles & 2)
template <int LOAD>
__global__ __launch_bounds__(64) void k_rotate(char* region, int iters, int roles, Result* res, uint64_t wait_ticks) {
    const unsigned lane = threadIdx.x;
    const int b = blockIdx.x;
    if (lane == 0) res->xcc[b] = xcc_id();
    if (b < kP) {
        if (!(roles & 1)) return;
        const int p = b;
        const char* x = region + p * kLine;
        uint64_t* flag = reinterpret_cast<uint64_t*>(region + kFlagOff + p * 256);
        uint64_t* ack = reinterpret_cast<uint64_t*>(region + kAckOff + p * 256);
        unsigned long long stale = 0, done = 0;
        if (lane == 0) st_sys64(ack, 1);
        for (int i = 1; i <= iters; ++i) {
            bool ok;
            const uint64_t seen = wait_ge(flag, (uint64_t)i, i == 1 ? 2000000000ull : wait_ticks, &ok);
            if (!ok) {
                if (lane == 0) {
                    atomicAdd(&res->timeouts, 1ull);
                    atomicCAS(&res->first_iter, 0ull, (unsigned long long)i);
                    atomicCAS(&res->first_seen, 0ull, (unsigned long long)seen + 1);
                }
                break;
            }
            const v4u v = load_kind<LOAD>(x, lane * 16);
            const uint32_t w = (uint32_t)i;
            stale += (v.x != w || v.y != w || v.z != w || v.w != w) ? 1 : 0;
            ++done;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) st_sys64(ack, (uint64_t)i + 1);
        }
        atomicAdd(&res->stale, stale);
        if (lane == 0) atomicAdd(&res->iters, done);
        return;
    }
    if (!(roles & 2)) return;
    const int wb = b - kP;
    const int p = wb % kP, k = wb / kP;  // writer k of pair p: XCD rotates with k
    char* x = region + p * kLine;
    uint64_t* flag = reinterpret_cast<uint64_t*>(region + kFlagOff + p * 256);
    uint64_t* ack = reinterpret_cast<uint64_t*>(region + kAckOff + p * 256);
    const __amdgpu_buffer_rsrc_t r = rsrc(x);
    for (int i = 1 + k; i <= iters; i += 8) {
        bool ok;
        (void)wait_ge(ack, (uint64_t)i, 2000000000ull, &ok);
        if (!ok) break;
        const uint32_t w = (uint32_t)i;
        __builtin_amdgcn_raw_buffer_store_b128(v4u{w, w, w, w}, r, lane * 16, 0, 17);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) st_sys64(flag, (uint64_t)i);
    }
}

typedef void (*KFn)(char*, int, int, Result*, uint64_t);
// LITMUS_WAIT_MS: per-iteration wait limit (default 10 ms)
static uint64_t wait_ticks() {
    const char* v = getenv("LITMUS_WAIT_MS");
    return (uint64_t)(v ? atof(v) : 10.0) * 100000ull;
}
static KFn kernel_for(int load) { return load == 0 ? k_rotate<0> : load == 1 ? k_rotate<1> : k_rotate<3>; }
static const char* kMem[] = {"hipMalloc", "uncached", "finegrained"};

static char* alloc_kind(int mem) {
    void* p = nullptr;
    if (mem == 0) CK(hipMalloc(&p, kRegion));
    else CK(hipExtMallocWithFlags(&p, kRegion, mem == 1 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
    CK(hipMemset(p, 0, kRegion));
    CK(hipDeviceSynchronize());
    return static_cast<char*>(p);
}
static void report(const char* mode, int mem, int load, const Result& r, int iters) {
    int rot = 0;
    for (int p = 0; p < kP; ++p) {
        unsigned seen = 0;
        for (int k = 0; k < 8; ++k) seen |= 1u << r.xcc[kP + k * kP + p];
        rot += __builtin_popcount(seen);
    }
    printf("{\"mode\": \"%s\", \"memory\": \"%s\", \"load\": %d, \"pairs\": %d, \"writer_xcds_per_pair\": %.2f, "
           "\"iters\": %d, \"reads\": %llu, \"stale_lanes\": %llu, \"timeouts\": %llu, \"first_timeout\": [%llu, %llu]}\n",
           mode, kMem[mem], load, kP, (double)rot / kP, iters, r.iters, r.stale, r.timeouts, r.first_iter,
           r.first_seen ? r.first_seen - 1 : 0);
    fflush(stdout);
}

__global__ void k_touch(uint32_t* p) {
    if (threadIdx.x == 0 && p) p[blockIdx.x] = 0;
}

// LITMUS_EXTRA_STREAMS=k: create k more streams and run a kernel on each, so
// that this process holds up to GPU_MAX_HW_QUEUES hardware queues (several
// processes doing so oversubscribe the GPU's queue slots: time-slicing)
static void extra_queues() {
    const char* v = getenv("LITMUS_EXTRA_STREAMS");
    const int k = v ? atoi(v) : 0;
    for (int i = 0; i < k; ++i) {
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, nullptr);
        CK(hipStreamSynchronize(s));
    }
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "local";
    extra_queues();
    Result* res = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&res), sizeof(Result), hipHostMallocCoherent));
    memset(res, 0, sizeof(Result));
    const int grid = kP + 8 * kP;
    if (mode == "local") {
        const int mem = argc > 2 ? atoi(argv[2]) : 1, load = argc > 3 ? atoi(argv[3]) : 1;
        const int iters = argc > 4 ? atoi(argv[4]) : 4000;
        char* reg = alloc_kind(mem);
        hipLaunchKernelGGL(kernel_for(load), dim3(grid), dim3(64), 0, 0, reg, iters, 3, res, wait_ticks());
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        report("local", mem, load, *res, iters);
        return 0;
    }
    if (argc < 3) return 2;
    const std::string dir = argv[2];
    if (mode == "owner") {
        const int mem = atoi(argv[3]), load = atoi(argv[4]);
        const int iters = argc > 5 ? atoi(argv[5]) : 4000;
        char* reg = alloc_kind(mem);
        hipIpcMemHandle_t h;
        CK(hipIpcGetMemHandle(&h, reg));
        FILE* f = fopen((dir + "/handle.tmp").c_str(), "wb");
        fwrite(&h, sizeof(h), 1, f);
        fwrite(&iters, sizeof(iters), 1, f);
        fclose(f);
        rename((dir + "/handle.tmp").c_str(), (dir + "/handle").c_str());
        hipLaunchKernelGGL(kernel_for(load), dim3(grid), dim3(64), 0, 0, reg, iters, 1, res, wait_ticks());
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        report("ipc (readers in the owner)", mem, load, *res, iters);
        if (res->timeouts) {  // what memory holds now, read by the host, beside what the readers last saw
            printf("{\"host_flags\": [");
            for (int p = 0; p < kP; ++p) {
                uint64_t v = 0;
                CK(hipMemcpy(&v, reg + kFlagOff + p * 256, 8, hipMemcpyDeviceToHost));
                printf("%s%llu", p ? ", " : "", (unsigned long long)v);
            }
            printf("]}\n");
        }
        return 0;
    }
    if (mode == "writer") {
        hipIpcMemHandle_t h;
        int iters = 0;
        FILE* f = nullptr;
        for (int t = 0; t < 600 && !(f = fopen((dir + "/handle").c_str(), "rb")); ++t) usleep(50000);
        if (!f) return 1;
        if (fread(&h, sizeof(h), 1, f) != 1 || fread(&iters, sizeof(iters), 1, f) != 1) return 1;
        fclose(f);
        void* reg = nullptr;
        CK(hipIpcOpenMemHandle(&reg, h, hipIpcMemLazyEnablePeerAccess));
        hipLaunchKernelGGL(kernel_for(0), dim3(grid), dim3(64), 0, 0, static_cast<char*>(reg), iters, 2, res, wait_ticks());
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipIpcCloseMemHandle(reg));
        return 0;
    }
    return 2;
}
