// MI355X (gfx950) kernels of the rdc path that do not depend on the reduction
// operator (broadcast, synthetic fill) and the (dtype, op) dispatch.
//   per-operator instantiations: rdc_kernels_{max,min,sum,bitor}.hip
//   device templates:            rdc_kernels_impl.h
#include "rdc_kernels_impl.h"

namespace rdc_amd {

__global__ __launch_bounds__(kBlock) void k_bcast(CollArgs a) {
    uint64_t seq;
    if (!launch_begin(a, &seq)) bcast_body(a, seq);
    launch_done(a, seq);
}

// ============================================================ allgather ===
// Allgather of per-rank buffers of any size (rdc::Allgather,
// include/core/rdc-inl.h:106-122; the reference runs it as TryAllgatherRing,
// src/comm/communicator_collective.cc:79-114).  A pure copy, so any route
// gives the reference's bytes: every rank pushes its own buffer's tiles into
// each peer's AG slot `rank` over all links at once (push blocks) and lands
// the peers' buffers from its own AG slots (gather blocks).  Like broadcast,
// receivers never answer, so pushes wait for the targets' done words.
__device__ void allgather_body(const CollArgs& a, uint64_t seq) {
    const int n = a.n, r = a.rank;
    Abort ab{a.err, wall_clock64() + a.timeout_ticks, a.poll_rmw};
    __shared__ uint64_t* s_flags[RDC_MAX_RANKS];
    int b = blockIdx.x;
    if (b < a.nb_scatter) {
        const int items = (n - 1) * a.tiles[r];
        if (b < items) {
            if (threadIdx.x < (unsigned)(n - 1)) s_flags[threadIdx.x] = done_word(a, r, (r + 1 + threadIdx.x) % n);
            __syncthreads();
            if (!block_wait(s_flags, n - 1, seq_prev(seq), ab, RDC_KERR_TIMEOUT_ALLGATHER, a.uc, false)) return;
        }
        for (int it = b; it < items; it += a.nb_scatter) {
            const int t = it / (n - 1);
            const int p = (r + 1 + it % (n - 1)) % n;
            const uint64_t toff = (uint64_t)t * a.tile_bytes;
            uint64_t tlen = a.len[r] - toff;
            if (tlen > a.tile_bytes) tlen = a.tile_bytes;
            block_copy<kDstPeer>(a.ag[p] + (uint64_t)r * a.slot_bytes + a.mis[r] + toff, a.cbuf[r] + a.off[r] + toff, tlen);
            block_publish1(flag_word(a, p, (uint64_t)(n + r) * a.max_tiles + t), seq, a.uc);
        }
        return;
    }
    b -= a.nb_scatter;
    int tmax = 0;
    for (int c = 0; c < n; ++c) tmax = a.tiles[c] > tmax ? a.tiles[c] : tmax;
    const int items = (n - 1) * tmax;
    for (int it = b; it < items; it += a.nb_gather) {
        const int t = it / (n - 1);
        const int c = (r + 1 + it % (n - 1)) % n;
        if (t >= a.tiles[c]) continue;
        if (threadIdx.x == 0) s_flags[0] = flag_word(a, r, (uint64_t)(n + c) * a.max_tiles + t);
        __syncthreads();
        if (!block_wait(s_flags, 1, seq, ab, RDC_KERR_TIMEOUT_ALLGATHER, a.uc)) return;
        const uint64_t toff = (uint64_t)t * a.tile_bytes;
        uint64_t tlen = a.len[c] - toff;
        if (tlen > a.tile_bytes) tlen = a.tile_bytes;
        char* land = a.ag[r] + (uint64_t)c * a.slot_bytes + a.mis[c] + toff;
        block_copy_pull(a.cbuf[c] + a.off[c] + toff, land, tlen);
        __syncthreads();
        if (a.poison) block_poison(land, tlen);  // writers gate on this rank's done word
    }
}

__global__ __launch_bounds__(kBlock) void k_allgather(CollArgs a) {
    uint64_t seq;
    if (!launch_begin(a, &seq)) allgather_body(a, seq);
    launch_done(a, seq);
}

// ============================================================ pack ===
// Coalesced allreduce (rdc_plan.h PlanCoalesced): copy every unit between its
// user buffer and the chunk-major staging image.  Unit table in device memory
// (buf = user address of the unit's first byte); unpack = image -> buffers.
__global__ __launch_bounds__(kBlock) void k_pack(const PackUnit* __restrict__ units, int nunits,
                                                 char* __restrict__ image, int unpack) {
    for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
        char* usr = reinterpret_cast<char*>(units[u].buf);
        char* img = image + units[u].packed;
        const uint64_t len = units[u].len;
        if (unpack) block_copy<kDstLocal>(usr, img, len);
        else block_copy<kDstLocal>(img, usr, len);
    }
}

// ============================================================ p2p copy ===
// Point-to-point pieces (rdc_p2p.cpp): a plain copy, 64 KiB per block step;
// dst may be a peer's IPC-mapped slot (remote stores over xGMI).  Never waits.
// The last block publishes the piece's sequence number into the host-mapped
// control block, so neither side's host needs to observe the kernel first.
__global__ __launch_bounds__(kBlock) void k_copy(char* __restrict__ dst, const char* __restrict__ src, uint64_t bytes,
                                                 uint32_t* arrive, uint64_t* word, uint64_t value) {
    constexpr uint64_t kStep = 64 << 10;
    for (uint64_t off = (uint64_t)blockIdx.x * kStep; off < bytes; off += (uint64_t)gridDim.x * kStep)
        block_copy<kDstPeer>(dst + off, src + off, bytes - off < kStep ? bytes - off : kStep);
    if (word == nullptr) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        if (atomicAdd(arrive, 1u) == gridDim.x - 1) {
            __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __hip_atomic_store(word, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ================================================================ probe ===
// Link probe (Communicator::Probe): the blocks are split evenly over the ndst
// targets; each target receives the same `bytes` from src with remote
// stores (16-B non-temporal lanes), all targets concurrently.  With t.src[d]
// set the blocks read that (remote) source instead: pull instead of push.
__global__ __launch_bounds__(kBlock) void k_push(PushTargets t, int ndst, const char* __restrict__ src,
                                                 uint64_t bytes) {
    const int per = gridDim.x / ndst;
    const int d = blockIdx.x % ndst, b = blockIdx.x / ndst;
    if (b >= per) return;
    constexpr uint64_t kStep = 64 << 10;
    for (uint64_t off = (uint64_t)b * kStep; off < bytes; off += (uint64_t)per * kStep)
        block_copy<kDstPeer>(t.dst[d] + off, (t.src[d] ? t.src[d] : src) + off, bytes - off < kStep ? bytes - off : kStep);
}

// ================================================================= fill ===
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ uint16_t f32_to_f16_bits(float f) {
    _Float16 h = (_Float16)f;
    return __builtin_bit_cast(uint16_t, h);
}

__global__ __launch_bounds__(kBlock) void k_fill(char* buf, uint64_t count, int dtype, uint64_t seed, int rank) {
    const uint64_t key = seed ^ ((uint64_t)rank << 40);
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < count; i += stride) {
        const uint64_t u = splitmix64(key ^ i);
        const float f = (float)(int32_t)(u >> 32) * 0x1p-31f;
        switch (dtype) {
            case RDC_DT_INT8: case RDC_DT_UINT8: reinterpret_cast<uint8_t*>(buf)[i] = (uint8_t)u; break;
            case RDC_DT_INT32: case RDC_DT_UINT32: reinterpret_cast<uint32_t*>(buf)[i] = (uint32_t)u; break;
            case RDC_DT_FLOAT32: reinterpret_cast<float*>(buf)[i] = f; break;
            case RDC_DT_FLOAT64: reinterpret_cast<double*>(buf)[i] = (double)(int64_t)u * 0x1p-63; break;
            case RDC_DT_FLOAT16: reinterpret_cast<uint16_t*>(buf)[i] = f32_to_f16_bits(f); break;
            case RDC_DT_BFLOAT16: reinterpret_cast<uint16_t*>(buf)[i] = f32_to_bf16(f); break;
            default: reinterpret_cast<uint64_t*>(buf)[i] = u; break;
        }
    }
}

bool pick_max(int dtype, KernelSet* ks);
bool pick_min(int dtype, KernelSet* ks);
bool pick_sum(int dtype, KernelSet* ks);
bool pick_bitor(int dtype, KernelSet* ks);

bool get_kernels(int dtype, int op, KernelSet* ks) {
    switch (op) {
        case RDC_OP_MAX: return pick_max(dtype, ks);
        case RDC_OP_MIN: return pick_min(dtype, ks);
        case RDC_OP_SUM: return pick_sum(dtype, ks);
        case RDC_OP_BITOR: return pick_bitor(dtype, ks);
        default: return false;
    }
}
namespace {
template <typename F>
int occupancy_of(F kernel, int* cache) {
    if (*cache > 0) return *cache;
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, kBlock, 0) != hipSuccess || b <= 0) {
        (void)hipGetLastError();
        b = 1;
    }
    *cache = b;
    return b;
}
}  // namespace

int occupancy_bcast() {
    static int c = 0;
    return occupancy_of(k_bcast, &c);
}

int occupancy_allgather() {
    static int c = 0;
    return occupancy_of(k_allgather, &c);
}

hipError_t launch_allgather(const CollArgs& a, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_allgather, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_bcast(const CollArgs& a, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_bcast, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_pack(const PackUnit* units, int nunits, char* image, int unpack, int grid, hipStream_t s) {
    if (nunits <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack, dim3(grid), dim3(kBlock), 0, s, units, nunits, image, unpack);
    return hipGetLastError();
}

hipError_t launch_copy(void* dst, const void* src, uint64_t bytes, hipStream_t s, uint32_t* arrive, uint64_t* word,
                       uint64_t value) {
    if (bytes == 0 && word == nullptr) return hipSuccess;
    uint64_t grid = (bytes + (64 << 10) - 1) >> 16;
    if (grid > 128) grid = 128;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(k_copy, dim3((unsigned)grid), dim3(kBlock), 0, s, (char*)dst, (const char*)src, bytes, arrive,
                       word, value);
    return hipGetLastError();
}

hipError_t launch_push(const PushTargets& t, int ndst, const void* src, uint64_t bytes, int grid, hipStream_t s) {
    if (ndst <= 0 || bytes == 0) return hipSuccess;
    grid = (grid / ndst) * ndst;
    if (grid < ndst) grid = ndst;
    hipLaunchKernelGGL(k_push, dim3((unsigned)grid), dim3(kBlock), 0, s, t, ndst, (const char*)src, bytes);
    return hipGetLastError();
}

hipError_t launch_fill(void* buf, uint64_t count, int dtype, uint64_t seed, int rank, hipStream_t s) {
    uint64_t blocks = (count + kBlock - 1) / kBlock;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill, dim3((unsigned)blocks), dim3(kBlock), 0, s, (char*)buf, count, dtype, seed, rank);
    return hipGetLastError();
}

}  // namespace rdc_amd
