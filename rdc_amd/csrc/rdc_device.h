// Device-side primitives for the MI355X (gfx950) rdc allreduce path.
//
//  * reduction operators with the reference's exact semantics
//    (op::Max/Min/Sum/BitOR::Reduce, include/core/mpi.h:85-112):
//        Max: dst = (dst < src) ? src : dst      (NaN in src ignored, NaN in dst sticky)
//        Min: dst = (dst > src) ? src : dst
//        Sum: dst = dst + src                    (signed ints wrap: computed unsigned)
//        BitOR: dst = dst | src
//    f16: native v_add_f16 (correctly rounded); bf16: f32 add + RNE to bf16.
//  * 16-byte vector reduce (v4u reinterpreted as 16/sizeof(T) lanes)
//  * cross-GPU hand-off: payload stores -> every wave's vmcnt(0) -> barrier ->
//    one lane: system-scope release fence, asm vmcnt(0), relaxed system-scope
//    flag store.  Consumer: one lane per flag polls relaxed/system, then a
//    system-scope acquire fence, vmcnt(0), barrier (MI355X_MICROARCH.md
//    "Workgroup dispatch ... visibility"; cdna_hip_programming.md G16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rdc_common.h"

namespace rdc_amd {

// ---------------------------------------------------------------- types ----
// native 16-byte vector (global_load/store_dwordx4)
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct bf16_t {
    uint16_t bits;
};

template <typename T> struct Arith { typedef T U; };
template <> struct Arith<int8_t> { typedef uint8_t U; };
template <> struct Arith<int32_t> { typedef uint32_t U; };
template <> struct Arith<int64_t> { typedef uint64_t U; };

__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
    return __uint_as_float((uint32_t)b << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    uint32_t x = __float_as_uint(f);
    if ((x & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((x >> 16) | 0x40);
    x += 0x7fffu + ((x >> 16) & 1u);
    return (uint16_t)(x >> 16);
}

template <int OP> struct OpF;
template <> struct OpF<RDC_OP_MAX> {
    template <typename T> __device__ __forceinline__ static T apply(T d, T s) { return (d < s) ? s : d; }
    __device__ __forceinline__ static bf16_t apply(bf16_t d, bf16_t s) {
        return (bf16_to_f32(d.bits) < bf16_to_f32(s.bits)) ? s : d;
    }
};
template <> struct OpF<RDC_OP_MIN> {
    template <typename T> __device__ __forceinline__ static T apply(T d, T s) { return (d > s) ? s : d; }
    __device__ __forceinline__ static bf16_t apply(bf16_t d, bf16_t s) {
        return (bf16_to_f32(d.bits) > bf16_to_f32(s.bits)) ? s : d;
    }
};
template <> struct OpF<RDC_OP_SUM> {
    template <typename T> __device__ __forceinline__ static T apply(T d, T s) {
        typedef typename Arith<T>::U U;
        return (T)((U)d + (U)s);
    }
    __device__ __forceinline__ static float apply(float d, float s) { return d + s; }
    __device__ __forceinline__ static double apply(double d, double s) { return d + s; }
    __device__ __forceinline__ static _Float16 apply(_Float16 d, _Float16 s) { return d + s; }
    // f32 add (exact inputs) then one RNE conversion = the correctly rounded
    // bf16 add; v_cvt_pk_bf16_f32 (gfx950) does the conversion in hardware
    __device__ __forceinline__ static bf16_t apply(bf16_t d, bf16_t s) {
        const __bf16 h = (__bf16)(bf16_to_f32(d.bits) + bf16_to_f32(s.bits));
        bf16_t r;
        r.bits = __builtin_bit_cast(uint16_t, h);
        return r;
    }
};
template <> struct OpF<RDC_OP_BITOR> {
    template <typename T> __device__ __forceinline__ static T apply(T d, T s) {
        typedef typename Arith<T>::U U;
        return (T)((U)d | (U)s);
    }
};

// Reduce two 16-byte vectors lane-wise: returns OP(d, s) per element.
template <int OP, typename T>
__device__ __forceinline__ v4u reduce16(v4u d, v4u s) {
    constexpr int K = 16 / sizeof(T);
    T a[K], b[K];
    __builtin_memcpy(a, &d, 16);
    __builtin_memcpy(b, &s, 16);
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = OpF<OP>::apply(a[k], b[k]);
    __builtin_memcpy(&d, a, 16);
    return d;
}

// bf16 Sum, two lanes per dword: v_pk_add_f32 + v_cvt_pk_bf16_f32 instead of
// a software round per element (the generic loop runs 4.35 TB/s, ALU-bound)
template <>
__device__ __forceinline__ v4u reduce16<RDC_OP_SUM, bf16_t>(v4u d, v4u s) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef __bf16 h2 __attribute__((ext_vector_type(2)));
    v4u out;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const f2 a = {__uint_as_float(d[k] << 16), __uint_as_float(d[k] & 0xffff0000u)};
        const f2 b = {__uint_as_float(s[k] << 16), __uint_as_float(s[k] & 0xffff0000u)};
        out[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(a + b, h2));
    }
    return out;
}

// ------------------------------------------------------- memory access ----
__device__ __forceinline__ v4u ld16(const void* p) { return *reinterpret_cast<const v4u*>(p); }
__device__ __forceinline__ void st16(void* p, v4u v) { *reinterpret_cast<v4u*>(p) = v; }
// streaming (non-temporal) forms for once-touched bytes
__device__ __forceinline__ v4u ld16_nt(const void* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
}
__device__ __forceinline__ void st16_nt(void* p, v4u v) {
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
}

// ------------------------------------------------------------- hand-off ----
__device__ __forceinline__ uint32_t flag_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void flag_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool seq_reached(uint32_t v, uint32_t seq) { return (int32_t)(v - seq) >= 0; }

// Called by EVERY thread of the block after its payload stores.  Lanes
// 0..nflags-1 of wave 0 then store flags[i] = seq.
// Every hand-off payload lives in the peers' scratch slots.  When all scratch
// is uncached (MTYPE UC, hipDeviceMallocUncached: `uc`), those stores are
// write-through — no XCD's L2 keeps them — and every storing wave's
// `s_waitcnt vmcnt(0)` (before the barrier) means they have been performed
// at memory: the write-through + drained-flag form of MI355X_MICROARCH.md
// ("Valid forms", R1), with uncached memory in place of `sc1` stores.  The
// system-scope release fence would only add an L2 write-back (buffer_wbl2
// sc0 sc1, 1.7-6.5 us per call) of cached lines no peer reads, so it is
// issued only for fine- / coarse-grained scratch (alloc fallbacks).
__device__ __forceinline__ void block_publish(uint32_t* const* flags, int nflags, uint32_t seq, int uc) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < (unsigned)nflags) {
        if (!uc) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        flag_store(flags[threadIdx.x], seq);
    }
}

__device__ __forceinline__ void block_publish1(uint32_t* flag, uint32_t seq, int uc) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!uc) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        flag_store(flag, seq);
    }
}

struct Abort {
    uint32_t* err;          // local error word (device memory), 0 = ok
    uint64_t deadline;      // wall_clock64() value after which we give up
};

// Block-wide wait until every flags[i] (i < nflags <= 64) reached seq.  Wave 0
// polls (one lane per flag), sleeping between polls; the other waves park at
// the barrier.  Returns false (uniformly) on timeout or if another block of
// this launch already aborted.  With cached scratch the matching lane then
// runs a system-scope acquire (L2 / L1 invalidate) so the block's plain loads
// of the handed-off bytes cannot hit stale lines; uncached scratch (`uc`) is
// never held in any GPU cache, so its loads after the matched poll read
// memory and need no invalidate (MI355X_MICROARCH.md: an acquire is ≈1.7 us).
__device__ __forceinline__ bool block_wait(uint32_t* const* flags, int nflags, uint32_t seq,
                                           const Abort& ab, uint32_t code, int uc) {
    __shared__ int s_ok;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        bool mine = lane >= nflags;
        bool ok = true;
        uint32_t spins = 0;
        while (true) {
            if (!mine) mine = seq_reached(flag_load(flags[lane]), seq);
            if (__all(mine)) break;
            if ((++spins & 63) == 0) {
                bool dead = wall_clock64() > ab.deadline ||
                            __hip_atomic_load(ab.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                if (__any(dead)) { ok = false; break; }
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (lane == 0) {
            if (ok && !uc) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else if (!ok) {
                uint32_t expected = 0;
                __hip_atomic_compare_exchange_strong(ab.err, &expected, code, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            s_ok = ok;
        }
    }
    __syncthreads();
    const bool ok = s_ok != 0;
    __syncthreads();  // s_ok reused by the next wait
    return ok;
}

// ------------------------------------------------------ block-wide moves ----
// Byte ranges [0,len).  Scratch images sit at the buffer-relative alignment
// (offset % 16), so they are congruent with the user buffer whenever the
// user pointer is 16-B aligned: then the middle runs as 16-byte lanes and
// only the <16-byte head/tail goes element-wise.  A rank whose pointer is
// not 16-B aligned takes the narrow path (units of the widest common
// alignment), still exact.

// dst[i] = src[i], dst and src congruent mod 16
__device__ __forceinline__ void block_copy_vec(char* __restrict__ dst, const char* __restrict__ src,
                                               uint64_t len) {
    const uint64_t mis = (uint64_t)(uintptr_t)src & 15;
    uint64_t head = mis ? (16 - mis) : 0;
    if (head > len) head = len;
    const uint64_t nvec = (len - head) >> 4;
    const uint64_t tail_start = head + (nvec << 4);
    const unsigned tid = threadIdx.x;
    if (tid < head) dst[tid] = src[tid];
    if (tid < len - tail_start) dst[tail_start + tid] = src[tail_start + tid];
    const v4u* s = reinterpret_cast<const v4u*>(src + head);
    v4u* d = reinterpret_cast<v4u*>(dst + head);
    constexpr int U = 8;  // 32 KiB in flight per 256-thread block
    const uint64_t step = (uint64_t)blockDim.x;
    uint64_t i = tid;
    for (; i + (U - 1) * step < nvec; i += U * step) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld16_nt(s + i + u * step);
#pragma unroll
        for (int u = 0; u < U; ++u) st16_nt(d + i + u * step, v[u]);
    }
    for (; i < nvec; i += step) st16_nt(d + i, ld16_nt(s + i));
}

template <typename W>
__device__ __forceinline__ void block_copy_words(char* dst, const char* src, uint64_t len) {
    const uint64_t mis = (uint64_t)(uintptr_t)src & (sizeof(W) - 1);
    uint64_t head = mis ? sizeof(W) - mis : 0;
    if (head > len) head = len;
    const uint64_t nw = (len - head) / sizeof(W);
    const uint64_t tail_start = head + nw * sizeof(W);
    const unsigned tid = threadIdx.x;
    if (tid < head) dst[tid] = src[tid];
    if (tid < len - tail_start) dst[tail_start + tid] = src[tail_start + tid];
    const W* s = reinterpret_cast<const W*>(src + head);
    W* d = reinterpret_cast<W*>(dst + head);
    for (uint64_t i = tid; i < nw; i += blockDim.x) d[i] = s[i];
}

__device__ __forceinline__ void block_copy(char* __restrict__ dst, const char* __restrict__ src, uint64_t len) {
    const uintptr_t x = ((uintptr_t)dst ^ (uintptr_t)src) & 15;
    if (x == 0) block_copy_vec(dst, src, len);
    else if ((x & 7) == 0) block_copy_words<uint64_t>(dst, src, len);
    else if ((x & 3) == 0) block_copy_words<uint32_t>(dst, src, len);
    else if ((x & 1) == 0) block_copy_words<uint16_t>(dst, src, len);
    else block_copy_words<uint8_t>(dst, src, len);
}

}  // namespace rdc_amd
