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
//  * cross-GPU hand-off: write-through (sc0 sc1) payload stores into the
//    peer's scratch -> every wave's vmcnt(0) -> barrier -> one lane: relaxed
//    system-scope flag store (plus a system-scope release fence when the
//    scratch is not uncached).  Consumer: one lane per flag polls
//    relaxed/system, barrier, loads of its own uncached scratch (an acquire
//    fence when it is not uncached) (MI355X_MICROARCH.md "Workgroup dispatch
//    ... visibility"; cdna_hip_programming.md G16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

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

// 8-bit integers, four lanes per dword without unpacking (the generic loop
// spends ~12 VALU ops and a register per byte: the int8 / uint8 one-shot
// needed 256 VGPRs and ran one wave per SIMD).  Sum wraps like the
// reference's `dst += src` on a byte: low 7 bits added without carry-out,
// top bit by XOR.  Max / Min: even and odd bytes as 16-bit lanes through
// v_pk_max_u16 / v_pk_min_u16; signed bytes compare as unsigned after
// flipping their sign bits.
namespace swar8 {
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) {
    return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ ((a ^ b) & 0x80808080u);
}
template <bool MAX>
__device__ __forceinline__ uint32_t pick_u(uint32_t a, uint32_t b) {
    const u16x2 ae = __builtin_bit_cast(u16x2, a & 0x00ff00ffu), be = __builtin_bit_cast(u16x2, b & 0x00ff00ffu);
    const u16x2 ao = __builtin_bit_cast(u16x2, (a >> 8) & 0x00ff00ffu), bo = __builtin_bit_cast(u16x2, (b >> 8) & 0x00ff00ffu);
    const u16x2 e = MAX ? __builtin_elementwise_max(ae, be) : __builtin_elementwise_min(ae, be);
    const u16x2 o = MAX ? __builtin_elementwise_max(ao, bo) : __builtin_elementwise_min(ao, bo);
    return __builtin_bit_cast(uint32_t, e) | (__builtin_bit_cast(uint32_t, o) << 8);
}
template <int OP, bool SIGNED>
__device__ __forceinline__ v4u reduce(v4u d, v4u s) {
    constexpr uint32_t flip = SIGNED ? 0x80808080u : 0u;
    v4u out;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (OP == RDC_OP_SUM) out[k] = add(d[k], s[k]);
        else if (OP == RDC_OP_BITOR) out[k] = d[k] | s[k];
        else out[k] = pick_u<OP == RDC_OP_MAX>(d[k] ^ flip, s[k] ^ flip) ^ flip;
    }
    return out;
}
}  // namespace swar8
template <>
__device__ __forceinline__ v4u reduce16<RDC_OP_SUM, uint8_t>(v4u d, v4u s) { return swar8::reduce<RDC_OP_SUM, false>(d, s); }
template <>
__device__ __forceinline__ v4u reduce16<RDC_OP_SUM, int8_t>(v4u d, v4u s) { return swar8::reduce<RDC_OP_SUM, true>(d, s); }
template <>
__device__ __forceinline__ v4u reduce16<RDC_OP_BITOR, uint8_t>(v4u d, v4u s) { return swar8::reduce<RDC_OP_BITOR, false>(d, s); }
template <>
__device__ __forceinline__ v4u reduce16<RDC_OP_BITOR, int8_t>(v4u d, v4u s) { return swar8::reduce<RDC_OP_BITOR, true>(d, s); }
template <>
__device__ __forceinline__ v4u reduce16<RDC_OP_MAX, uint8_t>(v4u d, v4u s) { return swar8::reduce<RDC_OP_MAX, false>(d, s); }
template <>
__device__ __forceinline__ v4u reduce16<RDC_OP_MAX, int8_t>(v4u d, v4u s) { return swar8::reduce<RDC_OP_MAX, true>(d, s); }
template <>
__device__ __forceinline__ v4u reduce16<RDC_OP_MIN, uint8_t>(v4u d, v4u s) { return swar8::reduce<RDC_OP_MIN, false>(d, s); }
template <>
__device__ __forceinline__ v4u reduce16<RDC_OP_MIN, int8_t>(v4u d, v4u s) { return swar8::reduce<RDC_OP_MIN, true>(d, s); }

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

// Write-through stores for bytes a PEER reads (its IPC-mapped scratch, over
// xGMI on a multi-GPU node).  `sc0 sc1` (system scope) stores leave no copy in
// this XCD's L2, so once the storing wave's vmcnt has drained they are at the
// target's memory whatever memory type the IPC import was mapped with (MTYPE
// UC if the driver carries the exporter's uncached flag over, NC — L2-cached,
// written back only by a system release — if it does not).  Plain or `nt`
// stores would depend on that mapping (MI355X_MICROARCH.md visibility table:
// `nt` is not write-through).  16-B form: buffer store with aux = sc0|sc1 from
// a wave-uniform base (cdna_hip_programming.md T8/T20); narrow form: relaxed
// system-scope atomic stores (global_store_{byte,short,dword,dwordx2} sc0 sc1).
constexpr int kWtAux = 1 | 16;  // CPol SC0 | SC1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
    const uint64_t b = (uint64_t)(uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, 0xffffffffu, 0x00020000);
}
// 16 bytes at base + off (off < 4 GiB; base wave-uniform)
__device__ __forceinline__ void st16_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, v4u v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kWtAux);
}
template <typename W>
__device__ __forceinline__ void st_wt(W* p, W v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// one element of type T (any 1/2/4/8-byte type) written through
template <typename T>
__device__ __forceinline__ void st_elem_wt(void* p, T v) {
    typedef typename std::conditional<sizeof(T) == 1, uint8_t,
            typename std::conditional<sizeof(T) == 2, uint16_t,
            typename std::conditional<sizeof(T) == 4, uint32_t, uint64_t>::type>::type>::type W;
    st_wt(reinterpret_cast<W*>(p), __builtin_bit_cast(W, v));
}

// Where a block_copy writes: this GPU's own memory (user buffers, local
// slots: streaming `nt` stores) or a peer's scratch (write-through, above).
enum { kDstLocal = 0, kDstPeer = 1 };

// System-scope loads for bytes READ FROM a peer's scratch (pull-mode mesh):
// `sc0 sc1` loads are coherent at system scope whatever memory type the
// driver gave the IPC import, so a line of the peer's memory cached in this
// XCD's L2 by an earlier launch (an NC import) is not returned stale — the
// load-side twin of the write-through stores above.  16-B form through a
// wave-uniform descriptor, narrow form as relaxed system-scope atomic loads.
__device__ __forceinline__ v4u ld16_sys(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kWtAux);
}
template <typename W>
__device__ __forceinline__ W ld_sys(const W* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// one element of type T (any 1/2/4/8-byte type) read at system scope
template <typename T>
__device__ __forceinline__ T ld_elem_sys(const void* p) {
    typedef typename std::conditional<sizeof(T) == 1, uint8_t,
            typename std::conditional<sizeof(T) == 2, uint16_t,
            typename std::conditional<sizeof(T) == 4, uint32_t, uint64_t>::type>::type>::type W;
    return __builtin_bit_cast(T, ld_sys(reinterpret_cast<const W*>(p)));
}

// ------------------------------------------------------------- hand-off ----
// Hand-off flags are 64-bit words holding a launch's sequence number:
//   seq = (counter << kTagBits) | tag
// counter: the channel's launch count (every communicator sharing a channel
// draws from one counter, 56 bits: it never wraps in practice, so a slot no
// launch has written yet (0) or one idle for any number of launches never
// looks "reached"); tag: the launching communicator's tag on that channel.
// Hand-off flags carry the whole word, so a rank waiting for launch k of
// communicator X that finds launch k of communicator Y — ranks that issued two
// communicators' collectives in different orders — fails with RDC_KERR_ORDER
// instead of folding unrelated buffers.  "Done" words (a peer finished launch
// k-1, whichever communicator issued it) compare the counter only.
constexpr uint32_t kTagBits = 8;
constexpr uint64_t kTagMask = (1ull << kTagBits) - 1ull;
__device__ __forceinline__ uint64_t flag_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void flag_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t seq_counter(uint64_t seq) { return seq >> kTagBits; }
// counter of v >= counter of seq (modulo 2^56)
__device__ __forceinline__ bool seq_reached(uint64_t v, uint64_t seq) {
    return (int64_t)((seq_counter(v) - seq_counter(seq)) << kTagBits) >= 0;
}
__device__ __forceinline__ bool same_tag(uint64_t v, uint64_t seq) { return ((v ^ seq) & kTagMask) == 0; }
// the previous launch's number (counter - 1, same tag; compared untagged)
__device__ __forceinline__ uint64_t seq_prev(uint64_t seq) { return seq - (1ull << kTagBits); }

// Called by EVERY thread of the block after its payload stores.  Lanes
// 0..nflags-1 of wave 0 then store flags[i] = seq.
// Every hand-off payload lives in the peers' scratch slots and is stored
// write-through (st16_wt / block_copy<kDstPeer>: sc0 sc1), so every storing
// wave's `s_waitcnt vmcnt(0)` (before the barrier) means it has been
// performed at the owner's memory: the write-through + drained-flag form of
// MI355X_MICROARCH.md ("Valid forms", R1) at system scope.  When the scratch
// is uncached (MTYPE UC, hipDeviceMallocUncached: `uc`) the owner's loads
// never hit a stale line either, and the system-scope release fence would
// only add an L2 write-back (buffer_wbl2 sc0 sc1, 1.7-6.5 us per call) of
// cached lines no peer reads, so it is issued only for fine- / coarse-grained
// scratch (alloc fallbacks).
// verify (RDC_VERIFY_PUBLISH, debug): each storing lane reads its flag back
// through the same mapping until it sees seq (bounded), and counts in
// verify[0] the stores it never saw, recording the last such flag address in
// verify[2..3] — does a store the writer made stay invisible to the writer too?
__device__ __forceinline__ void verify_flag(uint64_t* f, uint64_t seq, uint32_t* verify) {
    for (int i = 0; i < (1 << 14); ++i) {
        if (seq_counter(flag_load(f)) == seq_counter(seq)) return;
        __builtin_amdgcn_s_sleep(2);
    }
    __hip_atomic_fetch_add(verify, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<uint64_t*>(verify + 2), (uint64_t)(uintptr_t)f, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void block_publish(uint64_t* const* flags, int nflags, uint64_t seq, int uc,
                                              uint32_t* verify = nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < (unsigned)nflags) {
        if (!uc) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        flag_store(flags[threadIdx.x], seq);
        if (verify) verify_flag(flags[threadIdx.x], seq, verify);
    }
}

__device__ __forceinline__ void block_publish1(uint64_t* flag, uint64_t seq, int uc) {
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
    int poll_rmw = 0;       // RDC_POLL_RMW (debug): poll with a system-scope atomic add of 0
};

// Block-wide wait until every flags[i] (i < nflags <= 64) reached seq.  Wave 0
// polls (one lane per flag), sleeping between polls; the other waves park at
// the barrier.  Returns false (uniformly) on timeout or if another block of
// this launch already aborted.  tagged (hand-off flags of this launch): a
// flag that reached the counter with another communicator's tag is an order
// violation (RDC_KERR_ORDER, immediate); untagged (done words): the counter only.  With cached scratch the matching lane then
// runs a system-scope acquire (L2 / L1 invalidate) so the block's plain loads
// of the handed-off bytes cannot hit stale lines; uncached scratch (`uc`) is
// never held in any GPU cache, so its loads after the matched poll read
// memory and need no invalidate (MI355X_MICROARCH.md: an acquire is ≈1.7 us).
__device__ __forceinline__ bool block_wait(uint64_t* const* flags, int nflags, uint64_t seq,
                                           const Abort& ab, uint32_t code, int uc, bool tagged = true) {
    __shared__ int s_ok;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        bool mine = lane >= nflags;
        bool ok = true;
        bool wrong = false;  // this lane's flag reached the counter with another tag
        uint32_t spins = 0;
        uint64_t seen = 0;   // this lane's last flag value
        while (true) {
            if (!mine) {
                const uint64_t v = ab.poll_rmw ? __hip_atomic_fetch_add(flags[lane], (uint64_t)0, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_SYSTEM)
                                               : flag_load(flags[lane]);
                seen = v;
                if (seq_reached(v, seq)) {
                    if (!tagged || same_tag(v, seq)) mine = true;
                    else wrong = true;
                }
            }
            if (__all(mine)) break;
            if (__any(wrong)) {
                code = RDC_KERR_ORDER;
                ok = false;
                break;
            }
            if ((++spins & 63) == 0) {
                bool dead = wall_clock64() > ab.deadline ||
                            __hip_atomic_load(ab.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                if (__any(dead)) { ok = false; break; }
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (!ok) {
            // the first wait to give up records what it waited for (err words
            // 64..71: claim, -, seq, flag value, flag address), before the
            // error word tells the other blocks to give up
            const uint64_t open = __ballot(!mine);
            if (open != 0 && lane == (int)__builtin_ctzll(open)) {
                uint32_t expected = 0;
                if (__hip_atomic_compare_exchange_strong(ab.err + 64, &expected, 1u, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    uint64_t* d = reinterpret_cast<uint64_t*>(ab.err + 66);
                    __hip_atomic_store(d, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(d + 1, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(d + 2, (uint64_t)(uintptr_t)flags[lane], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    // the same flag read five ways once more (err words 96..107):
                    // a relaxed system-scope load, an atomic add of 0 at system
                    // scope, a load after a system-scope acquire (L1 / L2
                    // invalidate), a non-temporal load, and this wave's XCC —
                    // which view still shows the old value after the wait gave up
                    uint64_t* f = flags[lane];
                    const uint64_t v1 = flag_load(f);
                    const uint64_t v2 = __hip_atomic_fetch_add(f, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                    const uint64_t v3 = flag_load(f);
                    const uint64_t v4 = __builtin_nontemporal_load(f);
                    const uint64_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf;
                    uint64_t* pr = reinterpret_cast<uint64_t*>(ab.err + 96);
                    __hip_atomic_store(pr, v1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(pr + 1, v2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(pr + 2, v3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(pr + 3, v4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(pr + 4, xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
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
//
// Where a block_copy reads: this rank's own bytes (user buffers, kSrcLocal:
// streaming `nt` loads) or bytes another rank handed off through scratch
// (kSrcHandoff: `sc0 sc1` loads, ld16_sys / ld_sys) — every load of a
// handed-off byte is a system-scope load, so the consumer side of every
// hand-off is the "sc0 sc1 stores and loads both sides" form of
// MI355X_MICROARCH.md ("Valid forms") whatever memory type backs the scratch
// or its IPC import.
enum { kSrcLocal = 0, kSrcHandoff = 1 };

template <int DST, typename W>
__device__ __forceinline__ void put_word(W* p, W v) {
    if (DST == kDstPeer) st_wt(p, v);
    else *p = v;
}
template <int SRC, typename W>
__device__ __forceinline__ W get_word(const W* p) {
    if (SRC == kSrcHandoff) return ld_sys(p);
    return *p;
}

// dst[i] = src[i], dst and src congruent mod 16.  The 16-B body walks windows
// of U x blockDim vectors; the window base is wave-uniform, so a peer
// destination or a handed-off source gets one buffer descriptor per window
// (offsets < 4 GiB).
template <int DST, int SRC>
__device__ __forceinline__ void block_copy_vec(char* __restrict__ dst, const char* __restrict__ src,
                                               uint64_t len) {
    const uint64_t mis = (uint64_t)(uintptr_t)src & 15;
    uint64_t head = mis ? (16 - mis) : 0;
    if (head > len) head = len;
    const uint64_t nvec = (len - head) >> 4;
    const uint64_t tail_start = head + (nvec << 4);
    const unsigned tid = threadIdx.x;
    if (tid < head) put_word<DST, char>(dst + tid, (char)get_word<SRC, uint8_t>(reinterpret_cast<const uint8_t*>(src) + tid));
    if (tid < len - tail_start)
        put_word<DST, char>(dst + tail_start + tid,
                            (char)get_word<SRC, uint8_t>(reinterpret_cast<const uint8_t*>(src) + tail_start + tid));
    const v4u* s = reinterpret_cast<const v4u*>(src + head);
    v4u* d = reinterpret_cast<v4u*>(dst + head);
    constexpr int U = 8;  // 32 KiB in flight per 256-thread block
    const uint64_t step = (uint64_t)blockDim.x;
    for (uint64_t ib = 0; ib < nvec; ib += U * step) {
        const uint64_t i = ib + tid;
        const __amdgpu_buffer_rsrc_t rsrc_s = wt_rsrc(SRC == kSrcHandoff ? s + ib : s);  // dead for kSrcLocal
        auto load = [&](int u) -> v4u {
            if (SRC == kSrcHandoff) return ld16_sys(rsrc_s, (uint32_t)((tid + u * step) * 16));
            return ld16_nt(s + i + u * step);
        };
        if (ib + U * step <= nvec) {
            v4u v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = load(u);
            if (DST == kDstPeer) {
                const __amdgpu_buffer_rsrc_t rs = wt_rsrc(d + ib);
#pragma unroll
                for (int u = 0; u < U; ++u) st16_wt(rs, (uint32_t)((tid + u * step) * 16), v[u]);
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) st16_nt(d + i + u * step, v[u]);
            }
        } else {
            const __amdgpu_buffer_rsrc_t rs = wt_rsrc(d + ib);
            for (int u = 0; u < U; ++u) {
                if (i + u * step >= nvec) break;
                const v4u v = load(u);
                if (DST == kDstPeer) st16_wt(rs, (uint32_t)((tid + u * step) * 16), v);
                else st16_nt(d + i + u * step, v);
            }
        }
    }
}

template <int DST, int SRC, typename W>
__device__ __forceinline__ void block_copy_words(char* dst, const char* src, uint64_t len) {
    const uint64_t mis = (uint64_t)(uintptr_t)src & (sizeof(W) - 1);
    uint64_t head = mis ? sizeof(W) - mis : 0;
    if (head > len) head = len;
    const uint64_t nw = (len - head) / sizeof(W);
    const uint64_t tail_start = head + nw * sizeof(W);
    const unsigned tid = threadIdx.x;
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(src);
    if (tid < head) put_word<DST, char>(dst + tid, (char)get_word<SRC, uint8_t>(sb + tid));
    if (tid < len - tail_start) put_word<DST, char>(dst + tail_start + tid, (char)get_word<SRC, uint8_t>(sb + tail_start + tid));
    const W* s = reinterpret_cast<const W*>(src + head);
    W* d = reinterpret_cast<W*>(dst + head);
    for (uint64_t i = tid; i < nw; i += blockDim.x) put_word<DST, W>(d + i, get_word<SRC, W>(s + i));
}

// DST: kDstLocal (this GPU's memory) or kDstPeer (a peer's IPC-mapped scratch);
// SRC: kSrcLocal (this rank's bytes) or kSrcHandoff (bytes a peer handed off)
template <int DST, int SRC = kSrcLocal>
__device__ __forceinline__ void block_copy(char* __restrict__ dst, const char* __restrict__ src, uint64_t len) {
    const uintptr_t x = ((uintptr_t)dst ^ (uintptr_t)src) & 15;
    if (x == 0) block_copy_vec<DST, SRC>(dst, src, len);
    else if ((x & 7) == 0) block_copy_words<DST, SRC, uint64_t>(dst, src, len);
    else if ((x & 3) == 0) block_copy_words<DST, SRC, uint32_t>(dst, src, len);
    else if ((x & 1) == 0) block_copy_words<DST, SRC, uint16_t>(dst, src, len);
    else block_copy_words<DST, SRC, uint8_t>(dst, src, len);
}

// dst (this GPU's memory) = src (a PEER's scratch or this rank's own scratch
// written by a peer), every load at system scope: landing handed-off bytes.
__device__ __forceinline__ void block_copy_pull(char* __restrict__ dst, const char* __restrict__ src, uint64_t len) {
    block_copy<kDstLocal, kSrcHandoff>(dst, src, len);
}

// ------------------------------------------------------------ poison mode ----
// RDC_POISON_SCRATCH=1 (CollArgs::poison): after its last read of a scratch
// range in a launch, the consumer overwrites it with 0xFF bytes (write-through:
// the range may be a peer's), before the signal that lets the producer reuse
// it.  A read of the range before the producer's next publish then folds or
// lands NaN / all-ones words instead of a plausible older value (DESIGN.md
// §4.2, debug mode; the tests run with it on).
__device__ __forceinline__ void block_poison(char* p, uint64_t len) {
    const uint64_t mis = (uint64_t)(uintptr_t)p & 15;
    uint64_t head = mis ? 16 - mis : 0;
    if (head > len) head = len;
    const uint64_t nvec = (len - head) >> 4;
    const uint64_t tail = head + (nvec << 4);
    const unsigned tid = threadIdx.x;
    if (tid < head) st_wt<uint8_t>(reinterpret_cast<uint8_t*>(p) + tid, 0xff);
    if (tid < len - tail) st_wt<uint8_t>(reinterpret_cast<uint8_t*>(p) + tail + tid, 0xff);
    const v4u ones = {~0u, ~0u, ~0u, ~0u};
    const uint64_t step = (uint64_t)blockDim.x;
    constexpr int U = 8;
    for (uint64_t ib = 0; ib < nvec; ib += U * step) {
        const __amdgpu_buffer_rsrc_t rs = wt_rsrc(p + head + ib * 16);
        for (int u = 0; u < U; ++u) {
            if (ib + tid + u * step >= nvec) break;
            st16_wt(rs, (uint32_t)((tid + u * step) * 16), ones);
        }
    }
}

}  // namespace rdc_amd
