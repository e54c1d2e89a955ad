// MI355X (gfx950) kernels of the rdc allreduce path — device templates shared by
// the per-operator translation units rdc_kernels_{max,min,sum,bitor}.hip.
//
//   k_reduce   : op::Reducer<OP,DType> on device (include/core/mpi.h:113-120):
//                dst[i] = OP::Reduce(dst[i], src[i]) — 16-B coalesced lanes,
//                4 independent 16-B loads per operand in flight per lane.
//   k_mesh     : allreduce over all links.  Rank r owns chunk r of
//                utils::Split(0,count,n) (include/utils/utils.h:59-70);
//                scatter blocks push every other chunk's tiles to their
//                owners' scratch; reduce blocks fold the n contributions in
//                the reference ring's order (communicator_collective.cc:
//                115-182 => s = x[r-1]; s = OP(x[r-2], s) ... s = OP(x[r], s))
//                and push the result to every peer; gather blocks land the
//                peers' results in the user buffer.  Bit-identical to the ring.
//   k_ring     : the reference schedule itself — TryReduceScatterRing
//                (:115-182) + TryAllgatherRing (:79-114): n-1 steps each,
//                send to prev=(r-1)%n, receive from next, pipelined per tile.
//   k_bcast    : root pushes every tile to all peers (src/comm/
//                communicator_collective.cc:44-69 semantics, correct for n>=4).
//   k_fill     : synthetic inputs, bit-identical to oracle rdc_oracle_fill.
#pragma once
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <type_traits>

#include "rdc_device.h"
#include "rdc_kernels.h"

namespace rdc_amd {

constexpr int kBlock = 256;

// flag number `idx` (row * max_tiles + tile, or a done word) of rank p's flag
// array: RDC_FLAG_STRIDE words apart, each flag in a line of its own
__device__ __forceinline__ uint64_t* flag_word(const CollArgs& a, int p, uint64_t idx) {
    return a.flags[p] + idx * RDC_FLAG_STRIDE;
}
// rank `owner`'s flag word that rank `writer` sets when it finished a launch
__device__ __forceinline__ uint64_t* done_word(const CollArgs& a, int owner, int writer) {
    return flag_word(a, owner, (uint64_t)(2 * a.n) * a.max_tiles + writer);
}

// ====================================================== launch sequencing ===
// Launch sequence numbers live on the device, so a captured hipGraph replays
// correctly: every block reads the communicator's launch counter when it
// starts (seq = launches completed + 1, identical on every rank because all
// ranks issue the same collectives), and the launch's last block advances it.
// seq = (counter << kTagBits) | the launching communicator's tag
// (rdc_device.h).
// Block start: thread 0 reads the launch counter and the channel's error word
// together (one round trip instead of two), the block shares them through LDS.
// A channel that failed (a peer missed a hand-off, an order violation) is
// unusable: later launches move nothing — in particular they push nothing
// into peers' scratch, where a peer still inside the failed launch would take
// a later launch's flags (>= its seq) for its own — and only advance the
// counters.  The host raises the recorded error at its next check.
// Returns true when the channel failed; *seq = this launch's sequence word.
__device__ __forceinline__ bool launch_begin(const CollArgs& a, uint64_t* seq) {
    __shared__ uint64_t s_done;
    __shared__ int s_failed;
    if (threadIdx.x == 0) {
        const uint64_t done = __hip_atomic_load(a.launch_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t e = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_done = done;
        s_failed = e != 0;
        if (a.tlog) {  // RDC_LAUNCH_TIMES: when this launch's blocks started (ticks only grow: max needs no reset)
            unsigned long long* ent = reinterpret_cast<unsigned long long*>(a.tlog + ((done + 1ull) & 63ull) * 4);
            const unsigned long long t = wall_clock64();
            if (blockIdx.x == 0) {
                __hip_atomic_store(ent, (unsigned long long)(done + 1ull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(ent + 1, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __hip_atomic_fetch_max(ent + 2, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (a.seq_check) {
            // RDC_SEQ_CHECK: every block of one launch must read the same
            // launch number.  The first block to start claims the launch's
            // check word with its number (the launch's last block clears it
            // in launch_done, after every block has started); a block that
            // finds another number there records both (err words 72..).
            // Device-side only, so graph replays are checked like eager launches.
            unsigned long long want = 0;
            unsigned long long* chk = reinterpret_cast<unsigned long long*>(a.err + 80);
            if (!__hip_atomic_compare_exchange_strong(chk, &want, (unsigned long long)(done + 1ull), __ATOMIC_RELAXED,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &&
                want != done + 1ull) {
                uint32_t expected = 0;
                if (__hip_atomic_compare_exchange_strong(a.err + 72, &expected, 1u, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    uint64_t* d = reinterpret_cast<uint64_t*>(a.err + 74);
                    __hip_atomic_store(d, done + 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(d + 1, (uint64_t)want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(d + 2, (uint64_t)blockIdx.x | ((uint64_t)gridDim.x << 32), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
                expected = 0;
                __hip_atomic_compare_exchange_strong(a.err, &expected, (uint32_t)RDC_KERR_SEQ, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    __syncthreads();
    *seq = ((s_done + 1ull) << kTagBits) | ((uint64_t)a.tag & kTagMask);
    const bool f = s_failed != 0;
    __syncthreads();
    return f;
}
__device__ __forceinline__ uint32_t prev_kind(const CollArgs& a) {
    return __hip_atomic_load(a.launch_kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Block-wide: wait until each listed peer finished launch seq-1 (its done word
// in MY flag array).  Used before writing into peers' scratch when no data
// dependency already orders the write.
__device__ __forceinline__ bool gate_on_peers(const CollArgs& a, uint64_t seq, int first, int count,
                                              const Abort& ab, uint32_t code) {
    __shared__ uint64_t* s_gate[RDC_MAX_RANKS];
    if (threadIdx.x < (unsigned)count) s_gate[threadIdx.x] = done_word(a, a.rank, (first + threadIdx.x) % a.n);
    __syncthreads();
    return block_wait(s_gate, count, seq_prev(seq), ab, code, a.uc, false);
}


// =============================================================== reduce ===
template <int OP, typename T>
__device__ __forceinline__ void reduce_elems(char* dst, const char* src, uint64_t nelem, uint64_t first,
                                             uint64_t stride) {
    T* d = reinterpret_cast<T*>(dst);
    const T* s = reinterpret_cast<const T*>(src);
    for (uint64_t i = first; i < nelem; i += stride) d[i] = OpF<OP>::apply(d[i], s[i]);
}

// dst and src congruent mod 16; nbytes a multiple of sizeof(T).  Grid-stride
// walk in which the whole grid sweeps one window of grid x 256 x U x 16 B
// per step; at one 256-thread block per CU and U = 2 that window is 2 MiB
// per stream and the kernel streams 6.44 TB/s (3 x S) vs 5.9 TB/s for
// per-block contiguous spans (tools/bench_reduce.hip sweep, MI355X, 1 GiB).
// Non-temporal loads and stores: every byte is touched once.
template <int OP, typename T, int U>
__global__ __launch_bounds__(kBlock) void k_reduce(char* __restrict__ dst, const char* __restrict__ src,
                                                   uint64_t nbytes) {
    const uint64_t mis = (uint64_t)(uintptr_t)dst & 15;
    uint64_t head = mis ? 16 - mis : 0;
    if (head > nbytes) head = nbytes;
    const uint64_t nvec = (nbytes - head) >> 4;
    const uint64_t tail = head + (nvec << 4);
    if (blockIdx.x == 0) {
        reduce_elems<OP, T>(dst, src, head / sizeof(T), threadIdx.x, kBlock);
        reduce_elems<OP, T>(dst + tail, src + tail, (nbytes - tail) / sizeof(T), threadIdx.x, kBlock);
    }
    v4u* d = reinterpret_cast<v4u*>(dst + head);
    const v4u* s = reinterpret_cast<const v4u*>(src + head);
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        v4u a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ld16_nt(d + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = ld16_nt(s + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) st16_nt(d + i + u * stride, reduce16<OP, T>(a[u], b[u]));
    }
    for (; i < nvec; i += stride) st16_nt(d + i, reduce16<OP, T>(ld16_nt(d + i), ld16_nt(s + i)));
}

// dst and src NOT congruent mod 16: element-wise grid-stride.
template <int OP, typename T>
__global__ __launch_bounds__(kBlock) void k_reduce_unaligned(char* dst, const char* src, uint64_t nelem) {
    reduce_elems<OP, T>(dst, src, nelem, (uint64_t)blockIdx.x * kBlock + threadIdx.x,
                        (uint64_t)gridDim.x * kBlock);
}

// ======================================================= mesh allreduce ===
// Fold one tile of chunk r: out = ring-order reduction of the n ranks'
// tile, written to the local user buffer and to every peer's allgather slot.
// one element at byte offset e of the tile: ring-order fold of the n ranks'
// values, stored to the local user buffer and every peer's allgather slot
template <int OP, typename T>
__device__ __forceinline__ void mesh_fold_elem(const CollArgs& a, char* own, const char* slot0, uint64_t soff,
                                               uint64_t e) {
    const int n = a.n, r = a.rank, f = a.fold[r];  // the ring order of chunk f
    // own values are this rank's; every other rank's came through its RS slot
    auto val = [&](int q) -> T {
        return q == r ? *reinterpret_cast<const T*>(own + e) : ld_elem_sys<T>(slot0 + q * a.slot_bytes + e);
    };
    T acc = val((f - 1 + n) % n);
    for (int k = 2; k <= n; ++k) acc = OpF<OP>::apply(val((f - k + n) % n), acc);
    *reinterpret_cast<T*>(own + e) = acc;
    for (int p = 0; p < n; ++p)
        if (p != r) st_elem_wt<T>(a.ag[p] + soff + e, acc);
}

// Fold `tlen` bytes: own (this rank's values, overwritten with the result),
// slot0 (rank q's copy at slot0 + q*slot_bytes) in ring order; the result also
// goes to every peer's allgather region at byte offset soff.
template <int OP, typename T, int NMAX>
__device__ __forceinline__ void mesh_reduce_range(const CollArgs& a, char* own, const char* slot0, uint64_t soff, uint64_t tlen) {
    const int n = a.n, r = a.rank, f = a.fold[r];
    const unsigned tid = threadIdx.x;
    if ((((uintptr_t)own ^ (uintptr_t)slot0) & 15) != 0) {
        // this rank's buffer is not 16-B aligned: exact, element by element
        for (uint64_t e = (uint64_t)tid * sizeof(T); e < tlen; e += (uint64_t)kBlock * sizeof(T))
            mesh_fold_elem<OP, T>(a, own, slot0, soff, e);
        return;
    }
    const uint64_t mis16 = (uint64_t)(uintptr_t)own & 15;
    uint64_t head = mis16 ? 16 - mis16 : 0;
    if (head > tlen) head = tlen;
    const uint64_t nvec = (tlen - head) >> 4;
    const uint64_t tail = head + (nvec << 4);
    {   // element-wise head / tail (< 16 bytes each)
        const uint64_t nh = head / sizeof(T), nt = (tlen - tail) / sizeof(T);
        if (tid < nh) mesh_fold_elem<OP, T>(a, own, slot0, soff, tid * sizeof(T));
        else if (tid >= 64 && tid - 64 < nt) mesh_fold_elem<OP, T>(a, own, slot0, soff, tail + (tid - 64) * sizeof(T));
    }
    // All n contributions of U positions are loaded before folding (NMAX x U
    // 16-B loads in flight per lane); folding one rank at a time inside a
    // runtime loop would leave the lane latency-bound at n = 8.
    constexpr int U = NMAX <= 8 ? 2 : 1;
    const uint64_t stride = kBlock;
    // peers' allgather regions at this range: one write-through descriptor
    // each per window of U x kBlock vectors (wave-uniform bases)
    __amdgpu_buffer_rsrc_t ag_rs[NMAX];
    for (uint64_t ib = 0; ib < nvec; ib += U * stride) {
        const uint64_t i = ib + tid;
#pragma unroll
        for (int p = 0; p < NMAX; ++p)
            if (p < n && p != r) ag_rs[p] = wt_rsrc(a.ag[p] + soff + head + ib * 16);
        v4u v[U][NMAX];
        bool live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) live[u] = i + u * stride < nvec;
#pragma unroll
        for (int k = 1; k <= NMAX; ++k) {
            if (k <= n) {  // (a `break` here stops full unrolling: v would live in scratch)
                const int q = (f - k + n) % n;  // k-th value in ring order: x[f-1], x[f-2], ..., x[f]
                if (q == r) {
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (live[u]) v[u][k - 1] = ld16_nt(own + head + (i + u * stride) * 16);
                } else {  // rank q's handed-off copy: system-scope loads (rdc_device.h kSrcHandoff)
                    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(slot0 + q * a.slot_bytes + head + ib * 16);
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (live[u]) v[u][k - 1] = ld16_sys(rs, (uint32_t)((tid + u * stride) * 16));
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!live[u]) continue;
            v4u acc = v[u][0];
#pragma unroll
            for (int k = 2; k <= NMAX; ++k)
                if (k <= n) acc = reduce16<OP, T>(v[u][k - 1], acc);
            const uint64_t b = head + (i + u * stride) * 16;
            st16(own + b, acc);
#pragma unroll
            for (int p = 0; p < NMAX; ++p)
                if (p < n && p != r) st16_wt(ag_rs[p], (uint32_t)((tid + u * stride) * 16), acc);
        }
    }
}

// Fold one tile of chunk r: out = ring-order reduction of the n ranks'
// tile, written to the local user buffer and to every peer's allgather slot.
template <int OP, typename T, int NMAX>
__device__ __forceinline__ void mesh_reduce_tile(const CollArgs& a, int t, uint64_t tlen) {
    const int r = a.rank;
    const uint64_t toff = (uint64_t)t * a.tile_bytes;
    mesh_reduce_range<OP, T, NMAX>(a, a.user + a.off[r] + toff, a.rs[r] + a.mis[r] + toff,
                                   (uint64_t)r * a.slot_bytes + a.mis[r] + toff, tlen);
}

// ---- coalesced mesh: packed chunk-major offsets -> user buffers.  The unit
// table (rdc_plan.h PlanCoalesced) is sorted by packed offset; a tile covers a
// run of units (gaps between segments are padding nobody reads).  Every role
// works on the unit pieces of its tile directly, so no staging image exists.
__device__ __forceinline__ int unit_first(const PackUnit* u, int nunits, uint64_t pos) {
    __shared__ int s_first;
    if (threadIdx.x < 64) {
        // first unit whose range ends after pos: a 64-ary search by wave 0
        // (each pass one load per lane, all in flight together) — 2 passes
        // for cfg5's 1024 buckets instead of 10 dependent loads by one lane.
        // ends(i) <= pos is monotone in i: the lanes that see it true are a
        // prefix, and the answer lies after the last of them.
        const int lane = threadIdx.x;
        int lo = 0, hi = nunits;  // answer in [lo, hi]
        while (lo < hi) {
            const int step = (hi - lo + 63) >> 6;
            const int idx = lo + lane * step;
            const bool before = idx < hi && u[idx].packed + u[idx].len <= pos;
            const int k = __popcll(__ballot(before));  // lanes 0..k-1 are before pos
            if (k == 0) {
                hi = lo;  // u[lo] already ends after pos
            } else {
                const int nlo = lo + (k - 1) * step + 1;
                const int nhi = lo + k * step;
                lo = nlo;
                if (nhi < hi) hi = nhi;
            }
        }
        if (lane == 0) s_first = lo;
    }
    __syncthreads();
    const int f = s_first;
    __syncthreads();
    return f;
}

// f(user pointer, packed offset, bytes) for every unit piece of packed [p0, p1)
// (first: the first unit of the range when the caller already knows it)
template <typename F>
__device__ __forceinline__ void for_unit_pieces(const CollArgs& a, uint64_t p0, uint64_t p1, F&& f, int first = -1) {
    const PackUnit* u = static_cast<const PackUnit*>(a.units);
    for (int i = first >= 0 ? first : unit_first(u, a.nunits, p0); i < a.nunits; ++i) {
        const uint64_t up = u[i].packed, ul = u[i].len;
        if (up >= p1) break;
        const uint64_t lo = up > p0 ? up : p0;
        const uint64_t hi = up + ul < p1 ? up + ul : p1;
        if (lo < hi) f(reinterpret_cast<char*>(u[i].buf) + (lo - up), lo, hi - lo);
    }
}

template <int OP, typename T, int NMAX>
__device__ __forceinline__ void mesh_body(const CollArgs& a, uint64_t seq) {
    const int n = a.n, r = a.rank;
    Abort ab{a.err, wall_clock64() + a.timeout_ticks, a.poll_rmw};
    int b = blockIdx.x;
    int tmax = 0;
    for (int c = 0; c < n; ++c) tmax = a.tiles[c] > tmax ? a.tiles[c] : tmax;
    __shared__ uint64_t* s_flags[RDC_MAX_RANKS];

    if (b < a.nb_scatter) {
        // ---- scatter: my copy of chunk c's tile t -> owner c's rs slot r
        const int items = (n - 1) * tmax;
        // after a one-shot launch the owners may still be reading their RS
        // slots (nothing in this launch orders that): wait for their done words
        if (b < items && prev_kind(a) == RDC_KIND_ONESHOT &&
            !gate_on_peers(a, seq, r + 1, n - 1, ab, RDC_KERR_TIMEOUT_RS))
            return;
        for (int it = b; it < items; it += a.nb_scatter) {
            const int t = it / (n - 1);
            const int c = (r + 1 + it % (n - 1)) % n;
            if (t >= a.tiles[c]) continue;
            const uint64_t toff = (uint64_t)t * a.tile_bytes;
            uint64_t tlen = a.len[c] - toff;
            if (tlen > a.tile_bytes) tlen = a.tile_bytes;
            char* dst = a.rs[c] + (uint64_t)r * a.slot_bytes + a.mis[c];
            if (a.units)
                for_unit_pieces(a, a.off[c] + toff, a.off[c] + toff + tlen, [&](char* usr, uint64_t p, uint64_t l) {
                    block_copy<kDstPeer>(dst + (p - a.off[c]), usr, l);
                });
            else
                block_copy<kDstPeer>(dst + toff, a.user + a.off[c] + toff, tlen);
            block_publish1(flag_word(a, c, (uint64_t)r * a.max_tiles + t), seq, a.uc);
        }
        return;
    }
    b -= a.nb_scatter;
    if (b < a.nb_reduce) {
        // ---- reduce: chunk r, tile t, once all n-1 contributions landed
        for (int t = b; t < a.tiles[r]; t += a.nb_reduce) {
            if (threadIdx.x < (unsigned)(n - 1)) {
                const int p = (r + 1 + threadIdx.x) % n;
                s_flags[threadIdx.x] = flag_word(a, r, (uint64_t)p * a.max_tiles + t);
            }
            __syncthreads();
            if (!block_wait(s_flags, n - 1, seq, ab, RDC_KERR_TIMEOUT_RS, a.uc)) return;
            const uint64_t toff = (uint64_t)t * a.tile_bytes;
            uint64_t tlen = a.len[r] - toff;
            if (tlen > a.tile_bytes) tlen = a.tile_bytes;
            if (a.units)
                for_unit_pieces(a, a.off[r] + toff, a.off[r] + toff + tlen, [&](char* usr, uint64_t p, uint64_t l) {
                    const uint64_t co = a.mis[r] + (p - a.off[r]);
                    mesh_reduce_range<OP, T, NMAX>(a, usr, a.rs[r] + co, (uint64_t)r * a.slot_bytes + co, l);
                });
            else
                mesh_reduce_tile<OP, T, NMAX>(a, t, tlen);
            if (a.poison) {  // every peer's copy of this tile was read: before the result's publish
                __syncthreads();
                for (int k = 1; k < n; ++k)
                    block_poison(a.rs[r] + (uint64_t)((r + k) % n) * a.slot_bytes + a.mis[r] + toff, tlen);
            }
            if (threadIdx.x < (unsigned)(n - 1)) {
                const int p = (r + 1 + threadIdx.x) % n;
                s_flags[threadIdx.x] = flag_word(a, p, (uint64_t)(n + r) * a.max_tiles + t);
            }
            block_publish(s_flags, n - 1, seq, a.uc);
            __syncthreads();
        }
        return;
    }
    b -= a.nb_reduce;
    // ---- gather: owner c's result tile t -> my user buffer
    const int items = (n - 1) * tmax;
    for (int it = b; it < items; it += a.nb_gather) {
        const int t = it / (n - 1);
        const int c = (r + 1 + it % (n - 1)) % n;
        if (t >= a.tiles[c]) continue;
        if (threadIdx.x == 0) s_flags[0] = flag_word(a, r, (uint64_t)(n + c) * a.max_tiles + t);
        __syncthreads();
        if (!block_wait(s_flags, 1, seq, ab, RDC_KERR_TIMEOUT_AG, a.uc)) return;
        const uint64_t toff = (uint64_t)t * a.tile_bytes;
        uint64_t tlen = a.len[c] - toff;
        if (tlen > a.tile_bytes) tlen = a.tile_bytes;
        char* src = a.ag[r] + (uint64_t)c * a.slot_bytes + a.mis[c];
        if (a.units)
            for_unit_pieces(a, a.off[c] + toff, a.off[c] + toff + tlen, [&](char* usr, uint64_t p, uint64_t l) {
                block_copy_pull(usr, src + (p - a.off[c]), l);
            });
        else
            block_copy_pull(a.user + a.off[c] + toff, src + toff, tlen);
        // owner c rewrites this slot only in its next launch, after this
        // rank's next scatter: after this kernel's end
        if (a.poison) {
            __syncthreads();
            block_poison(src + toff, tlen);
        }
    }
}

// ================================================== pull-mode mesh ===
// The same owner-computes exchange and fold order as k_mesh, moved by REMOTE
// LOADS instead of remote stores (algo RDC_ALGO_MESH_PULL, an autotune
// candidate beside push: which direction xGMI serves faster is measured, not
// assumed — bench.py's xgmi_probe times both):
//   stage  : every other chunk c's tile t -> MY OWN scratch, RS slot c
//            (local write-through stores), then owner c's flag (row r, t);
//   reduce : owner r loads its chunk's tile from every peer's RS slot r
//            (system-scope loads over the link), folds in the ring order of
//            chunk r, stores the user tile and MY AG slot r (local), then
//            every peer's flag (row n + r, t);
//   gather : tile t of chunk c loaded from owner c's AG slot c (remote).
// Every element still folds x[r-1], x[r-2], ..., x[r] — bit-identical to the
// ring.  Scratch reuse across launches needs no gate in either direction: a
// rank finishes a launch only after gathering every tile of every chunk,
// which each owner folds only after loading every staged tile of it, and an
// owner overwrites its AG slot for tile t only after folding the NEXT
// launch's tile t, which needs every peer's next-launch stage.
template <int OP, typename T, int NMAX>
__device__ __forceinline__ void pull_fold_range(const CollArgs& a, char* own, const char* const* src, char* res, uint64_t tlen) {
    const int n = a.n, r = a.rank, f = a.fold[r];  // the ring order of chunk f
    const unsigned tid = threadIdx.x;
    auto fold_elem = [&](uint64_t e) {
        auto val = [&](int q) -> T {
            return q == r ? *reinterpret_cast<const T*>(own + e) : ld_elem_sys<T>(src[q] + e);
        };
        T acc = val((f - 1 + n) % n);
        for (int k = 2; k <= n; ++k) acc = OpF<OP>::apply(val((f - k + n) % n), acc);
        *reinterpret_cast<T*>(own + e) = acc;
        st_elem_wt<T>(res + e, acc);
    };
    const int q0 = (r + 1) % n;  // every src[q] and res share one alignment (slot base + mis)
    if ((((uintptr_t)own ^ (uintptr_t)src[q0]) & 15) != 0) {
        for (uint64_t e = (uint64_t)tid * sizeof(T); e < tlen; e += (uint64_t)kBlock * sizeof(T)) fold_elem(e);
        return;
    }
    const uint64_t mis16 = (uint64_t)(uintptr_t)own & 15;
    uint64_t head = mis16 ? 16 - mis16 : 0;
    if (head > tlen) head = tlen;
    const uint64_t nvec = (tlen - head) >> 4;
    const uint64_t tail = head + (nvec << 4);
    {
        const uint64_t nh = head / sizeof(T), nt = (tlen - tail) / sizeof(T);
        if (tid < nh) fold_elem(tid * sizeof(T));
        else if (tid >= 64 && tid - 64 < nt) fold_elem(tail + (tid - 64) * sizeof(T));
    }
    constexpr int U = NMAX <= 8 ? 2 : 1;
    const uint64_t stride = kBlock;
    for (uint64_t ib = 0; ib < nvec; ib += U * stride) {
        const uint64_t i = ib + tid;
        v4u v[U][NMAX];
        bool live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) live[u] = i + u * stride < nvec;
#pragma unroll
        for (int k = 1; k <= NMAX; ++k) {
            if (k <= n) {
                const int q = (f - k + n) % n;  // x[f-1], x[f-2], ..., x[f]
                if (q == r) {
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (live[u]) v[u][k - 1] = ld16(own + head + (i + u * stride) * 16);
                } else {
                    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(src[q] + head + ib * 16);
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (live[u]) v[u][k - 1] = ld16_sys(rs, (uint32_t)((tid + u * stride) * 16));
                }
            }
        }
        const __amdgpu_buffer_rsrc_t res_rs = wt_rsrc(res + head + ib * 16);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!live[u]) continue;
            v4u acc = v[u][0];
#pragma unroll
            for (int k = 2; k <= NMAX; ++k)
                if (k <= n) acc = reduce16<OP, T>(v[u][k - 1], acc);
            st16(own + head + (i + u * stride) * 16, acc);
            st16_wt(res_rs, (uint32_t)((tid + u * stride) * 16), acc);
        }
    }
}

// One work item of each pull-mesh role.
// stage: my copy of chunk c's tile t -> my RS slot c, then owner c's flag
__device__ __forceinline__ void pull_stage_item(const CollArgs& a, uint64_t seq, int t, int c) {
    const int r = a.rank;
    const uint64_t toff = (uint64_t)t * a.tile_bytes;
    uint64_t tlen = a.len[c] - toff;
    if (tlen > a.tile_bytes) tlen = a.tile_bytes;
    char* dst = a.rs[r] + (uint64_t)c * a.slot_bytes + a.mis[c];
    if (a.units)
        for_unit_pieces(a, a.off[c] + toff, a.off[c] + toff + tlen, [&](char* usr, uint64_t p, uint64_t l) {
            block_copy<kDstPeer>(dst + (p - a.off[c]), usr, l);
        });
    else
        block_copy<kDstPeer>(dst + toff, a.user + a.off[c] + toff, tlen);
    block_publish1(flag_word(a, c, (uint64_t)r * a.max_tiles + t), seq, a.uc);
    __syncthreads();
}

// reduce: chunk r, tile t, once all n-1 peers staged it; false: the wait gave up
template <int OP, typename T, int NMAX>
__device__ __forceinline__ bool pull_reduce_item(const CollArgs& a, uint64_t seq, const Abort& ab, int t) {
    const int n = a.n, r = a.rank;
    __shared__ uint64_t* s_flags[RDC_MAX_RANKS];
    __shared__ const char* s_src[RDC_MAX_RANKS];
    if (threadIdx.x < (unsigned)(n - 1)) {
        const int p = (r + 1 + threadIdx.x) % n;
        s_flags[threadIdx.x] = flag_word(a, r, (uint64_t)p * a.max_tiles + t);
    }
    __syncthreads();
    if (!block_wait(s_flags, n - 1, seq, ab, RDC_KERR_TIMEOUT_RS, a.uc)) return false;
    const uint64_t toff = (uint64_t)t * a.tile_bytes;
    uint64_t tlen = a.len[r] - toff;
    if (tlen > a.tile_bytes) tlen = a.tile_bytes;
    const uint64_t slot_r = (uint64_t)r * a.slot_bytes;
    if (a.units) {
        for_unit_pieces(a, a.off[r] + toff, a.off[r] + toff + tlen, [&](char* usr, uint64_t p, uint64_t l) {
            const uint64_t co = a.mis[r] + (p - a.off[r]);
            if (threadIdx.x < (unsigned)n) s_src[threadIdx.x] = a.rs[threadIdx.x] + slot_r + co;
            __syncthreads();
            pull_fold_range<OP, T, NMAX>(a, usr, s_src, a.ag[r] + slot_r + co, l);
            __syncthreads();  // s_src is rewritten for the next piece
        });
    } else {
        const uint64_t co = a.mis[r] + toff;
        if (threadIdx.x < (unsigned)n) s_src[threadIdx.x] = a.rs[threadIdx.x] + slot_r + co;
        __syncthreads();
        pull_fold_range<OP, T, NMAX>(a, a.user + a.off[r] + toff, s_src, a.ag[r] + slot_r + co, tlen);
    }
    if (a.poison) {  // peer q restages its slot r only after gathering this tile's result
        __syncthreads();
        for (int k = 1; k < n; ++k) block_poison(a.rs[(r + k) % n] + slot_r + a.mis[r] + toff, tlen);
    }
    if (threadIdx.x < (unsigned)(n - 1)) {
        const int p = (r + 1 + threadIdx.x) % n;
        s_flags[threadIdx.x] = flag_word(a, p, (uint64_t)(n + r) * a.max_tiles + t);
    }
    block_publish(s_flags, n - 1, seq, a.uc);
    __syncthreads();
    return true;
}

// gather: owner c's result tile t (its AG slot c) -> my user buffer; false: gave up
__device__ __forceinline__ bool pull_gather_item(const CollArgs& a, uint64_t seq, const Abort& ab, int t, int c) {
    const int n = a.n, r = a.rank;
    __shared__ uint64_t* s_flag[1];
    if (threadIdx.x == 0) s_flag[0] = flag_word(a, r, (uint64_t)(n + c) * a.max_tiles + t);
    __syncthreads();
    if (!block_wait(s_flag, 1, seq, ab, RDC_KERR_TIMEOUT_AG, a.uc)) return false;
    const uint64_t toff = (uint64_t)t * a.tile_bytes;
    uint64_t tlen = a.len[c] - toff;
    if (tlen > a.tile_bytes) tlen = a.tile_bytes;
    const char* src = a.ag[c] + (uint64_t)c * a.slot_bytes + a.mis[c];
    if (a.units)
        for_unit_pieces(a, a.off[c] + toff, a.off[c] + toff + tlen, [&](char* usr, uint64_t p, uint64_t l) {
            block_copy_pull(usr, src + (p - a.off[c]), l);
        });
    else
        block_copy_pull(a.user + a.off[c] + toff, src + toff, tlen);
    __syncthreads();
    return true;
}

template <int OP, typename T, int NMAX>
__device__ __forceinline__ void mesh_pull_body(const CollArgs& a, uint64_t seq) {
    const int n = a.n, r = a.rank;
    Abort ab{a.err, wall_clock64() + a.timeout_ticks, a.poll_rmw};
    int b = blockIdx.x;
    int tmax = 0;
    for (int c = 0; c < n; ++c) tmax = a.tiles[c] > tmax ? a.tiles[c] : tmax;
    if (b < a.nb_scatter) {
        const int items = (n - 1) * tmax;
        for (int it = b; it < items; it += a.nb_scatter) {
            const int t = it / (n - 1);
            const int c = (r + 1 + it % (n - 1)) % n;
            if (t < a.tiles[c]) pull_stage_item(a, seq, t, c);
        }
        return;
    }
    b -= a.nb_scatter;
    if (b < a.nb_reduce) {
        for (int t = b; t < a.tiles[r]; t += a.nb_reduce)
            if (!pull_reduce_item<OP, T, NMAX>(a, seq, ab, t)) return;
        return;
    }
    b -= a.nb_reduce;
    const int items = (n - 1) * tmax;
    for (int it = b; it < items; it += a.nb_gather) {
        const int t = it / (n - 1);
        const int c = (r + 1 + it % (n - 1)) % n;
        if (t < a.tiles[c] && !pull_gather_item(a, seq, ab, t, c)) return;
    }
}

// ============================================ direct (registered buffers) ===
// RDC_ALGO_DIRECT (Communicator::AllreduceDirect): every rank's user buffer
// is mapped into every peer (HIP IPC, once per allocation; a host rendezvous
// per call agrees on the buffers), so owner r folds chunk r straight out of
// the n user buffers and writes the result straight back into all of them.
// No scratch: each rank's kernels read its buffer once and write it once
// (2 S of memory traffic per rank, against the pull mesh's (5n-2)/n S).
// Hand-offs (rows of the ordinary flag array, tile 0):
//   ready: first thing in its launch, rank q tells every owner r its buffer
//          holds this launch's input (owner r's row q) — stream order made it so;
//   done : launch_done's done words (every owner tile written and drained),
//          and a direct launch ends only once every peer's done word arrived,
//          so no owner reads or writes a rank's buffer after that rank's
//          stream moves on.
// Fold order per element: chunk r's ring order, as every schedule.  All ranks'
// buffers are congruent mod 16 (checked at the rendezvous), so one 16-B path.
template <int OP, typename T, int NMAX>
__device__ __forceinline__ void direct_fold_range(const CollArgs& a, char* const* buf, uint64_t tlen) {
    const int n = a.n, r = a.rank, f = a.fold[r];
    const unsigned tid = threadIdx.x;
    auto fold_elem = [&](uint64_t e) {
        auto val = [&](int q) -> T {
            return q == r ? *reinterpret_cast<const T*>(buf[q] + e) : ld_elem_sys<T>(buf[q] + e);
        };
        T acc = val((f - 1 + n) % n);
        for (int k = 2; k <= n; ++k) acc = OpF<OP>::apply(val((f - k + n) % n), acc);
        for (int q = 0; q < n; ++q) {
            if (q == r) *reinterpret_cast<T*>(buf[q] + e) = acc;
            else st_elem_wt<T>(buf[q] + e, acc);
        }
    };
    const uint64_t mis16 = (uint64_t)(uintptr_t)buf[r] & 15;
    uint64_t head = mis16 ? 16 - mis16 : 0;
    if (head > tlen) head = tlen;
    const uint64_t nvec = (tlen - head) >> 4;
    const uint64_t tail = head + (nvec << 4);
    {
        const uint64_t nh = head / sizeof(T), nt = (tlen - tail) / sizeof(T);
        if (tid < nh) fold_elem(tid * sizeof(T));
        else if (tid >= 64 && tid - 64 < nt) fold_elem(tail + (tid - 64) * sizeof(T));
    }
    constexpr int U = NMAX <= 8 ? 2 : 1;
    const uint64_t stride = kBlock;
    for (uint64_t ib = 0; ib < nvec; ib += U * stride) {
        const uint64_t i = ib + tid;
        v4u v[U][NMAX];
        bool live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) live[u] = i + u * stride < nvec;
#pragma unroll
        for (int k = 1; k <= NMAX; ++k) {
            if (k <= n) {
                const int q = (f - k + n) % n;  // x[f-1], x[f-2], ..., x[f]
                if (q == r) {
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (live[u]) v[u][k - 1] = ld16_nt(buf[r] + head + (i + u * stride) * 16);
                } else {
                    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(buf[q] + head + ib * 16);
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (live[u]) v[u][k - 1] = ld16_sys(rs, (uint32_t)((tid + u * stride) * 16));
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!live[u]) continue;
            v4u acc = v[u][0];
#pragma unroll
            for (int k = 2; k <= NMAX; ++k)
                if (k <= n) acc = reduce16<OP, T>(v[u][k - 1], acc);
            v[u][0] = acc;
        }
#pragma unroll
        for (int q = 0; q < NMAX; ++q) {
            if (q >= n) continue;
            if (q == r) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (live[u]) st16_nt(buf[r] + head + (i + u * stride) * 16, v[u][0]);
            } else {
                const __amdgpu_buffer_rsrc_t rs = wt_rsrc(buf[q] + head + ib * 16);
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (live[u]) st16_wt(rs, (uint32_t)((tid + u * stride) * 16), v[u][0]);
            }
        }
    }
}

template <int OP, typename T, int NMAX>
__device__ __forceinline__ void direct_body(const CollArgs& a, uint64_t seq) {
    const int n = a.n, r = a.rank;
    Abort ab{a.err, wall_clock64() + a.timeout_ticks, a.poll_rmw};
    __shared__ uint64_t* s_flags[RDC_MAX_RANKS];
    __shared__ char* s_buf[RDC_MAX_RANKS];
    // ready: this rank's buffer holds this launch's input (block 0, before any wait)
    if (blockIdx.x == 0 && threadIdx.x < (unsigned)(n - 1))
        flag_store(flag_word(a, (r + 1 + threadIdx.x) % n, (uint64_t)r * a.max_tiles), seq);
    if (threadIdx.x < (unsigned)(n - 1))
        s_flags[threadIdx.x] = flag_word(a, r, (uint64_t)((r + 1 + threadIdx.x) % n) * a.max_tiles);
    if (threadIdx.x < (unsigned)n) s_buf[threadIdx.x] = a.cbuf[threadIdx.x] + a.off[r];
    __syncthreads();
    if (!block_wait(s_flags, n - 1, seq, ab, RDC_KERR_TIMEOUT_RS, a.uc)) return;
    __shared__ char* s_tile[RDC_MAX_RANKS];
    if (a.units) {
        // coalesced list: item t = piece of chunk r of buffer it[0], at byte
        // it[1], it[2] bytes; rank q's buffer b at ptr[q * dnbuf + b]
        const uint64_t* items = static_cast<const uint64_t*>(a.units);
        const uint64_t* ptr = items + 3 * (uint64_t)a.nunits;
        const int rot = a.rotate ? (int)((int64_t)a.nunits * r / n) : 0;
        for (int i = blockIdx.x; i < a.nunits; i += gridDim.x) {
            const int t = i + rot < a.nunits ? i + rot : i + rot - a.nunits;
            const uint64_t b = items[3 * (uint64_t)t], so = items[3 * (uint64_t)t + 1];
            const uint64_t tlen = items[3 * (uint64_t)t + 2];
            if (threadIdx.x < (unsigned)n)
                s_tile[threadIdx.x] = reinterpret_cast<char*>(ptr[(uint64_t)threadIdx.x * a.dnbuf + b]) + so;
            __syncthreads();
            direct_fold_range<OP, T, NMAX>(a, s_tile, tlen);
            __syncthreads();  // s_tile is rewritten for the next item
        }
        return;
    }
    // owners walk their chunks from staggered points (rotate): at any moment
    // the n owners touch offsets that are not all exactly S/n apart in every
    // buffer.  tools/placement_probe.py (profiles/r05/direct/placement/): one
    // buffer placement in three runs ~20 % slower at n = 4 with or without
    // it; the stagger gains 1-3 % at n = 4 and up to 8 % at n = 8, never loses
    const int ntiles = a.tiles[r];
    const int rot = a.rotate ? (int)((int64_t)ntiles * r / n) : 0;
    for (int i = blockIdx.x; i < ntiles; i += gridDim.x) {
        const int t = i + rot < ntiles ? i + rot : i + rot - ntiles;
        const uint64_t toff = (uint64_t)t * a.tile_bytes;
        uint64_t tlen = a.len[r] - toff;
        if (tlen > a.tile_bytes) tlen = a.tile_bytes;
        if (threadIdx.x < (unsigned)n) s_tile[threadIdx.x] = s_buf[threadIdx.x] + toff;
        __syncthreads();
        direct_fold_range<OP, T, NMAX>(a, s_tile, tlen);
        __syncthreads();  // s_tile is rewritten for the next tile
    }
}

// ======================================================= ring allreduce ===
// own[i] = OP(own[i], recv[i]) — reducer(src=reducebuf, dst=sendrecvbuf)
// (communicator_collective.cc:174-176), element-wise head/tail + 16-B body.
// recv is this rank's RS slot, written by the next rank: system-scope loads.
template <int OP, typename T>
__device__ void block_reduce_into(char* own, const char* recv, uint64_t len) {
    const unsigned tid = threadIdx.x;
    auto fold_elem = [&](uint64_t e) {
        T* d = reinterpret_cast<T*>(own + e);
        *d = OpF<OP>::apply(*d, ld_elem_sys<T>(recv + e));
    };
    if ((((uintptr_t)own ^ (uintptr_t)recv) & 15) != 0) {  // buffer not 16-B aligned: element-wise
        for (uint64_t e = (uint64_t)tid * sizeof(T); e < len; e += (uint64_t)kBlock * sizeof(T)) fold_elem(e);
        return;
    }
    const uint64_t mis16 = (uint64_t)(uintptr_t)own & 15;
    uint64_t head = mis16 ? 16 - mis16 : 0;
    if (head > len) head = len;
    const uint64_t nvec = (len - head) >> 4;
    const uint64_t tail = head + (nvec << 4);
    if (tid < head / sizeof(T)) fold_elem(tid * sizeof(T));
    if (tid < (len - tail) / sizeof(T)) fold_elem(tail + tid * sizeof(T));
    v4u* d = reinterpret_cast<v4u*>(own + head);
    constexpr int U = 4;
    for (uint64_t ib = 0; ib < nvec; ib += U * kBlock) {
        const __amdgpu_buffer_rsrc_t rs = wt_rsrc(recv + head + ib * 16);
        const uint64_t i = ib + tid;
        if (ib + U * kBlock <= nvec) {
            v4u x[U], y[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = ld16(d + i + u * kBlock);
#pragma unroll
            for (int u = 0; u < U; ++u) y[u] = ld16_sys(rs, (uint32_t)((tid + u * kBlock) * 16));
#pragma unroll
            for (int u = 0; u < U; ++u) st16(d + i + u * kBlock, reduce16<OP, T>(x[u], y[u]));
        } else {
            for (int u = 0; u < U; ++u) {
                if (i + u * kBlock >= nvec) break;
                st16(d + i + u * kBlock,
                     reduce16<OP, T>(ld16(d + i + u * kBlock), ld16_sys(rs, (uint32_t)((tid + u * kBlock) * 16))));
            }
        }
    }
}

// Chunk c's user bytes [off[c] + toff, + tlen) as (user pointer, offset from
// off[c], bytes) pieces: one piece of the buffer, or — coalesced lists
// (a.units) — the unit pieces the packed range covers (rdc_plan.h
// PlanCoalesced: user slices and scratch images are congruent mod 16).
// The ring touches every (chunk, tile) range twice — received at one step,
// sent on at the next, or sent in the reduce-scatter and received in the
// allgather — so a block remembers each chunk's first unit for its current
// tile (UnitCache, block-shared) and searches the table once per range.
struct UnitCache {
    uint64_t toff[RDC_MAX_RANKS];
    int first[RDC_MAX_RANKS];
};
__device__ __forceinline__ void unit_cache_reset(UnitCache& uc) {
    if (threadIdx.x < RDC_MAX_RANKS) uc.toff[threadIdx.x] = ~0ull;
    __syncthreads();
}
template <typename F>
__device__ __forceinline__ void chunk_pieces(const CollArgs& a, int c, uint64_t toff, uint64_t tlen, F&& f,
                                             UnitCache* uc = nullptr) {
    if (a.units) {
        int first = -1;
        if (uc) {
            if (uc->toff[c] == toff) {
                first = uc->first[c];
            } else {
                first = unit_first(static_cast<const PackUnit*>(a.units), a.nunits, a.off[c] + toff);
                __syncthreads();  // every thread has read the old entry
                if (threadIdx.x == 0) {
                    uc->toff[c] = toff;
                    uc->first[c] = first;
                }
                __syncthreads();
            }
        }
        for_unit_pieces(a, a.off[c] + toff, a.off[c] + toff + tlen,
                        [&](char* usr, uint64_t p, uint64_t l) { f(usr, p - a.off[c], l); }, first);
    } else {
        f(a.user + a.off[c] + toff, toff, tlen);
    }
}

template <int OP, typename T>
__device__ void ring_body(const CollArgs& a, uint64_t seq) {
    const int n = a.n, r = a.rank;
    const int prev = (r - 1 + n) % n;
    Abort ab{a.err, wall_clock64() + a.timeout_ticks, a.poll_rmw};
    if (prev_kind(a) == RDC_KIND_ONESHOT && !gate_on_peers(a, seq, prev, 1, ab, RDC_KERR_TIMEOUT_RING)) return;
    __shared__ uint64_t* s_flag[1];
    __shared__ UnitCache s_units;
    UnitCache* ucp = a.units ? &s_units : nullptr;
    if (ucp) unit_cache_reset(s_units);
    int tmax = 0;
    for (int c = 0; c < n; ++c) tmax = a.tiles[c] > tmax ? a.tiles[c] : tmax;
    for (int t = blockIdx.x; t < tmax; t += gridDim.x) {
        const uint64_t toff = (uint64_t)t * a.tile_bytes;
        // ---- TryReduceScatterRing: step j sends chunk (r+1+j)%n to prev,
        //      receives chunk (r+2+j)%n from next and reduces it in place.
        for (int j = 0; j < n - 1; ++j) {
            const int cs = (r + 1 + j) % n;
            if (t < a.tiles[cs]) {
                uint64_t tlen = a.len[cs] - toff;
                if (tlen > a.tile_bytes) tlen = a.tile_bytes;
                char* dst = a.rs[prev] + (uint64_t)j * a.slot_bytes + a.mis[cs];
                chunk_pieces(a, cs, toff, tlen, [&](char* usr, uint64_t co, uint64_t l) {
                    block_copy<kDstPeer>(dst + co, usr, l);
                }, ucp);
                block_publish1(flag_word(a, prev, (uint64_t)j * a.max_tiles + t), seq, a.uc);
            }
            const int cr = (r + 2 + j) % n;
            if (t < a.tiles[cr]) {
                if (threadIdx.x == 0) s_flag[0] = flag_word(a, r, (uint64_t)j * a.max_tiles + t);
                __syncthreads();
                if (!block_wait(s_flag, 1, seq, ab, RDC_KERR_TIMEOUT_RING, a.uc)) return;
                uint64_t tlen = a.len[cr] - toff;
                if (tlen > a.tile_bytes) tlen = a.tile_bytes;
                char* src = a.rs[r] + (uint64_t)j * a.slot_bytes + a.mis[cr];
                chunk_pieces(a, cr, toff, tlen, [&](char* usr, uint64_t co, uint64_t l) {
                    block_reduce_into<OP, T>(usr, src + co, l);
                }, ucp);
                __syncthreads();
                if (a.poison) block_poison(src + toff, tlen);
            }
        }
        // ---- TryAllgatherRing: step j sends chunk (r+j)%n to prev and
        //      receives chunk (r+1+j)%n from next (in place).
        for (int j = 0; j < n - 1; ++j) {
            const int cs = (r + j) % n;
            if (t < a.tiles[cs]) {
                uint64_t tlen = a.len[cs] - toff;
                if (tlen > a.tile_bytes) tlen = a.tile_bytes;
                char* dst = a.ag[prev] + (uint64_t)j * a.slot_bytes + a.mis[cs];
                chunk_pieces(a, cs, toff, tlen, [&](char* usr, uint64_t co, uint64_t l) {
                    block_copy<kDstPeer>(dst + co, usr, l);
                }, ucp);
                block_publish1(flag_word(a, prev, (uint64_t)(n + j) * a.max_tiles + t), seq, a.uc);
            }
            const int cr = (r + 1 + j) % n;
            if (t < a.tiles[cr]) {
                if (threadIdx.x == 0) s_flag[0] = flag_word(a, r, (uint64_t)(n + j) * a.max_tiles + t);
                __syncthreads();
                if (!block_wait(s_flag, 1, seq, ab, RDC_KERR_TIMEOUT_RING, a.uc)) return;
                uint64_t tlen = a.len[cr] - toff;
                if (tlen > a.tile_bytes) tlen = a.tile_bytes;
                char* src = a.ag[r] + (uint64_t)j * a.slot_bytes + a.mis[cr];
                chunk_pieces(a, cr, toff, tlen, [&](char* usr, uint64_t co, uint64_t l) {
                    block_copy_pull(usr, src + co, l);
                }, ucp);
                __syncthreads();
                if (a.poison) block_poison(src + toff, tlen);
            }
        }
    }
}

// =================================================== one-shot allreduce ===
// Small buffers: every rank pushes its WHOLE buffer into every peer's RS slot
// `rank` (one hand-off instead of the mesh's two), then folds all n
// contributions itself.  Element i of chunk c (utils::Split) is folded in the
// ring's order for c — s = x[c-1]; s = OP(x[c-2], s) ... s = OP(x[c], s) —
// so every rank computes the reference's bits without a second exchange.
// Consecutive one-shot launches alternate between the two halves of each
// slot (seq parity): a peer can be at most one launch ahead, so it never
// overwrites the half a slower rank is still folding.

// What a one-shot / tree fold reads and writes: this rank's values `own`,
// rank q's copy at slots + q * slot_bytes, the tree program, and where the
// result goes (`out`: `own` itself for the collective kernels, the host
// mailbox for the small-allreduce service k_svc).
struct FoldView {
    int n, r;
    const char* own;
    char* out;
    const char* slots;
    uint64_t slot_bytes;
    int tree_len;
    const int8_t* tree_dst;
    const int8_t* tree_src;
};

// fold bytes [lo, hi) of the buffer, all inside chunk c
template <int OP, typename T, int NMAX>
__device__ void oneshot_fold_range(const FoldView& a, int c, uint64_t lo, uint64_t hi) {
    const int n = a.n, r = a.r;
    const char* own = a.own;
    char* out = a.out;
    const char* slots = a.slots;
    const unsigned tid = threadIdx.x;
    auto src = [&](int q) -> const char* { return q == r ? own : slots + (uint64_t)q * a.slot_bytes; };
    // own values are this rank's; the others were handed off (system-scope loads)
    auto val = [&](int q, uint64_t x) -> T {
        return q == r ? *reinterpret_cast<const T*>(own + x) : ld_elem_sys<T>(src(q) + x);
    };
    auto fold_elem = [&](uint64_t x) {
        T acc = val((c - 1 + n) % n, x);
        for (int k = 2; k <= n; ++k) acc = OpF<OP>::apply(val((c - k + n) % n, x), acc);
        *reinterpret_cast<T*>(out + x) = acc;
    };
    if (((((uintptr_t)own ^ (uintptr_t)slots) | ((uintptr_t)out ^ (uintptr_t)slots)) & 15) != 0) {  // not 16-B aligned
        for (uint64_t x = lo + (uint64_t)tid * sizeof(T); x < hi; x += (uint64_t)kBlock * sizeof(T)) fold_elem(x);
        return;
    }
    uint64_t vlo = (lo + 15) & ~(uint64_t)15;
    if (vlo > hi) vlo = hi;
    const uint64_t vhi = vlo + ((hi - vlo) & ~(uint64_t)15);
    {
        const uint64_t nh = (vlo - lo) / sizeof(T), nt = (hi - vhi) / sizeof(T);
        if (tid < nh) fold_elem(lo + tid * sizeof(T));
        else if (tid >= 64 && tid - 64 < nt) fold_elem(vhi + (tid - 64) * sizeof(T));
    }
    constexpr int U = NMAX <= 8 ? 2 : 1;
    const uint64_t nvec = (vhi - vlo) >> 4;
    for (uint64_t ib = 0; ib < nvec; ib += U * kBlock) {
        const uint64_t i = ib + tid;
        v4u v[U][NMAX];
        bool live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) live[u] = i + u * kBlock < nvec;
#pragma unroll
        for (int k = 1; k <= NMAX; ++k) {
            if (k <= n) {
                const int q = (c - k + n) % n;
                if (q == r) {
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (live[u]) v[u][k - 1] = ld16_nt(own + vlo + (i + u * kBlock) * 16);
                } else {
                    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(src(q) + vlo + ib * 16);
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (live[u]) v[u][k - 1] = ld16_sys(rs, (uint32_t)((tid + u * kBlock) * 16));
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!live[u]) continue;
            v4u acc = v[u][0];
#pragma unroll
            for (int k = 2; k <= NMAX; ++k)
                if (k <= n) acc = reduce16<OP, T>(v[u][k - 1], acc);
            st16(out + vlo + (i + u * kBlock) * 16, acc);
        }
    }
}

// ---- tree order (rdc_reduce_ring_mincount, TryAllreduceTree): every element
// of [lo, hi) folded over the n ranks' values with the host-planned program
// acc[d] = OP(acc[d], acc[s]) (rdc_plan.h PlanTreeProgram), result acc[0] —
// the reference root's bits, which its broadcast hands to every rank.  The
// program's indices are run-time values, so the n values live in LDS as
// [rank][thread] (a register array indexed that way becomes scratch memory).
template <int OP, typename T, int NMAX>
__device__ void tree_fold_range(const FoldView& a, uint64_t lo, uint64_t hi) {
    __shared__ v4u s_acc[NMAX * kBlock];
    const int n = a.n, r = a.r;
    const char* own = a.own;
    char* out = a.out;
    const char* slots = a.slots;
    const unsigned tid = threadIdx.x;
    auto src = [&](int q) -> const char* { return q == r ? own : slots + (uint64_t)q * a.slot_bytes; };
    auto fold_elem = [&](uint64_t x) {
        T* v = reinterpret_cast<T*>(s_acc + tid);  // v[q * 16 / sizeof(T) * kBlock]: rank q's value
        constexpr int S = 16 / sizeof(T) * kBlock;
#pragma unroll
        for (int k = 0; k < NMAX; ++k)
            if (k < n) v[k * S] = k == r ? *reinterpret_cast<const T*>(own + x) : ld_elem_sys<T>(src(k) + x);
        for (int i = 0; i < a.tree_len; ++i) {
            const int d = a.tree_dst[i], s = a.tree_src[i];
            v[d * S] = OpF<OP>::apply(v[d * S], v[s * S]);
        }
        *reinterpret_cast<T*>(out + x) = v[0];
    };
    if (((((uintptr_t)own ^ (uintptr_t)slots) | ((uintptr_t)out ^ (uintptr_t)slots)) & 15) != 0) {  // not 16-B aligned
        for (uint64_t x = lo + (uint64_t)tid * sizeof(T); x < hi; x += (uint64_t)kBlock * sizeof(T)) fold_elem(x);
        return;
    }
    uint64_t vlo = (lo + 15) & ~(uint64_t)15;
    if (vlo > hi) vlo = hi;
    const uint64_t vhi = vlo + ((hi - vlo) & ~(uint64_t)15);
    {
        const uint64_t nh = (vlo - lo) / sizeof(T), nt = (hi - vhi) / sizeof(T);
        if (tid < nh) fold_elem(lo + tid * sizeof(T));
        else if (tid >= 64 && tid - 64 < nt) fold_elem(vhi + (tid - 64) * sizeof(T));
    }
    const uint64_t nvec = (vhi - vlo) >> 4;
    v4u* v = s_acc + tid;  // v[q * kBlock]: rank q's vector
    for (uint64_t ib = 0; ib < nvec; ib += kBlock) {
        const uint64_t i = ib + tid;
        if (i >= nvec) break;  // the last window (no barrier inside the loop)
        v4u x[NMAX];
#pragma unroll
        for (int k = 0; k < NMAX; ++k)
            if (k < n) x[k] = k == r ? ld16_nt(own + vlo + i * 16)
                                     : ld16_sys(wt_rsrc(src(k) + vlo + ib * 16), (uint32_t)(tid * 16));
#pragma unroll
        for (int k = 0; k < NMAX; ++k)
            if (k < n) v[k * kBlock] = x[k];
        for (int j = 0; j < a.tree_len; ++j) {
            const int d = a.tree_dst[j], s = a.tree_src[j];
            v[d * kBlock] = reduce16<OP, T>(v[d * kBlock], v[s * kBlock]);
        }
        st16(out + vlo + i * 16, v[0]);
    }
}

template <int OP, typename T, int NMAX, bool TREE = false>
__device__ void oneshot_body(const CollArgs& a, uint64_t seq) {
    const int n = a.n, r = a.rank;
    Abort ab{a.err, wall_clock64() + a.timeout_ticks, a.poll_rmw};
    __shared__ uint64_t* s_flags[RDC_MAX_RANKS];
    const uint64_t half = (seq_counter(seq) & 1u) ? a.half_bytes : 0;
    const uint64_t total = a.total_bytes;
    const int ntiles = a.tiles[0];
    // 1) push every tile of my buffer into every peer's slot r (never waits)
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t toff = (uint64_t)t * a.tile_bytes;
        uint64_t tlen = total - toff;
        if (tlen > a.tile_bytes) tlen = a.tile_bytes;
        for (int k = 1; k < n; ++k)
            block_copy<kDstPeer>(a.rs[(r + k) % n] + (uint64_t)r * a.slot_bytes + half + toff, a.user + toff, tlen);
        if (threadIdx.x < (unsigned)(n - 1))
            s_flags[threadIdx.x] = flag_word(a, (r + 1 + threadIdx.x) % n, (uint64_t)r * a.max_tiles + t);
        block_publish(s_flags, n - 1, seq, a.uc, a.verify);
        __syncthreads();
    }
    // 2) fold my tiles once every peer's copy landed
    const FoldView fv{n, r, a.user, a.user, a.rs[r] + half, a.slot_bytes, a.tree_len, a.tree_dst, a.tree_src};
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        if (threadIdx.x < (unsigned)(n - 1))
            s_flags[threadIdx.x] = flag_word(a, r, (uint64_t)((r + 1 + threadIdx.x) % n) * a.max_tiles + t);
        __syncthreads();
        if (!block_wait(s_flags, n - 1, seq, ab, RDC_KERR_TIMEOUT_RS, a.uc)) return;
        const uint64_t lo = (uint64_t)t * a.tile_bytes;
        const uint64_t hi = lo + a.tile_bytes < total ? lo + a.tile_bytes : total;
        if (TREE) {
            tree_fold_range<OP, T, NMAX>(fv, lo, hi);
        } else {
            for (int c = 0; c < n; ++c) {
                if (a.len[c] == 0) continue;
                const uint64_t clo = a.off[c] > lo ? a.off[c] : lo;
                const uint64_t chi = a.off[c] + a.len[c] < hi ? a.off[c] + a.len[c] : hi;
                if (clo < chi) oneshot_fold_range<OP, T, NMAX>(fv, a.fold[c], clo, chi);
            }
        }
        __syncthreads();
        // a peer rewrites this half two launches later, after this kernel's end
        if (a.poison)
            for (int k = 1; k < n; ++k) block_poison(a.rs[r] + (uint64_t)((r + k) % n) * a.slot_bytes + half + lo, hi - lo);
    }
}

// ============================================================ broadcast ===
// piece = [off[0], off[0]+len[0]) of the user buffer; tiles[0] tiles.
// direct (bcast_split == 0): the root pushes every tile to all n-1 peers - one
//   hop, but the root's egress is (n-1) x S: for small pieces.
// split (n >= 3): tile t goes from the root to ONE forwarder, the
//   (t mod (n-1))-th rank after the root, which lands it and pushes it on to
//   the other n-2 non-root ranks.  Two hops, but every link out of the root
//   carries S/(n-1) and every forwarder link S/(n-1): up to (n-1)/2 x the
//   direct rate when the links are the bound (8 GPUs: 3.5x).
// Either way a rank's flag (n+root, t) has one writer per launch: the root
// (direct, or the forwarder's own flag) or the tile's forwarder.
__device__ __forceinline__ int bcast_forwarder(int n, int root, int t) { return (root + 1 + t % (n - 1)) % n; }

__device__ void bcast_body(const CollArgs& a, uint64_t seq) {
    const int n = a.n, r = a.rank, root = a.root;
    const bool split = a.bcast_split != 0 && n >= 3;
    Abort ab{a.err, wall_clock64() + a.timeout_ticks, a.poll_rmw};
    __shared__ uint64_t* s_flags[RDC_MAX_RANKS];
    __shared__ int s_cnt;
    if (blockIdx.x < a.tiles[0] && (r == root || split)) {
        // A broadcast's receivers never report back, so before overwriting a
        // peer's allgather region a writer waits until that peer finished
        // its previous launch (done word >= seq-1): the root for every peer,
        // a forwarder (split) for the other non-root ranks.  Allreduce
        // launches need no such gate: their peer writes depend on data the
        // target only sends once it has entered the same launch.
        if (threadIdx.x == 0) {
            int k = 0;
            for (int q = 0; q < n; ++q)
                if (q != r && q != root) s_flags[k++] = done_word(a, r, q);
            s_cnt = k;
        }
        __syncthreads();
        if (!block_wait(s_flags, s_cnt, seq_prev(seq), ab, RDC_KERR_TIMEOUT_BCAST, a.uc, false)) return;
    }
    for (int t = blockIdx.x; t < a.tiles[0]; t += gridDim.x) {
        const uint64_t toff = (uint64_t)t * a.tile_bytes;
        uint64_t tlen = a.len[0] - toff;
        if (tlen > a.tile_bytes) tlen = a.tile_bytes;
        char* mine = a.user + a.off[0] + toff;
        const uint64_t soff = a.mis[0] + toff;
        const uint64_t frow = (uint64_t)(n + root) * a.max_tiles + t;
        if (r == root) {
            if (split) {
                const int f = bcast_forwarder(n, root, t);
                block_copy<kDstPeer>(a.ag[f] + soff, mine, tlen);
                block_publish1(flag_word(a, f, frow), seq, a.uc);
            } else {
                for (int k = 1; k < n; ++k) block_copy<kDstPeer>(a.ag[(root + k) % n] + soff, mine, tlen);
                if (threadIdx.x < (unsigned)(n - 1)) s_flags[threadIdx.x] = flag_word(a, (root + 1 + threadIdx.x) % n, frow);
                block_publish(s_flags, n - 1, seq, a.uc);
            }
            __syncthreads();
        } else {
            if (threadIdx.x == 0) s_flags[0] = flag_word(a, r, frow);
            __syncthreads();
            if (!block_wait(s_flags, 1, seq, ab, RDC_KERR_TIMEOUT_BCAST, a.uc)) return;
            char* land = a.ag[r] + soff;
            if (split && bcast_forwarder(n, root, t) == r) {
                for (int k = 1; k < n; ++k) {
                    const int q = (r + k) % n;
                    if (q != root) block_copy<kDstPeer, kSrcHandoff>(a.ag[q] + soff, land, tlen);
                }
                if (threadIdx.x == 0) {
                    int k = 0;
                    for (int q = 0; q < n; ++q)
                        if (q != r && q != root) s_flags[k++] = flag_word(a, q, frow);
                }
                block_publish(s_flags, n - 2, seq, a.uc);  // its barrier orders thread 0's list before use
            }
            block_copy_pull(mine, land, tlen);
            __syncthreads();
            // writers gate on this rank's done word (this kernel's end) before rewriting
            if (a.poison) block_poison(land, tlen);
        }
    }
}

// Every block of every collective launch ends here exactly once (also after
// a timeout).  The last block to arrive resets the local arrival counter,
// publishes done = seq into every peer's flag array (row 2n, column = this
// rank: "this rank finished reading its scratch for launch seq") and
// advances the launch counter.
// The done words mean "finished READING my scratch for launch seq": every
// wave's loads have returned once it passed `s_waitcnt vmcnt(0)`, so with
// uncached scratch and no host memory involved the arrival add and the done
// stores need no fence (the next launch of this communicator sees this one's
// buffer writes through the kernel boundary).  A launch that writes host
// memory (zero-copy host path: `notify`) or uses cached scratch keeps the
// system-scope fences, so the host reads the results after the notify word.
__device__ __forceinline__ void launch_done(const CollArgs& a, uint64_t seq) {
    const bool fence = a.notify != nullptr || !a.uc;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (fence) __threadfence_system();
        // a one-block launch is its own last block: no arrival round trip
        // (small messages run one block)
        const bool last = gridDim.x == 1 || atomicAdd(a.done_ctr, 1u) == gridDim.x - 1;
        if (last) {
            if (gridDim.x > 1) __hip_atomic_store(a.done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (a.seq_check)
                __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.err + 80), 0ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            // the other blocks' writes reach the host (zero-copy results) or
            // cached scratch through this block's release, which its acquire
            // side is the host's read of `notify` (the arrivals are
            // relaxed agent-scope adds, so without it the host-visible order
            // would rest on hardware ordering alone)
            if (fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            for (int p = 0; p < a.n; ++p)
                if (p != a.rank) flag_store(done_word(a, p, a.rank), seq);
            if (a.kind == RDC_KIND_DIRECT) {
                // registered buffers: every owner finished writing into this
                // rank's buffer before its stream moves on (done words of this
                // launch from every peer; bounded like every wait)
                const uint64_t deadline = wall_clock64() + a.timeout_ticks;
                bool gave_up = false;
                for (int p = 0; p < a.n && !gave_up; ++p) {
                    if (p == a.rank) continue;
                    const uint64_t* w = done_word(a, a.rank, p);
                    while (!seq_reached(flag_load(w), seq)) {
                        if (wall_clock64() > deadline ||
                            __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                            uint32_t expected = 0;
                            __hip_atomic_compare_exchange_strong(a.err, &expected, (uint32_t)RDC_KERR_TIMEOUT_AG,
                                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT);
                            gave_up = true;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
            }
            __hip_atomic_store(a.launch_kind, (uint32_t)a.kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (a.tlog)
                __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.tlog + (seq_counter(seq) & 63ull) * 4 + 3),
                                   (unsigned long long)wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.launch_ctr, seq_counter(seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // the host reads the (sticky) error word here after a stream sync: no
            // copy needed.  The mirror starts at 0 and only ever changes to an
            // error, so the PCIe write (whose completion the kernel's end waits
            // for) is made only when there is one — and then completed before
            // the notify word, which the host reads first
            const uint32_t e = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (e != 0) {
                __hip_atomic_store(a.err_mirror, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (a.notify) __hip_atomic_store(a.notify, a.notify_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// RdcCommTraceNext: every block of the traced launch records when it started
// and when its role finished (wall_clock64, 100 MHz) — role timelines for tuning
__device__ __forceinline__ void trace_block(const CollArgs& a, uint64_t t0) {
    if (a.trace && threadIdx.x == 0) {
        a.trace[2 * blockIdx.x] = t0;
        a.trace[2 * blockIdx.x + 1] = wall_clock64();
    }
}

template <int OP, typename T, int NMAX>
__global__ __launch_bounds__(kBlock) void k_mesh(CollArgs a) {
    const uint64_t t0 = wall_clock64();
    uint64_t seq;
    if (!launch_begin(a, &seq)) {
        if (a.pull) mesh_pull_body<OP, T, NMAX>(a, seq);
        else mesh_body<OP, T, NMAX>(a, seq);
    }
    trace_block(a, t0);
    launch_done(a, seq);
}

template <int OP, typename T, int NMAX>
__global__ __launch_bounds__(kBlock) void k_oneshot(CollArgs a) {
    uint64_t seq;
    if (!launch_begin(a, &seq)) oneshot_body<OP, T, NMAX>(a, seq);
    launch_done(a, seq);
}

template <int OP, typename T, int NMAX>
__global__ __launch_bounds__(kBlock) void k_tree(CollArgs a) {
    uint64_t seq;
    if (!launch_begin(a, &seq)) oneshot_body<OP, T, NMAX, true>(a, seq);
    launch_done(a, seq);
}

template <int OP, typename T>
__global__ __launch_bounds__(kBlock) void k_ring(CollArgs a) {
    const uint64_t t0 = wall_clock64();
    uint64_t seq;
    if (!launch_begin(a, &seq)) ring_body<OP, T>(a, seq);
    trace_block(a, t0);
    launch_done(a, seq);
}


template <int OP, typename T, int NMAX>
__global__ __launch_bounds__(kBlock) void k_direct(CollArgs a) {
    uint64_t seq;
    if (!launch_begin(a, &seq)) direct_body<OP, T, NMAX>(a, seq);
    launch_done(a, seq);
}

// ================================================ small-allreduce service ===
// One block per rank, resident while requests keep coming (rdc_service.h).
// Request k: copy the mailbox input into this rank's own slot of half k&1,
// push it into every peer's slot [k&1][rank] (uncached), publish an arrival
// word per peer, wait for the n-1 peers' words, fold every element in its
// Split chunk's ring order (or the tree's order) exactly as the one-shot
// does, and copy the result back into the mailbox; then `done` = k.  A rank
// is at most one request ahead of any peer (it cannot finish k+1 before every
// peer has sent k+1, i.e. finished k), so the two halves never collide.
// Exit conditions, all reached by the one block: `stop` set by the host,
// RDC_HOST_SERVICE_IDLE_US without a request (state EXITING, one more look
// at `req` so a request posted meanwhile is served), or a peer that never
// arrives (error, exit).
// The mailbox is pinned host memory allocated hipHostMallocUncached (MTYPE
// UC: no GPU cache holds it), so plain loads read what the host wrote last and
// plain stores are performed at host memory once `s_waitcnt vmcnt(0)` returns
// (measured: with the default, L2-cacheable host memory the result stores
// stayed in L2 and the host read its own input back).  Control words are
// still system-coherent relaxed atomics; no acquire / release fence (an L2
// invalidate / write-back) on the request path.
__device__ __forceinline__ uint32_t box_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t box_load64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void box_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- exchange between the ranks' service blocks: LL words.  Each 16-byte
// vector i of a rank's input travels as two 16-byte stores {x, seq, y, seq}
// {z, seq, w, seq} into its slot of every peer's region (half next & 1): the
// receiver polls the words themselves, so a vector is complete when its four
// sequence words match — no write drain before a flag, no flag poll, no
// second read of the payload.  8-byte {data, seq} pairs inside a 16-byte
// store are written whole.  A peer is at most one request ahead (it needs
// this rank's next contribution to finish its own), so it never overwrites
// the half this rank is still reading.
__device__ __forceinline__ v4u vload16(const char* p) { return *reinterpret_cast<const volatile v4u*>(p); }

// chunk of element e under utils::Split (rdc_plan.cpp SplitRanges): the
// first m chunks hold k + 1 elements; positions past `count` (the vector
// round-up) map to the last chunk
__device__ __forceinline__ int split_chunk(uint64_t e, uint64_t k, uint64_t m, int n) {
    const uint64_t big = m * (k + 1);
    uint64_t c = e < big ? e / (k + 1) : (k ? m + (e - big) / k : (uint64_t)n - 1);
    return c < (uint64_t)n ? (int)c : n - 1;
}

__device__ __forceinline__ bool ll_match(const v4u& lo, const v4u& hi, uint32_t seq) {
    return lo.y == seq && lo.w == seq && hi.y == seq && hi.w == seq;
}

// Header bits: 31 tree order, 30 LL input, 29 LL result, 28 host exchange,
// 0-27 bytes.
//   LL input (<= RDC_HOST_SERVICE_LL_BYTES): the host writes its input as LL
//     words, so the poll that finds the header can already hold the data (the
//     first `eager` threads read their vector every round): one PCIe round
//     trip fewer; otherwise the input as is, read after the header is seen.
//   LL result: the result as LL words the host polls (no drain, no `done`
//     wait on the host); otherwise as is, drained, then `done`.
//   Host exchange (a.hx, small n * bytes): every rank's host writes its LL
//     input into its slot of ONE shared host region, and every rank's block
//     reads all n inputs from there over PCIe — no send to the peers' slots,
//     no xGMI hand-off; the first `hx_eager` threads poll every rank's words
//     of their vector with the header.  The halves alternate with seq like the
//     slots (a rank is at most one request ahead of any peer's reads).
// LL words are PLANAR: vector i's {w0, seq, w1, seq} at plane 0 + 16 i and
// {w2, seq, w3, seq} at plane 1 + 16 i, so the 64 lanes of one instruction
// touch 1 KiB of contiguous memory (an interleaved 32-byte pair per lane made
// every instruction 64 separate 16-byte requests).
// HX: compiled with the host exchange (a.hx set); the default variant keeps
// its polling arrays out of the register budget
template <int OP, typename T, int NMAX, int BS, bool HX>
__global__ __launch_bounds__(BS) void k_svc(SvcArgs a) {
    constexpr int L = 16 / sizeof(T);  // elements per vector
    constexpr int U = 4;               // input vectors in flight per thread
    typedef typename std::conditional<sizeof(T) == 1, uint8_t,
            typename std::conditional<sizeof(T) == 2, uint16_t,
            typename std::conditional<sizeof(T) == 4, uint32_t, uint64_t>::type>::type>::type UT;
    const int n = a.n, r = a.rank;
    const unsigned tid = threadIdx.x;
    SvcBox* box = a.box;
    SvcIn* in = a.in;
    const bool hxm = HX && a.hx != nullptr;
    const uint32_t all = (n >= 32 ? ~0u : (1u << n) - 1u);
    __shared__ v4u s_in[RDC_SVC_MAX_BYTES / 16];  // this rank's input, read once over PCIe
    __shared__ v4u s_pv[NMAX * BS];               // [q][thread]: rank q's vector being folded
    __shared__ uint32_t s_next;
    __shared__ int s_go, s_err;
    __shared__ uint64_t s_req;
    if (tid == 0) {
        s_next = box_load(&box->done) + 1u;
        s_err = 0;
        box_store(&box->state, RDC_SVC_RUNNING);
    }
    __syncthreads();
    for (;;) {
        // ---- wait for a request (rounds: every thread's loads, one barrier)
        const uint32_t seq = s_next;
        const uint64_t t0 = wall_clock64();
        const bool eager = !hxm && tid < (unsigned)a.eager;
        const bool heager = hxm && tid < (unsigned)a.hx_eager;
        const char* hxh = hxm ? a.hx + (uint64_t)(seq & 1u) * (uint64_t)n * RDC_SVC_HX_RANK_BYTES : nullptr;
        uint32_t hpend = all;  // heager: ranks whose words of vector tid are not in s_pv yet
        v4u elo = {0, 0, 0, 0}, ehi = {0, 0, 0, 0};
        int go = 0;
        // tid 0: the round's decision from its header / stop reads (shared
        // with the host-exchange loop below)
        auto decide = [&](uint64_t q, uint32_t stop) {
            int g = 0;  // 0 poll again, 1 request, -1 leave
            if ((uint32_t)(q >> 32) == seq) {
                g = 1;
            } else if (stop) {
                g = -1;
            } else if (wall_clock64() - t0 > a.idle_ticks) {
                // leaving: EXITING, then one more look at the header (the
                // host posts it and then reads `state`; seq_cst both sides)
                box_store(&box->state, RDC_SVC_EXITING);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
                g = -1;
                q = box_load64(&in->hdr);
                if ((uint32_t)(q >> 32) == seq) {
                    box_store(&box->state, RDC_SVC_RUNNING);
                    g = 1;
                }
            }
            s_req = q;
            s_go = g;
        };
        if (!HX && a.pipe) {
            // RDC_HOST_SERVICE_PIPELINE=1: two rounds in flight — round k+1's
            // reads go out before round k is examined, so a request that lands
            // is seen about 1.25 PCIe round trips later instead of 1.5 (loads
            // return in order; the compiler waits only for the older round).
            // Twice the reads while idle: on one shared link the trace's
            // poll + done fell 4.9 -> 4.1 us but small_latency's 4 B call rose
            // 6.2 -> 7.7 us (profiles/r04/svc_pipeline/), so it is opt-in.
            v4u loA = {0, 0, 0, 0}, hiA = {0, 0, 0, 0}, loB = {0, 0, 0, 0}, hiB = {0, 0, 0, 0};
            uint64_t qA = 0, qB = 0;
            uint32_t sA = 0, sB = 0;
            // branch-free (every lane reads; lanes past the eager range and
            // waves other than 0 re-read vector 0 and the header, one request
            // per wave), so the compiler's wait for a round's reads leaves the
            // next round's in flight
            const uint64_t ev = eager ? tid : 0;
            auto issue = [&](v4u& lo, v4u& hi, uint64_t& q, uint32_t& st) {
                lo = ld16_nt(in->data + 16 * ev);
                hi = ld16_nt(in->data + RDC_SVC_LL_MAX + 16 * ev);
                q = box_load64(&in->hdr);
                st = box_load(&in->stop);
            };
            auto round = [&](uint64_t q, uint32_t st) {
                if (tid == 0) decide(q, st);
                __syncthreads();
                const int g = s_go;
                __syncthreads();  // s_go is rewritten by the next round
                return g;
            };
            issue(loA, hiA, qA, sA);
            for (;;) {
                issue(loB, hiB, qB, sB);
                go = round(qA, sA);
                if (go != 0) {
                    elo = loA;
                    ehi = hiA;
                    break;
                }
                issue(loA, hiA, qA, sA);
                go = round(qB, sB);
                if (go != 0) {
                    elo = loB;
                    ehi = hiB;
                    break;
                }
            }
        }
        for (; HX || !a.pipe;) {
            if (eager) {
                elo = ld16_nt(in->data + 16 * tid);
                ehi = ld16_nt(in->data + RDC_SVC_LL_MAX + 16 * tid);
            }
            if (heager && hpend) {  // pending ranks' loads in flight four at a time, then the matches
                constexpr int G = 4;      // (all NMAX at once spilled VGPRs to scratch)
#pragma unroll
                for (int g = 0; g < NMAX; g += G) {
                    v4u hl[G], hh[G];
#pragma unroll
                    for (int j = 0; j < G; ++j)
                        if ((hpend >> (g + j)) & 1u) {
                            const char* p = hxh + (uint64_t)(g + j) * RDC_SVC_HX_RANK_BYTES + 16 * tid;
                            hl[j] = ld16_nt(p);
                            hh[j] = ld16_nt(p + RDC_SVC_LL_MAX);
                        }
#pragma unroll
                    for (int j = 0; j < G; ++j)
                        if (((hpend >> (g + j)) & 1u) && ll_match(hl[j], hh[j], seq)) {
                            s_pv[(g + j) * BS + tid] = v4u{hl[j].x, hl[j].z, hh[j].x, hh[j].z};
                            hpend &= ~(1u << (g + j));
                        }
                }
            }
            if (tid == 0) {
                const uint64_t q = box_load64(&in->hdr);
                const uint32_t stop = box_load(&in->stop);  // issued with the header read: one round trip
                decide(q, stop);
            }
            __syncthreads();
            go = s_go;
            __syncthreads();  // s_go is rewritten by the next round
            if (go != 0) break;
            if (tid == 0) __builtin_amdgcn_s_sleep(1);
        }
        if (go < 0) break;
        uint64_t ts[4];
        if (a.trace) ts[0] = wall_clock64();
        const uint64_t req = s_req;
        const uint64_t bytes = req & 0x0fffffffu;
        const bool tree = (req >> 31) & 1u, ll = (req >> 30) & 1u, ll_out = (req >> 29) & 1u;
        const bool hx = hxm && ((req >> 28) & 1u);
        const uint64_t nvec = (bytes + 15) >> 4;  // rounded up: the mailbox and slots have room
        const uint64_t half = (uint64_t)(seq & 1u) * (uint64_t)n * RDC_SVC_SLOT_BYTES;
        const uint64_t deadline = wall_clock64() + a.timeout_ticks;
        bool ok = true;
        // 1) my input (U vectors in flight per thread), kept in LDS and sent as
        //    LL words into my slot of every peer's region
        auto send = [&](uint64_t i, const v4u& x) {
            s_in[i] = x;
            for (int k = 1; k < n; ++k) {
                const __amdgpu_buffer_rsrc_t rs =
                    wt_rsrc(a.region[(r + k) % n] + half + (uint64_t)r * RDC_SVC_SLOT_BYTES);
                st16_wt(rs, (uint32_t)(16 * i), v4u{x.x, seq, x.y, seq});
                st16_wt(rs, (uint32_t)(16 * i + RDC_SVC_MAX_BYTES), v4u{x.z, seq, x.w, seq});
            }
        };
        if (hx) {
            // nothing to send: the peers read this rank's input where its host wrote it
        } else if (ll) {
            const bool have0 = eager && ll_match(elo, ehi, seq);
            for (uint64_t i0 = tid; i0 < nvec && ok; i0 += (uint64_t)U * BS) {
                v4u lo[U], hi[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint64_t i = i0 + (uint64_t)u * BS;
                    if (u == 0 && i0 == tid && have0) {
                        lo[u] = elo;
                        hi[u] = ehi;
                    } else if (i < nvec) {
                        lo[u] = ld16_nt(in->data + 16 * i);
                        hi[u] = ld16_nt(in->data + RDC_SVC_LL_MAX + 16 * i);
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint64_t i = i0 + (uint64_t)u * BS;
                    if (i >= nvec || !ok) continue;
                    uint32_t spins = 0;
                    while (!ll_match(lo[u], hi[u], seq)) {  // written before the header, so rarely taken
                        if ((++spins & 63) == 0 && wall_clock64() > deadline) {
                            ok = false;
                            break;
                        }
                        asm volatile("" ::: "memory");
                        lo[u] = ld16_nt(in->data + 16 * i);
                        hi[u] = ld16_nt(in->data + RDC_SVC_LL_MAX + 16 * i);
                    }
                    if (ok) send(i, v4u{lo[u].x, lo[u].z, hi[u].x, hi[u].z});
                }
            }
        } else {
            for (uint64_t i0 = tid; i0 < nvec; i0 += (uint64_t)U * BS) {
                v4u x[U];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (i0 + (uint64_t)u * BS < nvec) x[u] = ld16_nt(in->data + 16 * (i0 + (uint64_t)u * BS));
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (i0 + (uint64_t)u * BS < nvec) send(i0 + (uint64_t)u * BS, x[u]);
            }
        }
        if (a.trace) ts[1] = wall_clock64();
        // 2) per vector: every peer's words (polled together), folded in the
        //    reference's order in registers, written straight to the mailbox
        //    (host exchange: every rank's words, this rank's included, from
        //    the shared host region)
        const char* src = hx ? hxh : a.region[r] + half;
        const uint64_t stride = hx ? RDC_SVC_HX_RANK_BYTES : RDC_SVC_SLOT_BYTES;
        const uint64_t plane = hx ? RDC_SVC_LL_MAX : RDC_SVC_MAX_BYTES;
        const uint32_t pending0 = hx ? all : all & ~(1u << r);
        const uint64_t count = bytes / sizeof(T), ck = count / (uint64_t)n, cm = count % (uint64_t)n;
#pragma unroll 1
        for (uint64_t i = tid; i < nvec && ok; i += BS) {
            v4u* pv = s_pv + tid;  // pv[q * BS]
            uint32_t pending = (hx && heager && i == tid) ? hpend : pending0;
            uint32_t spins = 0;
            while (pending) {
                asm volatile("" ::: "memory");  // a fresh load of every pending word per pass
#pragma unroll
                for (int q = 0; q < NMAX; ++q)
                    if ((pending >> q) & 1u) {
                        const char* p = src + (uint64_t)q * stride + 16 * i;
                        const v4u lo = ld16_nt(p), hi = ld16_nt(p + plane);
                        if (ll_match(lo, hi, seq)) {
                            pv[q * BS] = v4u{lo.x, lo.z, hi.x, hi.z};
                            pending &= ~(1u << q);
                        }
                    }
                if (pending && (++spins & 63) == 0 && wall_clock64() > deadline) {
                    ok = false;
                    break;
                }
            }
            if (!ok) break;
            if (a.trace && i == tid) ts[2] = wall_clock64();
            const v4u own = hx ? pv[r * BS] : s_in[i];
            if (!hx) pv[r * BS] = own;
            v4u res;
            if (tree) {  // acc[d] = OP(acc[d], acc[s]) over the host-planned program; result acc[0]
                for (int j = 0; j < a.tree_len; ++j) {
                    const int d = a.tree_dst[j], sidx = a.tree_src[j];
                    pv[d * BS] = reduce16<OP, T>(pv[d * BS], pv[sidx * BS]);
                }
                res = pv[0];
            } else {
                const uint64_t e0 = i * (uint64_t)L;
                const int c0 = split_chunk(e0, ck, cm, n), c1 = split_chunk(e0 + L - 1, ck, cm, n);
                res = own;
                for (int c = c0; c <= c1; ++c) {  // ring order of chunk c: x[c-1], then x[c-2] ... x[c]
                    v4u acc = pv[((c - 1 + n) % n) * BS];
                    for (int kk = 2; kk <= n; ++kk) acc = reduce16<OP, T>(pv[((c - kk + n) % n) * BS], acc);
                    if (c0 == c1) {
                        res = acc;
                    } else {  // a vector across chunk boundaries: each lane from its own chunk's fold
                        UT rl[L], al[L];
                        __builtin_memcpy(rl, &res, 16);
                        __builtin_memcpy(al, &acc, 16);
#pragma unroll
                        for (int l = 0; l < L; ++l)
                            if (split_chunk(e0 + l, ck, cm, n) == c) rl[l] = al[l];
                        __builtin_memcpy(&res, rl, 16);
                    }
                }
            }
            if (ll_out) {  // LL result words, planar like the input; the host polls them
                st16(box->out + 16 * i, v4u{res.x, seq, res.y, seq});
                st16(box->out + RDC_SVC_LL_MAX + 16 * i, v4u{res.z, seq, res.w, seq});
            } else {
                st16(box->out + 16 * i, res);
            }
        }
        if (!ok) s_err = 1;
        // plain result: every wave's stores performed at host memory before
        // `done` (LL result words carry their own sequence number)
        if (!ll_out) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (s_err) {
            if (tid == 0) {
                __hip_atomic_store(a.derr, (uint32_t)RDC_KERR_TIMEOUT_RS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                box_store(&box->err, RDC_KERR_TIMEOUT_RS);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                box_store(&box->done, seq);  // the host reads err
            }
            break;
        }
        if (tid == 0) {
            if (a.trace) {
                ts[3] = wall_clock64();
                for (int t = 0; t < 4; ++t)
                    __hip_atomic_store(&box->trace[t], ts[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stamps before `done`
            }
            if (a.strict) __threadfence_system();
            box_store(&box->done, seq);
            s_next = seq + 1u;
        }
        __syncthreads();
    }
    if (tid == 0) box_store(&box->state, RDC_SVC_EXITED);
}

// ============================================================ dispatch ===
// RDC_DEBUG_LDS_PAD=<bytes>: dynamic LDS reserved by every collective launch
// (and counted by the occupancy queries, so the resident-grid clamp follows):
// a debug knob that lowers the blocks per CU, e.g. 96 KiB = one block per CU,
// to rehearse a kernel at another occupancy without changing its code
// (round 4's lost one-shot hand-off happened at one block per CU).
inline unsigned debug_lds_pad() {
    static const unsigned pad = [] {
        const char* v = getenv("RDC_DEBUG_LDS_PAD");
        const long x = v ? atol(v) : 0;
        return (unsigned)(x > 0 && x <= (150l << 10) ? x : 0);
    }();
    return pad;
}

template <int OP, typename T>
struct Kernels {
    static hipError_t reduce(char* dst, const char* src, uint64_t nbytes, int grid, hipStream_t s) {
        if ((((uintptr_t)dst ^ (uintptr_t)src) & 15) == 0) {
            hipLaunchKernelGGL((k_reduce<OP, T, 2>), dim3(grid), dim3(kBlock), 0, s, dst, src, nbytes);
        } else {
            hipLaunchKernelGGL((k_reduce_unaligned<OP, T>), dim3(grid), dim3(kBlock), 0, s, dst, src,
                               nbytes / sizeof(T));
        }
        return hipGetLastError();
    }
    static hipError_t mesh(const CollArgs& a, int grid, hipStream_t s) {
        if (a.n <= 8)
            hipLaunchKernelGGL((k_mesh<OP, T, 8>), dim3(grid), dim3(kBlock), debug_lds_pad(), s, a);
        else
            hipLaunchKernelGGL((k_mesh<OP, T, 16>), dim3(grid), dim3(kBlock), debug_lds_pad(), s, a);
        return hipGetLastError();
    }
    static hipError_t oneshot(const CollArgs& a, int grid, hipStream_t s) {
        if (a.n <= 8)
            hipLaunchKernelGGL((k_oneshot<OP, T, 8>), dim3(grid), dim3(kBlock), debug_lds_pad(), s, a);
        else
            hipLaunchKernelGGL((k_oneshot<OP, T, 16>), dim3(grid), dim3(kBlock), debug_lds_pad(), s, a);
        return hipGetLastError();
    }
    static hipError_t direct(const CollArgs& a, int grid, hipStream_t s) {
        if (a.n <= 8)
            hipLaunchKernelGGL((k_direct<OP, T, 8>), dim3(grid), dim3(kBlock), debug_lds_pad(), s, a);
        else
            hipLaunchKernelGGL((k_direct<OP, T, 16>), dim3(grid), dim3(kBlock), debug_lds_pad(), s, a);
        return hipGetLastError();
    }
    static hipError_t ring(const CollArgs& a, int grid, hipStream_t s) {
        hipLaunchKernelGGL((k_ring<OP, T>), dim3(grid), dim3(kBlock), debug_lds_pad(), s, a);
        return hipGetLastError();
    }
    static hipError_t svc(const SvcArgs& a, hipStream_t s) {
        const bool hx = a.hx != nullptr;
        if (a.n <= 8 && hx)
            hipLaunchKernelGGL((k_svc<OP, T, 8, 512, true>), dim3(1), dim3(512), 0, s, a);
        else if (a.n <= 8)
            hipLaunchKernelGGL((k_svc<OP, T, 8, 512, false>), dim3(1), dim3(512), 0, s, a);
        else if (hx)
            hipLaunchKernelGGL((k_svc<OP, T, 16, 256, true>), dim3(1), dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL((k_svc<OP, T, 16, 256, false>), dim3(1), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    static hipError_t tree(const CollArgs& a, int grid, hipStream_t s) {
        if (a.n <= 8)
            hipLaunchKernelGGL((k_tree<OP, T, 8>), dim3(grid), dim3(kBlock), debug_lds_pad(), s, a);
        else
            hipLaunchKernelGGL((k_tree<OP, T, 16>), dim3(grid), dim3(kBlock), debug_lds_pad(), s, a);
        return hipGetLastError();
    }
    static int occupancy(int kind, int n) {
        // [mesh 8, mesh 16, oneshot 8, oneshot 16, ring, tree 8, tree 16, direct 8, direct 16]; 0 = not queried yet
        static int cache[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        const int wide = n > 8 ? 1 : 0;
        const int slot = kind == RDC_KIND_RING      ? 4
                         : kind == RDC_KIND_TREE    ? 5 + wide
                         : kind == RDC_KIND_ONESHOT ? 2 + wide
                         : kind == RDC_KIND_DIRECT  ? 7 + wide
                                                    : wide;
        if (cache[slot] > 0) return cache[slot];
        int b = 0;
        hipError_t e = hipSuccess;
        switch (slot) {
            case 0: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_mesh<OP, T, 8>, kBlock, debug_lds_pad()); break;
            case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_mesh<OP, T, 16>, kBlock, debug_lds_pad()); break;
            case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_oneshot<OP, T, 8>, kBlock, debug_lds_pad()); break;
            case 3: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_oneshot<OP, T, 16>, kBlock, debug_lds_pad()); break;
            case 5: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_tree<OP, T, 8>, kBlock, debug_lds_pad()); break;
            case 6: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_tree<OP, T, 16>, kBlock, debug_lds_pad()); break;
            case 7: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_direct<OP, T, 8>, kBlock, debug_lds_pad()); break;
            case 8: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_direct<OP, T, 16>, kBlock, debug_lds_pad()); break;
            default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_ring<OP, T>, kBlock, debug_lds_pad()); break;
        }
        if (e != hipSuccess || b <= 0) {
            (void)hipGetLastError();
            b = 1;  // unknown: one block per CU is always resident
        }
        cache[slot] = b;
        return b;
    }
};


#define RDC_SET(T)                        \
    ks->reduce = &Kernels<OP, T>::reduce; \
    ks->mesh = &Kernels<OP, T>::mesh;     \
    ks->ring = &Kernels<OP, T>::ring;     \
    ks->direct = &Kernels<OP, T>::direct; \
    ks->oneshot = &Kernels<OP, T>::oneshot; \
    ks->tree = &Kernels<OP, T>::tree;       \
    ks->svc = &Kernels<OP, T>::svc;         \
    ks->occupancy = &Kernels<OP, T>::occupancy; \
    return true;

// integer element types (every operator)
template <int OP>
inline bool pick_int(int dtype, KernelSet* ks) {
    switch (dtype) {
        case RDC_DT_INT8: RDC_SET(int8_t)
        case RDC_DT_UINT8: RDC_SET(uint8_t)
        case RDC_DT_INT32: RDC_SET(int32_t)
        case RDC_DT_UINT32: RDC_SET(uint32_t)
        case RDC_DT_INT64: case RDC_DT_LONGLONG: RDC_SET(int64_t)
        case RDC_DT_UINT64: case RDC_DT_ULONGLONG: RDC_SET(uint64_t)
        default: return false;
    }
}

// integer and floating element types (Max, Min, Sum)
template <int OP>
inline bool pick_arith(int dtype, KernelSet* ks) {
    if (pick_int<OP>(dtype, ks)) return true;
    switch (dtype) {
        case RDC_DT_FLOAT32: RDC_SET(float)
        case RDC_DT_FLOAT64: RDC_SET(double)
        case RDC_DT_FLOAT16: RDC_SET(_Float16)
        case RDC_DT_BFLOAT16: RDC_SET(bf16_t)
        default: return false;
    }
}
#undef RDC_SET

}  // namespace rdc_amd
