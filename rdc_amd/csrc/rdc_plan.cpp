// Host-side planning (see rdc_plan.h).
#include "rdc_plan.h"

#include <string.h>

#include <algorithm>
#include <functional>
#include <queue>
#include <unordered_map>
#include <unordered_set>

namespace rdc_amd {

namespace {
size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
size_t round_down(size_t x, size_t a) { return x / a * a; }
}  // namespace

Layout MakeLayout(int n, size_t scratch_bytes) {
    Layout L;
    const size_t region = std::min<size_t>(scratch_bytes / 2, kMaxRegionBytes);
    size_t slot = round_down(region / (size_t)n, 4096);
    if (slot < 64 * 1024 || n == 1) slot = 64 * 1024;  // world size 1 never moves data
    L.slot_bytes = slot;
    L.region_bytes = slot * (size_t)n;
    L.max_tiles = (uint32_t)(L.region_bytes / RDC_MIN_TILE + 2);
    // [2n][max_tiles] hand-off flags + done[n] (one word per peer, rdc_kernels.hip launch_done)
    L.flag_bytes = round_up(((size_t)2 * n * L.max_tiles + (size_t)n) * sizeof(uint64_t) * RDC_FLAG_STRIDE, 4096);
    return L;
}

void SplitRanges(int64_t count, int n, int64_t* b, int64_t* e) {
    const int64_t k = count / n, m = count % n;
    for (int i = 0; i < n; ++i) {
        b[i] = (int64_t)i * k + std::min<int64_t>(i, m);
        e[i] = (int64_t)(i + 1) * k + std::min<int64_t>(i + 1, m);
    }
}

int ResidentGrid(int want, int blocks_per_cu, int cus, int ranks_per_gpu, int xcds, int reserve_cus) {
    const long bpc = std::max(1, blocks_per_cu), ranks = std::max(1, ranks_per_gpu);
    cus = std::max(1, cus);
    if (xcds < 1 || cus % xcds != 0) xcds = 1;
    // a dispatch sends workgroup i to XCD i % xcds, so each XCD must hold
    // every rank's share of it; reserved CUs (resident service blocks) may
    // all sit on one XCD, so every XCD gives them up
    long per_xcd = bpc * (cus / xcds) - bpc * std::max(0, reserve_cus);
    // Five or more ranks sharing a GPU at one block per CU keep 3/8 of every
    // XCD's CUs free: with 5 processes x 3 hardware queues, grids filling 30
    // (and 25) of an XCD's 32 CUs left one rank's next kernel undispatched
    // behind its peers' spinning ones in every run (3 of 3), 20 of 32 never
    // (3 of 3), and 5 of 32 passed too (DESIGN.md §4.2 failure 2,
    // profiles/r06/queues/).  2-4 ranks ran full grids through rounds 4-6
    // with no such stall, and the slack cost them 5-7 % (k_direct, N = 2 / 4
    // rehearsals); one rank per GPU never shares.
    if (ranks >= 5 && bpc == 1 && xcds > 1) per_xcd = per_xcd * 5 / 8;
    const long cap = std::max(1L, per_xcd / ranks * xcds);
    return (int)std::max(1L, std::min<long>(want, cap));
}

void PlanTiles(size_t chunk_bytes, int n, int algo, size_t cfg_tile, int max_blocks, Piece* p, MeshSplit split) {
    const int s16 = std::min(std::max(split.s16, 1), 14), r16 = std::min(std::max(split.r16, 1), 15 - s16);
    size_t t = cfg_tile;
    if (t == 0) {
        // ring: each block walks 2(n-1) hand-offs per tile, so one tile per
        // block.  mesh: ~2 tiles per reduce block, at least 64 KiB — every
        // tile costs a flag hand-off per role, and the tile sweep on one GPU
        // (profiles/r01/mesh_tile_sweep_group2.log)
        // found 4 tiles per reduce block too fine below 64 MB (16 MB:
        // 0.115 ms at 22 KiB tiles vs 0.071-0.075 ms at 64-128 KiB), and
        // 16 KiB floors slow at 4 MB (0.044 vs 0.034 ms at 64 KiB).
        const size_t G = (size_t)std::max(1, max_blocks);
        size_t want, lo = RDC_MIN_TILE;
        if (algo == RDC_ALGO_RING) {
            want = chunk_bytes / (G * (size_t)(split.tpb > 0 ? split.tpb : 1));
        } else {
            want = chunk_bytes / ((size_t)(split.tpb > 0 ? split.tpb : 2) * std::max<size_t>(1, G * (size_t)r16 / 16));
            lo = (size_t)64 << 10;
        }
        t = std::min<size_t>(std::max<size_t>(want, lo), (size_t)1 << 20);
    }
    t = std::max<size_t>(round_up(t, RDC_SLOT_ALIGN), RDC_MIN_TILE);
    p->tile_bytes = t;
    const int T = (int)((chunk_bytes + t - 1) / t);
    const int G = std::max(1, max_blocks);
    if (algo == RDC_ALGO_RING) {
        p->nb_scatter = std::max(1, std::min(T, G));
        p->nb_reduce = p->nb_gather = 0;
        return;
    }
    const int items_s = (n - 1) * T;
    const int s = std::max(1, std::min(items_s, G * s16 / 16));
    const int r = std::max(1, std::min(T, G * r16 / 16));
    const int g = std::max(1, std::min(items_s, G - s - r));
    p->nb_scatter = s;
    p->nb_reduce = r;
    p->nb_gather = g;
}

std::vector<Piece> PlanAllreduceRanges(int n, const uint64_t* off, const uint64_t* len, size_t esz,
                                       const Layout& L, int algo, size_t cfg_tile, int max_blocks, MeshSplit split) {
    std::vector<Piece> out;
    if (n <= 1 || esz == 0) return out;
    uint64_t maxlen = 0;
    for (int c = 0; c < n; ++c) maxlen = std::max<uint64_t>(maxlen, len[c]);
    if (maxlen == 0) return out;
    // a piece occupies at most slot - 256 bytes (+ < 16 bytes of alignment slack)
    const uint64_t pe = (uint64_t)(round_down(L.slot_bytes - RDC_SLOT_ALIGN, RDC_SLOT_ALIGN) / esz) * esz;
    const uint64_t npieces = (maxlen + pe - 1) / pe;
    for (uint64_t k = 0; k < npieces; ++k) {
        Piece p;
        memset(&p, 0, sizeof(p));
        size_t chunk_max = 0;
        for (int c = 0; c < n; ++c) {
            const uint64_t b0 = k * pe;
            if (len[c] > b0) {
                p.off[c] = off[c] + b0;
                p.len[c] = std::min<uint64_t>(len[c] - b0, pe);
            }
            // buffer-relative: every rank places chunk c's bytes identically
            p.mis[c] = (uint32_t)(p.off[c] % 16);
            chunk_max = std::max<size_t>(chunk_max, p.len[c]);
        }
        PlanTiles(chunk_max, n, algo, cfg_tile, max_blocks, &p, split);
        for (int c = 0; c < n; ++c) p.tiles[c] = (int)((p.len[c] + p.tile_bytes - 1) / p.tile_bytes);
        out.push_back(p);
    }
    return out;
}

std::vector<Piece> PlanAllreduce(int n, uint64_t count, size_t esz, const Layout& L, int algo, size_t cfg_tile,
                                 int max_blocks) {
    if (n <= 1 || count == 0 || esz == 0) return std::vector<Piece>();
    int64_t cb[RDC_MAX_RANKS], ce[RDC_MAX_RANKS];
    SplitRanges((int64_t)count, n, cb, ce);
    uint64_t off[RDC_MAX_RANKS] = {0}, len[RDC_MAX_RANKS] = {0};
    for (int c = 0; c < n; ++c) {
        off[c] = (uint64_t)cb[c] * esz;
        len[c] = (uint64_t)(ce[c] - cb[c]) * esz;
    }
    return PlanAllreduceRanges(n, off, len, esz, L, algo, cfg_tile, max_blocks);
}

uint64_t OneshotHalfBytes(const Layout& L) { return round_down(L.slot_bytes / 2, RDC_SLOT_ALIGN); }

bool OneshotEligible(int n, uint64_t bytes, const Layout& L, uint64_t push_max) {
    return n > 1 && bytes > 0 && bytes <= OneshotHalfBytes(L) && bytes * (uint64_t)(n - 1) <= push_max;
}

bool OneshotAuto(int n, uint64_t bytes, const Layout& L, uint64_t push_max) {
    if (push_max) return OneshotEligible(n, bytes, L, push_max);  // RDC_ONESHOT_BYTES given: (n-1) x S <= it
    if (!OneshotEligible(n, bytes, L, ~(uint64_t)0)) return false;
    // the one-shot pushes (n-1) x S per rank where the mesh pushes 2(n-1)/n x S,
    // and hands off once instead of twice: worth it while the extra egress
    // (n-1)(n-2)/n x S stays small, and while S is small enough that fixed
    // costs, not bandwidth, decide (n = 2: no extra bytes at all)
    const uint64_t extra = bytes * (uint64_t)(n - 1) * (uint64_t)(n - 2) / (uint64_t)n;
    return bytes <= kOneshotAutoMaxBytes && extra <= kOneshotAutoExtraBytes;
}

int AutoAlgo(int n, uint64_t bytes, const Layout& L, uint64_t push_max) {
    if (OneshotAuto(n, bytes, L, push_max)) return RDC_ALGO_ONESHOT;
    // two ranks: one link either way, and the ring's two steps hand off less
    // than the mesh's three roles; the mesh's all-links egress pays from n = 3
    return n == 2 ? RDC_ALGO_RING : RDC_ALGO_MESH;
}

bool DirectAuto(int n, uint64_t bytes, const Layout& L, uint64_t push_max, uint64_t direct_min) {
    if (n < 2 || direct_min == 0) return false;
    if (direct_min != kDirectMinAuto) return bytes >= direct_min;
    if (bytes < (n == 2 ? kDirectAutoMinBytes2 : kDirectAutoMinBytes)) return false;
    const int a = AutoAlgo(n, bytes, L, push_max);
    return a == RDC_ALGO_RING || a == RDC_ALGO_MESH;
}

Piece PlanOneshot(int n, uint64_t count, size_t esz, const Layout& L, size_t cfg_tile, int max_blocks) {
    int64_t cb[RDC_MAX_RANKS], ce[RDC_MAX_RANKS];
    SplitRanges((int64_t)count, n, cb, ce);
    uint64_t off[RDC_MAX_RANKS] = {0}, len[RDC_MAX_RANKS] = {0};
    for (int c = 0; c < n; ++c) {
        if (ce[c] > cb[c]) {
            off[c] = (uint64_t)cb[c] * esz;
            len[c] = (uint64_t)(ce[c] - cb[c]) * esz;
        }
    }
    return PlanOneshotRanges(n, off, len, count * esz, L, cfg_tile, max_blocks);
}

Piece PlanOneshotRanges(int n, const uint64_t* off, const uint64_t* len, uint64_t total, const Layout& L,
                        size_t cfg_tile, int max_blocks) {
    Piece p;
    memset(&p, 0, sizeof(p));
    for (int c = 0; c < n; ++c) {
        p.off[c] = len[c] ? off[c] : 0;
        p.len[c] = len[c];
    }
    const int G = std::max(1, max_blocks);
    size_t t = cfg_tile ? cfg_tile : std::max<size_t>(total / (size_t)G, RDC_MIN_TILE);
    t = std::max<size_t>(round_up(t, RDC_SLOT_ALIGN), RDC_MIN_TILE);
    (void)L;
    p.tile_bytes = t;
    p.tiles[0] = (int)((total + t - 1) / t);
    p.nb_scatter = std::max(1, std::min(p.tiles[0], G));
    return p;
}

std::vector<Piece> PlanAllgather(int n, const uint64_t* sizes, const Layout& L, size_t cfg_tile, int max_blocks) {
    std::vector<Piece> out;
    if (n <= 1) return out;
    const uint64_t cap = round_down(L.slot_bytes - RDC_SLOT_ALIGN, RDC_SLOT_ALIGN);
    uint64_t maxlen = 0;
    for (int c = 0; c < n; ++c) maxlen = std::max<uint64_t>(maxlen, sizes[c]);
    const uint64_t npieces = (maxlen + cap - 1) / cap;
    const int G = std::max(1, max_blocks);
    for (uint64_t k = 0; k < npieces; ++k) {
        Piece p;
        memset(&p, 0, sizeof(p));
        uint64_t chunk_max = 0;
        for (int c = 0; c < n; ++c) {
            const uint64_t b0 = k * cap;
            if (sizes[c] > b0) {
                p.off[c] = b0;
                p.len[c] = std::min<uint64_t>(cap, sizes[c] - b0);
            }
            p.mis[c] = (uint32_t)(p.off[c] % 16);
            chunk_max = std::max<uint64_t>(chunk_max, p.len[c]);
        }
        size_t t = cfg_tile ? cfg_tile
                            : std::min<size_t>(std::max<size_t>(chunk_max / (size_t)std::max(1, G / 2), RDC_MIN_TILE),
                                               (size_t)1 << 20);
        t = std::max<size_t>(round_up(t, RDC_SLOT_ALIGN), RDC_MIN_TILE);
        p.tile_bytes = t;
        int T = 0;
        for (int c = 0; c < n; ++c) {
            p.tiles[c] = (int)((p.len[c] + t - 1) / t);
            T = std::max(T, p.tiles[c]);
        }
        p.nb_scatter = std::max(1, std::min((n - 1) * T, G / 2));
        p.nb_gather = std::max(1, std::min((n - 1) * T, G - G / 2));
        out.push_back(p);
    }
    return out;
}

std::vector<Piece> PlanBroadcast(uint64_t bytes, const Layout& L, size_t cfg_tile, int max_blocks) {
    std::vector<Piece> out;
    const size_t cap = round_down(L.region_bytes - RDC_SLOT_ALIGN, RDC_SLOT_ALIGN);
    const int G = std::max(1, max_blocks);
    for (uint64_t off = 0; off < bytes; off += cap) {
        Piece p;
        memset(&p, 0, sizeof(p));
        p.off[0] = off;
        p.len[0] = std::min<uint64_t>(cap, bytes - off);
        p.mis[0] = (uint32_t)(off % 16);
        size_t t = cfg_tile ? cfg_tile
                            : std::min<size_t>(std::max<size_t>(p.len[0] / (size_t)G, RDC_MIN_TILE), (size_t)1 << 20);
        t = std::max<size_t>(round_up(t, RDC_SLOT_ALIGN), RDC_MIN_TILE);
        p.tile_bytes = t;
        p.tiles[0] = (int)((p.len[0] + t - 1) / t);
        p.nb_scatter = std::max(1, std::min(p.tiles[0], G));
        out.push_back(p);
    }
    return out;
}

CoalescedPlan PlanCoalesced(int n, const uint64_t* counts, int nbuf, size_t esz, uint64_t unit_max) {
    CoalescedPlan P;
    memset(P.off, 0, sizeof(P.off));
    memset(P.len, 0, sizeof(P.len));
    P.total = 0;
    unit_max = std::max<uint64_t>(round_down(unit_max, 16), 16);
    std::vector<int64_t> cb((size_t)nbuf * RDC_MAX_RANKS), ce((size_t)nbuf * RDC_MAX_RANKS);
    for (int b = 0; b < nbuf; ++b) SplitRanges((int64_t)counts[b], n, &cb[(size_t)b * RDC_MAX_RANKS], &ce[(size_t)b * RDC_MAX_RANKS]);
    uint64_t end = 0;
    for (int c = 0; c < n; ++c) {
        uint64_t at = round_up(end, RDC_SLOT_ALIGN);  // every packed chunk starts 256-B aligned (mis = 0)
        P.off[c] = at;
        for (int b = 0; b < nbuf; ++b) {
            const int64_t b0 = cb[(size_t)b * RDC_MAX_RANKS + c], e0 = ce[(size_t)b * RDC_MAX_RANKS + c];
            if (e0 <= b0) continue;
            const uint64_t so = (uint64_t)b0 * esz, sl = (uint64_t)(e0 - b0) * esz;
            // the segment sits at the same offset mod 16 as its first byte in
            // a 16-B aligned buffer (so % 16: a Split slice of a bucket need
            // not start on 16 B, e.g. 1 MiB / 3), so user memory and scratch
            // stay congruent and every role takes the 16-byte path; packing
            // at 16 B instead made n = 3 / 5 lists run element-wise (2x the
            // plain buffer's time).  Depends on counts only: rank-independent.
            at += so % 16;
            for (uint64_t x = 0; x < sl; x += unit_max) {
                PackUnit u;
                u.buf = (uint64_t)b;
                u.buf_off = so + x;
                u.packed = at + x;
                u.len = std::min<uint64_t>(unit_max, sl - x);
                P.units.push_back(u);
            }
            at = round_up(at + sl, 16);  // next segment from a 16-B boundary
        }
        P.len[c] = at - P.off[c];
        if (P.len[c] == 0) P.off[c] = 0;
        else end = at;
    }
    P.total = end;
    return P;
}

std::vector<uint64_t> PlanDirectItems(int n, int rank, const uint64_t* bytes, int nbuf, size_t esz, uint64_t tile) {
    std::vector<uint64_t> items;
    for (int b = 0; b < nbuf; ++b) {
        int64_t cb[RDC_MAX_RANKS], ce[RDC_MAX_RANKS];
        SplitRanges((int64_t)(bytes[b] / esz), n, cb, ce);
        const uint64_t so = (uint64_t)cb[rank] * esz, sl = (uint64_t)(ce[rank] - cb[rank]) * esz;
        for (uint64_t x = 0; x < sl; x += tile) {
            items.push_back((uint64_t)b);
            items.push_back(so + x);
            items.push_back(std::min<uint64_t>(tile, sl - x));
        }
    }
    return items;
}

// The reference derives the tree in three hash-container passes whose
// iteration order decides who folds first (topo.cc:20-115, communicator_base.cc:
// 136-149, graph.h:70-83, communicator_collective.cc:16-27).  The same
// container operations are replayed here on libstdc++'s unordered_map /
// unordered_set (the toolchain's standard library, as the reference's), so
// each rank's children come out in the reference's order; the CPU tests
// compare every n = 1..16 with the oracle's independent restatement
// (oracle/tree_order.cc).
int PlanTreeProgram(int n, int* dst, int* src) {
    if (n < 2) return 0;
    typedef std::unordered_map<int, std::vector<int>> NbMap;
    // heap tree: parent (r+1)/2-1, children 2r+1, 2r+2 (topo.cc:3-30)
    NbMap heap;
    std::unordered_map<int, int> up;
    for (int r = 0; r < n; ++r) {
        std::vector<int>& v = heap[r];
        if (r > 0) v.push_back((r + 1) / 2 - 1);
        for (int c = 2 * r + 1; c <= 2 * r + 2; ++c)
            if (c < n) v.push_back(c);
        up[r] = (r + 1) / 2 - 1;
    }
    // ring positions: DFS order with the last child's segment reversed (topo.cc:32-94)
    std::function<std::vector<int>(int)> walk = [&](int r) {
        std::vector<int> seq(1, r), kids;
        for (int x : heap[r])
            if (x != up[r]) kids.push_back(x);
        for (size_t i = 0; i < kids.size(); ++i) {
            std::vector<int> part = walk(kids[i]);
            if (i + 1 == kids.size()) std::reverse(part.begin(), part.end());
            seq.insert(seq.end(), part.begin(), part.end());
        }
        return seq;
    };
    const std::vector<int> order = walk(0);
    std::vector<int> pos((size_t)n);
    for (int i = 0; i < n; ++i) pos[(size_t)order[(size_t)i]] = i;
    // relabelled neighbour lists, built by walking the heap map (topo.cc:95-106)
    NbMap rel;
    for (const auto& kv : NbMap(heap))
        for (int x : kv.second) rel[pos[(size_t)kv.first]].push_back(pos[(size_t)x]);
    // adjacency sets from the edge list of a copy (communicator_base.cc:136-149),
    // with graph.h:79-80's insertion of `to` into its own set
    std::unordered_map<int, std::unordered_set<int>> adj;
    for (const auto& kv : NbMap(rel))
        for (int x : kv.second) {
            std::unordered_set<int>& a = adj[kv.first];
            if (!a.count(x)) a.emplace(x);
            std::unordered_set<int>& b = adj[x];
            if (!b.count(kv.first)) b.emplace(x);
        }
    // levels from rank 0 (graph.h:45-67); children in the order a fresh
    // unordered_set returns them (communicator_collective.cc:19-27)
    std::vector<int> level((size_t)n, -1);
    std::queue<int> q;
    q.push(0);
    level[0] = 0;
    while (!q.empty()) {
        const int v = q.front();
        q.pop();
        for (int w : adj[v])
            if (level[(size_t)w] < 0) {
                level[(size_t)w] = level[(size_t)v] + 1;
                q.push(w);
            }
    }
    std::vector<std::vector<int>> kids((size_t)n);
    for (int r = 0; r < n; ++r) {
        std::unordered_set<int> from;
        for (int x : std::unordered_set<int>(adj[r]))
            if (level[(size_t)x] == level[(size_t)r] + 1) from.insert(x);
        kids[(size_t)r].assign(from.begin(), from.end());
    }
    int k = 0;
    std::function<void(int)> emit = [&](int v) {  // post-order: a subtree is complete before it is folded
        for (int c : kids[(size_t)v]) {
            emit(c);
            dst[k] = v;
            src[k] = c;
            ++k;
        }
    };
    emit(0);
    return k;
}

// Bytes one rank's kernels load and store for an allreduce of `count`
// elements (16-B lanes and element-wise edges alike, each byte once per
// access), per the kernels' loops (rdc_kernels_impl.h), with chunk c =
// utils::Split(0, count, n) = len[c] bytes:
//   ring (TryReduceScatterRing + TryAllgatherRing):
//     RS step j: send chunk (r+1+j)%n (load user, store into prev's scratch),
//                receive chunk (r+2+j)%n (load scratch + user, store user);
//     AG step j: send chunk (r+j)%n (load user, store into prev's scratch),
//                receive chunk (r+1+j)%n (load scratch, store user)
//   mesh: scatter every other chunk to its owner (load user, store remote);
//         fold own chunk (load n-1 slots + user, store user + n-1 remote);
//         gather every other chunk (load own AG slot, store user)
//   mesh (pull): stage every other chunk in own scratch (load user, store
//         local); fold own chunk (load n-1 peers' staged tiles remotely +
//         user, store user + own AG slot); gather (load owners' AG, store user)
//   one-shot / tree: push the whole buffer to n-1 peers (each push loads the
//         user bytes again), fold every element over the n inputs (load
//         n-1 slots + user, store user)
// A remote store or load is counted at the rank that issues it (the counters
// of the issuing GPU's L2 see it); egress = bytes that leave this rank's
// memory for a peer (its remote stores; for the pull mode, what peers load).
HbmBytes ModelHbmBytes(int n, uint64_t count, size_t esz, int algo) {
    HbmBytes h;
    if (n < 2 || count == 0) return h;
    int64_t cb[RDC_MAX_RANKS], ce[RDC_MAX_RANKS];
    SplitRanges((int64_t)count, n, cb, ce);
    uint64_t len[RDC_MAX_RANKS];
    for (int c = 0; c < n; ++c) len[c] = (uint64_t)(ce[c] - cb[c]) * esz;
    const uint64_t S = count * esz;
    for (int r = 0; r < n; ++r) {  // every rank; the rank-averaged figure is reported
        uint64_t rd = 0, wr = 0, eg = 0;
        if (algo == RDC_ALGO_RING) {
            for (int j = 0; j + 1 < n; ++j) {
                const uint64_t cs = len[(r + 1 + j) % n], cr = len[(r + 2 + j) % n];
                rd += cs + 2 * cr;
                wr += cs + cr;
                eg += cs;
                const uint64_t as = len[(r + j) % n], ar = len[(r + 1 + j) % n];
                rd += as + ar;
                wr += as + ar;
                eg += as;
            }
        } else if (algo == RDC_ALGO_MESH) {
            const uint64_t others = S - len[r];
            rd += others + (uint64_t)n * len[r] + others;
            wr += others + (uint64_t)n * len[r] + others;
            eg += others + (uint64_t)(n - 1) * len[r];
        } else if (algo == RDC_ALGO_MESH_PULL) {
            // stage others locally; fold loads n-1 peers' staged tiles (remote
            // loads, counted here: this GPU's L2 issues them) + user, stores
            // user + own AG slot; gather loads owners' results (remote)
            const uint64_t others = S - len[r];
            rd += others + (uint64_t)n * len[r] + others;
            wr += others + 2 * len[r] + others;
            eg += others + (uint64_t)(n - 1) * len[r];  // what peers load from this rank's memory
        } else if (algo == RDC_ALGO_DIRECT) {
            // owner r loads chunk r of all n user buffers (n-1 of them remote)
            // and stores the result into all n; no scratch
            rd += (uint64_t)n * len[r];
            wr += (uint64_t)n * len[r];
            eg += (uint64_t)(n - 1) * len[r] + (S - len[r]);  // pushed results + what peers load from here
        } else {  // one-shot / tree order
            rd += (uint64_t)(n - 1) * S + (uint64_t)n * S;
            wr += (uint64_t)(n - 1) * S + S;
            eg += (uint64_t)(n - 1) * S;
        }
        h.read_max = std::max(h.read_max, rd);
        h.write_max = std::max(h.write_max, wr);
        h.read_sum += rd;
        h.write_sum += wr;
        h.egress_max = std::max(h.egress_max, eg);
    }
    return h;
}

// the intersection of piece [lo, hi) with every Split chunk, relative to lo:
// range q = the piece's bytes of chunk q, owned by rank q (its ring order)
static void piece_ranges(uint64_t lo, uint64_t hi, int n, const int64_t* cb, const int64_t* ce, size_t esz, uint64_t* roff,
                  uint64_t* rlen, int8_t* fold) {
    for (int q = 0; q < n; ++q) {
        const uint64_t a = std::max<uint64_t>(lo, (uint64_t)cb[q] * esz);
        const uint64_t b = std::min<uint64_t>(hi, (uint64_t)ce[q] * esz);
        roff[q] = b > a ? a - lo : 0;
        rlen[q] = b > a ? b - a : 0;
        fold[q] = (int8_t)q;
    }
}

// The same piece as n BALANCED ranges.  A contiguous piece lies in one or two
// Split chunks, so with piece_ranges one owner folds (nearly) all of it and
// every other rank only copies — on one GPU per rank that puts the piece's
// whole exchange on the owner's links.  Here the bytes of each chunk the
// piece meets are cut into parts over the ranks (in proportion to their
// length, at least one rank per chunk); every part is folded by its rank in
// the ring order of the chunk it belongs to (fold), so every element keeps
// its reference bits.  false (use piece_ranges) when the piece meets more
// chunks than there are ranks.
static bool balanced_ranges(uint64_t lo, uint64_t hi, int n, const int64_t* cb, const int64_t* ce, size_t esz,
                     uint64_t* roff, uint64_t* rlen, int8_t* fold) {
    int segc[RDC_MAX_RANKS], m = 0;
    uint64_t sega[RDC_MAX_RANKS], segb[RDC_MAX_RANKS];
    for (int q = 0; q < n; ++q) {
        const uint64_t a = std::max<uint64_t>(lo, (uint64_t)cb[q] * esz);
        const uint64_t b = std::min<uint64_t>(hi, (uint64_t)ce[q] * esz);
        if (b > a) {
            segc[m] = q;
            sega[m] = a;
            segb[m] = b;
            ++m;
        }
    }
    if (m == 0 || m > n) return false;
    int k[RDC_MAX_RANKS];
    for (int s = 0; s < m; ++s) k[s] = 1;
    for (int extra = n - m; extra > 0; --extra) {  // the next rank to the segment with the most bytes per rank
        int best = 0;
        for (int s = 1; s < m; ++s)
            if ((segb[s] - sega[s]) * (uint64_t)k[best] > (segb[best] - sega[best]) * (uint64_t)k[s]) best = s;
        ++k[best];
    }
    int i = 0;
    for (int s = 0; s < m; ++s) {
        const uint64_t E = (segb[s] - sega[s]) / esz, base = E / (uint64_t)k[s], rem = E % (uint64_t)k[s];
        uint64_t at = sega[s];
        for (int j = 0; j < k[s]; ++j, ++i) {
            const uint64_t cnt = base + ((uint64_t)j < rem ? 1 : 0);
            roff[i] = at - lo;
            rlen[i] = cnt * esz;
            fold[i] = (int8_t)segc[s];
            at += cnt * esz;
        }
    }
    return true;
}


void HostPieceRanges(uint64_t lo, uint64_t hi, int n, const int64_t* cb, const int64_t* ce, size_t esz, bool balanced,
                     uint64_t* roff, uint64_t* rlen, int8_t* fold) {
    if (!balanced || !balanced_ranges(lo, hi, n, cb, ce, esz, roff, rlen, fold))
        piece_ranges(lo, hi, n, cb, ce, esz, roff, rlen, fold);
}

std::vector<int> GroupCoalesced(const uint64_t* counts, int nbuf, size_t esz, uint64_t fuse_bytes) {
    std::vector<int> bounds;
    bounds.push_back(0);
    uint64_t acc = 0;
    for (int b = 0; b < nbuf; ++b) {
        const uint64_t s = counts[b] * esz;
        if (b > bounds.back() && acc + s > fuse_bytes) {
            bounds.push_back(b);
            acc = 0;
        }
        acc += s;
    }
    if (nbuf > 0) bounds.push_back(nbuf);
    return bounds;
}

}  // namespace rdc_amd
