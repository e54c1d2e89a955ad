// Host-side planning of one device collective: chunk map, pieces, tiles and
// block roles.  Pure functions (no HIP calls), so the CPU tests exercise the
// exact logic the launches use (exported as RdcPlanAllreduce/RdcPlanLayout).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "rdc_common.h"

namespace rdc_amd {

// scratch geometry of one communicator (identical on every rank)
struct Layout {
    size_t slot_bytes = 0;    // one slot = one chunk piece (+ alignment slack)
    size_t region_bytes = 0;  // n slots; RS and AG regions are separate allocations
    uint32_t max_tiles = 0;   // flag-row length
    size_t flag_bytes = 0;    // [2n][max_tiles] + done[n] uint64 sequence words, rounded to 4 KiB
};
// RS / AG regions are capped below 2 GiB: on ROCm 7.2 (dmabuf IPC)
// hipIpcOpenMemHandle of an allocation >= 2 GiB never returns
// (measured on MI355X: 2044 MiB opens, 2048 MiB hangs).
constexpr size_t kMaxRegionBytes = (size_t)2040 << 20;
Layout MakeLayout(int n, size_t scratch_bytes);

// utils::Split (include/utils/utils.h:59-70) in 64-bit arithmetic: the first
// count % n chunks get one extra element; same ranges as the reference for
// every count its int version can represent.
void SplitRanges(int64_t count, int n, int64_t* begin, int64_t* end);

struct Piece {
    uint64_t off[RDC_MAX_RANKS];  // byte offset of chunk c's piece in the user buffer
    uint64_t len[RDC_MAX_RANKS];  // byte length (0 = chunk c has nothing in this piece)
    uint32_t mis[RDC_MAX_RANKS];  // off % 16: where the piece sits inside its scratch slot
    int tiles[RDC_MAX_RANKS];     // ceil(len / tile_bytes)
    uint64_t tile_bytes;
    int nb_scatter, nb_reduce, nb_gather;  // mesh roles; ring uses nb_scatter as its grid
};

// Mesh role split of the grid in sixteenths: scatter s16/16, reduce r16/16,
// gather the rest (default 4 / 8 / 4: profiles/r02/ split sweep, 2 ranks on one GPU,
// 1 GiB 1.69 -> 1.54 ms at 512 blocks against 6 / 6 / 4 — the reduce role has
// the most work per byte: n loads, n stores).
struct MeshSplit {
    int s16 = 4, r16 = 8;
    // automatic tiles per block (0 = default: 2 per mesh reduce block, 1 per
    // ring block); bounded to [64 KiB (mesh) / RDC_MIN_TILE (ring), 1 MiB].
    // Set by Communicator::Autotune; scales with the buffer like the default.
    int tpb = 0;
};
// Grid of a launch whose blocks wait on peers' blocks.  Every waiting block of
// every rank must be resident at once, or a rank's waiters can occupy the CUs
// its own (or a co-located rank's) producers need: the launch then ends in the
// device timeout (4 ranks on one GPU, k_ring at 768 blocks each, round 1).
// Residency = blocks_per_cu (hipOccupancyMaxActiveBlocksPerMultiprocessor of
// the kernel) x cus / ranks_per_gpu (the most ranks sharing one physical GPU).
// Every rank computes it from the same exchanged values, so the grid — and
// the tile plan derived from it — is identical on all ranks.
int ResidentGrid(int want, int blocks_per_cu, int cus, int ranks_per_gpu, int xcds = 1, int reserve_cus = 0);

// tile size and grid for a piece whose largest chunk is chunk_bytes
void PlanTiles(size_t chunk_bytes, int n, int algo, size_t cfg_tile, int max_blocks, Piece* p,
               MeshSplit split = MeshSplit());

// Every launch of an allreduce of `count` elements of `esz` bytes.
std::vector<Piece> PlanAllreduce(int n, uint64_t count, size_t esz, const Layout& L, int algo, size_t cfg_tile,
                                 int max_blocks);

// One-shot allreduce (whole buffer pushed to every peer): eligible when the
// buffer fits half a slot and the total pushed bytes (n-1) x S stay within
// push_max.  off/len = the Split chunk byte ranges; tiles[0] tiles over the
// whole buffer; nb_scatter = grid.
bool OneshotEligible(int n, uint64_t bytes, const Layout& L, uint64_t push_max);
// The automatic choice between one-shot and mesh.  push_max != 0
// (RDC_ONESHOT_BYTES set): one-shot while (n-1) x bytes <= push_max.  0: one-
// shot while bytes <= kOneshotAutoMaxBytes and the extra egress over the mesh,
// (n-1)(n-2)/n x bytes, <= kOneshotAutoExtraBytes — n = 2: up to 8 MiB, n = 3:
// 6 MiB, n = 4: 2.7 MiB, n = 8: 0.76 MiB.  Measured with 2-4 ranks on one GPU
// (tools/algo_sweep.py, profiles/r02/algo_sweep_*.log): the one-shot is the
// fastest schedule up to 8 MiB at n = 2 (1.6x the mesh at 2-8 MiB) and up to
// 8-16 MiB at n = 3, 4.
constexpr uint64_t kOneshotAutoMaxBytes = (uint64_t)8 << 20;
constexpr uint64_t kOneshotAutoExtraBytes = (uint64_t)4 << 20;
bool OneshotAuto(int n, uint64_t bytes, const Layout& L, uint64_t push_max);
// RDC_ALGO=auto: the one-shot by OneshotAuto, else the ring at n = 2 (one link
// either way; measured 16 MiB 0.028 vs 0.036 ms, 1 GiB 1.71 vs 1.74 ms with 2
// ranks on one GPU) and the mesh from n = 3 (all n-1 links)
int AutoAlgo(int n, uint64_t bytes, const Layout& L, uint64_t push_max);
// Round 6: the registered-buffer schedule (RDC_ALGO_DIRECT) for an untuned
// RDC_ALGO=auto call on a multi-process channel whose direct self-check
// passed.  direct_min (RDC_DIRECT_BYTES): kDirectMinAuto (the default) = where
// AutoAlgo picks a two-hand-off schedule (ring or mesh, i.e. above the
// one-shot sizes) and the buffer is at least kDirectAutoMinBytes (n >= 3) or
// kDirectAutoMinBytes2 (n = 2); 0 = never; otherwise from direct_min bytes.
// Why there: the direct schedule moves 2 S of HBM per rank where the ring
// moves 9(n-1)/n S and the pull mesh (5n-2)/n S (ModelHbmBytes), the same
// link bytes as the mesh, and pays one host rendezvous per call (two
// shared-memory stamps: 2-3 us at n = 2, 6-11 us at n = 8, export ~1 us of
// it) and one hand-off where the mesh has two.  Per-size sweep, ranks on one
// GPU (tools/algo_sweep.py, profiles/r06/direct_default/): n = 8 direct
// 0.117 vs pull mesh 0.103 ms at 4 MiB, 0.142 vs 0.164 at 16 MiB, 0.81 vs
// 1.92 at 256 MiB; n = 2 direct 0.0315 vs ring 0.0258 ms at 16 MiB, 0.064 vs
// 0.090 at 64 MiB.
constexpr uint64_t kDirectMinAuto = ~(uint64_t)0;
constexpr uint64_t kDirectAutoMinBytes = (uint64_t)16 << 20;
constexpr uint64_t kDirectAutoMinBytes2 = (uint64_t)32 << 20;
bool DirectAuto(int n, uint64_t bytes, const Layout& L, uint64_t push_max, uint64_t direct_min);
uint64_t OneshotHalfBytes(const Layout& L);
Piece PlanOneshot(int n, uint64_t count, size_t esz, const Layout& L, size_t cfg_tile, int max_blocks);

// Allgather of n per-rank buffers of sizes[c] bytes: pieces of at most one
// slot per source rank (off/len/mis/tiles per source c; nb_scatter = push
// blocks, nb_gather = gather blocks).
std::vector<Piece> PlanAllgather(int n, const uint64_t* sizes, const Layout& L, size_t cfg_tile, int max_blocks);

// Broadcast pieces of `bytes` (use off/len/mis/tiles [0]).
std::vector<Piece> PlanBroadcast(uint64_t bytes, const Layout& L, size_t cfg_tile, int max_blocks);

// Allreduce pieces over explicit per-chunk byte ranges [off[c], off[c]+len[c])
// of one buffer (PlanAllreduce is this with the Split ranges; the coalesced
// path passes the packed chunk ranges).  Each range length is a multiple of esz.
std::vector<Piece> PlanAllreduceRanges(int n, const uint64_t* off, const uint64_t* len, size_t esz,
                                       const Layout& L, int algo, size_t cfg_tile, int max_blocks,
                                       MeshSplit split = MeshSplit());
Piece PlanOneshotRanges(int n, const uint64_t* off, const uint64_t* len, uint64_t total, const Layout& L,
                        size_t cfg_tile, int max_blocks);

// ------------------------------------------------------ tree allreduce ---
// rdc_reduce_ring_mincount (communicator_manager.cc:46): TryAllreduce takes
// TryAllreduceTree for buffers of at most that many bytes
// (communicator_collective.cc:6-13): TryReduceTree to rank 0 over the tree of
// GetLinkMap (src/utils/topo.cc:80-115) as the communicator's UndirectedGraph
// holds it (communicator_base.cc:113-150, include/utils/graph.h:45-83), then
// TryBroadcast from rank 0.  Rank r folds its children's subtree results
// into its own buffer one by one, own = OP(own, child), in the iteration
// order of the unordered_set the reference collects them in (:14-33).
// The fold as a post-order program over the n inputs: acc[dst[i]] =
// OP(acc[dst[i]], acc[src[i]]) for i < n-1, result acc[0].  Returns n-1.
int PlanTreeProgram(int n, int* dst, int* src);

// ---------------------------------------------------- coalesced allreduce ---
// Many buffers reduced as one launch sequence (BASELINE cfg5: 1024 x 1 MiB,
// test/mallreduce.cc's back-to-back shape).  The ring order of an element
// depends only on its Split chunk index c (s = x[c-1]; ...;
// s = OP(x[c], s)), so chunk c of EVERY buffer can be owned and folded
// together: the buffers are packed chunk-major into one staging image
//     [ chunk 0: buf0.c0 | buf1.c0 | ... ][ chunk 1: buf0.c1 | buf1.c1 | ... ] ...
// (each segment 16-B aligned), the normal schedule runs on that image with
// chunk c = the packed chunk-c range, and the segments are copied back.
// Every element is folded in its own buffer's ring order: bit-identical to
// one rdc::Allreduce per buffer.
struct PackUnit {       // one copy between a user buffer and the staging image
    uint64_t buf;       // buffer index (host plan) / user address (device table)
    uint64_t buf_off;   // byte offset in that buffer
    uint64_t packed;    // byte offset in the staging image
    uint64_t len;       // bytes (<= unit_max)
};
struct CoalescedPlan {
    uint64_t off[RDC_MAX_RANKS];  // packed chunk c = [off[c], off[c]+len[c])
    uint64_t len[RDC_MAX_RANKS];
    uint64_t total;               // staging bytes
    std::vector<PackUnit> units;
};
constexpr uint64_t kPackUnitMax = 128 << 10;
CoalescedPlan PlanCoalesced(int n, const uint64_t* counts, int nbuf, size_t esz, uint64_t unit_max = kPackUnitMax);

// Owner `rank`'s items of a coalesced direct launch (k_direct over a list):
// Split chunk `rank` of every buffer (bytes[b] / esz elements) in pieces of
// at most `tile` bytes, as {buffer, byte offset in it, bytes} triples.
std::vector<uint64_t> PlanDirectItems(int n, int rank, const uint64_t* bytes, int nbuf, size_t esz, uint64_t tile);
// Cut the buffer list (in order) into fusion groups of at most fuse_bytes of
// data each; a buffer larger than fuse_bytes forms a group of its own.
// Returns group boundaries: group g = buffers [bounds[g], bounds[g+1]).
std::vector<int> GroupCoalesced(const uint64_t* counts, int nbuf, size_t esz, uint64_t fuse_bytes);

// One host-path piece [lo, hi) (rdc_host.cpp) as the n ranges of its
// allreduce: range q = [lo + roff[q], + rlen[q]) owned by rank q, folded in
// the ring order of Split chunk fold[q].  Chunk-owned (the piece's bytes of
// chunk q to rank q) or, `balanced`, each chunk's bytes cut over the ranks.
// (cb, ce: the Split element ranges; esz: element bytes.)
void HostPieceRanges(uint64_t lo, uint64_t hi, int n, const int64_t* cb, const int64_t* ce, size_t esz, bool balanced,
                     uint64_t* roff, uint64_t* rlen, int8_t* fold);

// HBM byte model of one allreduce (rdc_plan.cpp ModelHbmBytes): bytes the
// kernels load / store, per rank (max over ranks) and summed over ranks,
// plus the most remote-store (link egress) bytes of any rank
struct HbmBytes {
    uint64_t read_max = 0, write_max = 0, read_sum = 0, write_sum = 0, egress_max = 0;
};
HbmBytes ModelHbmBytes(int n, uint64_t count, size_t esz, int algo);

}  // namespace rdc_amd
