// Device communicator of the MI355X rdc path — the counterpart of the
// reference's comm::Communicator (include/comm/communicator_base.h:37-283)
// with its TCP link mesh replaced by IPC-mapped HBM scratch on every peer GPU.
//
// HBM layout per rank (uncached allocations, IPC-exported, each < 2 GiB):
//   RS region : n slots x slot_bytes      AG region : n slots x slot_bytes
// and a flag array (uncached, IPC-exported): uint32 [2n][max_tiles] + done[n].
//   mesh : RS slot p  <- rank p's copy of my chunk;   AG slot c <- owner c's result
//   ring : RS slot j  <- reduce-scatter step j;       AG slot j <- allgather step j
//   bcast: the whole AG region holds the root's piece
// Every launch carries seq (same on all ranks, +1 per launch); a flag word
// equal to seq means "this tile of this launch has landed".
#pragma once
#include <hip/hip_runtime_api.h>

#include <map>
#include <mutex>
#include <set>
#include <memory>
#include <string>
#include <vector>

#include "rdc_bootstrap.h"
#include "rdc_common.h"
#include "rdc_plan.h"

#include "rdc_vmem.h"

namespace rdc_amd {

struct CommConfig {
    size_t scratch_bytes = (size_t)4080 << 20;  // RS + AG regions (2 x 2040 MiB), per rank
    int algo = RDC_ALGO_AUTO;
    int max_blocks = 0;                      // 0 = auto
    size_t tile_bytes = 0;                   // 0 = auto
    double timeout_s = 60.0;                 // device-side wait limit
    size_t oneshot_push_max = 0;  // RDC_ONESHOT_BYTES: 0 = size/rank-aware rule (rdc_plan.h OneshotAuto)
    size_t fuse_bytes = (size_t)256 << 20;      // coalesced allreduce: data bytes per fusion group
    size_t p2p_slot_bytes = (size_t)4 << 20;    // Send/Recv: piece size (2 slots per ordered rank pair)
    bool coalesce_fused = true;                 // coalesced mesh reads/writes user buffers directly (no image)
    size_t fuse_bytes_direct = (size_t)16 << 30;  // ... in groups of up to this many data bytes
    size_t bcast_split_bytes = (size_t)1 << 20;   // broadcast pieces from this size: root -> forwarders -> ranks
    MeshSplit mesh_split;                          // mesh roles in sixteenths of the grid (RDC_MESH_SPLIT=s,r)
    // rdc_reduce_ring_mincount (src/comm/communicator_manager.cc:46, default 1
    // byte): allreduces of at most this many bytes take the reference's tree
    // order instead of the ring's (communicator_collective.cc:6-13)
    size_t ring_mincount = 1;
    // RDC_DIRECT_BYTES: which untuned automatic allreduces on multi-process
    // channels take the registered-buffer schedule (RDC_ALGO_DIRECT) when every
    // rank's buffer can be mapped and the channel's self-check passed: "auto"
    // (kDirectMinAuto, the default: rdc_plan.h DirectAuto), 0 = only when
    // asked for (algo 6, RDC_ALGO=direct) or autotuned, N = from N bytes
    uint64_t direct_min = kDirectMinAuto;
    // RDC_POISON_SCRATCH=1: consumers overwrite every scratch range they
    // finished reading with 0xFF bytes (debug mode, rdc_device.h block_poison)
    int poison = 0;
};

struct KernelSet;
struct P2PCtl;
class P2PEngine;
class WorkComp;
class SmallService;

// The collective state of one set of ranks: the RS / AG scratch regions, the
// flag array, the device error word and launch counter, and the peers' IPC
// mappings of all of them.  Communicators created over the same bootstrap
// (every named communicator of the process: "main", "second", the
// checkpoint-style ones) SHARE one channel instead of 4 GiB of scratch and
// n-1 peer mappings each: their launches are serialised on the channel in
// issue order (stream order; a launch on another stream than the channel's
// previous one waits for it by event), which every rank issues identically —
// the reference's collectives block the caller, so its communicators see
// one global order too.  Point-to-point stays per communicator (messages on
// different communicators must not match each other).  RDC_SHARE_SCRATCH=0
// gives every communicator its own channel.
struct Channel {
    ~Channel();  // closes the peers' mappings (collective over bs) and frees
    // serialise a call on `s` behind the channel's previous one (only when
    // several communicators use the channel) / record the call's end on `s`
    void Order(hipStream_t s);
    void Mark(hipStream_t s);

    Bootstrap* bs = nullptr;   // not owned; null for single-process groups
    uint64_t id = 0;           // per-bootstrap creation index (equal on every rank)
    int rank = 0, n = 1, device = 0;
    bool ipc = false;          // peers' regions opened through IPC
    Layout L;
    int alloc_kind = 0;
    // kind of each region (scratch, ag, flags, service slots; rdc_comm.cpp
    // "Region kinds": 0 hipDeviceMallocUncached = MTYPE CC, 3 HSA-uncached =
    // MTYPE UC, ...), their sizes, and the kinds of the peers' regions mapped here
    int region_kind[4] = {};
    size_t region_bytes[4] = {};
    int8_t peer_kind[4][RDC_MAX_RANKS] = {};
    char* scratch = nullptr;
    char* scratch_ag = nullptr;
    uint64_t* flags = nullptr;
    uint32_t* err = nullptr;           // [0] error word, [16] arrivals, [32] launches, [48] last kind
    uint32_t* err_host = nullptr;      // pinned: [0] error mirror, [4] notify token
    uint32_t* err_host_dev = nullptr;
    char* peer_scratch[RDC_MAX_RANKS] = {};
    char* peer_ag[RDC_MAX_RANKS] = {};
    uint64_t* peer_flags[RDC_MAX_RANKS] = {};
    // small-allreduce service slots (rdc_service.h): [2 halves][n] x
    // RDC_SVC_SLOT_BYTES of LL words per rank, IPC-mapped
    char* svc_region = nullptr;
    char* peer_svc_region[RDC_MAX_RANKS] = {};
    // the service's host exchange: [2 halves][n] x RDC_SVC_HX_RANK_BYTES of
    // shared host memory every rank maps (null: RDC_HOST_SERVICE_HX_BYTES=0)
    std::shared_ptr<char> svc_hx;
    std::unique_ptr<SmallService> svc;  // started on first use
    bool svc_enabled = false;          // agreed at creation: the service may run on this channel
    bool svc_counted = false;          // counted in the process's per-device service registry
    std::mutex mu;
    int users = 0;                     // communicators attached
    uint32_t attached = 0;             // communicators ever attached (the next one's tag)
    uint32_t notify_token = 0;
    hipEvent_t last_ev = nullptr;
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    // registered-buffer allreduce (RDC_ALGO_DIRECT, Communicator::AllreduceDirect):
    // per-call rendezvous slots in shared host memory ([2 parities][n] DirectDesc,
    // multi-process channels only), the rendezvous count, the peers' buffers
    // mapped here (by (peer, HIP buffer id); open until the channel closes or
    // RdcCommDirectRelease) and this rank's exported allocations by base
    // address (kept for the channel's life: see AllreduceDirect)
    std::shared_ptr<char> dreg;
    uint64_t dcalls = 0;
    struct DirectMap {
        char* ptr = nullptr;
        size_t size = 0;
    };
    std::map<std::pair<int, uint64_t>, DirectMap> dmaps;
    struct DirectExport {
        hipIpcMemHandle_t handle;
        uint64_t id = 0;
        size_t size = 0;
        bool verified = false;  // a call ran direct on it: its importers checked the canary
    };
    std::map<uintptr_t, DirectExport> dexports;
    uintptr_t dscan = 0;              // retirement scan cursor (a base address in dexports)
    hipEvent_t dlast = nullptr;       // recorded after this rank's latest direct launch
    // round 6, RDC_DIRECT_IMPORT=vmem: peers' allocations mapped at addresses
    // this process chooses (dma-buf + ROCr vmem, rdc_vmem.h); null: HIP IPC
    // (the default, or a rank could not set it up)
    std::unique_ptr<VmemImporter> vmem;
    // address ranges this process unmapped (closed peer mappings) or whose
    // allocation it retired (own exports): a new peer mapping that lands
    // partly over one is refused (DirectMapPeers; round 5 and round 6 faulted
    // at the first launch through such a mapping), and the peer allocation
    // it maps stays refused
    std::vector<std::pair<uintptr_t, size_t>> dclosed;
    std::set<std::pair<int, uint64_t>> drefused;
    // host cost of the per-call rendezvous (RdcCommGetParam "direct_*")
    uint64_t dstat_calls = 0, dstat_rdv_ns = 0, dstat_export_ns = 0, dstat_closed = 0, dstat_retired = 0;
    uint64_t dstat_close_wait_ns = 0, dstat_refused = 0;
    // calls that fell back (every rank alike), calls whose lists were not
    // usable, mapping failures on this rank and the last one's reason
    // (1 table full, 2 refused earlier, 3 open failed, 4 a mapping already
    // held, 5 lands partly over unmapped ranges: refused, 6 the canary shows
    // another buffer object: refused)
    uint64_t dstat_fallback = 0, dstat_unusable = 0, dstat_mapfail = 0, dfail_reason = 0;
    // exports of this rank's allocations that HIP refused, the last hipError_t
    uint64_t dstat_exportfail = 0, dexport_err = 0;
    bool direct_off = false;  // RdcCommDirectRelease ran: the direct schedule stays off
    void* tune_buf = nullptr;  // Autotune's buffer, kept (peers map it) until the channel closes
    size_t tune_bytes = 0;
    std::vector<void*> tune_old;  // outgrown tune buffers: never freed before the channel closes (a
                                  // freed address handed out again could not be exported)
    int direct_check = 0;         // DirectSelfCheck: 0 not run, 1 passed, 2 failed
    uint64_t* tlog = nullptr;     // RDC_LAUNCH_TIMES=1: 64 x {seq, block 0 start, latest block start, end} ticks
    // the canary check of new peer mappings: a private stream and a pinned word
    hipStream_t dpeek_stream = nullptr;
    uint64_t* dpeek_host = nullptr;
    uint64_t dstat_canary = 0;    // new peer mappings checked by their canary
};

// One rank's slot of the registered-buffer rendezvous (shared host memory):
// the call's buffers (one, or a coalesced list), each as (allocation, offset),
// and the allocations they live in with their IPC handles.
constexpr int kDirectAllocsMax = 1024;  // allocations per call (torch's small pool: 2 MiB segments)
constexpr int kDirectBufsMax = 4096;    // buffers per call (a longer list takes the scratch schedules)
struct DirectAlloc {
    uint64_t id;                        // HIP_POINTER_ATTRIBUTE_BUFFER_ID
    hipIpcMemHandle_t handle;
    // exported in this call: canary_len (<= 8) bytes at canary_off hold the
    // low bytes of `nonce` until the second rendezvous stamp (every importer
    // reads them through its new mapping); canary_len 0 = not checked
    uint64_t nonce, canary_off, canary_len;
};

// the read (<= 8 bytes) an importer checks a new mapping with (rdc_peek.hip)
hipError_t Peek(const void* src, uint32_t len, void* dst, hipStream_t s);
// the exporter's write of the canary (and of the original bytes back)
hipError_t Poke(void* dst, uint32_t len, uint64_t v, hipStream_t s);
struct DirectBuf {
    uint32_t alloc;                     // index into alloc[]
    uint32_t mis16;                     // address % 16 (every rank's must agree per buffer)
    uint64_t off;                       // address - allocation base
    uint64_t bytes;
};
constexpr int kDirectRetireMax = 256;  // retired allocations one rank announces per call
struct DirectDesc {
    uint64_t stamp0;          // rendezvous number whose descriptor this slot holds (release-stored last)
    int32_t valid;            // every buffer in an exportable device allocation
    int32_t ok;               // phase 1: every peer's buffers are mapped here
    uint64_t stamp1;          // rendezvous number of `ok` (release-stored last)
    uint32_t nalloc, nbuf;
    uint32_t nretired, pad_;
    uint64_t retired[kDirectRetireMax];  // ids of this rank's exported allocations that are gone: peers close them
    DirectAlloc alloc[kDirectAllocsMax];
    DirectBuf buf[kDirectBufsMax];
};

class Communicator {
public:
    // Multi-process: one communicator per process, peers found through `bs`
    // (collective over bs).
    static Communicator* Create(const std::string& name, Bootstrap* bs, int device, const CommConfig& cfg);
    // Sub-communicator over parent ranks `ranks` (group rank i = ranks[i];
    // CreateGroup, include/api.h:124-125, include/comm/communicator.h:133-134).
    // Collective over every rank of `parent`; non-members get null.
    static Communicator* CreateSubset(const std::string& name, Communicator* parent, const std::vector<int>& ranks,
                                      const CommConfig& cfg);
    // Single process driving n ranks (devices may repeat, e.g. n ranks on one GPU).
    static void CreateGroup(const std::string& name, int n, const int* devices, const CommConfig& cfg,
                            std::vector<Communicator*>* out);
    ~Communicator();

    // in-place device allreduce, stream-ordered; returns hipError_t-style code
    void Allreduce(void* buf, size_t count, int dtype, int op, hipStream_t stream, int algo = RDC_ALGO_AUTO);
    // bucketed allreduce: the result of Allreduce on every buffer in order
    // (bit-identical), moved as fused launches over a chunk-major staging image
    void AllreduceCoalesced(void* const* bufs, const size_t* counts, int nbuf, int dtype, int op,
                            hipStream_t stream, int algo = RDC_ALGO_AUTO);
    // allreduce of explicit byte ranges of buf, range c = [off[c], off[c]+len[c])
    // owned by rank c and folded in the ring order of Split chunk fold[c]
    // (fold null: c): one piece of a larger buffer (host path pipeline).  A
    // fold other than the identity needs an owner-computes schedule (mesh,
    // pull mesh, one-shot): a ring pick becomes the mesh.
    void AllreduceRanges(void* buf, const uint64_t* off, const uint64_t* len, int dtype, int op,
                         hipStream_t stream, const int8_t* fold = nullptr);
    void Broadcast(void* buf, size_t bytes, int root, hipStream_t stream);
    // bufs[c] (device) holds sizes[c] bytes; bufs[rank] is this rank's data
    void Allgather(void* const* bufs, const uint64_t* sizes, hipStream_t stream);
    // waits for `stream`, then reads the device error word; throws on error
    void Check(hipStream_t stream);
    // split form of Check: after the caller synchronised the stream of its
    // launches, RaiseIfError(HostErrorWord()) (the last block of every launch
    // mirrors the device error word into pinned host memory)
    uint32_t HostErrorWord() const;
    // Synchronous callers: ArmNotify() before ONE Allreduce / AllreduceRanges,
    // WaitNotify(token, stream) after it.  The call's final launch stores the
    // token into pinned host memory after a system-scope fence; the host spins
    // on it (a stream sync costs ~5 us more per call, tools/sync_latency.hip),
    // then raises a device-side error like Check.  A call that launched
    // nothing returns at once.
    uint32_t ArmNotify();
    void WaitNotify(uint32_t token, hipStream_t stream);
    void RaiseIfError(uint32_t e) const;
    // Synchronous allreduce of a small HOST buffer through the resident
    // service (rdc_service.h); false if it does not apply (too large,
    // disabled, world size 1) and the caller takes the launch path.
    bool SmallHostAllreduce(void* host, size_t count, int dtype, int op);
    // point-to-point (rdc_p2p.h): bytes of buf to / from one peer, matched in
    // order per pair; device copies start after the work queued on `after`
    WorkComp* ISend(const void* buf, size_t bytes, int dest, hipStream_t after);
    WorkComp* IRecv(void* buf, size_t bytes, int src, hipStream_t after);

    // xGMI probe (diagnostics; no collective may be in flight on any rank):
    // push `bytes` into each target peer's scratch (mode 0: rank+1 only, one
    // link one direction; mode 1: every peer at once) `reps` times on
    // `stream`; returns the average ms per push round (HIP events).
    // Overwrites scratch contents only, which every collective rewrites.
    double Probe(int mode, size_t* bytes, int reps, hipStream_t stream);  // *bytes: asked in, used out

    // tuning between collectives (stream order keeps launches consistent: the
    // plan is made on the host per call, every rank must use the same values):
    // mesh role split in sixteenths (s16 + r16 <= 15), grid (0 = auto), tile
    // bytes (0 = auto).  Throws std::invalid_argument on a bad split.
    void Tune(int s16, int r16, int max_blocks, size_t tile_bytes);
    void SetPoison(bool on) { cfg_.poison = on ? 1 : 0; }
    // closes this rank's mappings of peer buffers and turns the direct
    // schedule off for this communicator's channel (RdcCommDirectRelease)
    void DirectUnmapAll();
    // collective: one direct allreduce against the ring on the same input,
    // read back through the caches; 1 passed, 2 failed (cached per channel);
    // Autotune only times the direct schedule on a node where it passed
    int DirectSelfCheck(hipStream_t stream);
    int DirectCheckResult() const { return ch_ ? ch_->direct_check : 0; }
    // the channel's direct-schedule counters: "direct_calls" (rendezvous),
    // "direct_rendezvous_ns" / "direct_export_ns" (host time, summed),
    // "direct_retired" / "direct_closed" / "direct_refused" (mapping life
    // cycle; direct_refused counts the calls this rank refused a peer mapping
    // in), "direct_close_wait_ns", "direct_maps" / "direct_exports" (held now),
    // "direct_fallback" / "direct_unusable" (calls that fell back; of them,
    // those whose buffer lists were not usable), "direct_map_failed" /
    // "direct_fail_reason" (this rank's mapping failures, the last one's code)
    uint64_t DirectStat(const std::string& key) const;

    // Collective (every rank, same arguments, no collective in flight): time
    // the schedules (ring, mesh, one-shot where it fits) and then the launch
    // shapes of the fastest
    // for `bytes` of `dtype` (mesh: role split, then grid, then tiles per
    // reduce block; ring: grid, then tiles per block — granularity that scales
    // with the buffer), `reps`
    // Max allreduces of synthetic data each on a scratch buffer, agree on the per-candidate
    // times by a MAX allreduce over this communicator (every rank gets the
    // same bits, so the same winner), and keep the fastest for allreduces of
    // the same size class ([2^k, 2^(k+1)) bytes: tuned_algo_ / tuned_; Tune
    // clears them; nothing is tuned while RDC_ALGO forces a schedule).
    // Noise: every stage times each candidate in kTuneRounds rounds of `reps`
    // calls, round-robin over the stage's candidates (drift hits them alike);
    // a candidate's time is the median over rounds of the slowest rank's time
    // (ms_min / ms_max the spread), and a stage's first candidate — the
    // automatic rule's schedule in stage 0, the previous stage's winner after
    // that, re-timed — stays unless another beats its median by more than
    // kTuneMargin.
    // Candidates in cand[] ({algo, s16, r16, grid, tpb, ms, ms_min, ms_max};
    // up to max_cand); returns their count and *best = the chosen index (-1:
    // nothing to tune, a tree-order size).  Results stay bit-identical
    // whatever wins.
    static constexpr int kTuneRounds = 3;
    static constexpr double kTuneMargin = 0.03;
    struct TuneCand {
        int algo;                 // RDC_ALGO_MESH / RDC_ALGO_RING / RDC_ALGO_ONESHOT
        int s16, r16, grid, tpb;  // tpb: automatic tiles per block (MeshSplit::tpb), 0 = default
        double ms;                // median over rounds (slowest rank per round)
        double ms_min, ms_max;    // spread over rounds
    };
    int Autotune(size_t bytes, int dtype, int reps, hipStream_t stream, TuneCand* cand, int max_cand, int* best);

    // diagnostics: the next allreduce's launches (mesh or ring) record per
    // block {start, end} wall_clock64 ticks into dev_words (>= 2 x grid words);
    // LastLaunch() = {grid, nb_scatter, nb_reduce, nb_gather, tile_bytes, algo}
    void TraceNext(uint64_t* dev_words, size_t nwords) {
        trace_ = dev_words;
        trace_words_ = nwords;
    }
    void LastLaunch(uint64_t* out6) const {
        for (int i = 0; i < 6; ++i) out6[i] = last_launch_[i];
    }
    // diagnostics: the channel's device launch counter (the counter half of
    // every hand-off sequence word, rdc_device.h).  SetLaunchCounter is
    // collective (every rank the same value, no collective in flight on any
    // communicator of the channel); tests use it to start past 2^32.
    uint64_t LaunchCounter();
    void SetLaunchCounter(uint64_t value);

    int rank() const { return rank_; }
    uint32_t* err_words() const { return err_; }  // device: [0] error, [16] arrivals, [32] launches (diagnostics)
    int size() const { return n_; }
    Bootstrap* bootstrap() const { return bs_; }
    int device() const { return device_; }
    const std::string& name() const { return name_; }
    int alloc_kind() const { return alloc_kind_; }  // 0 uncached, 1 fine-grained, 2 coarse
    // the kind of the channel's region r (0 scratch, 1 ag, 2 flags, 3 service slots)
    int region_kind(int r) const { return ch_ && r >= 0 && r < 4 ? ch_->region_kind[r] : -1; }
    size_t slot_bytes() const { return slot_bytes_; }
    uint32_t seq() const { return seq_; }
    bool shares_channel() const;  // another communicator uses this one's scratch
    const CommConfig& config() const { return cfg_; }
    Layout layout() const;
    // requested grids (RDC_NBLOCKS / Tune, else automatic); every launch is then
    // clamped to what stays resident next to the other ranks on its GPU
    // (LaunchGrid, rdc_plan.h ResidentGrid)
    int max_blocks() const;
    int mesh_blocks() const;
    // Launch shape of a mesh / ring allreduce of `total` bytes: the shape
    // Autotune recorded for its size class (floor(log2(total))) and schedule,
    // else the communicator's configuration (defaults, RDC_* env, Tune).
    // (A coalesced list of the same size class takes the same schedule and
    // shape over its unit table.)
    struct Shape {
        MeshSplit split;
        int max_blocks = 0;
        size_t tile_bytes = 0;
    };
    Shape ShapeFor(uint64_t total, int algo) const;
    static int SizeClass(uint64_t bytes);
    std::map<int, Shape> tuned_;     // Autotune results by size class * 8 + algo; cleared by Tune
    std::map<int, int> tuned_algo_;  // Autotune's schedule by size class (PickAlgo); cleared by Tune
    int LaunchGrid(int want, int blocks_per_cu) const;
    bool shared_gpu() const { return share_max_ > 1; }
    int ranks_per_gpu() const { return share_max_; }

private:
    Communicator();
    void AllocLocal();                                   // a fresh channel + this communicator's p2p region
    void AllocChannel();
    void AllocP2P();
    void Attach(const std::shared_ptr<Channel>& ch);     // one more user of the channel, then Alias()
    void Alias();                                        // copy the channel's pointers into the names below
    void FillArgsCommon(CollArgs* a) const;
    int PickAlgo(int algo) const;
    int PickAlgo(int algo, uint64_t bytes) const;
    // units != null: coalesced mesh over a device PackUnit table (off/len = packed chunk ranges)
    void LaunchRanges(const KernelSet& ks, char* buf, const uint64_t* off, const uint64_t* len, uint64_t total,
                      size_t esz, int algo, hipStream_t stream, const PackUnit* units = nullptr, int nunits = 0,
                      const int8_t* fold = nullptr);
    struct PackEntry {
        PackUnit* dtable = nullptr;  // device unit table (user addresses)
        int nunits = 0;
        uint64_t off[RDC_MAX_RANKS] = {}, len[RDC_MAX_RANKS] = {};
        uint64_t total = 0;
        uint64_t last_use = 0;
        std::shared_ptr<std::vector<PackUnit>> host;  // the upload's source, alive until the copy is done
    };
    static constexpr size_t kPackCacheMax = 64;
    const PackEntry& PackTable(void* const* bufs, const size_t* counts, int nbuf, size_t esz, hipStream_t stream);
    char* Image(uint64_t bytes, hipStream_t stream);
    void LaunchTree(const KernelSet& ks, char* buf, uint64_t total, hipStream_t stream);
    // registered user buffers (k_direct): false when the rendezvous finds any
    // rank's buffer unusable (the caller takes the scratch schedules; every
    // rank decides alike)
    bool DirectEligible(int algo, uint64_t bytes, hipStream_t stream) const;
    // one buffer (nbuf = 1) or a coalesced list; bytes[b] > 0 for every b
    bool AllreduceDirect(const KernelSet& ks, char* const* bufs, const uint64_t* bytes, int nbuf, size_t esz,
                         hipStream_t stream);
    void TuneBuffer(size_t bytes);
    // fresh: the allocations exported in this call, as (index in me.alloc,
    // the canary: the first bytes of one of this call's buffers)
    bool DirectExport(DirectDesc& me, char* const* bufs, const uint64_t* bytes, int nbuf, uint64_t call,
                      std::vector<char*>* own_base, std::vector<std::pair<uint32_t, std::pair<char*, uint32_t>>>* fresh);
    bool DirectMapPeers(const DirectDesc* slots, const std::vector<char*>& own_base, uint64_t call,
                        std::vector<char*>* amap);
    void DirectCloseRetired(const DirectDesc* slots, uint64_t call);
    bool CanaryOk(const DirectAlloc& al, char* mapped, size_t size, int p, uint64_t call);
    // device tables of coalesced direct launches: owner items + every rank's
    // buffer addresses, cached by the call's layout
    struct DirectTable {
        void* dtable = nullptr;
        std::shared_ptr<std::vector<uint64_t>> host;  // the upload's source
        int nitems = 0;
        uint64_t tile = 0;
        uint64_t last_use = 0;
    };
    std::map<std::vector<uint64_t>, DirectTable> direct_tables_;
    const DirectTable& DirectTableFor(const DirectDesc* slots, const uint64_t* bytes, int nbuf, size_t esz,
                                      uint64_t tile, const std::vector<char*>& amap, hipStream_t stream);
    std::vector<std::pair<hipEvent_t, std::shared_ptr<std::vector<uint64_t>>>> direct_retired_;
    uint64_t direct_tick_ = 0;
    void CoalescedTree(const KernelSet& ks, void* const* bufs, const size_t* counts, int nbuf, size_t esz,
                       hipStream_t stream);
    void CoalescedStaged(const KernelSet& ks, void* const* bufs, const size_t* counts, int nbuf, int dtype, int op,
                         size_t esz, int algo, hipStream_t stream);

    std::string name_;
    int rank_ = 0, n_ = 1, device_ = 0;
    CommConfig cfg_;
    Bootstrap* bs_ = nullptr;       // not owned (unless owned_bs_ holds it: group communicators)
    std::unique_ptr<Bootstrap> owned_bs_;
    std::shared_ptr<Channel> ch_;   // scratch_ ... peer_flags_ below alias its resources
    bool owns_peers_ipc_ = false;   // peers' p2p regions opened through IPC
    char* scratch_ = nullptr;       // RS region
    char* scratch_ag_ = nullptr;    // AG region
    uint64_t* flags_ = nullptr;
    uint32_t* err_ = nullptr;
    uint32_t* err_host_ = nullptr;  // pinned mirror of *err_ (kernel-written)
    uint32_t* err_host_dev_ = nullptr;
    uint32_t* notify_ = nullptr;    // armed: device address of the pinned notify word
    uint32_t notify_val_ = 0;
    uint64_t* trace_ = nullptr;     // TraceNext
    size_t trace_words_ = 0;
    uint64_t last_launch_[6] = {};
    int tree_len_ = 0, tree_dst_[RDC_MAX_RANKS] = {}, tree_src_[RDC_MAX_RANKS] = {};  // PlanTreeProgram(n)
    size_t slot_bytes_ = 0, region_bytes_ = 0, flag_bytes_ = 0;
    uint32_t max_tiles_ = 0;
    uint32_t seq_ = 0;
    uint32_t tag_ = 0;              // bits 24-31 of this communicator's launch sequence numbers
public:
    int coalesced_misaligned_ = 0;  // buckets of the last coalesced call not 16-B aligned (element-wise folds)
private:
    int alloc_kind_ = 0;
    int num_cus_ = 256;             // this GPU
    int cus_min_ = 256;             // fewest CUs of any rank's GPU (grids are planned identically on all ranks)
    int num_xcds_ = 1;              // this GPU's XCDs
    int xcds_max_ = 1;              // most XCDs of any rank's GPU (ResidentGrid's per-XCD clamp)
    int share_max_ = 1;             // most ranks of this communicator on one physical GPU
    int wall_khz_ = 100000;         // wall_clock64() rate
    char* peer_scratch_[RDC_MAX_RANKS] = {};
    char* peer_ag_[RDC_MAX_RANKS] = {};
    uint64_t* peer_flags_[RDC_MAX_RANKS] = {};
    std::map<std::vector<uint64_t>, PackEntry> pack_cache_;
    std::vector<std::pair<hipEvent_t, std::shared_ptr<std::vector<PackUnit>>>> retired_;  // evicted host copies
    uint64_t pack_tick_ = 0;
    char* image_ = nullptr;         // coalesced staging image (local HBM)
    uint64_t image_bytes_ = 0;
    // point-to-point: slot region [n senders][kP2PSlots] x p2p_slot_bytes (uncached, IPC-exported),
    // a control block shared by the group (POSIX shm across processes), engine started on first use
    P2PEngine* P2P();
    char* p2p_ = nullptr;
    char* peer_p2p_[RDC_MAX_RANKS] = {};
    std::shared_ptr<P2PCtl> p2p_ctl_;
    std::unique_ptr<P2PEngine> p2p_engine_;
    std::mutex p2p_mu_;
};

// op::Reducer<OP,DType> on device: dst = OP(dst, src) element-wise
void DeviceReduce(void* dst, const void* src, size_t count, int dtype, int op, hipStream_t stream, int grid = 0);
void DeviceFill(void* buf, size_t count, int dtype, uint64_t seed, int rank, hipStream_t stream);

}  // namespace rdc_amd
