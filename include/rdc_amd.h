/*
 * rdc_amd.h — C ABI of the MI355X-native rdc allreduce path (librdc_amd.so).
 *
 * The reference ships NO C ABI: its Python package calls `_LIB.Rdc*` symbols
 * that exist nowhere in src/ (SURVEY.md §0 finding 3).  The entry points below
 * are exactly the ones those callers bind, with the signatures the call sites
 * imply, plus device-resident extensions for the MI355X path.
 * Plain pointers and sizes only; no torch types.
 *
 * Conventions
 *   - every function returns 0 on success and a non-zero code on failure
 *     (RdcGetLastError() then describes it), except the getters
 *     RdcGetRank/RdcGetWorldSize/RdcIsDistributed/RdcCommRank/RdcCommSize;
 *     the reference aborts via CHECK_F instead — the C++ header include/rdc.h
 *     restores that behaviour on top of these codes.
 *   - dtype: mpi::DataType (include/core/mpi.h:19-30) = rdc/core.py:160-169:
 *       0 int8, 1 uint8, 2 int32, 3 uint32, 4 int64, 5 uint64, 6 float32,
 *       7 float64, 8 long long, 9 unsigned long long
 *     MI355X additions: 10 float16 (IEEE binary16), 11 bfloat16.
 *   - op: mpi::OpType (include/core/mpi.h:12-17) = rdc/core.py:16-20:
 *       0 MAX, 1 MIN, 2 SUM, 3 BITOR (integer dtypes only)
 *   - results are bit-identical to the reference's CPU ring allreduce
 *     (src/comm/communicator_collective.cc:115-203) on the same inputs.
 */
#ifndef RDC_AMD_H_
#define RDC_AMD_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ */
/* Reference-bound entry points (the names rdc/core.py & rdc/comm.py call) */
/* ------------------------------------------------------------------ */

/* rdc::Init (include/rdc.h:58-61, include/core/rdc-inl.h:21-23;
 * rdc/core.py:29-49 calls RdcInit(len(args), arr)).  argv entries of the form
 * key=val override environment variables (communicator_manager.cc:87-104).
 * Keys: RDC_RANK, RDC_WORLD_SIZE|rdc_world_size, RDC_TRACKER_URI,
 * RDC_TRACKER_PORT, rdc_reduce_ring_mincount, RDC_DEVICE, RDC_SCRATCH_BYTES,
 * RDC_ALGO (mesh|mesh_pull|ring|oneshot), RDC_NBLOCKS, RDC_TILE_BYTES, RDC_TIMEOUT, RDC_ONESHOT_BYTES,
 * RDC_FUSE_BYTES, RDC_FUSE_BYTES_DIRECT, RDC_COALESCE_FUSED, RDC_HOST_ZC_BYTES,
 * RDC_BCAST_SPLIT_BYTES, RDC_P2P_SLOT_BYTES.
 * Falls back to torchrun's RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/MASTER_PORT
 * (tracker port = MASTER_PORT+1).  Does not touch the GPU. */
int RdcInit(int argc, char** argv);
/* rdc::Finalize (include/rdc.h:75; rdc/core.py:52-57) */
int RdcFinalize(void);
/* rdc::GetRank / GetWorldSize / IsDistributed (include/rdc.h:76-80;
 * rdc/core.py:66-87) */
int RdcGetRank(void);
int RdcGetWorldSize(void);
int RdcIsDistributed(void);
/* rdc::TrackerPrint (include/api.h:9; rdc/core.py:90-103) */
int RdcTrackerPrint(const char* msg);
/* rdc/core.py:106-118 */
int RdcGetProcessorName(char* buf, unsigned long* out_len, unsigned long max_len);
/* rdc::Barrier (include/api.h:14) */
int RdcBarrier(void);

/* rdc::Allreduce<OP,DType> (include/api.h:62-64, include/core/rdc-inl.h:125-135)
 * on the "main" communicator; rdc/core.py:204-216 calls
 * RdcAllreduce(ptr, size, dtype_enum, int(op), prepare_fun|NULL, NULL).
 * sendrecv may be host or device memory (detected); synchronous, in place.
 * prepare_fun(prepare_arg), when given, runs before the reduction. */
int RdcAllreduce(void* sendrecv, size_t count, int dtype, int op, void (*prepare_fun)(void*),
                 void* prepare_arg);
/* rdc::Broadcast(void*, size, root) (include/api.h:23-24, rdc-inl.h:71-75;
 * rdc/core.py:143-154).  Host or device memory; synchronous. */
int RdcBroadcast(void* sendrecv, unsigned long size, int root);

/* The same two calls on a named communicator (rdc::Allreduce<OP,DType>(buf,
 * count, comm_name), include/api.h:62-64; rdc::Broadcast(..., comm_name),
 * include/api.h:23-26).  Host or device memory; synchronous. */
int RdcAllreduceOn(void* comm, void* sendrecv, size_t count, int dtype, int op);
int RdcBroadcastOn(void* comm, void* sendrecv, size_t size, int root);

/* rdc::Allgather (include/api.h:47-52, include/core/rdc-inl.h:106-122;
 * TryAllgatherRing, communicator_collective.cc:79-114): bufs[c] holds
 * sizes[c] bytes; on entry bufs[rank] holds this rank's data, on return every
 * bufs[c] holds rank c's data.  All host or all device memory; synchronous.
 * RdcAllgather uses the "main" communicator. */
int RdcAllgather(void** bufs, const size_t* sizes);
int RdcAllgatherOn(void* comm, void** bufs, const size_t* sizes);

/* Coalesced (bucketed) allreduce: the result of one RdcAllreduce per buffer,
 * in order, bit-identical, but the buffers move in fused launches (BASELINE
 * cfg5 / test/mallreduce.cc's back-to-back shape).  A list takes the schedule
 * and launch shape one buffer of its total size would get (the automatic rule,
 * or what RdcCommAutotune chose for that size class); the mesh and the ring
 * read and write the buffers in place through a cached unit table (groups of
 * up to RDC_FUSE_BYTES_DIRECT, default 16 GiB); one-shot lists are packed
 * chunk-major into an HBM staging image in groups of RDC_FUSE_BYTES (default
 * 256 MiB).  Buckets whose addresses are 16-B aligned take the vector paths;
 * a bucket that is only element-aligned folds element by element (correct,
 * slower): RdcCommGetParam(comm, "coalesced_misaligned") counts them in the
 * last coalesced call.
 * bufs[b] holds counts[b] elements of `dtype`; all host or all device memory;
 * synchronous.  RdcAllreduceCoalesced uses the "main" communicator. */
int RdcAllreduceCoalesced(void** bufs, const size_t* counts, int nbuf, int dtype, int op);
int RdcAllreduceCoalescedOn(void* comm, void** bufs, const size_t* counts, int nbuf, int dtype, int op);

/* rdc::NewCommunicator / GetCommunicator (include/rdc.h:62-71;
 * rdc/comm.py:90-93,106-109 call RdcNewCommunicator(byref(handle), name)).
 * NewCommunicator is collective over all ranks.  Named communicators over the
 * same ranks share one scratch channel (one pool of uncached HBM per rank):
 * every rank must then issue the collectives of ALL those communicators in
 * the same order (the SPMD order rdc programs follow; the reference's
 * Allreduce is not thread-safe either, communicator.h:87).  Ranks that
 * interleave two communicators differently — e.g. from two threads — need
 * RDC_SHARE_SCRATCH=0 (a channel per communicator, as the reference's
 * independent TCP meshes behave). */
int RdcNewCommunicator(void** out, const char* name);
int RdcGetCommunicator(void** out, const char* name);
/* rdc::CreateGroup / ICommunicator::CreateGroup (include/api.h:124-125,
 * include/comm/communicator.h:133-134; declared, never defined in the
 * reference): a communicator over `ranks` (ranks of `parent`, NULL = "main";
 * group rank i = ranks[i]) named `name` ("" = "group<k>").  Collective over
 * every rank of the parent, all passing the same list; *out = NULL on ranks
 * not in it.  Members rendezvous through node-local shared memory and get
 * their own scratch; destroy with RdcCommDestroy (collective over members). */
int RdcCreateGroup(void** out, void* parent, const int* ranks, int nranks, const char* name);

/* Point-to-point (ICommunicator::ISend/IRecv, include/comm/communicator.h:
 * 56-80; rdc/comm.py:46-80 binds RdcISend / RdcIRecv / RdcWorkCompletion*).
 * Buffers are rdc Buffer handles (rdc/buffer.py:34-38: RdcNewBuffer(byref(h),
 * addr, size, pinned)) over host OR device memory; `pinned` page-locks a host
 * range (hipHostRegister) for the buffer's lifetime (whole pages only: a
 * page-aligned address and size).  A host allreduce (RdcAllreduce /
 * RdcCommAllreduce on a host pointer) whose buffer lies inside such a range
 * DMAs straight from and into it, with no copy through staging memory.  Data moves GPU to GPU
 * over xGMI through the receiver's IPC-mapped slots; messages on one (src,
 * dst) pair are matched in order and must have equal sizes on both sides.
 * A request that makes no progress for RDC_TIMEOUT seconds ends in error.
 * Completion handles are freed with RdcDelWorkCompletion (safe while
 * pending).  RdcIRecv returns the handle (NULL on failure), as comm.py:73
 * expects; every other function returns a status code. */
int RdcNewBuffer(void** out, void* addr, size_t size, int pinned);
int RdcDelBuffer(void* buf);
int RdcISend(void** wc, void* comm, void* buf, int dest);
void* RdcIRecv(void* comm, void* buf, int src);
/* 0 = finished, 1 = error (RdcWorkCompletionError describes it) */
int RdcWorkCompletionWait(void* wc);
/* WorkStatus (include/core/work_request.h:23-30): 2 pending, 8 finished, 64 error */
int RdcWorkCompletionStatus(void* wc);
const char* RdcWorkCompletionError(void* wc);
int RdcDelWorkCompletion(void* wc);
/* blocking rdc::Send / rdc::Recv on "main" (include/api.h:10-11) */
int RdcSend(void* buf, size_t size, int dest);
int RdcRecv(void* buf, size_t size, int src);
/* raw-pointer forms on `comm`; for device memory the copies start after the
 * work already queued on `stream` (NULL = default stream) */
int RdcCommISend(void** wc, void* comm, const void* buf, size_t bytes, int dest, void* stream);
int RdcCommIRecv(void** wc, void* comm, void* buf, size_t bytes, int src, void* stream);

/* ------------------------------------------------------------------ */
/* MI355X device-resident extensions                                    */
/* ------------------------------------------------------------------ */

/* In-place allreduce of device memory on `comm`, enqueued on `stream`
 * (hipStream_t; NULL = default stream).  Asynchronous: errors raised inside
 * the kernels (a peer that never joins) surface at RdcCommCheck. */
int RdcCommAllreduce(void* comm, void* dev_buf, size_t count, int dtype, int op, void* stream);
/* algo: 0 auto, 1 ring (the reference schedule), 2 mesh (all links, pushed by remote stores),
 * 6 direct (registered buffers, one process per rank: every rank's buffer is mapped into every
 * peer through HIP IPC once per allocation — a host rendezvous over shared memory agrees on the
 * buffers each call — and owner r folds chunk r straight out of the n buffers and writes the
 * result back into all of them: no scratch, one read and one write of each buffer; falls back
 * to the automatic rule on every rank when any buffer cannot be mapped, the addresses differ mod
 * 16, the stream is being captured or the ranks share one process; RDC_DIRECT_BYTES=<n> takes it
 * automatically from n bytes),
 * 5 pull-mode mesh (the same exchange by remote loads: ranks stage their chunks in their own
 * scratch, owners load and fold, peers load the results; RdcCommAutotune times it against
 * the push mesh), 3 one-shot (small buffers:
 * every rank pushes the whole buffer to every peer, one hand-off); auto = one-shot when
 * the one-shot while bytes <= 8 MiB and its extra egress over the mesh,
 * (n-1)(n-2)/n x bytes, is <= 4 MiB (n = 2: 8 MiB, n = 8: 0.76 MiB; with
 * RDC_ONESHOT_BYTES set: while (n-1) x bytes <= it), else the ring at n = 2
 * and the mesh from n = 3.  All bit-identical.
 * Whatever the algo, a buffer of at most rdc_reduce_ring_mincount bytes (default 1) takes
 * the reference's TREE order (TryAllreduce, src/comm/communicator_collective.cc:6-13: the
 * fold of TryReduceTree to rank 0, every rank receiving the root's bits) as one one-shot
 * style hand-off; algo 4 forces that tree order for any size. */
int RdcCommAllreduceEx(void* comm, void* dev_buf, size_t count, int dtype, int op, int algo, void* stream);
/* device-resident coalesced allreduce (see RdcAllreduceCoalesced), stream-ordered.
 * The per-group unit table is cached by (buffers, counts): after a first
 * (warm-up) call with the same buckets, launches need no host->device copy
 * and can be captured in a hipGraph.  algo 6 (or an Autotune'd direct
 * schedule for the list's total size) runs the whole list as ONE direct
 * launch between the ranks' buffers (every buffer's allocation mapped into
 * the peers, <= 4096 buffers in <= 64 allocations per call; else the
 * scratch schedules). */
int RdcCommAllreduceCoalesced(void* comm, void* const* dev_bufs, const size_t* counts, int nbuf, int dtype, int op,
                              int algo, void* stream);
int RdcCommBroadcast(void* comm, void* dev_buf, size_t bytes, int root, void* stream);
/* device-resident allgather of per-rank buffers (see RdcAllgather), stream-ordered */
int RdcCommAllgather(void* comm, void** dev_bufs, const size_t* sizes, void* stream);
/* synchronise `stream` and report any device-side collective failure */
int RdcCommCheck(void* comm, void* stream);
/* A communicator's parameter: "rdc_reduce_ring_mincount", "RDC_SCRATCH_BYTES",
 * "RDC_TILE_BYTES", "RDC_NBLOCKS", "RDC_ONESHOT_BYTES", "slot_bytes",
 * "ranks_per_gpu" (most ranks of it sharing one physical GPU), "coalesced_misaligned"
 * (buckets of the last coalesced call not 16-B aligned), "shares_scratch"
 * (1 when another communicator uses the same scratch channel: every named
 * communicator over the same ranks shares one, RDC_SHARE_SCRATCH=0 disables),
 * "host_registered_calls" (host allreduces of this process that DMA'd in place
 * from a pinned RdcNewBuffer range), "RDC_DIRECT_BYTES" (RDC_DIRECT_MIN_AUTO =
 * the default rule), "direct_check" (the channel's direct self-check, run at
 * creation: 0 not run, 1 passed, 2 failed), "flags_kind" / "scratch_kind" (3 =
 * HSA-uncached, MTYPE UC; 0 = hipDeviceMallocUncached, MTYPE CC on gfx950),
 * and the direct schedule's counters "direct_calls", "direct_rendezvous_ns",
 * "direct_export_ns", "direct_retired", "direct_closed", "direct_refused",
 * "direct_close_wait_ns", "direct_maps", "direct_exports", "direct_fallback"
 * (calls that fell back, alike on every rank), "direct_unusable" (of them, the
 * calls whose buffer lists could not run direct), "direct_map_failed" and
 * "direct_fail_reason" (this rank's peer-mapping failures and the last one's
 * code: 1 table full, 2 refused earlier, 3 open failed, 4 a mapping already
 * held, 5 lands partly over unmapped ranges, 6 the mapping did not show
 * the exporter's canary: another buffer object), "direct_canary" (new peer
 * mappings checked by their canary), "direct_export_failed" /
 * "direct_export_error" (exports of this rank's allocations HIP refused and
 * the last hipError_t), "direct_import" (1: peers mapped from dma-bufs at
 * chosen addresses, RDC_DIRECT_IMPORT=vmem; 0: HIP IPC) and "direct_pending"
 * (dma-bufs received and not mapped). */
int RdcCommGetParam(void* comm, const char* key, uint64_t* value);
int RdcCommRank(void* comm);
int RdcCommSize(void* comm);
int RdcCommDevice(void* comm);
/* 0 uncached, 1 fine-grained, 2 coarse-grained scratch */
int RdcCommAllocKind(void* comm);

/* xGMI link probe (diagnostics, bench.py at N > 1): push `bytes` per target
 * from this rank's scratch into peers' scratch `reps` times on `stream`, all
 * targets at once, with the copy kernel the collectives use for remote
 * stores.  mode 0: rank+1 only (one link, one direction); mode 1: every peer
 * (all n-1 links out of this GPU); modes 2 / 3: the same links read instead
 * (pull from rank+1 / from every peer into local scratch).  *ms_out = average ms per round;
 * *bytes_out (may be NULL) = bytes per target actually pushed (clamped to
 * the scratch slot).  Call it
 * between collectives with every rank idle (e.g. after a barrier): it
 * overwrites scratch, which every collective rewrites before reading. */
int RdcCommProbe(void* comm, int mode, size_t bytes, int reps, void* stream, double* ms_out, size_t* bytes_out);

/* Re-tune one communicator between collectives (every rank of it must pass
 * the same values; the plan is made per call on each host): mesh role split
 * in sixteenths of the grid (RDC_MESH_SPLIT; mesh_s16 + mesh_r16 <= 15, the
 * gather role gets the rest), grid size (RDC_NBLOCKS; 0 = auto) and tile
 * bytes (RDC_TILE_BYTES; 0 = auto, else a multiple of 256).  Results stay
 * bit-identical (the fold order is per element).  No reference counterpart:
 * the reference's schedule has no such knobs; bench.py sweeps them at N>1. */
int RdcCommTune(void* comm, int mesh_s16, int mesh_r16, int max_blocks, size_t tile_bytes);

/* Debug mode (RDC_POISON_SCRATCH; every rank of `comm` should pass the same
 * value, though ranks that differ stay correct): with on != 0 every consumer
 * of a hand-off overwrites the scratch range it finished reading with 0xFF
 * bytes before the signal that lets the producer reuse it, so a read of a
 * range before its producer's next publish lands NaN / all-ones words instead
 * of a plausible older value.  Results are unchanged; each launch stores its
 * consumed scratch bytes once more.  No reference counterpart. */
int RdcCommSetPoison(void* comm, int on);

/* The direct schedule (algo 6) maps each peer's buffer into this process once
 * per allocation and keeps the mapping while the communicator lives; a
 * mapping keeps the peer's allocation alive after the peer frees it, and an
 * allocation at an address this rank exported before for another allocation
 * is not exported again (those calls take the scratch schedules).  This
 * closes all of this rank's mappings (after waiting for the device) and turns
 * the direct schedule off for the communicator, releasing the peers' freed
 * allocations.  Call it on every rank.  No reference counterpart. */
int RdcCommDirectRelease(void* comm);

/* Autotune (collective: every rank of `comm`, same arguments, no collective in
 * flight; blocks the host): time the ring, the mesh pushed and pulled (RDC_ALGO_MESH_PULL),
 * (where it fits half a slot) the one-shot schedule and (ranks in processes of
 * their own) the direct schedule, then the launch shapes of the fastest, for
 * `bytes` of `dtype` on this node — mesh: role split, then grid, then
 * tiles per reduce block; ring: grid, then tiles per block (a granularity, so
 * the chosen tiles scale with later buffers' sizes) — `reps` Max allreduces of synthetic data each on a scratch
 * buffer, in 3 rounds per candidate taken round-robin over each stage; agree
 * on the per-round times with a MAX allreduce over `comm` (identical on every
 * rank, so every rank keeps the same winner); a candidate's time is the median
 * of its rounds, and each stage keeps its first candidate (stage 0: the
 * automatic rule's schedule; later: the previous winner) unless another is
 * faster by more than 3 %; keep the chosen schedule and shape for allreduces of that size class ([2^k,
 * 2^(k+1)) bytes; other sizes keep the automatic rule and the configured
 * shape, RdcCommTune clears every autotuned one, and nothing is tuned while
 * RDC_ALGO forces a schedule; with RDC_TUNE_FILE set, rank 0 appends the
 * winner there and later communicators of the same rank and CU count start
 * from it).  cand (room for max_cand; 24 suffices)
 * receives every timed candidate with its slowest-rank ms; *ncand their count,
 * *best the chosen index (-1 and nothing changed for sizes that take the
 * tree order, rdc_reduce_ring_mincount).  Results stay bit-identical whatever wins.  No
 * reference counterpart (the reference's schedule has no launch shape). */
typedef struct {
    int algo;                           /* RDC_ALGO_RING (1), RDC_ALGO_MESH (2), RDC_ALGO_ONESHOT (3),
                                           RDC_ALGO_MESH_PULL (5) */
    int mesh_s16, mesh_r16, max_blocks; /* max_blocks 0 = automatic grid */
    int tiles_per_block;                /* 0 = default (mesh 2 per reduce block, ring 1) */
    double ms;                          /* per allreduce: median over rounds of the slowest rank's time */
    double ms_min, ms_max;              /* spread of that time over the rounds */
} RdcTuneCand;
int RdcCommAutotune(void* comm, size_t bytes, int dtype, int reps, void* stream, RdcTuneCand* cand, int max_cand,
                    int* ncand, int* best);

/* Diagnostics (bench.py at N > 1): the next allreduce on `comm` (mesh or
 * ring schedule) records, per block, {start, end} wall_clock64 ticks
 * (100 MHz) into dev_words (device memory, >= 2 x grid uint64 words; a launch
 * with a larger grid is not traced).  RdcCommLastLaunch: {grid, nb_scatter,
 * nb_reduce, nb_gather, tile_bytes, algo} of the last allreduce launch
 * (mesh roles: blocks [0, s) scatter, [s, s+r) reduce, the rest gather). */
int RdcCommTraceNext(void* comm, void* dev_words, size_t nwords);
int RdcCommLastLaunch(void* comm, uint64_t* out6);

/* Diagnostics: the device launch counter of comm's scratch channel — the
 * counter half of every 64-bit hand-off sequence word (seq = counter << 8 |
 * communicator tag; 56-bit counters, compared modulo 2^56, so flag slots never
 * written or idle for any number of launches never read as "reached").
 * RdcCommSetLaunchCounter is collective: every rank of the channel sets the
 * same value with no collective in flight (tests start it past 2^32). */
int RdcCommLaunchCounter(void* comm, uint64_t* value);
int RdcCommSetLaunchCounter(void* comm, uint64_t value);

/* Single process driving n ranks (devices[i] = HIP device of rank i; devices
 * may repeat).  comms[i] receives rank i's handle.  scratch_bytes 0 = default. */
int RdcCommInitAll(void** comms, int n, const int* devices, size_t scratch_bytes);
/* Destroy a communicator (collective for communicators made by
 * RdcNewCommunicator; local for RdcCommInitAll groups). */
int RdcCommDestroy(void* comm);

/* op::Reducer<OP,DType>(src, dst, count) (include/core/mpi.h:113-120) on
 * device memory: dst[i] = OP::Reduce(dst[i], src[i]).  Stream-ordered. */
int RdcReduce(void* dst, const void* src, size_t count, int dtype, int op, void* stream);
/* Synchronous copy between any two of host / device memory (the C++ header's
 * custom-reducer path stages device buffers with it). */
int RdcMemcpy(void* dst, const void* src, size_t bytes);
/* Synthetic inputs: u = splitmix64(seed ^ (rank<<40) ^ i) mapped per dtype
 * (identical to the CPU oracle's generator).  Stream-ordered. */
int RdcFill(void* dev_buf, size_t count, int dtype, uint64_t seed, int rank, void* stream);

/* Host-side planning, no GPU needed (what the launches of a collective will
 * be; used by the CPU tests).  RdcPlanLayout: out = {slot_bytes,
 * region_bytes, max_tiles, flag_bytes} of a communicator of n ranks.
 * RdcPlanAllreduce: one record of RDC_PLAN_WORDS uint64 per launch:
 *   [tile_bytes, nb_scatter, nb_reduce, nb_gather,
 *    off[16], len[16], mis[16], tiles[16]]   (per chunk c < n)
 * *out_pieces = number of launches (records written: min(that, max_pieces)). */
#define RDC_PLAN_WORDS 68
/* Grid of a collective launch whose blocks wait on other ranks' blocks: the
 * requested grid `want` clamped so that every rank's blocks stay resident at
 * once, min(want, blocks_per_cu x cus / ranks_per_gpu) (at least 1).
 * Communicators apply it to every ring / mesh / one-shot / tree / broadcast /
 * allgather launch, including grids forced by RDC_NBLOCKS or RdcCommTune;
 * blocks_per_cu is the kernel's occupancy, ranks_per_gpu the most ranks of
 * the communicator on one physical GPU, cus the fewest CUs of any rank's GPU.
 * Returns the grid (not a status). */
int RdcPlanResidentGrid(int want, int blocks_per_cu, int cus, int ranks_per_gpu);
/* The clamp communicators apply (round 4): a dispatch sends workgroup i to
 * XCD i % xcds, so the grid is min(want, xcds x floor((blocks_per_cu x
 * cus / xcds - blocks_per_cu x reserve_cus) / ranks_per_gpu)) — every XCD
 * holds every rank's share even when the reserve_cus CUs kept for resident
 * service blocks all sit on one XCD (xcds = 1 when it does not divide cus).
 * With xcds = 1 and reserve_cus = 0 it is RdcPlanResidentGrid.  Communicators
 * pass hipDeviceAttributeNumberOfXccs (the most of any rank) and reserve one
 * CU per rank on the GPU. */
int RdcPlanResidentGridXcd(int want, int blocks_per_cu, int cus, int ranks_per_gpu, int xcds, int reserve_cus);
/* The tree allreduce's fold for n ranks (rdc_reduce_ring_mincount path): the
 * post-order program acc[dst[i]] = OP(acc[dst[i]], acc[src[i]]), i < n-1,
 * over the n ranks' inputs (acc[q] = rank q's value); the result is acc[0].
 * dst/src hold >= 16 ints.  Returns n-1, or -1 on bad arguments. */
int RdcPlanTree(int n, int* dst, int* src);
int RdcPlanLayout(int n, size_t scratch_bytes, uint64_t* out4);
/* The host-buffer pipeline's contiguous pieces for `bytes` (RDC_HOST_PIECE_BYTES,
 * RDC_HOST_PIECE_RAMP): bounds[0..*out_n) = {0, ..., bytes}, piece k = [bounds[k],
 * bounds[k+1]) (one piece up to 16 MiB).  Writes at most max_bounds entries. */
int RdcPlanHostPieces(size_t bytes, uint64_t* bounds, int max_bounds, int* out_n);
/* The ranges of one host-path piece [lo, hi) (byte offsets of a buffer of
 * `count` elements of `dtype`) over n ranks: off[q], len[q] (relative to lo)
 * owned by rank q and folded in the ring order of Split chunk fold[q].
 * balanced 0: the piece's bytes of chunk q go to rank q (fold[q] = q);
 * balanced 1: each chunk's bytes are cut over the ranks in proportion to
 * their length (RDC_HOST_BALANCE; the default with one rank per GPU). */
int RdcPlanHostPieceRanges(int n, size_t count, int dtype, uint64_t lo, uint64_t hi, int balanced, uint64_t* off,
                           uint64_t* len, int* fold);
/* The automatic schedule for an allreduce of `bytes` over n ranks: returns
 * RDC_ALGO_ONESHOT (3), RDC_ALGO_RING (1, n = 2 beyond the one-shot) or
 * RDC_ALGO_MESH (2) (negative on bad arguments).
 * oneshot_bytes = RDC_ONESHOT_BYTES (0 = the default size / rank-aware rule). */
int RdcPlanAutoAlgo(int n, size_t bytes, size_t scratch_bytes, size_t oneshot_bytes);
/* Whether an untuned automatic allreduce of `bytes` over n processes takes the
 * registered-buffer schedule (RDC_ALGO_DIRECT) when every rank's buffer can be
 * mapped and the channel's direct self-check passed: 1 / 0 (negative on bad
 * arguments).  direct_min = RDC_DIRECT_BYTES: RDC_DIRECT_MIN_AUTO (the
 * default) = beyond the one-shot sizes and from 16 MiB (32 MiB at n = 2); 0 = never; N = from N
 * bytes.  Replaces nothing in the reference (its one schedule is the ring);
 * the drop-in rdc::Allreduce / rdc.allreduce calls get it without tuning. */
#define RDC_DIRECT_MIN_AUTO (~(uint64_t)0)
int RdcPlanDirectAuto(int n, size_t bytes, size_t scratch_bytes, size_t oneshot_bytes, uint64_t direct_min);
/* HBM byte model of one allreduce of `count` elements over n ranks with
 * schedule `algo` (1 ring, 2 mesh, 3 one-shot, 4 tree, 5 pull-mode mesh, 6 direct): the
 * bytes the kernels load and store, counted per access as their loops issue
 * them, a remote store or load counted at the rank that issues it.  out5 = {read bytes, write bytes
 * (both the most of any rank), read bytes, write bytes (both summed over the
 * ranks), link egress bytes (the most of any rank)}.  bench.py's N > 1
 * roofline divides this by the measured time. */
int RdcPlanHbmBytes(int n, size_t count, int dtype, int algo, uint64_t* out5);
int RdcPlanAllreduce(int n, size_t count, int dtype, size_t scratch_bytes, int algo, size_t tile_bytes,
                     int max_blocks, uint64_t* out, int max_pieces, int* out_pieces);

/* RdcPlanCoalesced: the staging image of one fusion group.  chunk_out (33
 * words): packed chunk offsets off[16], lengths len[16], total bytes.  units_out:
 * 4 words per copy unit {buffer index, byte offset in the buffer, byte offset
 * in the image, bytes}.  RdcPlanFuseGroups: group boundaries (group g =
 * buffers [bounds[g], bounds[g+1])); fuse_bytes 0 = default. */
int RdcPlanCoalesced(int n, const size_t* counts, int nbuf, int dtype, uint64_t* chunk_out, uint64_t* units_out,
                     int max_units, int* out_units);
/* RdcPlanDirectItems: owner `rank`'s items of a coalesced direct launch
 * (algo 6 over a list): Split chunk `rank` of every buffer in pieces of at
 * most `tile` bytes, 3 words each {buffer, byte offset, bytes}. */
int RdcPlanDirectItems(int n, int rank, const size_t* counts, int nbuf, int dtype, uint64_t tile, uint64_t* out,
                       int max_items, int* out_items);
int RdcPlanFuseGroups(const size_t* counts, int nbuf, int dtype, size_t fuse_bytes, int* bounds_out, int max_bounds,
                      int* out_n);

/* Set a parameter (same keys as RdcInit argv). */
int RdcSetParam(const char* name, const char* value);
/* Description of the last failure on this thread ("" if none). */
const char* RdcGetLastError(void);
const char* RdcVersion(void);

#ifdef __cplusplus
}
#endif
#endif /* RDC_AMD_H_ */
