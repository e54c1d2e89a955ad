// Shared host/device definitions for the MI355X rdc allreduce path.
#pragma once
#include <stddef.h>
#include <stdint.h>

// mpi::DataType (include/core/mpi.h:19-30) + MI355X-build additions
enum {
    RDC_DT_INT8 = 0,
    RDC_DT_UINT8 = 1,
    RDC_DT_INT32 = 2,
    RDC_DT_UINT32 = 3,
    RDC_DT_INT64 = 4,
    RDC_DT_UINT64 = 5,
    RDC_DT_FLOAT32 = 6,
    RDC_DT_FLOAT64 = 7,
    RDC_DT_LONGLONG = 8,
    RDC_DT_ULONGLONG = 9,
    RDC_DT_FLOAT16 = 10,
    RDC_DT_BFLOAT16 = 11,
    RDC_DT_COUNT = 12
};
// mpi::OpType (include/core/mpi.h:12-17)
enum { RDC_OP_MAX = 0, RDC_OP_MIN = 1, RDC_OP_SUM = 2, RDC_OP_BITOR = 3, RDC_OP_COUNT = 4 };

// allreduce data-movement schedules
enum {
    RDC_ALGO_AUTO = 0,
    RDC_ALGO_RING = 1,  // the reference's ring: n-1 reduce-scatter + n-1 allgather steps
    RDC_ALGO_MESH = 2,  // direct all-links exchange, same per-chunk accumulation order
    RDC_ALGO_ONESHOT = 3,  // small buffers: every rank pushes all of it, every rank folds (one hand-off)
    RDC_ALGO_TREE = 4,     // the reference's tree ORDER (TryAllreduceTree, buffers <= rdc_reduce_ring_mincount),
                           // moved like the one-shot: every rank folds all n inputs in the tree's order
    RDC_ALGO_MESH_PULL = 5,  // the mesh moved by remote LOADS: ranks stage their chunks in their own scratch,
                             // owners pull and fold, peers pull the results (same fold order)
    RDC_ALGO_DIRECT = 6      // registered user buffers: owners fold straight out of every rank's buffer and
                             // write the result straight back (no scratch; multi-process, device buffers)
};

// launch kinds (recorded on the device: the next launch reads the previous kind)
// (tree launches use the one-shot's slot protocol and record RDC_KIND_ONESHOT;
// RDC_KIND_TREE only names the kernel in occupancy queries)
enum { RDC_KIND_NONE = 0, RDC_KIND_MESH = 1, RDC_KIND_RING = 2, RDC_KIND_BCAST = 3, RDC_KIND_ALLGATHER = 4,
       RDC_KIND_ONESHOT = 5, RDC_KIND_TREE = 6, RDC_KIND_DIRECT = 7 };

#define RDC_MAX_RANKS 16
// 64-bit words from one hand-off flag to the next: 1 = packed (the default);
// a build with 16 puts each flag in a 128-B line of its own (tried in round 5
// against the lost hand-off of DESIGN.md §4.2: no effect; it costs 16x the
// flag memory, 255 MiB per rank at n = 8 and the default scratch)
#ifndef RDC_FLAG_STRIDE
#define RDC_FLAG_STRIDE 1
#endif
#define RDC_SLOT_ALIGN 256         // scratch images keep the user buffer's address mod 256
#define RDC_MIN_TILE (16u << 10)   // smallest tile, bytes

// device error codes written to the communicator's error word
enum {
    RDC_KERR_NONE = 0,
    RDC_KERR_TIMEOUT_RS = 1,
    RDC_KERR_TIMEOUT_AG = 2,
    RDC_KERR_TIMEOUT_BCAST = 3,
    RDC_KERR_TIMEOUT_RING = 4,
    RDC_KERR_TIMEOUT_ALLGATHER = 5,
    // a peer's hand-off carried this launch's sequence number but another
    // communicator's tag: ranks issued the collectives of communicators that
    // share a channel in different orders (rdc_device.h kTagBits)
    RDC_KERR_ORDER = 6,
    // RDC_SEQ_CHECK: two blocks of one launch read different launch numbers
    RDC_KERR_SEQ = 7
};

static inline size_t rdc_dtype_size(int dtype) {
    switch (dtype) {
        case RDC_DT_INT8: case RDC_DT_UINT8: return 1;
        case RDC_DT_INT32: case RDC_DT_UINT32: case RDC_DT_FLOAT32: return 4;
        case RDC_DT_INT64: case RDC_DT_UINT64: case RDC_DT_FLOAT64:
        case RDC_DT_LONGLONG: case RDC_DT_ULONGLONG: return 8;
        case RDC_DT_FLOAT16: case RDC_DT_BFLOAT16: return 2;
        default: return 0;
    }
}
static inline int rdc_dtype_is_float(int dtype) {
    return dtype == RDC_DT_FLOAT32 || dtype == RDC_DT_FLOAT64 || dtype == RDC_DT_FLOAT16 ||
           dtype == RDC_DT_BFLOAT16;
}

// Everything one collective launch needs.  Passed by value as the kernel
// argument (< 1.5 KiB).  Peer pointers are IPC-mapped (multi-process) or
// direct (single-process); index [rank] is the local one.
struct CollArgs {
    char* user;                          // local in-place buffer (byte 0 of the whole buffer)
    int n;                               // ranks
    int rank;
    int root;                            // broadcast root
    uint64_t tile_bytes;                 // multiple of RDC_SLOT_ALIGN
    int tiles[RDC_MAX_RANKS];            // tiles in chunk c for this launch
    uint64_t off[RDC_MAX_RANKS];         // byte offset of chunk c's piece in `user`
    uint64_t len[RDC_MAX_RANKS];         // byte length of chunk c's piece
    uint32_t mis[RDC_MAX_RANKS];         // off[c] % 16: scratch image alignment (rank-independent)
    int8_t fold[RDC_MAX_RANKS];          // range c is folded in the ring order of Split chunk fold[c]
                                         //   (= c for a whole buffer; host pieces cut one chunk's range
                                         //   into n ranges, one per owner, all folding in its order)
    uint64_t slot_bytes;                 // scratch slot stride
    uint32_t max_tiles;                  // flag array row stride (in flags)
    char* rs[RDC_MAX_RANKS];             // rank p's reduce-scatter scratch region
    char* ag[RDC_MAX_RANKS];             // rank p's allgather scratch region
    uint64_t* flags[RDC_MAX_RANKS];      // rank p's flag region: [2n][max_tiles] + done[n] (rdc_device.h seq)
    char* cbuf[RDC_MAX_RANKS];           // allgather: local buffer of rank c's data (off/len index into it)
    int nb_scatter, nb_reduce, nb_gather;  // mesh block roles (allgather: push / -, gather)
    uint32_t* err;                       // local device error word
    uint32_t* err_mirror;                // host-pinned copy of *err, refreshed by every launch's last block
    uint32_t* notify;                    // optional pinned word: the last block stores notify_val there when
    uint32_t notify_val;                 //   the launch is complete (host spins on it instead of a stream sync)
    uint32_t* done_ctr;                  // local per-launch block arrival counter (self-resetting)
    uint64_t* launch_ctr;                // local count of completed launches (device-side seq counter)
    uint32_t* launch_kind;               // local: kind of the last completed launch
    uint32_t tag;                        // communicator's tag on its channel: bits 0-7 of every seq
    int kind;                            // this launch's RDC_KIND_*
    int pull;                            // mesh: 1 = pull mode (RDC_ALGO_MESH_PULL, mesh_pull_body)
    int bcast_split;                     // broadcast: root -> forwarder per tile -> other ranks (n >= 3)
    uint64_t half_bytes;                 // one-shot: offset of the slot half used by odd seq
    uint64_t total_bytes;                // one-shot: whole buffer bytes
    int tree_len;                        // tree: fold program acc[tree_dst[i]] = OP(acc[tree_dst[i]],
    int8_t tree_dst[RDC_MAX_RANKS];      //   acc[tree_src[i]]), i < tree_len, over the n inputs indexed
    int8_t tree_src[RDC_MAX_RANKS];      //   by rank; the result is acc[0] (rdc_plan.h PlanTreeProgram)
    const void* units;                   // coalesced mesh: device PackUnit table (off/len are packed
    int nunits;                          //   offsets; user bytes reached through the units), else null;
                                         //   coalesced direct: nunits items {buffer, offset, length}
                                         //   (3 words each), then every rank's dnbuf buffer addresses
    int dnbuf;                           // coalesced direct: buffers in the list
    int rotate;                          // direct: owner r starts its tile (item) walk r/n of the way in
    uint64_t timeout_ticks;              // wall_clock64 ticks (100 MHz) before giving up
    int uc;                              // 1: every scratch region is uncached (hand-offs need no L2
                                         //   write-back, rdc_device.h block_publish)
    uint64_t* trace;                     // optional (mesh/ring): per block {start, end} wall_clock64 ticks
    int seq_check;                       // RDC_SEQ_CHECK: every block checks it read the launch number the
                                         //   launch's first block read (err words 80-81; a mismatch is
                                         //   recorded in err words 72..79)
    uint32_t* verify;                    // RDC_VERIFY_PUBLISH (debug): publish read-back counters (err words 84..)
    int poll_rmw;                        // RDC_POLL_RMW (debug): hand-off polls as atomic adds of 0
    int poison;                          // RDC_POISON_SCRATCH: consumers overwrite scratch ranges they
                                         //   finished reading with 0xFF (rdc_device.h block_poison)
    uint64_t* tlog;                      // RDC_LAUNCH_TIMES (debug): per launch {seq, block 0 start, latest block
                                         //   start, last block end} (wall_clock64) in a ring of 64 entries
};

// ------------------------------------------------ small-allreduce service --
// A resident one-block kernel per rank (k_svc) that serves small synchronous
// HOST-buffer allreduces from a pinned mailbox without a kernel launch per
// call; it exits after RDC_HOST_SERVICE_IDLE_US of idleness (rdc_service.h).
#define RDC_SVC_MAX_BYTES (64u << 10)  // largest buffer it serves
#define RDC_SVC_SLOT_BYTES (2u * RDC_SVC_MAX_BYTES)  // one rank's LL words: two planes of RDC_SVC_MAX_BYTES
#define RDC_SVC_LL_MAX (16u << 10)  // largest input sent over PCIe as LL words
// host exchange (rdc_service.h): every rank's LL input in one POSIX shared
// host region, [2 halves][n ranks][RDC_SVC_HX_RANK_BYTES], read by every
// rank's service block over PCIe (no xGMI hand-off)
#define RDC_SVC_HX_RANK_BYTES (2u * RDC_SVC_LL_MAX)
enum { RDC_SVC_NEVER = 0, RDC_SVC_RUNNING = 1, RDC_SVC_EXITING = 2, RDC_SVC_EXITED = 3 };

// The request side of a rank's mailbox, written by the host, polled by the
// resident block: device memory the CPU writes through the PCIe BAR when the
// runtime gives the CPU access to the GPU's fine-grained uncached pool (the
// block then polls local HBM instead of reading host memory over PCIe every
// round: round trip 1.8 vs 2.6 us, tools/mailbox_rtt.hip), else pinned
// uncached host memory.
struct SvcIn {
    // request header, itself an LL word:
    //   (seq << 32) | tree << 31 | LL input << 30 | LL result << 29 | host exchange << 28 | bytes
    alignas(64) uint64_t hdr;
    alignas(64) uint32_t stop;    // host: exit now
    // the input: LL words {4 payload bytes, seq} in two planes of RDC_SVC_LL_MAX
    // (k_svc), or as is
    alignas(256) char data[RDC_SVC_MAX_BYTES];
};

struct SvcBox {  // the answer side: pinned host memory, hipHostMallocUncached; one per rank
    alignas(64) uint32_t done;    // device: last completed request
    alignas(64) uint32_t state;   // device: RDC_SVC_*
    alignas(64) uint32_t err;     // device: RDC_KERR_* of a failed request (sticky)
    alignas(64) uint64_t trace[4];  // RDC_SVC_TRACE: wall clock at request seen / input sent / peers in / result out
    alignas(256) char out[RDC_SVC_MAX_BYTES];  // the result: LL words (two planes) or as is
};

struct SvcArgs {
    SvcBox* box;                    // device address of this rank's mailbox (answers)
    SvcIn* in;                      // device address of its request side (VRAM or pinned host memory)
    char* region[RDC_MAX_RANKS];    // rank p's service slots: [2 halves][n] x RDC_SVC_SLOT_BYTES (uncached)
    uint32_t* derr;                 // device error word of the service (the mailbox gets a copy)
    int n, rank;
    int strict;                     // RDC_STRICT_FENCES: system fence before `done`
    int trace;                      // RDC_SVC_TRACE: stamp SvcBox::trace per request
    int eager;                      // threads that read their LL input vector while polling the header
    char* hx;                       // device address of the host exchange region, or null
    int hx_eager;                   // threads that poll every rank's exchange words of their vector
                                    //   while polling the header
    int pipe;                       // RDC_HOST_SERVICE_PIPELINE: two poll rounds in flight
    uint64_t idle_ticks;            // wall_clock64 ticks without a request before exiting
    uint64_t timeout_ticks;         // waiting for a peer's contribution
    int tree_len;
    int8_t tree_dst[RDC_MAX_RANKS];
    int8_t tree_src[RDC_MAX_RANKS];
};
