// Host-resident allreduce (rdc's own setting: buffers begin and end in host
// memory — rdc/core.py:172-217, test/allreduce.cc), pipelined over PCIe.
//
// The buffer is cut into K contiguous pieces (RDC_HOST_PIECE_BYTES); piece k's
// allreduce gets the Split chunk ranges (include/utils/utils.h:59-70) it
// intersects, so every element is still folded in its own chunk's ring order
// (bit-identical to one whole-buffer allreduce) while each piece moves as one
// copy in, one H2D and one D2H.
// Per piece, on three streams:
//   host threads memcpy the slices into a pinned slot -> H2D DMA (copy stream)
//   -> allreduce of the slices on the communicator's stream
//   -> a drain thread waits for it and copies the slices straight back into
//      the pageable buffer (D2H on a second copy stream),
// so piece k+1's H2D and piece k-1's D2H run under piece k's allreduce.
// On the box pageable H2D runs 12-22 GB/s but pinned DMA 57 GB/s, while
// pageable D2H already runs 56 GB/s (tools/host_copy_bench.cpp):
// stage the input only.
#pragma once
#include <hip/hip_runtime_api.h>

#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rdc_comm.h"
#include "rdc_copypool.h"

namespace rdc_amd {

// RDC_HOST_PIECE_BYTES (default 16 MiB): every rank cuts a pipelined host
// buffer into the same pieces, so it is one of the plan keys agreed at
// communicator creation (rdc_comm.cpp PlanKey)
size_t HostPieceBytes();
// RDC_HOST_PIECE_RAMP (default 1): small first and last pieces (a plan key too)
bool HostPieceRamp();
// RDC_HOST_INLINE_BYTES (default 16 MiB): host buffers up to this size go as
// ONE piece on the caller's thread, larger ones through the pipeline (a plan key)
size_t HostInlineBytes();
// the pipeline's piece boundaries for an S-byte host buffer: {0, ..., S}
std::vector<uint64_t> HostPieceBounds(uint64_t S);

// Host ranges page-locked through RdcNewBuffer(..., pinned = 1) (rdc/buffer.py:
// 34-38, the reference's registered Buffer).  A host allreduce whose whole
// buffer lies in one of them skips the pinned slots, the copy pool and the
// drain thread: the DMA engines read and write the user's pages directly
// (HostPath::AllreduceRegistered).  The caller keeps a registered range alive
// until RdcDelBuffer, as with any registration.
void HostRegistryAdd(const void* p, size_t bytes);
void HostRegistryRemove(const void* p);
// RDC_HOST_BALANCE: -1 unset (balanced host pieces with one rank per GPU), 0 off, 1 on
int HostBalanceSetting();
// *base (may be null) = the registered range's start
bool HostRegistryCovers(const void* p, size_t bytes, const void** base = nullptr);
// RDC_HOST_REG_ZC=1: registered host buffers are reduced in place over PCIe (no DMA)
bool RegisteredZeroCopy();
// RDC_HOST_REG_KCOPY (default 1): the registered path copies with kernels, not DMA
bool RegisteredKernelCopy();
// host allreduces of this process that took the registered path
uint64_t HostRegisteredCalls();

class HostPath {
public:
    // buffers up to kSmall: one pinned round trip, one synchronisation (no DMA)
    static constexpr size_t kSmall = (size_t)1 << 20;
    // zc_max: buffers up to this many bytes run zero-copy on pinned memory
    HostPath(int device, size_t zc_max);
    ~HostPath();
    // in place; synchronous (returns after the result is back in `host`)
    void Allreduce(Communicator* c, void* host, size_t count, int dtype, int op, hipStream_t comm_stream);
    // Bring up the copy path before the first timed call: H2D and D2H copies
    // of 64 KiB / 1 MiB / 16 MiB on every stream the host path copies on.
    // The first copies a process makes through the DMA engines stall ~7 ms
    // each while the runtime brings its SDMA queues up (measured: the first
    // two 64 MiB registered calls at n = 2 took 17 and 6.2 ms, every later
    // one ~4.3 ms; with HSA_ENABLE_SDMA=0 no call stalls;
    // profiles/r04/host_registered_events/).  Idempotent; RDC_HOST_WARM=0
    // skips it.
    void Warm(hipStream_t comm_stream);

private:
    static constexpr int kSlots = 3;
    struct Drain {                 // one piece for the drain thread
        hipEvent_t ready;          // the piece's allreduce finished
        int nslice;
        uint64_t off[RDC_MAX_RANKS], len[RDC_MAX_RANKS];
    };
    void Reserve(size_t piece_bytes, size_t total_bytes, int pieces, hipStream_t comm_stream);
    void QuiesceForRegrow(hipStream_t comm_stream);
    // parallel memcpy; to_pinned: into a staging slot only the DMA reads (streaming stores)
    void Copy(char* dst, const char* src, size_t bytes, bool to_pinned = false);
    void DrainLoop();

    void AllreduceSmall(Communicator* c, char* host, size_t count, size_t bytes, int dtype, int op,
                        hipStream_t comm_stream);
    // the same pieces and collectives as the pipeline, with the H2D / D2H DMA
    // straight from / into a registered user buffer, all stream-ordered
    void AllreduceRegistered(Communicator* c, char* host, size_t count, int dtype, int op, hipStream_t comm_stream,
                             const std::vector<uint64_t>& bounds, const int64_t* cb, const int64_t* ce);
    // RDC_HOST_REG_ZC: every piece's collective on the caller's registered pages
    void AllreduceRegisteredZeroCopy(Communicator* c, char* host, size_t count, int dtype, int op,
                                     hipStream_t comm_stream, const std::vector<uint64_t>& bounds,
                                     const int64_t* cb, const int64_t* ce);
    std::vector<hipEvent_t> h2d_done_;  // registered path: one per piece
    // RDC_HOST_EVENT_TRACE=1 (diagnostics): timing events around every
    // piece's H2D, allreduce and D2H of the registered path, summarised per
    // call on stderr — a complete timeline (every copy has its events)
    std::vector<hipEvent_t> tev_;
    void TraceRegistered(int K, const std::vector<uint64_t>& bounds, double host_ms);

    int device_;
    bool warm_ = false;
    hipStream_t h2d_ = nullptr, d2h_ = nullptr;
    char* pin_small_ = nullptr;      // kSmall bytes + the error word
    hipEvent_t small_done_ = nullptr;  // the staged small path's D2H
    static void SpinEvent(hipEvent_t e, const char* what);
    char* pin_small_dev_ = nullptr;  // its device address
    size_t zc_max_ = 0;
    char* dev_small_ = nullptr;
    hipEvent_t in_done_[kSlots] = {};
    std::vector<hipEvent_t> ar_done_;  // one per piece of the current call
    char* pin_in_[kSlots] = {};
    size_t slot_bytes_ = 0;
    char* dev_ = nullptr;  // device image of the buffer
    size_t dev_bytes_ = 0;
    CopyPool pool_;
    // drain thread: D2H of finished pieces into the user's buffer
    std::thread drain_;
    std::mutex dmu_;
    std::condition_variable dcv_, ddone_cv_;
    std::vector<Drain> queue_;
    size_t qhead_ = 0, drained_ = 0;
    char* dst_ = nullptr;          // user buffer of the current call
    std::string derr_;             // first drain-thread error of the current call
    bool dstop_ = false;
};

}  // namespace rdc_amd
