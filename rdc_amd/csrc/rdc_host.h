// Host-resident allreduce (rdc's own setting: buffers begin and end in host
// memory — rdc/core.py:172-217, test/allreduce.cc), pipelined over PCIe.
//
// The buffer's Split chunks (include/utils/utils.h:59-70) are cut into K
// pieces; piece k holds the k-th slice of EVERY chunk, so each piece is a
// balanced allreduce in its own right and every element is still folded in
// its chunk's ring order (bit-identical to one whole-buffer allreduce).
// Per piece, on three streams, all issued by the caller in stream order:
//   host threads memcpy the slices into a pinned input slot -> H2D DMA (copy
//   stream) -> allreduce of the slices on the communicator's stream -> D2H DMA
//   into a pinned output slot (second copy stream, waiting on the allreduce's
//   event) -> a drain thread's copy pool memcpys the slices back into the
//   pageable buffer,
// so the DMA engines never wait for a host thread to wake up: piece k's D2H
// starts when its allreduce ends, piece k+1's H2D runs beside it.  Pinned DMA
// runs 57 GB/s each way (48 GB/s duplex); pageable H2D 12-22 GB/s, and a
// pageable D2H blocks the issuing thread (tools/host_copy_bench.cpp, DESIGN.md
// §5.3), so both directions are staged through pinned slots.
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

// RDC_HOST_PIECE_BYTES (default 8 MiB): every rank cuts a pipelined host
// buffer into the same pieces, so it is one of the plan keys agreed at
// communicator creation (rdc_comm.cpp PlanKey)
size_t HostPieceBytes();

// fixed pool of memcpy threads; Run(n, f) calls f(0..n-1) across the pool
// and the caller, returning when all are done

class HostPath {
public:
    // zc_max: buffers up to this many bytes run zero-copy on pinned memory
    HostPath(int device, size_t zc_max);
    ~HostPath();
    // in place; synchronous (returns after the result is back in `host`)
    void Allreduce(Communicator* c, void* host, size_t count, int dtype, int op, hipStream_t comm_stream);

private:
    static constexpr int kSlots = 3;     // pinned input slots
    static constexpr int kOutSlots = 4;  // pinned output slots
    struct Drain {                 // one piece for the drain thread
        hipEvent_t ready;          // the piece's D2H into its output slot finished
        int nslice;
        int oslot;
        uint64_t off[RDC_MAX_RANKS], len[RDC_MAX_RANKS], pos[RDC_MAX_RANKS];
    };
    void Reserve(size_t piece_bytes, size_t total_bytes, int pieces, hipStream_t comm_stream);
    void QuiesceForRegrow(hipStream_t comm_stream);
    static void Copy(CopyPool& pool, char* dst, const char* src, size_t bytes);  // parallel memcpy
    void Copy(char* dst, const char* src, size_t bytes) { Copy(pool_, dst, src, bytes); }
    void DrainLoop();

    // buffers up to kSmall: one pinned round trip, one synchronisation
    static constexpr size_t kSmall = (size_t)1 << 20;
    void AllreduceSmall(Communicator* c, char* host, size_t count, size_t bytes, int dtype, int op,
                        hipStream_t comm_stream);

    int device_;
    hipStream_t h2d_ = nullptr, d2h_ = nullptr;
    char* pin_small_ = nullptr;      // kSmall bytes + the error word
    hipEvent_t small_done_ = nullptr;  // the staged small path's D2H
    static void SpinEvent(hipEvent_t e, const char* what);
    char* pin_small_dev_ = nullptr;  // its device address
    size_t zc_max_ = 0;
    char* dev_small_ = nullptr;
    hipEvent_t in_done_[kSlots] = {};
    std::vector<hipEvent_t> ar_done_;   // one per piece of the current call: allreduce finished
    std::vector<hipEvent_t> out_done_;  // ... and its D2H into the output slot
    char* pin_in_[kSlots] = {};
    char* pin_out_[kOutSlots] = {};
    size_t slot_bytes_ = 0;
    char* dev_ = nullptr;  // device image of the buffer
    size_t dev_bytes_ = 0;
    CopyPool pool_;      // the caller's copies (input)
    CopyPool out_pool_;  // the drain thread's copies (output)
    // drain thread: output slots of finished pieces -> the user's buffer
    std::thread drain_;
    std::mutex dmu_;
    std::condition_variable dcv_, ddone_cv_;
    std::vector<Drain> queue_;
    size_t qhead_ = 0, drained_ = 0;  // drained_: pieces copied out (their output slots free again)
    char* dst_ = nullptr;          // user buffer of the current call
    std::string derr_;             // first drain-thread error of the current call
    bool dstop_ = false;
};

}  // namespace rdc_amd
