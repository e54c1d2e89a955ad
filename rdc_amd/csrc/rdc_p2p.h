// Point-to-point Send/Recv on the device path — the counterpart of the
// reference's ICommunicator::Send/Recv/ISend/IRecv (include/comm/
// communicator.h:56-80, src/comm/communicator_base.cc:303-320) and of the
// WorkCompletion it returns (include/core/work_request.h:240-270), which rdc's
// Python package binds as RdcISend/RdcIRecv/RdcWorkCompletion* (rdc/comm.py).
//
// Data moves GPU to GPU: the sender's copy kernel writes each piece (<= one
// slot) straight into the receiver's IPC-mapped p2p slot for this sender over
// xGMI; the receiver copies it out.  No kernel ever waits: the hand-off lives
// in a small control block of host shared memory (POSIX shm between the
// node's processes, registered for device access), one writer per word,
// written by the copy kernels' last block:
//     posted[src][dst]   pieces src has landed in dst's slots
//     consumed[src][dst] pieces dst has copied out (slot reusable)
// and a per-communicator progress thread drives both directions for every
// peer, so an IRecv posted before the matching ISend, or exchanges in any
// order, make progress (the reference's epoll + thread pool role).
// Messages are matched in order per (src, dst) pair and must have equal
// sizes on both sides (the reference's byte stream is used that way by its
// callers, test/sendrecv.cc); a size mismatch is reported as an error.
#pragma once
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rdc_common.h"

namespace rdc_amd {

constexpr int kP2PSlots = 2;

// reference WorkStatus values (include/core/work_request.h:23-30)
enum { RDC_WS_PENDING = 1 << 1, RDC_WS_RUNNING = 1 << 2, RDC_WS_FINISHED = 1 << 3, RDC_WS_ERROR = 1 << 6 };

// Control block.  Lives on pages of its own (a POSIX shm mapping, or a
// hipHostMalloc'd block for single-process groups), registered for device
// access as ONE range: the copy kernels' only host-memory access is the
// system-scope store of `posted` / `consumed` into it.  Round 1 saw one
// illegal address in test_device_to_device when the group block was a
// heap object registered with hipHostRegister: the registration covered
// whole pages shared with unrelated heap allocations, and the runtime pins
// and unpins pageable pages around its own copies, which can drop the GPU
// mapping of exactly those pages; k_copy's `word` store (the last block's
// release of posted / consumed) was the only access to such a page — its
// `arrive` counter is hipMalloc'd HBM and its data pointers are HBM slots
// and the user's device buffer.  P2PEngine now refuses a block that is not
// page-aligned and mapped as one contiguous range (checked_ctl_mapping), and
// every launch checks its slot range, arrival counter and control word.
struct P2PCtl {  // 64-B lines; 16 pages
    struct alignas(64) Word {
        std::atomic<uint64_t> v;
    };
    Word posted[RDC_MAX_RANKS][RDC_MAX_RANKS];
    Word consumed[RDC_MAX_RANKS][RDC_MAX_RANKS];
    Word len[RDC_MAX_RANKS][RDC_MAX_RANKS][kP2PSlots];  // bytes of the piece in each slot
};

// The reference's WorkCompletion (work_request.h:240-270).  Two owners: the
// caller (released by RdcDelWorkCompletion) and the engine (released when the
// request finishes), so dropping a pending completion is safe.
class WorkComp {
public:
    int Wait();                 // blocks; 0 = finished, else error
    int Status() const { return status_.load(); }
    std::string error();
    void Release();             // drop one owner; the last one frees

private:
    friend class P2PEngine;
    void Finish(int status, const std::string& err);
    std::atomic<int> status_{RDC_WS_PENDING};
    std::atomic<int> refs_{2};
    std::mutex mu_;
    std::condition_variable cv_;
    std::string err_;
};

class P2PEngine {
public:
    // rank r's view: local slot region, peers' regions (IPC-mapped), shared control block
    // a lane with queued requests that moves nothing for timeout_s fails them
    P2PEngine(int rank, int n, int device, size_t slot_bytes, char* local, char* const* peers, P2PCtl* ctl,
              double timeout_s);
    ~P2PEngine();
    // `after` (may be null): the engine's copies start after the work queued
    // on this stream so far (the producer of a send / last reader of a recv)
    WorkComp* ISend(const void* buf, size_t bytes, int dest, hipStream_t after);
    WorkComp* IRecv(void* buf, size_t bytes, int src, hipStream_t after);

private:
    struct Req {
        WorkComp* wc;
        char* buf;
        size_t bytes;
        bool host;                  // buf is host memory
        hipEvent_t ready = nullptr; // recorded on the caller's stream at post time
        size_t issued = 0;          // bytes whose piece has been issued
        size_t done = 0;            // bytes whose piece completed
        std::deque<std::pair<uint64_t, size_t>> inflight;  // (piece seq, piece bytes)
    };
    struct Lane {           // one direction with one peer
        std::deque<Req> q;
        uint64_t seq_issued = 0, seq_done = 0;  // pieces
        hipStream_t stream = nullptr;
        char* bounce = nullptr;                 // send side: device staging of host pieces, kP2PSlots slots
        std::chrono::steady_clock::time_point last;  // last movement (or first request)
    };
    WorkComp* Post(Lane& L, char* buf, size_t bytes, hipStream_t after);
    void Loop();
    bool Progress();        // one pass; true if anything moved
    bool Complete(Lane& L, const std::atomic<uint64_t>& word);
    uint64_t* DevWord(const std::atomic<uint64_t>& w) const;  // device address of a control word (range-checked)
    void CheckLaunch(const char* slot_base, size_t slot_off, size_t len, const uint32_t* arrive) const;
    bool StepSend(int peer, Lane& L);
    bool StepRecv(int peer, Lane& L);
    void Ready(Lane& L, Req& r);
    hipEvent_t Event();
    void Fail(Lane& L, const std::string& err);

    int rank_, n_, device_;
    size_t slot_bytes_;
    double timeout_s_;
    char* local_;
    char* peers_[RDC_MAX_RANKS];
    P2PCtl* ctl_;
    char* ctl_dev_ = nullptr;      // the control block's device address (host-registered)
    uint32_t* arrive_ = nullptr;   // device: copy-kernel arrival counters [send n | recv n]
    Lane send_[RDC_MAX_RANKS], recv_[RDC_MAX_RANKS];
    std::vector<hipEvent_t> free_events_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
    int pending_ = 0;       // queued requests
    std::thread th_;
};

}  // namespace rdc_amd
