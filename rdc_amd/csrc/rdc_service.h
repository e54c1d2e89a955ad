// Small-allreduce service: synchronous allreduces of small HOST buffers (the
// reference's own setting, rdc/core.py:172-217 — BASELINE cfg1 is a 4 KiB
// fp32 allreduce) without a kernel launch per call.
//
// A launch-per-call path pays the host launch, the GPU dispatch and the
// kernel's completion before the caller sees its result (DESIGN.md §5.3:
// 14.6 us for a 4 KiB allreduce of device memory at n = 2, 17.4 us from host
// memory).  Here each rank keeps ONE resident block (k_svc) while calls keep
// coming.  The host writes its input into a pinned, GPU-uncached mailbox —
// up to RDC_HOST_SERVICE_LL_BYTES as LL words (4 payload bytes + the request's
// sequence number per 8, planar) — and then one header word (seq, tree order,
// LL input, LL result, bytes).  The block polls the header together with the
// first 4 KiB of LL input (so a small request's data usually arrives with the
// poll that finds it), stores its input as LL words into its slot of every
// peer's service region (xGMI), then each thread polls the peers' words for
// its own vectors, folds every element in the reference's order (Split chunk
// ring order, or the tree's order at or below rdc_reduce_ring_mincount)
// through LDS, and writes the result into the mailbox: as LL words the host
// polls (<= 256 B), or as is, drained, followed by `done`.
//
// The block exits after RDC_HOST_SERVICE_IDLE_US (default 1000) without a
// request, when the host sets `stop` (another (dtype, op), teardown) or when
// a peer never arrives (RDC_TIMEOUT): nothing stays resident, and a
// device-wide synchronisation waits at most the idle time.  The next call
// relaunches it (state EXITING closes the race with a request posted while it
// leaves: host store header / load state, device store state / fence / load
// header).  Its slots are its own, not the channel's scratch, so it never
// races the channel's stream-ordered launches.
//
// Host exchange (round 4, opt-in): when n * bytes <= RDC_HOST_SERVICE_HX_BYTES
// (default 0 = off; e.g. 32768) and the input goes as LL words, every rank's host writes
// them into its slot of ONE region of POSIX shared host memory that every
// rank maps and registers (uncached on the GPU side), and every rank's block
// reads all n inputs from it — the xGMI send and the peers' polls leave the
// critical path (request seen -> input sent -> peers in was 1.9-2.3 us of a
// 7.9 us call, profiles/r04/host_registered_events/svc4k_trace.txt).  Each GPU
// then reads n * bytes of LL words over its own PCIe link, so it is for small
// n * bytes only.  The first RDC_HOST_SERVICE_HX_EAGER_BYTES of the ranks'
// inputs together (default 8 KiB) are polled with the header.
// RDC_HOST_SERVICE=0 disables it; with more than RDC_HOST_SERVICE_SHARE_MAX
// (default 4) ranks on one GPU it is not used (their persistent blocks'
// queues get time-sliced by the hardware scheduler).
#pragma once
#include <hip/hip_runtime_api.h>

#include <mutex>
#include <vector>

#include "rdc_common.h"
#include "rdc_kernels.h"

namespace rdc_amd {

class SmallService {
public:
    // region: every rank's service slots (peers' IPC-mapped or direct); derr:
    // a device word for the kernel's errors
    // hx: this process's mapping of the channel's host exchange region
    // ([2][n] x RDC_SVC_HX_RANK_BYTES, registered for the device), or null
    SmallService(int rank, int n, int device, char* const* region, uint32_t* derr,
                 int tree_len, const int* tree_dst, const int* tree_src, double timeout_s, int wall_khz,
                 char* hx = nullptr);
    // n * bytes budget of the host exchange (RDC_HOST_SERVICE_HX_BYTES, default
    // 0 = off): a plan key, every rank must agree
    static uint64_t HxBytes();
    ~SmallService();
    static bool Enabled();
    // most ranks per GPU it runs with (RDC_HOST_SERVICE_SHARE_MAX, default 4)
    static int ShareMax();
    // false when the uncached mailbox could not be allocated (no service then)
    bool Usable() const;
    // in place on `host` (bytes <= RDC_SVC_MAX_BYTES); the kernel derives the
    // Split chunks from bytes / sizeof(T); tree: fold in the tree's order.
    // Synchronous; throws on a device-side failure (the service is then unusable).
    void Allreduce(const KernelSet& ks, int kind, char* host, uint64_t bytes, bool tree);

private:
    void Stop();
    void EnsureRunning(const KernelSet& ks, int kind);

    int rank_, device_;
    double timeout_s_;
    SvcArgs args_;
    SvcBox* box_ = nullptr;       // host address
    SvcIn* in_ = nullptr;         // host (CPU) address of the request side
    bool in_vram_ = false;        // in_ is device memory written through the BAR (else pinned host memory)
    hipStream_t stream_ = nullptr;
    int kind_ = -1;               // (dtype, op) of the kernel launched last, -1 none
    bool launched_ = false;
    bool broken_ = false;
    uint32_t req_ = 0;
    int n_ = 1;
    char* hx_ = nullptr;  // host address of the exchange region, or null
    int wall_khz_ = 100000;
    uint64_t ll_bytes_ = RDC_SVC_LL_MAX;  // LL input up to this many bytes
    uint64_t ll_out_bytes_ = 0;           // LL result up to this many bytes (set from the env in the ctor)
    // 8-byte LL word of payload word j in the planar layout (k_svc)
    static uint64_t ll_index(uint64_t j) { return ((j >> 1) & 1) * (RDC_SVC_LL_MAX / 8) + 2 * (j >> 2) + (j & 1); }
    std::vector<uint64_t> stage_ = std::vector<uint64_t>(RDC_SVC_LL_MAX / 4);  // LL input words, built here
    double tr_[4] = {0, 0, 0, 0};  // RDC_SVC_TRACE sums: host us, device ticks per phase
    long traced_ = 0;
    double ht_[1] = {0};  // RDC_SVC_TRACE: LL encode time
    std::mutex mu_;
};

}  // namespace rdc_amd
