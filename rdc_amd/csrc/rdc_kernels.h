// Host-visible launchers of the gfx950 kernels (rdc_kernels.hip).
#pragma once
#include <hip/hip_runtime_api.h>

#include "rdc_common.h"
#include "rdc_plan.h"

namespace rdc_amd {

struct KernelSet {
    hipError_t (*reduce)(char* dst, const char* src, uint64_t nbytes, int grid, hipStream_t s);
    hipError_t (*mesh)(const CollArgs& a, int grid, hipStream_t s);
    hipError_t (*ring)(const CollArgs& a, int grid, hipStream_t s);
    hipError_t (*oneshot)(const CollArgs& a, int grid, hipStream_t s);
    hipError_t (*tree)(const CollArgs& a, int grid, hipStream_t s);
    hipError_t (*direct)(const CollArgs& a, int grid, hipStream_t s);  // registered user buffers (k_direct)
    hipError_t (*svc)(const SvcArgs& a, hipStream_t s);  // the small-allreduce service (one block)
    // resident blocks per CU of the kernel a launch of `kind` (RDC_KIND_MESH /
    // RING / ONESHOT / TREE) on n ranks uses (hipOccupancyMaxActiveBlocksPerMultiprocessor,
    // cached); the grid clamp of ResidentGrid (rdc_plan.h)
    int (*occupancy)(int kind, int n);
};

// false if (dtype, op) is not a valid reference combination
bool get_kernels(int dtype, int op, KernelSet* ks);
// resident blocks per CU of k_bcast / k_allgather
int occupancy_bcast();
int occupancy_allgather();
hipError_t launch_bcast(const CollArgs& a, int grid, hipStream_t s);
hipError_t launch_allgather(const CollArgs& a, int grid, hipStream_t s);
// coalesced allreduce: units[i].buf = user address; unpack = image -> buffers
hipError_t launch_pack(const PackUnit* units, int nunits, char* image, int unpack, int grid, hipStream_t s);
// plain device copy (dst may be IPC-mapped peer memory); never waits.
// With `word` (host-mapped): the last block to finish stores `value` there
// (system-scope release, after every block's system fence); `arrive` is a
// zeroed device counter owned by the stream (reset by that last block).
hipError_t launch_copy(void* dst, const void* src, uint64_t bytes, hipStream_t s, uint32_t* arrive = nullptr,
                       uint64_t* word = nullptr, uint64_t value = 0);
// xGMI probe: block b copies its share of `bytes` from src (or srcs[b % ndst]
// when set: remote reads) into dsts[b % ndst]
struct PushTargets {
    char* dst[RDC_MAX_RANKS];
    const char* src[RDC_MAX_RANKS];
};
hipError_t launch_push(const PushTargets& t, int ndst, const void* src, uint64_t bytes, int grid, hipStream_t s);
hipError_t launch_fill(void* buf, uint64_t count, int dtype, uint64_t seed, int rank, hipStream_t s);

}  // namespace rdc_amd
