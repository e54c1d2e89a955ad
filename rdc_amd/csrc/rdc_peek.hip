// The bytes [src, src + len) (len <= 8) read through a peer mapping, for the
// direct schedule's check that a newly mapped peer allocation is the buffer
// its exporter holds now (the canary of Communicator::AllreduceDirect,
// DESIGN.md §4.3).  System-scope loads of the aligned words that hold them:
// the mapping is new, but its physical pages may have been read through
// another mapping before.  Only words that overlap the range are read.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rdc_amd {

__global__ void k_peek(const char* src, uint32_t len, uint8_t* dst) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>((uintptr_t)src & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)((uintptr_t)src & 7);
    const uint64_t lo = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t hi = sh + len > 8 ? __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
    for (uint32_t i = 0; i < len; ++i) {  // no local array: registers only
        const uint32_t k = sh + i;
        dst[i] = (uint8_t)((k < 8 ? lo : hi) >> (8 * (k & 7)));
    }
}

// dst[0, len) = the low len bytes of v, then a system-scope release: the
// bytes are in memory (not only in this XCD's L2) when the kernel ends, for a
// peer reading them through its mapping from another XCD or another GPU
__global__ void k_poke(char* dst, uint32_t len, uint64_t v) {
    for (uint32_t i = 0; i < len; ++i) dst[i] = (char)(v >> (8 * i));
    __threadfence_system();
}

hipError_t Poke(void* dst, uint32_t len, uint64_t v, hipStream_t s) {
    if (len > 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_poke, dim3(1), dim3(1), 0, s, static_cast<char*>(dst), len, v);
    return hipGetLastError();
}

hipError_t Peek(const void* src, uint32_t len, void* dst, hipStream_t s) {
    if (len > 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_peek, dim3(1), dim3(1), 0, s, static_cast<const char*>(src), len, static_cast<uint8_t*>(dst));
    return hipGetLastError();
}

}  // namespace rdc_amd
