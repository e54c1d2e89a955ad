// Peer allocations of the direct schedule imported at addresses this process
// chooses (round 6).  HIP IPC (hipIpcOpenMemHandle) places a
// new peer mapping wherever the runtime likes, and a mapping placed partly
// over ranges the process unmapped faulted the GPU at its first use (rounds 5
// and 6), so such calls had to fall back.  Here the exporter hands each
// allocation over as a dma-buf (hsa_amd_portable_export_dmabuf), passed to
// every peer over a unix socket (SCM_RIGHTS; pidfd_getfd is not permitted on
// the pool's boxes), and the importer maps it with ROCr's virtual-memory API
// (hsa_amd_vmem_import_shareable_handle / hsa_amd_vmem_map / set_access) into
// an address arena it reserved: every mapping gets either addresses no mapping
// ever used or exactly the range of an unmapped one of the same size (the
// placement that never faulted), never a partial overlap.
// tools/vmem_import_probe.hip shows the mechanism on the box
// (profiles/r06/vmem/).
#pragma once

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace rdc_amd {

class Bootstrap;

class VmemImporter {
public:
    // Collective over `bs` (every rank calls it): a SOCK_SEQPACKET unix-socket
    // connection between every pair of ranks.  Null (and *why) when this rank
    // cannot take part; the caller agrees across ranks.
    static std::unique_ptr<VmemImporter> Create(Bootstrap* bs, int rank, int n, hsa_agent_t agent, double timeout_s,
                                                std::string* why);
    ~VmemImporter();

    // exporter: a dma-buf of the allocation [base, base + size) sent to every
    // peer, tagged with `id`; false (and *why) when it cannot be exported
    bool Export(void* base, size_t size, uint64_t id, std::string* why);
    // exporter: the allocation `id` is dead (retired).  Its dma-buf stays open
    // until then, so that a later export which the runtime resolves to this
    // same buffer object gets the same dma-buf file back and is refused
    void Release(uint64_t id);
    // importer: every peer's messages so far (non-blocking) into the pending
    // table; the exporter sent before the rendezvous stamp the caller waited on
    void Drain();
    // peer p's allocation `id` (received earlier) mapped here; *base = the
    // allocation's first byte.  False (and *why) when it was not received or
    // cannot be mapped.
    bool Map(int p, uint64_t id, char** base, size_t* size, std::string* why);
    // undo Map (the caller made sure no launch reads through it any more)
    void Unmap(char* base);
    // a received allocation never mapped whose exporter retired it
    void Forget(int p, uint64_t id);
    size_t pending() const { return pending_.size(); }
    size_t arena_bytes() const;

private:
    VmemImporter() = default;
    struct Msg {
        uint64_t id, offset, size;
    };
    struct Pending {
        int fd = -1;
        uint64_t offset = 0, size = 0;
    };
    struct Mapping {
        char* va = nullptr;   // start of the mapping (the dma-buf's first byte)
        size_t span = 0;      // mapped bytes (the dma-buf's size)
        hsa_amd_vmem_alloc_handle_t h{};
    };
    char* PlaceRange(size_t span);
    bool Recv(int p, bool block);

    int rank_ = 0, n_ = 0;
    hsa_agent_t agent_{};
    std::vector<int> sock_;                          // by peer rank (-1 for self)
    std::map<std::pair<int, uint64_t>, Pending> pending_;
    std::map<char*, Mapping> maps_;                  // by the base handed out
    struct Arena {
        char* base = nullptr;
        size_t size = 0, used = 0;
    };
    std::vector<Arena> arenas_;
    std::map<size_t, std::vector<char*>> free_;      // unmapped ranges by span: reused only whole
    std::map<uint64_t, uint64_t> sent_ino_;          // dma-buf inode -> the allocation id it was sent for
    std::map<uint64_t, int> live_fd_;                // exported allocation id -> its dma-buf (open)
};

}  // namespace rdc_amd
