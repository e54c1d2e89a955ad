// Peer allocations imported at addresses this process chooses: see rdc_vmem.h.
#include "rdc_vmem.h"

#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <stddef.h>
#include <string.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <random>

#include "rdc_bootstrap.h"

namespace rdc_amd {

namespace {

constexpr size_t kGranule = 2u << 20;          // mappings start on 2 MiB boundaries
constexpr size_t kArenaBytes = 64ull << 30;    // address space reserved at a time

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

socklen_t sock_name(uint64_t token, int rank, sockaddr_un* a) {
    memset(a, 0, sizeof(*a));
    a->sun_family = AF_UNIX;
    char name[64];
    const int len = snprintf(name, sizeof(name), "rdc-vmem-%016llx-%d", (unsigned long long)token, rank);
    memcpy(a->sun_path + 1, name, (size_t)len);  // abstract namespace: nothing on the file system
    return (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + (size_t)len);
}

bool wait_fd(int fd, short ev, double timeout_s) {
    pollfd p{fd, ev, 0};
    const int ms = (int)(timeout_s * 1000);
    int r;
    do {
        r = poll(&p, 1, ms);
    } while (r < 0 && errno == EINTR);
    return r == 1 && (p.revents & ev);
}

// one message, optionally carrying one descriptor
bool send_msg(int sock, const void* data, size_t bytes, int fd) {
    iovec iov{const_cast<void*>(data), bytes};
    char ctl[CMSG_SPACE(sizeof(int))];
    memset(ctl, 0, sizeof(ctl));
    msghdr m{};
    m.msg_iov = &iov;
    m.msg_iovlen = 1;
    if (fd >= 0) {
        m.msg_control = ctl;
        m.msg_controllen = sizeof(ctl);
        cmsghdr* c = CMSG_FIRSTHDR(&m);
        c->cmsg_level = SOL_SOCKET;
        c->cmsg_type = SCM_RIGHTS;
        c->cmsg_len = CMSG_LEN(sizeof(int));
        memcpy(CMSG_DATA(c), &fd, sizeof(int));
    }
    ssize_t r;
    do {
        r = sendmsg(sock, &m, MSG_NOSIGNAL);
    } while (r < 0 && errno == EINTR);
    return r == (ssize_t)bytes;
}

// 1 = a message (and *fd, -1 if none), 0 = nothing waiting (non-blocking), -1 = error
int recv_msg(int sock, void* data, size_t bytes, int* fd, bool block) {
    iovec iov{data, bytes};
    char ctl[CMSG_SPACE(sizeof(int))];
    msghdr m{};
    m.msg_iov = &iov;
    m.msg_iovlen = 1;
    m.msg_control = ctl;
    m.msg_controllen = sizeof(ctl);
    ssize_t r;
    do {
        r = recvmsg(sock, &m, MSG_CMSG_CLOEXEC | (block ? 0 : MSG_DONTWAIT));
    } while (r < 0 && errno == EINTR);
    if (r < 0) return errno == EAGAIN || errno == EWOULDBLOCK ? 0 : -1;
    if (r != (ssize_t)bytes) return -1;
    *fd = -1;
    for (cmsghdr* c = CMSG_FIRSTHDR(&m); c; c = CMSG_NXTHDR(&m, c))
        if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_RIGHTS) memcpy(fd, CMSG_DATA(c), sizeof(int));
    return 1;
}

}  // namespace

std::unique_ptr<VmemImporter> VmemImporter::Create(Bootstrap* bs, int rank, int n, hsa_agent_t agent,
                                                   double timeout_s, std::string* why) {
    std::unique_ptr<VmemImporter> v(new VmemImporter());
    v->rank_ = rank;
    v->n_ = n;
    v->agent_ = agent;
    v->sock_.assign((size_t)n, -1);
    // an exporter keeps one dma-buf open per live exported allocation (up to
    // kDirectExportsMax): the soft descriptor limit goes up to the hard one
    rlimit rl;
    if (getrlimit(RLIMIT_NOFILE, &rl) == 0 && rl.rlim_cur < rl.rlim_max) {
        rl.rlim_cur = rl.rlim_max;
        (void)setrlimit(RLIMIT_NOFILE, &rl);
    }
    // 1) every rank listens on rdc-vmem-<rank 0's token>-<rank>
    struct Hello {
        uint64_t token;
        int32_t ok, rank;
    };
    Hello mine{0, 1, rank};
    if (rank == 0) mine.token = std::random_device{}() * 0x9E3779B97F4A7C15ull ^ (uint64_t)getpid();
    std::vector<Hello> all((size_t)n);
    bs->allgather(&mine, sizeof(mine), all.data());
    const uint64_t token = all[0].token;
    const int ls = socket(AF_UNIX, SOCK_SEQPACKET | SOCK_CLOEXEC, 0);
    sockaddr_un sa;
    socklen_t sl = sock_name(token, rank, &sa);
    mine.ok = ls >= 0 && bind(ls, (sockaddr*)&sa, sl) == 0 && listen(ls, n) == 0;
    if (!mine.ok) *why = std::string("unix socket: ") + strerror(errno);
    bs->allgather(&mine, sizeof(mine), all.data());
    bool ok = true;
    for (const Hello& h : all) ok = ok && h.ok;
    // 2) rank r connects to every lower rank and accepts every higher one
    if (ok) {
        for (int q = 0; q < rank && mine.ok; ++q) {
            const int s = socket(AF_UNIX, SOCK_SEQPACKET | SOCK_CLOEXEC, 0);
            sockaddr_un qa;
            const socklen_t ql = sock_name(token, q, &qa);
            int32_t me = rank;
            if (s < 0 || connect(s, (sockaddr*)&qa, ql) != 0 || !send_msg(s, &me, sizeof(me), -1)) {
                *why = std::string("connect to rank ") + std::to_string(q) + ": " + strerror(errno);
                mine.ok = 0;
                if (s >= 0) close(s);
                break;
            }
            v->sock_[(size_t)q] = s;
        }
        for (int k = rank + 1; k < n && mine.ok; ++k) {
            int32_t from = -1, fd = -1;
            const int s = wait_fd(ls, POLLIN, timeout_s) ? accept4(ls, nullptr, nullptr, SOCK_CLOEXEC) : -1;
            if (s < 0 || !wait_fd(s, POLLIN, timeout_s) || recv_msg(s, &from, sizeof(from), &fd, true) != 1 ||
                from <= rank || from >= n || v->sock_[(size_t)from] >= 0) {
                *why = "accepting the peers' connections failed";
                mine.ok = 0;
                if (s >= 0) close(s);
                break;
            }
            v->sock_[(size_t)from] = s;
        }
    }
    if (ls >= 0) close(ls);
    bs->allgather(&mine, sizeof(mine), all.data());
    for (const Hello& h : all) ok = ok && h.ok;
    if (!ok) {
        if (why->empty()) *why = "a peer could not set up its sockets";
        return nullptr;  // the destructor closes what was opened
    }
    return v;
}

VmemImporter::~VmemImporter() {
    for (auto& m : maps_) {
        hsa_amd_vmem_unmap(m.second.va, m.second.span);
        hsa_amd_vmem_handle_release(m.second.h);
    }
    for (auto& p : pending_) close(p.second.fd);
    for (auto& f : live_fd_) hsa_amd_portable_close_dmabuf(f.second);
    for (auto& a : arenas_) hsa_amd_vmem_address_free(a.base, a.size);
    for (int s : sock_)
        if (s >= 0) close(s);
}

bool VmemImporter::Export(void* base, size_t size, uint64_t id, std::string* why) {
    // ROCr's record of the allocation at `base` must be the one HIP reports:
    // after an allocation at the same base was exported and freed, the
    // runtime handed out a dma-buf of that earlier buffer object
    // (profiles/r06/vmem/: 16 MiB for a new 64 MiB allocation)
    hsa_amd_pointer_info_t info;
    memset(&info, 0, sizeof(info));
    info.size = sizeof(info);
    if (hsa_amd_pointer_info(base, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        info.agentBaseAddress != base || info.sizeInBytes != size) {
        *why = "the runtime's record at this base is another allocation (" + std::to_string(info.sizeInBytes) +
               " B)";
        return false;
    }
    int fd = -1;
    uint64_t off = 0;
    const hsa_status_t s = hsa_amd_portable_export_dmabuf(base, size, &fd, &off);
    if (s != HSA_STATUS_SUCCESS || fd < 0) {
        *why = "hsa_amd_portable_export_dmabuf " + std::to_string((int)s);
        return false;
    }
    // the dma-buf must cover the allocation HIP reports (a smaller one would
    // be another buffer object: never handed to a peer)
    const off_t end = lseek(fd, 0, SEEK_END);
    if (end < 0 || (uint64_t)end < off + size) {
        *why = "dma-buf of " + std::to_string((long long)end) + " B for an allocation of " + std::to_string(size) +
               " B at offset " + std::to_string(off);
        hsa_amd_portable_close_dmabuf(fd);
        return false;
    }
    // a dma-buf file this rank already sent for another allocation is that
    // allocation's buffer object (dma-buf inode numbers are not reused; the
    // dma-buf of every allocation retired in this call is still open here,
    // so the runtime hands back that same file for its buffer object)
    struct stat st;
    if (fstat(fd, &st) != 0) {
        *why = std::string("fstat on the dma-buf: ") + strerror(errno);
        hsa_amd_portable_close_dmabuf(fd);
        return false;
    }
    auto seen = sent_ino_.find((uint64_t)st.st_ino);
    if (seen != sent_ino_.end() && seen->second != id) {
        *why = "the dma-buf of an earlier allocation (id " + std::to_string(seen->second) + ")";
        hsa_amd_portable_close_dmabuf(fd);
        return false;
    }
    sent_ino_[(uint64_t)st.st_ino] = id;
    const Msg m{id, off, size};
    bool ok = true;
    for (int p = 0; p < n_; ++p)
        if (p != rank_) ok = send_msg(sock_[(size_t)p], &m, sizeof(m), fd) && ok;
    if (!ok) {
        *why = std::string("sending the dma-buf: ") + strerror(errno);
        hsa_amd_portable_close_dmabuf(fd);
        return false;
    }
    auto old = live_fd_.find(id);
    if (old != live_fd_.end()) hsa_amd_portable_close_dmabuf(old->second);
    live_fd_[id] = fd;  // open until Release (the allocation retired)
    return true;
}

void VmemImporter::Release(uint64_t id) {
    auto it = live_fd_.find(id);
    if (it == live_fd_.end()) return;
    hsa_amd_portable_close_dmabuf(it->second);
    live_fd_.erase(it);
}

bool VmemImporter::Recv(int p, bool block) {
    Msg m;
    int fd = -1;
    if (recv_msg(sock_[(size_t)p], &m, sizeof(m), &fd, block) != 1) return false;
    if (fd < 0) return true;
    auto key = std::make_pair(p, m.id);
    auto it = pending_.find(key);
    if (it != pending_.end()) close(it->second.fd);  // buffer ids are not reused: not expected
    Pending pd;
    pd.fd = fd;
    pd.offset = m.offset;
    pd.size = m.size;
    pending_[key] = pd;
    return true;
}

void VmemImporter::Drain() {
    for (int p = 0; p < n_; ++p)
        if (p != rank_)
            while (Recv(p, false)) {
            }
}

char* VmemImporter::PlaceRange(size_t span) {
    auto f = free_.find(span);
    if (f != free_.end() && !f->second.empty()) {  // exactly where an unmapped one of this size was
        char* va = f->second.back();
        f->second.pop_back();
        return va;
    }
    for (Arena& a : arenas_)
        if (a.size - a.used >= span) {  // addresses no mapping used before
            char* va = a.base + a.used;
            a.used += span;
            return va;
        }
    for (size_t want : {std::max(kArenaBytes, span), span}) {
        void* va = nullptr;
        if (hsa_amd_vmem_address_reserve_align(&va, want, 0, kGranule, 0) == HSA_STATUS_SUCCESS && va) {
            Arena a;
            a.base = static_cast<char*>(va);
            a.size = want;
            a.used = span;
            arenas_.push_back(a);
            return a.base;
        }
    }
    return nullptr;
}

bool VmemImporter::Map(int p, uint64_t id, char** base, size_t* size, std::string* why) {
    const auto key = std::make_pair(p, id);
    auto it = pending_.find(key);
    if (it == pending_.end()) {
        Drain();
        it = pending_.find(key);
    }
    if (it == pending_.end()) {
        *why = "dma-buf not received";
        return false;
    }
    const Pending pd = it->second;
    pending_.erase(it);
    const off_t end = lseek(pd.fd, 0, SEEK_END);
    hsa_amd_vmem_alloc_handle_t h{};
    if (end <= 0 || (uint64_t)end < pd.offset + pd.size) {
        close(pd.fd);
        *why = "dma-buf of " + std::to_string((long long)end) + " B for an allocation of " + std::to_string(pd.size) +
               " B at offset " + std::to_string(pd.offset);
        return false;
    }
    const hsa_status_t si = hsa_amd_vmem_import_shareable_handle(pd.fd, &h);
    close(pd.fd);  // the handle holds the allocation
    if (si != HSA_STATUS_SUCCESS) {
        *why = "hsa_amd_vmem_import_shareable_handle " + std::to_string((int)si);
        return false;
    }
    const size_t span = (size_t)end;
    const size_t slot = round_up(span, kGranule);
    char* va = PlaceRange(slot);
    if (!va) {
        hsa_amd_vmem_handle_release(h);
        *why = "no address range left";
        return false;
    }
    hsa_status_t s = hsa_amd_vmem_map(va, span, 0, h, 0);
    if (s == HSA_STATUS_SUCCESS) {
        hsa_amd_memory_access_desc_t d;
        d.permissions = HSA_ACCESS_PERMISSION_RW;
        d.agent_handle = agent_;
        s = hsa_amd_vmem_set_access(va, span, &d, 1);
        if (s != HSA_STATUS_SUCCESS) hsa_amd_vmem_unmap(va, span);
    }
    if (s != HSA_STATUS_SUCCESS) {
        hsa_amd_vmem_handle_release(h);
        free_[slot].push_back(va);
        *why = "hsa_amd_vmem_map / set_access " + std::to_string((int)s);
        return false;
    }
    Mapping mp;
    mp.va = va;
    mp.span = span;
    mp.h = h;
    *base = va + pd.offset;
    *size = pd.size;
    maps_[*base] = mp;
    return true;
}

void VmemImporter::Unmap(char* base) {
    auto it = maps_.find(base);
    if (it == maps_.end()) return;
    hsa_amd_vmem_unmap(it->second.va, it->second.span);
    hsa_amd_vmem_handle_release(it->second.h);
    free_[round_up(it->second.span, kGranule)].push_back(it->second.va);
    maps_.erase(it);
}

void VmemImporter::Forget(int p, uint64_t id) {
    auto it = pending_.find(std::make_pair(p, id));
    if (it == pending_.end()) return;
    close(it->second.fd);
    pending_.erase(it);
}

size_t VmemImporter::arena_bytes() const {
    size_t s = 0;
    for (const Arena& a : arenas_) s += a.size;
    return s;
}

}  // namespace rdc_amd
