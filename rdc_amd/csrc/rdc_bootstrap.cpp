// TCP star bootstrap (see rdc_bootstrap.h).
#include "rdc_bootstrap.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <stdexcept>
#include <string>

namespace rdc_amd {

namespace {

double now_s() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

[[noreturn]] void fail(const std::string& what) {
    throw std::runtime_error("rdc bootstrap: " + what + " (" + strerror(errno) + ")");
}

void send_all(int fd, const void* buf, size_t n) {
    const char* p = static_cast<const char*>(buf);
    while (n) {
        ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR) continue;
            fail("send");
        }
        p += k;
        n -= (size_t)k;
    }
}

void recv_all(int fd, void* buf, size_t n) {
    char* p = static_cast<char*>(buf);
    while (n) {
        ssize_t k = ::recv(fd, p, n, 0);
        if (k == 0) {
            errno = ECONNRESET;
            fail("peer closed");
        }
        if (k < 0) {
            if (errno == EINTR) continue;
            fail("recv");
        }
        p += k;
        n -= (size_t)k;
    }
}

bool resolve(const std::string& host, int port, sockaddr_in* out) {
    memset(out, 0, sizeof(*out));
    out->sin_family = AF_INET;
    out->sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, host.c_str(), &out->sin_addr) == 1) return true;
    addrinfo hints;
    memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_INET;
    addrinfo* res = nullptr;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) return false;
    out->sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
    freeaddrinfo(res);
    return true;
}

void set_nodelay(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

}  // namespace

void Bootstrap::barrier() {
    std::vector<char> all((size_t)size());
    char c = 0;
    allgather(&c, 1, all.data());
}

void Bootstrap::broadcast(void* buf, size_t bytes, int root) {
    std::vector<char> all((size_t)size() * bytes);
    allgather(buf, bytes, all.data());
    memcpy(buf, all.data() + (size_t)root * bytes, bytes);
}

void SoloBootstrap::allgather(const void* mine, size_t bytes, void* all) { memcpy(all, mine, bytes); }

// ------------------------------------------------------------ ShmBootstrap --
struct ShmBootstrap::Block {  // followed by size x kSlotBytes allgather slots
    alignas(64) std::atomic<uint32_t> arrive;
    alignas(64) std::atomic<uint32_t> gen;
};

namespace {
size_t block_bytes(int size) { return sizeof(ShmBootstrap::Block) + (size_t)size * ShmBootstrap::kSlotBytes; }
char* slot_of(ShmBootstrap::Block* b, int q) {
    return reinterpret_cast<char*>(b) + sizeof(ShmBootstrap::Block) + (size_t)q * ShmBootstrap::kSlotBytes;
}
}  // namespace

Bootstrap* ShmBootstrap::CreateGroup(Bootstrap* parent, const std::vector<int>& members, double timeout_s) {
    const int np = parent->size(), pr = parent->rank();
    const int n = (int)members.size();
    // every parent rank must pass the same list
    std::vector<int> sorted(members);
    std::sort(sorted.begin(), sorted.end());
    bool ok = n >= 1 && std::unique(sorted.begin(), sorted.end()) == sorted.end() && sorted.front() >= 0 &&
              sorted.back() < np;
    uint64_t h = 1469598103934665603ull ^ (uint64_t)n;
    for (int m : members) h = (h ^ (uint64_t)(uint32_t)m) * 1099511628211ull;
    std::vector<uint64_t> all((size_t)np);
    parent->allgather(&h, sizeof(h), all.data());
    for (uint64_t x : all) ok = ok && x == h;
    if (!ok) throw std::invalid_argument("rdc: CreateGroup needs the same list of distinct ranks on every rank");
    int me = -1;
    for (int i = 0; i < n; ++i)
        if (members[(size_t)i] == pr) me = i;
    const int leader = members[0];
    char name[64];
    memset(name, 0, sizeof(name));
    int fd = -1;
    std::string err;
    if (pr == leader) {
        static std::atomic<int> counter{0};
        snprintf(name, sizeof(name), "/rdc_grp_%d_%d", (int)getpid(), counter++);
        fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, (off_t)block_bytes(n)) != 0) {
            err = std::string("rdc: cannot create group shared memory ") + name + ": " + strerror(errno);
            if (fd >= 0) {
                ::close(fd);
                shm_unlink(name);
            }
            fd = -1;
            memset(name, 0, sizeof(name));
        }
    }
    parent->broadcast(name, sizeof(name), leader);
    if (!name[0]) throw std::runtime_error(err.empty() ? "rdc: the group's first rank could not create its segment" : err);
    void* p = MAP_FAILED;
    if (me >= 0) {
        if (pr != leader) fd = shm_open(name, O_RDWR, 0600);
        if (fd >= 0) {
            p = mmap(nullptr, block_bytes(n), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            ::close(fd);
        }
    }
    const char failed = (me >= 0 && p == MAP_FAILED) ? 1 : 0;
    std::vector<char> fails((size_t)np);
    parent->allgather(&failed, 1, fails.data());  // everyone mapped (or failed) before the name goes
    if (pr == leader) shm_unlink(name);
    for (char f : fails)
        if (f) {
            if (p != MAP_FAILED) munmap(p, block_bytes(n));
            throw std::runtime_error("rdc: a group member could not map the group segment");
        }
    if (me < 0) return nullptr;
    return new ShmBootstrap(me, n, static_cast<Block*>(p), timeout_s);
}

ShmBootstrap::~ShmBootstrap() {
    if (blk_) munmap(blk_, block_bytes(size_));
}

void ShmBootstrap::wait_all() {
    const uint32_t g = blk_->gen.load(std::memory_order_acquire);
    if (blk_->arrive.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)size_) {
        blk_->arrive.store(0, std::memory_order_relaxed);
        blk_->gen.fetch_add(1, std::memory_order_release);
        return;
    }
    const double deadline = now_s() + timeout_s_;
    for (uint32_t spins = 0; blk_->gen.load(std::memory_order_acquire) == g; ++spins) {
        if (spins < 4096) {
            sched_yield();
            continue;
        }
        usleep(50);
        if ((spins & 255) == 0 && now_s() > deadline) {
            errno = ETIMEDOUT;
            fail("group barrier: a member did not arrive");
        }
    }
}

void ShmBootstrap::allgather(const void* mine, size_t bytes, void* all) {
    char* out = static_cast<char*>(all);
    const char* in = static_cast<const char*>(mine);
    for (size_t off = 0; off < bytes || (bytes == 0 && off == 0); off += kSlotBytes) {  // slot-sized rounds
        const size_t len = std::min(kSlotBytes, bytes - off);
        if (len) memcpy(slot_of(blk_, rank_), in + off, len);
        wait_all();
        for (int q = 0; q < size_; ++q)
            if (len) memcpy(out + (size_t)q * bytes + off, slot_of(blk_, q), len);
        wait_all();  // nobody overwrites a slot before every member read it
        if (bytes == 0) break;
    }
}

TcpBootstrap::TcpBootstrap(int rank, int size, const std::string& host, int port, double timeout_s)
    : rank_(rank), size_(size) {
    if (size < 1 || rank < 0 || rank >= size) {
        errno = EINVAL;
        fail("bad rank/size");
    }
    if (size == 1) return;
    sockaddr_in addr;
    if (!resolve(host, port, &addr)) {
        errno = EINVAL;
        fail("cannot resolve tracker host " + host);
    }
    const double deadline = now_s() + timeout_s;
    if (rank == 0) {
        listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
        if (listen_fd_ < 0) fail("socket");
        int one = 1;
        setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        sockaddr_in any = addr;
        if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&any), sizeof(any)) != 0)
            fail("bind " + host + ":" + std::to_string(port));
        if (::listen(listen_fd_, size) != 0) fail("listen");
        peer_fds_.assign((size_t)size, -1);
        int got = 0;
        while (got < size - 1) {
            pollfd pfd{listen_fd_, POLLIN, 0};
            int left_ms = (int)((deadline - now_s()) * 1000);
            if (left_ms <= 0) {
                errno = ETIMEDOUT;
                fail("waiting for " + std::to_string(size - 1 - got) + " ranks to connect");
            }
            int pr = ::poll(&pfd, 1, left_ms);
            if (pr < 0 && errno == EINTR) continue;
            if (pr <= 0) continue;
            int fd = ::accept(listen_fd_, nullptr, nullptr);
            if (fd < 0) {
                if (errno == EINTR) continue;
                fail("accept");
            }
            set_nodelay(fd);
            int32_t hello[2];
            recv_all(fd, hello, sizeof(hello));
            if (hello[0] != 0x52444341 || hello[1] <= 0 || hello[1] >= size || peer_fds_[(size_t)hello[1]] >= 0) {
                ::close(fd);
                continue;
            }
            peer_fds_[(size_t)hello[1]] = fd;
            ++got;
        }
    } else {
        for (;;) {
            root_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
            if (root_fd_ < 0) fail("socket");
            if (::connect(root_fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) == 0) break;
            ::close(root_fd_);
            root_fd_ = -1;
            if (now_s() > deadline) {
                errno = ETIMEDOUT;
                fail("connect to tracker " + host + ":" + std::to_string(port));
            }
            usleep(20000);
        }
        set_nodelay(root_fd_);
        int32_t hello[2] = {0x52444341, rank};
        send_all(root_fd_, hello, sizeof(hello));
    }
    barrier();
}

TcpBootstrap::~TcpBootstrap() {
    for (int fd : peer_fds_)
        if (fd >= 0) ::close(fd);
    if (root_fd_ >= 0) ::close(root_fd_);
    if (listen_fd_ >= 0) ::close(listen_fd_);
}

void TcpBootstrap::allgather(const void* mine, size_t bytes, void* all) {
    char* out = static_cast<char*>(all);
    if (size_ == 1) {
        memcpy(out, mine, bytes);
        return;
    }
    uint64_t len = bytes;
    if (rank_ == 0) {
        memcpy(out, mine, bytes);
        for (int p = 1; p < size_; ++p) {
            uint64_t plen = 0;
            recv_all(peer_fds_[(size_t)p], &plen, sizeof(plen));
            if (plen != len) {
                errno = EPROTO;
                fail("allgather size mismatch from rank " + std::to_string(p));
            }
            recv_all(peer_fds_[(size_t)p], out + (size_t)p * bytes, bytes);
        }
        for (int p = 1; p < size_; ++p) send_all(peer_fds_[(size_t)p], out, (size_t)size_ * bytes);
    } else {
        send_all(root_fd_, &len, sizeof(len));
        send_all(root_fd_, mine, bytes);
        recv_all(root_fd_, out, (size_t)size_ * bytes);
    }
}

}  // namespace rdc_amd
