// TCP star bootstrap (see rdc_bootstrap.h).
#include "rdc_bootstrap.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <time.h>
#include <unistd.h>

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
