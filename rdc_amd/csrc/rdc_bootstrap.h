// Rank bootstrap for the MI355X rdc path.
//
// Replaces the reference's tracker handshake (src/comm/tracker.cc:115-242,
// tracker/tracker.py:137-213) for the only thing the device data path needs
// from it: rank / world size and a byte allgather used to exchange HIP IPC
// handles (instead of building the reference's TCP data mesh,
// src/comm/communicator_base.cc:162-297).  Rank 0 listens on
// RDC_TRACKER_URI:RDC_TRACKER_PORT; the others connect to it (star).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace rdc_amd {

class Bootstrap {
public:
    virtual ~Bootstrap() {}
    virtual int rank() const = 0;
    virtual int size() const = 0;
    // every rank contributes `bytes` bytes; `all` receives size()*bytes, rank-major
    virtual void allgather(const void* mine, size_t bytes, void* all) = 0;
    void barrier();
    // root's `bytes` bytes land in buf on every rank
    void broadcast(void* buf, size_t bytes, int root);
};

class TcpBootstrap : public Bootstrap {
public:
    TcpBootstrap(int rank, int size, const std::string& host, int port, double timeout_s);
    ~TcpBootstrap() override;
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    void allgather(const void* mine, size_t bytes, void* all) override;

private:
    int rank_, size_;
    int listen_fd_ = -1;
    int root_fd_ = -1;             // non-root: socket to rank 0
    std::vector<int> peer_fds_;    // root: socket per rank (index = rank)
};

// Members of a sub-communicator (CreateGroup, include/api.h:124-125): a
// node-local rendezvous in POSIX shared memory (the xGMI path needs every
// rank on one node anyway).  Created collectively over the parent's
// bootstrap: the group's first rank creates the segment, the name travels
// over the parent, then only members take part in barriers / allgathers.
class ShmBootstrap : public Bootstrap {
public:
    // collective over `parent`: every parent rank calls it with the same
    // `members` (parent ranks, group rank i = members[i]); non-members get null
    static Bootstrap* CreateGroup(Bootstrap* parent, const std::vector<int>& members, double timeout_s);
    ~ShmBootstrap() override;
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    void allgather(const void* mine, size_t bytes, void* all) override;

    static constexpr size_t kSlotBytes = 4096;
    struct Block;  // barrier words, then size x kSlotBytes allgather slots

private:
    ShmBootstrap(int rank, int size, Block* blk, double timeout_s) : rank_(rank), size_(size), blk_(blk),
                                                                       timeout_s_(timeout_s) {}
    void wait_all();  // generation barrier over the members
    int rank_, size_;
    Block* blk_;
    double timeout_s_;
};

// One process owning every rank (single-process multi-GPU): trivially local.
class SoloBootstrap : public Bootstrap {
public:
    int rank() const override { return 0; }
    int size() const override { return 1; }
    void allgather(const void* mine, size_t bytes, void* all) override;
};

}  // namespace rdc_amd
