// ORACLE (_ref) — TEST INFRASTRUCTURE ONLY.
//
// Builds a CPU ring-allreduce simulator whose arithmetic and chunking are the
// reference's OWN code, compiled from the headers where they lie under
// /root/reference (nothing is copied into this repo):
//   rdc::op::Reducer<OP,DType>, op::Max/Min/Sum/BitOR   include/core/mpi.h:84-120
//   rdc::utils::Split                                   include/utils/utils.h:59-70
// The schedule (which chunk each rank sends/receives per step) is restated from
// src/comm/communicator_collective.cc:79-203; the survey verified this
// combination bit-exact against the running (shimmed) reference for
// n in {2,3,5,8}.  The full reference library itself does not
// compile as shipped (SURVEY.md §0 finding 1), so only these header-only parts
// are built; see oracle/Makefile and DESIGN.md.
//
// Output goes only to oracle/_ref/ (git-ignored).
#include <cstdint>
#include <cstddef>
#include <cstring>
#include <vector>
#include <utility>
#include <algorithm>

#include "core/mpi.h"     // from /root/reference/include
#include "utils/utils.h"  // from /root/reference/include

namespace {

template <typename OP, typename DType>
void ReduceChunk(const void* src, void* dst, uint64_t len) {
    rdc::op::Reducer<OP, DType>(src, dst, len);
}

typedef void (*ReduceFn)(const void*, void*, uint64_t);

template <typename DType>
ReduceFn PickArith(int op) {
    switch (op) {
        case rdc::mpi::kMax: return &ReduceChunk<rdc::op::Max, DType>;
        case rdc::mpi::kMin: return &ReduceChunk<rdc::op::Min, DType>;
        case rdc::mpi::kSum: return &ReduceChunk<rdc::op::Sum, DType>;
        default: return nullptr;
    }
}
template <typename DType>
ReduceFn PickInt(int op) {
    if (op == rdc::mpi::kBitwiseOR) return &ReduceChunk<rdc::op::BitOR, DType>;
    return PickArith<DType>(op);
}

// dtype enum follows rdc::mpi::DataType (mpi.h:19-30) with the C++ types
// GetType<> maps them from (mpi.h:40-81).
bool Pick(int dtype, int op, ReduceFn* fn, size_t* esz) {
    switch (dtype) {
        case rdc::mpi::kChar: *fn = PickInt<char>(op); *esz = 1; break;
        case rdc::mpi::kUChar: *fn = PickInt<unsigned char>(op); *esz = 1; break;
        case rdc::mpi::kInt: *fn = PickInt<int>(op); *esz = 4; break;
        case rdc::mpi::kUInt: *fn = PickInt<unsigned int>(op); *esz = 4; break;
        case rdc::mpi::kLong: *fn = PickInt<long>(op); *esz = 8; break;
        case rdc::mpi::kULong: *fn = PickInt<unsigned long>(op); *esz = 8; break;
        case rdc::mpi::kFloat: *fn = PickArith<float>(op); *esz = 4; break;
        case rdc::mpi::kDouble: *fn = PickArith<double>(op); *esz = 8; break;
        case rdc::mpi::kLongLong: *fn = PickInt<long long>(op); *esz = 8; break;
        case rdc::mpi::kULongLong: *fn = PickInt<unsigned long long>(op); *esz = 8; break;
        default: return false;
    }
    return *fn != nullptr;
}

}  // namespace

extern "C" {

// The reference's op::Reducer over one buffer pair (mpi.h:113-120).
int ref_reducer(const void* src, void* dst, uint64_t len, int dtype, int op) {
    ReduceFn fn;
    size_t esz;
    if (!Pick(dtype, op, &fn, &esz)) return -1;
    fn(src, dst, len);
    return 0;
}

// The reference's utils::Split (utils.h:59-70) — int arithmetic, as shipped.
int ref_split(int begin, int end, int nparts, int* out_begin, int* out_end) {
    auto ranges = rdc::utils::Split(begin, end, nparts);
    for (int i = 0; i < nparts; ++i) {
        out_begin[i] = ranges[i].first;
        out_end[i] = ranges[i].second;
    }
    return 0;
}

// n simulated ranks, bufs[r] = rank r's in-place sendrecvbuf.  Lock-step ring:
// TryReduceScatterRing (communicator_collective.cc:115-182) then
// TryAllgatherRing (:79-114), prev=(r-1+n)%n, next=(r+1)%n (topo.cc:80-115).
int ref_allreduce_ring(void** bufs, int n, uint64_t count, int dtype, int op) {
    ReduceFn fn;
    size_t esz;
    if (!Pick(dtype, op, &fn, &esz) || n < 1) return -1;
    if (n == 1 || count == 0) return 0;  // communicator_base.h:133-138
    const auto ranges = rdc::utils::Split(0, static_cast<int>(count), n);
    // per-rank state of the reduce-scatter loop (:119-133)
    std::vector<uint64_t> write_idx(n), read_idx(n), reduce_idx(n), stop_read(n), stop_write(n);
    for (int r = 0; r < n; ++r) {
        uint64_t next = (uint64_t)((r + 1) % n);
        write_idx[r] = next;
        read_idx[r] = next + 1;
        reduce_idx[r] = read_idx[r];
        stop_read[r] = n + next;
        stop_write[r] = n + r;
        if (stop_write[r] > stop_read[r]) stop_write[r] -= n;
    }
    for (int step = 0; step < n - 1; ++step) {
        // this step's sends: snapshot the chunk each rank ISends to prev (:145-155)
        std::vector<std::vector<char>> sent(n);
        std::vector<int> sent_pos(n, -1);
        for (int r = 0; r < n; ++r) {
            if (write_idx[r] < reduce_idx[r] && write_idx[r] != stop_write[r]) {
                int pos = (int)(write_idx[r] % n);
                size_t b = (size_t)ranges[pos].first * esz;
                size_t len = (size_t)(ranges[pos].second - ranges[pos].first) * esz;
                sent[r].assign((char*)bufs[r] + b, (char*)bufs[r] + b + len);
                sent_pos[r] = pos;
                write_idx[r]++;
            }
        }
        // receives from next into reducebuf, then reducer(reducebuf, sendrecvbuf) (:156-178)
        for (int r = 0; r < n; ++r) {
            if (read_idx[r] == stop_read[r]) continue;
            int nx = (r + 1) % n;
            int pos = (int)(read_idx[r] % n);
            if (sent_pos[nx] != pos) return -2;
            size_t b = (size_t)ranges[pos].first * esz;
            uint64_t cnt = (uint64_t)(ranges[pos].second - ranges[pos].first);
            fn(sent[nx].data(), (char*)bufs[r] + b, cnt);
            read_idx[r]++;
            reduce_idx[r]++;
        }
    }
    // TryAllgatherRing (:79-114) over chunk views of the sendrecvbuf (:190-201)
    std::vector<uint64_t> w(n), rd(n), sw(n), sr(n);
    for (int r = 0; r < n; ++r) {
        w[r] = r; rd[r] = r + 1; sw[r] = n + r - 1; sr[r] = n + r;
    }
    for (int step = 0; step < n - 1; ++step) {
        std::vector<std::vector<char>> sent(n);
        std::vector<int> sent_pos(n, -1);
        for (int r = 0; r < n; ++r) {
            if (w[r] < rd[r] && w[r] != sw[r]) {
                int pos = (int)(w[r] % n);
                size_t b = (size_t)ranges[pos].first * esz;
                size_t len = (size_t)(ranges[pos].second - ranges[pos].first) * esz;
                sent[r].assign((char*)bufs[r] + b, (char*)bufs[r] + b + len);
                sent_pos[r] = pos;
                w[r]++;
            }
        }
        for (int r = 0; r < n; ++r) {
            if (rd[r] == sr[r]) continue;
            int nx = (r + 1) % n;
            int pos = (int)(rd[r] % n);
            if (sent_pos[nx] != pos) return -3;
            size_t b = (size_t)ranges[pos].first * esz;
            if (!sent[nx].empty()) std::memcpy((char*)bufs[r] + b, sent[nx].data(), sent[nx].size());
            rd[r]++;
        }
    }
    return 0;
}

}  // extern "C"
