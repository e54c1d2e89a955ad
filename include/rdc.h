/*!
 * rdc.h — the reference's C++ interface (include/rdc.h, include/api.h,
 * include/core/rdc-inl.h, include/core/mpi.h of akkaze/rdc) over the
 * MI355X device path in librdc_amd.so.
 *
 * Drop-in for the allreduce/broadcast surface: same namespaces, names,
 * template parameters and argument meaning.  Differences, all deliberate:
 *   - the collectives work on host OR device (hipMalloc'd) pointers and are
 *     bit-identical to the reference's CPU ring allreduce;
 *   - comm::ICommunicator's collectives are real virtual calls (the
 *     reference's are non-virtual no-ops, include/comm/communicator.h:92-108);
 *   - failures abort with a message, like the reference's CHECK_F.
 * Link with -lrdc_amd.  Header-only otherwise.
 */
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "rdc_amd.h"

namespace rdc {

/*! \brief name of the default communicator (include/comm/communicator.h:21) */
static const std::string kMainCommName = "main";

namespace mpi {
/*! \brief reduction operators (include/core/mpi.h:12-17) */
enum OpType { kMax = 0, kMin = 1, kSum = 2, kBitwiseOR = 3 };
/*! \brief element types (include/core/mpi.h:19-30) */
enum DataType {
    kChar = 0,
    kUChar = 1,
    kInt = 2,
    kUInt = 3,
    kLong = 4,
    kULong = 5,
    kFloat = 6,
    kDouble = 7,
    kLongLong = 8,
    kULongLong = 9
};
template <typename DType>
inline DataType GetType(void);
template <> inline DataType GetType<char>(void) { return kChar; }
template <> inline DataType GetType<signed char>(void) { return kChar; }
template <> inline DataType GetType<unsigned char>(void) { return kUChar; }
template <> inline DataType GetType<int>(void) { return kInt; }
template <> inline DataType GetType<unsigned int>(void) { return kUInt; }
template <> inline DataType GetType<long>(void) { return kLong; }                       // NOLINT
template <> inline DataType GetType<unsigned long>(void) { return kULong; }             // NOLINT
template <> inline DataType GetType<float>(void) { return kFloat; }
template <> inline DataType GetType<double>(void) { return kDouble; }
template <> inline DataType GetType<long long>(void) { return kLongLong; }              // NOLINT
template <> inline DataType GetType<unsigned long long>(void) { return kULongLong; }    // NOLINT
}  // namespace mpi

/*! \brief reduction operators (include/core/mpi.h:84-112) */
namespace op {
struct Max { static const mpi::OpType kType = mpi::kMax; };
struct Min { static const mpi::OpType kType = mpi::kMin; };
struct Sum { static const mpi::OpType kType = mpi::kSum; };
struct BitOR { static const mpi::OpType kType = mpi::kBitwiseOR; };
}  // namespace op

namespace detail {
inline void Check(int rc, const char* what) {
    if (rc != 0) {
        fprintf(stderr, "rdc: %s failed: %s\n", what, RdcGetLastError());
        abort();
    }
}
}  // namespace detail

/*! \brief completion of an ISend / IRecv (include/core/work_request.h:240-270).
 *  Owned by the caller; deleting a pending completion is safe. */
class WorkCompletion {
public:
    explicit WorkCompletion(void* h) : h_(h) {}
    ~WorkCompletion() { RdcDelWorkCompletion(h_); }
    WorkCompletion(const WorkCompletion&) = delete;
    WorkCompletion& operator=(const WorkCompletion&) = delete;
    /*! \brief block until done; true on success (the reference's Wait) */
    bool Wait() { return RdcWorkCompletionWait(h_) == 0; }
    /*! \brief WorkStatus bits: 2 pending, 8 finished, 64 error */
    int Status() const { return RdcWorkCompletionStatus(h_); }
    std::string Error() const { return RdcWorkCompletionError(h_); }

private:
    void* h_;
};

namespace comm {
/*! \brief a named communicator (include/comm/communicator.h:41-146) */
class ICommunicator {
public:
    ICommunicator(void* handle, const std::string& name) : handle_(handle), name_(name) {}
    virtual ~ICommunicator() {}
    /*! \brief in-place allreduce of count elements (host or device memory) */
    virtual void Allreduce(void* sendrecvbuf, uint64_t count, mpi::DataType dtype, mpi::OpType op) {
        detail::Check(RdcAllreduceOn(handle_, sendrecvbuf, count, (int)dtype, (int)op), "Allreduce");
    }
    /*! \brief bucketed allreduce: Allreduce of every bufs[b] (counts[b] items), fused launches */
    virtual void AllreduceCoalesced(void** bufs, const size_t* counts, int nbuf, mpi::DataType dtype,
                                    mpi::OpType op) {
        detail::Check(RdcAllreduceCoalescedOn(handle_, bufs, counts, nbuf, (int)dtype, (int)op), "AllreduceCoalesced");
    }
    /*! \brief broadcast size bytes from root (host or device memory) */
    virtual void Broadcast(void* sendrecvaddr, uint64_t size, int root) {
        detail::Check(RdcBroadcastOn(handle_, sendrecvaddr, size, root), "Broadcast");
    }
    /*! \brief bufs[c] holds sizes[c] bytes; bufs[rank] is this rank's data */
    virtual void Allgather(void** bufs, const size_t* sizes) {
        detail::Check(RdcAllgatherOn(handle_, bufs, sizes), "Allgather");
    }
    /*! \brief non-blocking point-to-point (communicator.h:69-80); host or device
     *  memory; messages on one (src, dst) pair match in order, equal sizes */
    virtual WorkCompletion* ISend(const void* sendaddr, uint64_t size_in_bytes, int dest) {
        void* wc = nullptr;
        detail::Check(RdcCommISend(&wc, handle_, sendaddr, size_in_bytes, dest, nullptr), "ISend");
        return new WorkCompletion(wc);
    }
    virtual WorkCompletion* IRecv(void* recvaddr, uint64_t size_in_bytes, int src) {
        void* wc = nullptr;
        detail::Check(RdcCommIRecv(&wc, handle_, recvaddr, size_in_bytes, src, nullptr), "IRecv");
        return new WorkCompletion(wc);
    }
    /*! \brief blocking point-to-point (communicator.h:56-67); aborts on failure */
    virtual void Send(const void* sendaddr, uint64_t size_in_bytes, int dest) {
        WorkCompletion* w = ISend(sendaddr, size_in_bytes, dest);
        if (!w->Wait()) {
            fprintf(stderr, "rdc: Send failed: %s\n", w->Error().c_str());
            abort();
        }
        delete w;
    }
    virtual void Recv(void* recvaddr, uint64_t size_in_bytes, int src) {
        WorkCompletion* w = IRecv(recvaddr, size_in_bytes, src);
        if (!w->Wait()) {
            fprintf(stderr, "rdc: Recv failed: %s\n", w->Error().c_str());
            abort();
        }
        delete w;
    }
    int GetRank() const { return RdcCommRank(handle_); }
    int GetWorldSize() const { return RdcCommSize(handle_); }
    std::string name() const { return name_; }
    void* handle() const { return handle_; }

private:
    void* handle_;
    std::string name_;
};

inline std::vector<ICommunicator*>& Registry() {
    static std::vector<ICommunicator*> r;
    return r;
}
}  // namespace comm

/*! \brief initialise rdc; argv key=val pairs are parameters (rdc-inl.h:21-23) */
inline void Init(int argc, char** argv) { detail::Check(RdcInit(argc, argv), "Init"); }
inline void Init() { Init(0, nullptr); }

inline comm::ICommunicator* Lookup(const std::string& name) {
    for (comm::ICommunicator* c : comm::Registry())
        if (c->name() == name) return c;
    return nullptr;
}
/*! \brief create (collectively) a communicator (rdc-inl.h:25-27) */
inline comm::ICommunicator* NewCommunicator(const std::string& name) {
    if (comm::ICommunicator* c = Lookup(name)) return c;
    void* h = nullptr;
    detail::Check(RdcNewCommunicator(&h, name.c_str()), "NewCommunicator");
    comm::ICommunicator* c = new comm::ICommunicator(h, name);
    comm::Registry().push_back(c);
    return c;
}
/*! \brief an existing communicator; "main" is created on first use (rdc-inl.h:29-31) */
inline comm::ICommunicator* GetCommunicator(const std::string& name = kMainCommName) {
    if (comm::ICommunicator* c = Lookup(name)) return c;
    void* h = nullptr;
    detail::Check(RdcGetCommunicator(&h, name.c_str()), "GetCommunicator");
    comm::ICommunicator* c = new comm::ICommunicator(h, name);
    comm::Registry().push_back(c);
    return c;
}
inline void Finalize() {
    for (comm::ICommunicator* c : comm::Registry()) delete c;
    comm::Registry().clear();
    detail::Check(RdcFinalize(), "Finalize");
}
inline int GetRank() { return RdcGetRank(); }
inline int GetWorldSize() { return RdcGetWorldSize(); }
inline bool IsDistributed() { return RdcIsDistributed() != 0; }
inline void TrackerPrint(const std::string& msg) { RdcTrackerPrint(msg.c_str()); }
inline void Barrier() { detail::Check(RdcBarrier(), "Barrier"); }

/*! \brief blocking point-to-point on a communicator (include/api.h:10-11, rdc-inl.h:53-66) */
inline void Send(const void* send_data, uint64_t size, int dest, const std::string& comm_name = kMainCommName) {
    GetCommunicator(comm_name)->Send(send_data, size, dest);
}
inline void Recv(void* recv_data, uint64_t size, int src, const std::string& comm_name = kMainCommName) {
    GetCommunicator(comm_name)->Recv(recv_data, size, src);
}

/*! \brief in-place allreduce (include/api.h:62-64, rdc-inl.h:125-135) */
template <typename OP, typename DType>
inline void Allreduce(DType* sendrecvbuf, uint64_t count, const std::string& comm_name = kMainCommName) {
    if (GetWorldSize() == 1 || count == 0) return;  // communicator_base.h:133-138
    GetCommunicator(comm_name)->Allreduce(sendrecvbuf, count, mpi::GetType<DType>(), OP::kType);
}

/*! \brief bucketed allreduce (MI355X addition; test/mallreduce.cc's back-to-back shape):
 *  the result of Allreduce<OP,DType>(bufs[b], counts[b]) for every b, bit-identical,
 *  moved in fused device launches */
template <typename OP, typename DType>
inline void AllreduceCoalesced(DType** bufs, const uint64_t* counts, int nbuf,
                               const std::string& comm_name = kMainCommName) {
    if (GetWorldSize() == 1 || nbuf == 0) return;
    std::vector<size_t> c((size_t)nbuf);
    for (int b = 0; b < nbuf; ++b) c[(size_t)b] = (size_t)counts[b];
    GetCommunicator(comm_name)->AllreduceCoalesced(reinterpret_cast<void**>(bufs), c.data(), nbuf,
                                                   mpi::GetType<DType>(), OP::kType);
}

/*! \brief broadcast a memory region from root (include/api.h:23-24) */
inline void Broadcast(void* sendrecv_data, uint64_t size, int root, const std::string& comm_name = kMainCommName) {
    if (GetWorldSize() == 1 || size == 0) return;
    GetCommunicator(comm_name)->Broadcast(sendrecv_data, size, root);
}
/*! \brief broadcast a vector, resizing receivers (rdc-inl.h:76-88) */
template <typename DType>
inline void Broadcast(std::vector<DType>& sendrecv_data, int root, const std::string& comm_name = kMainCommName) {
    uint64_t size = sendrecv_data.size();
    Broadcast(&size, sizeof(size), root, comm_name);
    if (sendrecv_data.size() != size) sendrecv_data.resize(size);
    if (size != 0) Broadcast(sendrecv_data.data(), size * sizeof(DType), root, comm_name);
}
/*! \brief broadcast a string, resizing receivers (rdc-inl.h:89-100) */
inline void Broadcast(std::string& sendrecv_data, int root, const std::string& comm_name = kMainCommName) {
    uint64_t size = sendrecv_data.length();
    Broadcast(&size, sizeof(size), root, comm_name);
    if (sendrecv_data.length() != size) sendrecv_data.resize(size);
    if (size != 0) Broadcast(&sendrecv_data[0], size, root, comm_name);
}

/*! \brief allgather of per-rank buffers (include/api.h:51-52): sendrecv_data[c]
 *  holds counts[c] items of type_nbytes bytes; this rank's own entry is the input */
inline void Allgather(void** sendrecv_data, size_t type_nbytes, size_t* counts,
                      const std::string& comm_name = kMainCommName) {
    const int n = GetWorldSize();
    if (n == 1) return;
    std::vector<size_t> sizes((size_t)n);
    for (int i = 0; i < n; ++i) sizes[(size_t)i] = counts[i] * type_nbytes;
    GetCommunicator(comm_name)->Allgather(sendrecv_data, sizes.data());
}
/*! \brief allgather of pre-sized vectors (include/api.h:47-49, rdc-inl.h:112-122) */
template <typename DType>
inline void Allgather(std::vector<std::vector<DType>>& sendrecv_data, const std::string& comm_name = kMainCommName) {
    const int n = GetWorldSize();
    if (n == 1) return;
    std::vector<void*> bufs((size_t)n);
    std::vector<size_t> sizes((size_t)n);
    for (int i = 0; i < n; ++i) {
        bufs[(size_t)i] = sendrecv_data[(size_t)i].data();
        sizes[(size_t)i] = sendrecv_data[(size_t)i].size() * sizeof(DType);
    }
    GetCommunicator(comm_name)->Allgather(bufs.data(), sizes.data());
}

}  // namespace rdc
