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
 *   - failures abort with a message, like the reference's CHECK_F;
 *   - custom reducers (ICommunicator::Allreduce(Buffer, ReduceFunction),
 *     Reducer<DType, freduce>, SerializeReducer<DType>) run the user's HOST
 *     function: the inputs move over the device path (allgather), then every
 *     rank folds its own Split chunk in the ring's order (or the whole buffer
 *     in the tree's order at <= rdc_reduce_ring_mincount bytes), calling
 *     reducer(src, dst) exactly as TryReduceScatterRing / TryReduceTree would
 *     (communicator_collective.cc:14-43,115-182), and the chunks are
 *     allgathered.  (The reference declares these; its Reducer /
 *     SerializeReducer::Allreduce call themselves, rdc-inl.h:187-196.)
 * Link with -lrdc_amd.  Header-only otherwise.
 */
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <functional>
#include <memory>
#include <string>
#include <type_traits>
#include <utility>
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

/*! \brief reduction operators (include/core/mpi.h:84-120).  kType names the
 *  device kernel the typed collectives launch; Reduce(dst, src) is the
 *  element rule that kernel applies (rdc_amd/csrc/rdc_device.h OpF), kept
 *  here on the host so code written against the reference — its reducer
 *  lambda `op::Reducer<OP,DType>(src.addr(), dst.addr(), src.Count())`
 *  (include/core/rdc-inl.h:130-132) — compiles and folds the same bits. */
namespace op {
struct Max {
    static const mpi::OpType kType = mpi::kMax;
    /*! \brief dst = src when dst < src (a NaN dst stays, a NaN src is ignored) */
    template <typename DType> inline static void Reduce(DType& dst, const DType& src) {  // NOLINT(*)
        if (dst < src) dst = src;
    }
};
struct Min {
    static const mpi::OpType kType = mpi::kMin;
    /*! \brief dst = src when dst > src */
    template <typename DType> inline static void Reduce(DType& dst, const DType& src) {  // NOLINT(*)
        if (dst > src) dst = src;
    }
};
struct Sum {
    static const mpi::OpType kType = mpi::kSum;
    template <typename DType> inline static void Reduce(DType& dst, const DType& src) {  // NOLINT(*)
        dst += src;
    }
};
struct BitOR {
    static const mpi::OpType kType = mpi::kBitwiseOR;
    template <typename DType> inline static void Reduce(DType& dst, const DType& src) {  // NOLINT(*)
        dst |= src;
    }
};
/*! \brief dst[i] = OP::Reduce(dst[i], src[i]) for i < len, on HOST memory, in
 *  index order (include/core/mpi.h:113-120).  Device buffers: RdcReduce, the
 *  same rule as a HIP kernel. */
template <typename OP, typename DType>
inline void Reducer(const void* src_, void* dst_, uint64_t len) {
    const DType* src = static_cast<const DType*>(src_);
    DType* dst = static_cast<DType*>(dst_);
    for (uint64_t i = 0; i < len; ++i) OP::Reduce(dst[i], src[i]);
}
}  // namespace op


/*! \brief a typed view of memory (include/transport/buffer.h:15-257): address,
 *  size in bytes, optional item size (Count()), byte offsets start/end of a
 *  Slice relative to its parent.  A view, never an owner — except through
 *  AllocTemp/FreeTemp or Alloc/Free (host memory).  Host or device memory.
 *  The reference's RDMA / shm registration and its memory pool are not part
 *  of this path; `pinned` is kept as a flag (RdcNewBuffer pins page-aligned
 *  host ranges for point-to-point). */
class Buffer {
public:
    Buffer() {}
    explicit Buffer(uint64_t size_in_bytes) : size_in_bytes_(size_in_bytes), end_(size_in_bytes) {}
    Buffer(void* addr, uint64_t size_in_bytes) : Buffer(addr, size_in_bytes, 0, size_in_bytes, false) {}
    Buffer(const void* addr, uint64_t size_in_bytes) : Buffer(addr, size_in_bytes, 0, size_in_bytes, false) {}
    Buffer(void* addr, uint64_t size_in_bytes, const bool& pinned)
        : Buffer(addr, size_in_bytes, 0, size_in_bytes, pinned) {}
    Buffer(const void* addr, uint64_t size_in_bytes, const bool& pinned)
        : Buffer(addr, size_in_bytes, 0, size_in_bytes, pinned) {}
    Buffer(void* addr, uint64_t size_in_bytes, uint64_t start, uint64_t end)
        : Buffer(addr, size_in_bytes, start, end, false) {}
    Buffer(const void* addr, uint64_t size_in_bytes, uint64_t start, uint64_t end)
        : Buffer(addr, size_in_bytes, start, end, false) {}
    Buffer(void* addr, uint64_t size_in_bytes, uint64_t start, uint64_t end, const bool& pinned)
        : addr_(addr), size_in_bytes_(size_in_bytes), is_mutable_(true), start_(start), end_(end), pinned_(pinned) {}
    Buffer(const void* addr, uint64_t size_in_bytes, uint64_t start, uint64_t end, const bool& pinned)
        : addr_(const_cast<void*>(addr)), size_in_bytes_(size_in_bytes), is_mutable_(false), start_(start),
          end_(end), pinned_(pinned) {}

    /*! \brief bytes [start, end) of this buffer, same item size (buffer.h:112-119) */
    Buffer Slice(const uint64_t& start, const uint64_t& end) const {
        Buffer b(static_cast<void*>(static_cast<int8_t*>(addr_) + start), end - start, start, end, pinned_);
        b.with_type_ = with_type_;
        b.item_size_ = item_size_;
        b.dtype_ = dtype_;
        b.is_mutable_ = is_mutable_;
        return b;
    }
    template <typename DType> DType* As() const { return reinterpret_cast<DType*>(addr_); }
    template <typename DType> DType* At(const uint32_t& index) { return reinterpret_cast<DType*>(addr_) + index; }
    void* addr() const { return addr_; }
    void set_addr(void* addr) { addr_ = addr; is_mutable_ = true; }
    void set_addr(const void* addr) { addr_ = const_cast<void*>(addr); is_mutable_ = false; }
    uint64_t size_in_bytes() const { return size_in_bytes_; }
    void set_size_in_bytes(const uint64_t& size_in_bytes) { size_in_bytes_ = size_in_bytes; }
    bool is_mutable() const { return is_mutable_; }
    void set_is_mutable(const bool& is_mutable) { is_mutable_ = is_mutable; }
    bool pinned() const { return pinned_; }
    /*! \brief number of items; needs an item size that divides the size (buffer.h:171-174) */
    uint64_t Count() const {
        if (!with_type_ || item_size_ == 0 || size_in_bytes_ % item_size_ != 0) {
            fprintf(stderr, "rdc: Buffer::Count needs an item size dividing the buffer (size %llu, item %llu)\n",
                    (unsigned long long)size_in_bytes_, (unsigned long long)item_size_);
            abort();
        }
        return size_in_bytes_ / item_size_;
    }
    bool with_type() const { return with_type_; }
    void set_with_type(const bool& with_type) { with_type_ = with_type; }
    uint64_t item_size() const { return item_size_; }
    void set_item_size(const uint64_t& item_size) { with_type_ = true; item_size_ = item_size; }
    uint64_t start() const { return start_; }
    uint64_t end() const { return end_; }
    void set_start(const uint64_t start) { start_ = start; }
    void set_end(const uint64_t end) { end_ = end; }
    /*! \brief MI355X addition: the element type, so Allreduce<OP>(Buffer&) can
     *  pick the device kernel (sets the item size too).  -1 = untyped. */
    template <typename DType> void set_type();
    int dtype() const { return dtype_; }
    void AllocTemp(const std::function<void*(const uint64_t&)>& alloc_func) {
        own_data_ = true;
        addr_ = alloc_func(size_in_bytes_);
        is_mutable_ = true;
    }
    void FreeTemp(const std::function<void(void*)>& free_func) {
        own_data_ = false;
        free_func(addr_);
        addr_ = nullptr;
    }
    /*! \brief host memory of size_in_bytes (the reference's pool, buffer.h:220-230) */
    void Alloc() {
        own_data_ = true;
        addr_ = malloc(size_in_bytes_ ? size_in_bytes_ : 1);
        is_mutable_ = true;
    }
    void Free() {
        own_data_ = false;
        free(addr_);
        addr_ = nullptr;
    }

private:
    void* addr_ = nullptr;
    uint64_t size_in_bytes_ = 0;
    bool is_mutable_ = true;
    bool with_type_ = false;
    uint64_t item_size_ = 0;
    int dtype_ = -1;
    bool own_data_ = false;
    uint64_t start_ = 0;
    uint64_t end_ = 0;
    bool pinned_ = false;
};

/*! \brief serialization streams for SerializeReducer (include/io/io.h:14-70,
 *  include/io/memory_io.h:4-32) */
class Stream {
public:
    virtual ~Stream() {}
    virtual size_t Read(void* ptr, size_t size) = 0;
    virtual void Write(const void* ptr, size_t size) = 0;
    template <typename T> void Write(const T& data) {
        static_assert(std::is_trivially_copyable<T>::value, "rdc::Stream::Write<T>: trivially copyable T only");
        Write(&data, sizeof(T));
    }
    template <typename T> bool Read(T* out) {
        static_assert(std::is_trivially_copyable<T>::value, "rdc::Stream::Read<T>: trivially copyable T only");
        return Read(out, sizeof(T)) == sizeof(T);
    }
};
class SeekStream : public Stream {
public:
    virtual void Seek(size_t pos) = 0;
    virtual size_t Tell() = 0;
};
/*! \brief a fixed-size memory region as a stream; writing past the end aborts */
class MemoryFixedSizeStream : public SeekStream {
public:
    MemoryFixedSizeStream(void* p_buffer, size_t buffer_size)
        : p_buffer_(static_cast<char*>(p_buffer)), buffer_size_(buffer_size) {}
    size_t Read(void* ptr, size_t size) override {
        const size_t n = curr_ptr_ + size <= buffer_size_ ? size : buffer_size_ - curr_ptr_;
        if (n) memcpy(ptr, p_buffer_ + curr_ptr_, n);
        curr_ptr_ += n;
        return n;
    }
    void Write(const void* ptr, size_t size) override {
        if (curr_ptr_ + size > buffer_size_) {
            fprintf(stderr, "rdc: MemoryFixedSizeStream: writing %zu bytes past a %zu-byte buffer\n", size,
                    buffer_size_);
            abort();
        }
        if (size) memcpy(p_buffer_ + curr_ptr_, ptr, size);
        curr_ptr_ += size;
    }
    using Stream::Read;
    using Stream::Write;
    void Seek(size_t pos) override { curr_ptr_ = pos; }
    size_t Tell() override { return curr_ptr_; }
    bool AtEnd() const { return curr_ptr_ == buffer_size_; }
    void* inner_buffer() const { return p_buffer_; }
    size_t inner_buffer_size() const { return buffer_size_; }

private:
    char* p_buffer_;
    size_t buffer_size_;
    size_t curr_ptr_ = 0;
};

template <typename DType> inline void Buffer::set_type() {
    set_item_size(sizeof(DType));
    dtype_ = (int)mpi::GetType<DType>();
}

namespace detail {
inline void Check(int rc, const char* what) {
    if (rc != 0) {
        fprintf(stderr, "rdc: %s failed: %s\n", what, RdcGetLastError());
        abort();
    }
}
inline void Fail(const char* what, const std::string& why) {
    fprintf(stderr, "rdc: %s failed: %s\n", what, why.c_str());
    abort();
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
/*! \brief reducer over a received chunk and this rank's chunk, dst = OP(dst, src)
 *  (include/comm/communicator.h:36) */
using ReduceFunction = std::function<void(Buffer src, Buffer dst)>;

/*! \brief a named communicator (include/comm/communicator.h:41-146) */
class ICommunicator {
public:
    ICommunicator(void* handle, const std::string& name) : handle_(handle), name_(name) {}
    virtual ~ICommunicator() {}
    /*! \brief in-place allreduce of count elements (host or device memory) */
    virtual void Allreduce(void* sendrecvbuf, uint64_t count, mpi::DataType dtype, mpi::OpType op) {
        detail::Check(RdcAllreduceOn(handle_, sendrecvbuf, count, (int)dtype, (int)op), "Allreduce");
    }
    /*! \brief allreduce with a custom HOST reducer (communicator.h:92-93, virtual
     *  here).  sendrecvbuf needs an item size (Count()).  Ring order per Split
     *  chunk above rdc_reduce_ring_mincount bytes, the tree's order at or below
     *  (TryAllreduce, communicator_collective.cc:6-13); reducer(src, dst) is
     *  called on chunk-sized Buffers exactly as the reference's ring / tree
     *  would call it.  Data moves over the device path (allgather). */
    virtual void Allreduce(Buffer sendrecvbuf, ReduceFunction reducer);
    /*! \brief bucketed allreduce: Allreduce of every bufs[b] (counts[b] items), fused launches */
    virtual void AllreduceCoalesced(void** bufs, const size_t* counts, int nbuf, mpi::DataType dtype,
                                    mpi::OpType op) {
        detail::Check(RdcAllreduceCoalescedOn(handle_, bufs, counts, nbuf, (int)dtype, (int)op), "AllreduceCoalesced");
    }
    /*! \brief broadcast size bytes from root (host or device memory) */
    virtual void Broadcast(void* sendrecvaddr, uint64_t size, int root) {
        detail::Check(RdcBroadcastOn(handle_, sendrecvaddr, size, root), "Broadcast");
    }
    /*! \brief broadcast a Buffer (communicator.h:100-101, virtual here) */
    virtual void Broadcast(Buffer sendrecvbuf, int root) {
        Broadcast(sendrecvbuf.addr(), sendrecvbuf.size_in_bytes(), root);
    }
    /*! \brief bufs[c] holds sizes[c] bytes; bufs[rank] is this rank's data */
    virtual void Allgather(void** bufs, const size_t* sizes) {
        detail::Check(RdcAllgatherOn(handle_, bufs, sizes), "Allgather");
    }
    /*! \brief Allgather of per-rank Buffers (communicator.h:107-119, virtual here) */
    virtual void Allgather(std::vector<Buffer> sendrecvbufs) {
        std::vector<void*> p(sendrecvbufs.size());
        std::vector<size_t> sz(sendrecvbufs.size());
        for (size_t i = 0; i < p.size(); ++i) {
            p[i] = sendrecvbufs[i].addr();
            sz[i] = sendrecvbufs[i].size_in_bytes();
        }
        Allgather(p.data(), sz.data());
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
    virtual WorkCompletion* ISend(Buffer sendbuf, int dest) {
        return ISend(sendbuf.addr(), sendbuf.size_in_bytes(), dest);
    }
    virtual WorkCompletion* IRecv(Buffer recvbuf, int src) {
        return IRecv(recvbuf.addr(), recvbuf.size_in_bytes(), src);
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
    virtual void Send(Buffer sendbuf, int dest) { Send(sendbuf.addr(), sendbuf.size_in_bytes(), dest); }
    virtual void Recv(Buffer recvbuf, int src) { Recv(recvbuf.addr(), recvbuf.size_in_bytes(), src); }
    /*! \brief sub-communicator over ranks of this one (communicator.h:133-134):
     *  collective over every rank of this communicator; null on non-members */
    std::unique_ptr<ICommunicator> CreateGroup(const std::vector<int>& ranks, const std::string& group_name = "");
    int GetRank() const { return RdcCommRank(handle_); }
    int GetWorldSize() const { return RdcCommSize(handle_); }
    bool IsDistributed() const { return GetWorldSize() > 1; }
    std::string name() const { return name_; }
    void* handle() const { return handle_; }

private:
    void* handle_;
    std::string name_;
};

/*! \brief a CreateGroup communicator: owned by its unique_ptr (destroying it is
 *  collective over the group's members) */
class GroupCommunicator : public ICommunicator {
public:
    using ICommunicator::ICommunicator;
    ~GroupCommunicator() override { RdcCommDestroy(handle()); }  // after Finalize: a no-op error code
};

inline std::unique_ptr<ICommunicator> ICommunicator::CreateGroup(const std::vector<int>& ranks,
                                                                 const std::string& group_name) {
    void* h = nullptr;
    detail::Check(RdcCreateGroup(&h, handle_, ranks.data(), (int)ranks.size(), group_name.c_str()), "CreateGroup");
    if (!h) return std::unique_ptr<ICommunicator>();
    return std::unique_ptr<ICommunicator>(new GroupCommunicator(h, group_name));
}

inline void ICommunicator::Allreduce(Buffer buf, ReduceFunction reducer) {
    const int n = GetWorldSize(), r = GetRank();
    const uint64_t S = buf.size_in_bytes();
    if (n <= 1 || S == 0) return;  // communicator_base.h:133-138
    const uint64_t isz = buf.item_size(), count = buf.Count();
    auto view = [&](std::vector<char>& v, uint64_t off, uint64_t len) {
        Buffer b(v.data() + off, len, off, off + len);
        b.set_item_size(isz);
        return b;
    };
    uint64_t mincount = 1;
    detail::Check(RdcCommGetParam(handle_, "rdc_reduce_ring_mincount", &mincount), "Allreduce");
    if (S <= mincount) {
        // TryAllreduceTree (communicator_collective.cc:14-43,71-78): the fold
        // to rank 0 in the tree's order over whole (small: <= the threshold)
        // buffers, then everyone gets rank 0's bytes
        std::vector<std::vector<char>> in((size_t)n, std::vector<char>((size_t)S));
        detail::Check(RdcMemcpy(in[(size_t)r].data(), buf.addr(), S), "Allreduce input copy");
        std::vector<void*> ptrs((size_t)n);
        std::vector<size_t> sizes((size_t)n, (size_t)S);
        for (int q = 0; q < n; ++q) ptrs[(size_t)q] = in[(size_t)q].data();
        Allgather(ptrs.data(), sizes.data());
        int dst[16], src[16];
        const int k = RdcPlanTree(n, dst, src);
        for (int i = 0; i < k; ++i) reducer(view(in[(size_t)src[i]], 0, S), view(in[(size_t)dst[i]], 0, S));
        detail::Check(RdcMemcpy(buf.addr(), in[0].data(), S), "Allreduce result copy");
        return;
    }
    // TryReduceScatterRing (:115-182): rank r ends with chunk r of
    // utils::Split(0, count, n) = x[r] (+) (x[r+1] (+) ... (+) x[r-1]), each
    // step reducer(src = received partial, dst = this rank's chunk).  Only
    // chunk r of every rank's input is needed for that: rank q sends its
    // chunk c straight to rank c (point-to-point over the device path, all
    // pairs at once), (n-1)/n x S in and out per rank — the reference ring's
    // reduce-scatter traffic — and the host holds S/n per peer, not S.
    std::vector<uint64_t> off((size_t)n), len((size_t)n);
    const uint64_t kq = count / (uint64_t)n, km = count % (uint64_t)n;
    for (int c = 0; c < n; ++c) {
        const uint64_t b = (uint64_t)c * kq + std::min<uint64_t>((uint64_t)c, km);
        const uint64_t e = (uint64_t)(c + 1) * kq + std::min<uint64_t>((uint64_t)(c + 1), km);
        off[(size_t)c] = b * isz;
        len[(size_t)c] = (e - b) * isz;
    }
    const uint64_t o = off[(size_t)r], l = len[(size_t)r];
    std::vector<std::vector<char>> x((size_t)n);  // x[q] = rank q's chunk r
    if (l > 0) {
        for (int q = 0; q < n; ++q) x[(size_t)q].resize((size_t)l);
        detail::Check(RdcMemcpy(x[(size_t)r].data(), static_cast<char*>(buf.addr()) + o, l), "Allreduce input copy");
    }
    std::vector<WorkCompletion*> pending;
    for (int k = 1; k < n; ++k) {
        const int q = (r + k) % n;  // send chunk q to rank q; receive chunk r from rank (r - k)
        const int p = (r - k + n) % n;
        if (len[(size_t)q] > 0) pending.push_back(ISend(static_cast<char*>(buf.addr()) + off[(size_t)q], len[(size_t)q], q));
        if (l > 0) pending.push_back(IRecv(x[(size_t)p].data(), l, p));
    }
    bool ok = true;
    std::string err;
    for (WorkCompletion* w : pending) {
        if (!w->Wait() && ok) {
            ok = false;
            err = w->Error();
        }
        delete w;
    }
    if (!ok) detail::Fail("Allreduce chunk exchange", err);
    if (l > 0) {
        std::vector<char> partial(x[(size_t)((r - 1 + n) % n)]);
        for (int j = 2; j <= n; ++j) {
            std::vector<char>& d = x[(size_t)((r - j + n) % n)];
            Buffer dv(d.data(), l, o, o + l);  // the same Slice(o, o + l) view the full-buffer form passed
            dv.set_item_size(isz);
            reducer(view(partial, 0, l), dv);
            partial.swap(d);  // d (now the new partial) is not needed as an input again
        }
        detail::Check(RdcMemcpy(static_cast<char*>(buf.addr()) + o, partial.data(), l), "Allreduce result copy");
    }
    // TryAllgatherRing (:79-114): chunk c from rank c, in place
    std::vector<void*> cb((size_t)n);
    std::vector<size_t> cs((size_t)n);
    for (int c = 0; c < n; ++c) {
        cb[(size_t)c] = static_cast<char*>(buf.addr()) + off[(size_t)c];
        cs[(size_t)c] = (size_t)len[(size_t)c];
    }
    Allgather(cb.data(), cs.data());
}

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
namespace comm {
/*! \brief the reference's allreduce glue (src/comm/communicator.cc:24-28): the
 *  named communicator's Allreduce(Buffer, ReduceFunction) with `red` as the
 *  reducer.  dtype / op describe the buffer for the caller's benefit only, as
 *  in the reference (which ignores them); the typed device path is
 *  rdc::Allreduce<OP,DType>. */
inline void Allreduce_(Buffer sendrecvbuf, ReduceFunction red, mpi::DataType dtype, mpi::OpType op,
                       const std::string& name) {
    (void)dtype;
    (void)op;
    GetCommunicator(name)->Allreduce(sendrecvbuf, red);
}
}  // namespace comm

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

/*! \brief point-to-point on Buffers (rdc-inl.h:53-58; include/api.h:12-13's
 *  size argument, when given, must not exceed the Buffer and limits the bytes) */
inline void Send(const Buffer& sendbuf, int dest) { GetCommunicator()->Send(sendbuf, dest); }
inline void Recv(Buffer& recvbuf, int src) { GetCommunicator()->Recv(recvbuf, src); }
inline void Send(const Buffer& send_buf, size_t size, int dest) {
    if (size > send_buf.size_in_bytes()) {
        fprintf(stderr, "rdc: Send of %zu bytes from a %llu-byte Buffer\n", size,
                (unsigned long long)send_buf.size_in_bytes());
        abort();
    }
    GetCommunicator()->Send(send_buf.addr(), size, dest);
}
inline void Recv(Buffer& recv_buf, size_t size, int src) {
    if (size > recv_buf.size_in_bytes()) {
        fprintf(stderr, "rdc: Recv of %zu bytes into a %llu-byte Buffer\n", size,
                (unsigned long long)recv_buf.size_in_bytes());
        abort();
    }
    GetCommunicator()->Recv(recv_buf.addr(), size, src);
}

/*! \brief sub-communicator of "main" over `ranks` (include/api.h:124-125):
 *  collective over every rank; null on ranks not in the group */
inline std::unique_ptr<comm::ICommunicator> CreateGroup(const std::vector<int>& ranks,
                                                        const std::string& group_name = "") {
    return GetCommunicator()->CreateGroup(ranks, group_name);
}

/*! \brief in-place allreduce (include/api.h:62-64, rdc-inl.h:125-135) */
template <typename OP, typename DType>
inline void Allreduce(DType* sendrecvbuf, uint64_t count, const std::string& comm_name = kMainCommName) {
    if (GetWorldSize() == 1 || count == 0) return;  // communicator_base.h:133-138
    GetCommunicator(comm_name)->Allreduce(sendrecvbuf, count, mpi::GetType<DType>(), OP::kType);
}

/*! \brief in-place allreduce of a typed Buffer (include/api.h:65-66; declared
 *  but never defined in the reference): the Buffer must carry its element
 *  type (Buffer::set_type<DType>()), which picks the device kernel */
template <typename OP>
inline void Allreduce(Buffer& sendrecvbuf, const std::string& comm_name = kMainCommName) {
    if (sendrecvbuf.dtype() < 0) {
        fprintf(stderr, "rdc: Allreduce<OP>(Buffer&) needs a typed Buffer (Buffer::set_type<DType>())\n");
        abort();
    }
    if (GetWorldSize() == 1 || sendrecvbuf.size_in_bytes() == 0) return;
    GetCommunicator(comm_name)->Allreduce(sendrecvbuf.addr(), sendrecvbuf.Count(), (mpi::DataType)sendrecvbuf.dtype(),
                                          OP::kType);
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
/*! \brief broadcast a Buffer (include/api.h:25-26, rdc-inl.h:71-75) */
inline void Broadcast(Buffer& buf, int root, const std::string& comm_name = kMainCommName) {
    if (GetWorldSize() == 1 || buf.size_in_bytes() == 0) return;
    GetCommunicator(comm_name)->Broadcast(buf, root);
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
/*! \brief allgather of per-rank Buffers (rdc-inl.h:106-110) */
inline void Allgather(std::vector<Buffer>& sendrecvbufs, const std::string& comm_name = kMainCommName) {
    if (GetWorldSize() == 1) return;
    GetCommunicator(comm_name)->Allgather(sendrecvbufs);
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

/*! \brief custom element-wise reduction (include/api.h:135-146): freduce(dst,
 *  src) on every item, as ReducerSafe_ applies it (rdc-inl.h:142-155: items
 *  copied out and back, no alignment assumed).  DType must be trivially
 *  copyable.  Runs on the host (see ICommunicator::Allreduce(Buffer, ...)). */
template <typename DType, void (*freduce)(DType& dst, const DType& src)>  // NOLINT(*)
class Reducer {
public:
    static_assert(std::is_trivially_copyable<DType>::value, "rdc::Reducer needs a trivially copyable DType");
    Reducer() {}
    void Allreduce(DType* sendrecvbuf, size_t count, const std::string& comm_name = kMainCommName) {
        if (GetWorldSize() == 1 || count == 0) return;
        Buffer b(static_cast<void*>(sendrecvbuf), (uint64_t)count * sizeof(DType));
        b.set_item_size(sizeof(DType));
        GetCommunicator(comm_name)->Allreduce(b, [](Buffer src, Buffer dst) {
            const char* ps = static_cast<const char*>(src.addr());
            char* pd = static_cast<char*>(dst.addr());
            for (uint64_t i = 0, n = src.Count(); i < n; ++i) {
                DType td, ts;
                memcpy(&td, pd + i * sizeof(DType), sizeof(DType));
                memcpy(&ts, ps + i * sizeof(DType), sizeof(DType));
                freduce(td, ts);
                memcpy(pd + i * sizeof(DType), &td, sizeof(DType));
            }
        });
    }
};

/*! \brief reduction of serializable objects (include/api.h:147-174): each of
 *  the `count` objects is saved into a max_nbyte slot (DType::Save(Stream&)
 *  const), slots are reduced with DType::Load(Stream&) + DType::Reduce(const
 *  DType& src, size_t max_nbyte) + Save, and loaded back (the closure of
 *  rdc-inl.h:168-184).  Runs on the host like Reducer. */
template <typename DType>
class SerializeReducer {
public:
    SerializeReducer() {}
    void Allreduce(DType* sendrecvobj, size_t max_nbyte, size_t count, const std::string& comm_name = kMainCommName) {
        if (GetWorldSize() == 1 || count == 0) return;
        buffer_.assign(max_nbyte * count, '\0');
        for (size_t i = 0; i < count; ++i) {
            MemoryFixedSizeStream fs(&buffer_[i * max_nbyte], max_nbyte);
            sendrecvobj[i].Save(fs);
        }
        Buffer b(static_cast<void*>(&buffer_[0]), (uint64_t)(max_nbyte * count));
        b.set_item_size(max_nbyte);
        GetCommunicator(comm_name)->Allreduce(b, [max_nbyte](Buffer src, Buffer dst) {
            char* ps = static_cast<char*>(src.addr());
            char* pd = static_cast<char*>(dst.addr());
            for (uint64_t i = 0, n = src.Count(); i < n; ++i) {
                DType tsrc, tdst;
                MemoryFixedSizeStream fsrc(ps + i * max_nbyte, max_nbyte), fdst(pd + i * max_nbyte, max_nbyte);
                tsrc.Load(fsrc);
                tdst.Load(fdst);
                tdst.Reduce(tsrc, max_nbyte);
                fdst.Seek(0);
                tdst.Save(fdst);
            }
        });
        for (size_t i = 0; i < count; ++i) {
            MemoryFixedSizeStream fs(&buffer_[i * max_nbyte], max_nbyte);
            sendrecvobj[i].Load(fs);
        }
    }

private:
    std::string buffer_;  // count slots of max_nbyte bytes
};

}  // namespace rdc
