// TEST SHIM — include/rdc.h's host op::Reducer<OP,DType> (the restatement of
// include/core/mpi.h:84-120) behind a C entry point, so tests/test_capi.py can
// compare it with oracle/_ref's ref_reducer (the reference's own header
// compiled) for every (dtype, op).
#include <stdint.h>

#include "rdc.h"

namespace {
template <typename OP, typename DType>
void run(const void* src, void* dst, uint64_t len) {
    rdc::op::Reducer<OP, DType>(src, dst, len);
}
template <typename DType>
int arith(int op, const void* src, void* dst, uint64_t len) {
    switch (op) {
        case rdc::mpi::kMax: run<rdc::op::Max, DType>(src, dst, len); return 0;
        case rdc::mpi::kMin: run<rdc::op::Min, DType>(src, dst, len); return 0;
        case rdc::mpi::kSum: run<rdc::op::Sum, DType>(src, dst, len); return 0;
        default: return 1;
    }
}
template <typename DType>
int integer(int op, const void* src, void* dst, uint64_t len) {
    if (op == rdc::mpi::kBitwiseOR) {
        run<rdc::op::BitOR, DType>(src, dst, len);
        return 0;
    }
    return arith<DType>(op, src, dst, len);
}
}  // namespace

// dtype: rdc::mpi::DataType with the C++ types GetType<> maps from
extern "C" int hdr_reducer(const void* src, void* dst, uint64_t len, int dtype, int op) {
    switch (dtype) {
        case rdc::mpi::kChar: return integer<char>(op, src, dst, len);
        case rdc::mpi::kUChar: return integer<unsigned char>(op, src, dst, len);
        case rdc::mpi::kInt: return integer<int>(op, src, dst, len);
        case rdc::mpi::kUInt: return integer<unsigned int>(op, src, dst, len);
        case rdc::mpi::kLong: return integer<long>(op, src, dst, len);                      // NOLINT
        case rdc::mpi::kULong: return integer<unsigned long>(op, src, dst, len);            // NOLINT
        case rdc::mpi::kFloat: return arith<float>(op, src, dst, len);
        case rdc::mpi::kDouble: return arith<double>(op, src, dst, len);
        case rdc::mpi::kLongLong: return integer<long long>(op, src, dst, len);             // NOLINT
        case rdc::mpi::kULongLong: return integer<unsigned long long>(op, src, dst, len);   // NOLINT
        default: return 1;
    }
}

// the op tags' kType values (mpi.h:85-112)
extern "C" int hdr_op_types(int* out4) {
    out4[0] = rdc::op::Max::kType;
    out4[1] = rdc::op::Min::kType;
    out4[2] = rdc::op::Sum::kType;
    out4[3] = rdc::op::BitOR::kType;
    return 0;
}
