/* ORACLE — TEST INFRASTRUCTURE ONLY (see rdc_oracle.c header). */
#ifndef RDC_ORACLE_H_
#define RDC_ORACLE_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RDC_ORACLE_MAX_RANKS 16

/* mpi::DataType (include/core/mpi.h:19-30) + MI355X-build additions */
enum {
    RDC_DT_INT8 = 0,
    RDC_DT_UINT8 = 1,
    RDC_DT_INT32 = 2,
    RDC_DT_UINT32 = 3,
    RDC_DT_INT64 = 4,
    RDC_DT_UINT64 = 5,
    RDC_DT_FLOAT32 = 6,
    RDC_DT_FLOAT64 = 7,
    RDC_DT_LONGLONG = 8,
    RDC_DT_ULONGLONG = 9,
    RDC_DT_FLOAT16 = 10,
    RDC_DT_BFLOAT16 = 11
};
/* mpi::OpType (include/core/mpi.h:12-17) */
enum { RDC_OP_MAX = 0, RDC_OP_MIN = 1, RDC_OP_SUM = 2, RDC_OP_BITOR = 3 };

size_t rdc_oracle_dtype_size(int dtype);
void rdc_oracle_split(int64_t begin, int64_t end, int nparts, int64_t* out_begin,
                      int64_t* out_end);
int rdc_oracle_reducer(const void* src, void* dst, uint64_t len, int dtype, int op);
int rdc_oracle_ring_schedule(int n, int rank, int* rs_send, int* rs_recv, int* ag_send,
                             int* ag_recv);
int rdc_oracle_allreduce_ring(void** bufs, int n, uint64_t count, int dtype, int op);
int rdc_oracle_allreduce_closed_form(const void* const* bufs, int n, uint64_t count,
                                     int dtype, int op, void* out);
uint64_t rdc_oracle_splitmix64(uint64_t x);
int rdc_oracle_fill(void* buf, uint64_t count, int dtype, uint64_t seed, int rank);
int rdc_oracle_fill_at(void* buf, uint64_t first, uint64_t count, int dtype, uint64_t seed, int rank);
int rdc_oracle_allreduce_window(const void* const* wins, int n, uint64_t total, uint64_t first, uint64_t m,
                                int dtype, int op, void* out);
float rdc_oracle_f16_to_f32(uint16_t h);
uint16_t rdc_oracle_f32_to_f16(float f);
float rdc_oracle_bf16_to_f32(uint16_t b);
uint16_t rdc_oracle_f32_to_bf16(float f);

#ifdef __cplusplus
}
#endif
#endif
