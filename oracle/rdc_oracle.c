/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of akkaze/rdc's allreduce hot path, used as the
 * parity checker for the MI355X HIP implementation in rdc_amd/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this file's
 * library; the product path (librdc_amd.so) never links or calls it.
 *
 * Parity pinning: the restatement is checked bit-for-bit against
 *   (1) oracle/_ref (oracle/ref_ring.cc), which runs the reference's OWN
 *       op::Reducer<OP,DType> (include/core/mpi.h:113-120) and utils::Split
 *       (include/utils/utils.h:59-70), compiled from /root/reference headers;
 *   (2) the reference's integer known-answer tests
 *       (test/allreduce.cc:17-55, test/mallreduce.cc:17-53);
 *   (3) the committed golden vectors in tests/golden/ (made by
 *       tests/golden/make_golden.py from (1)).
 * The ring accumulation order restated here was verified bit-exact against
 * the running (shimmed) reference by the survey (SURVEY.md §0 finding 7, §8c).
 *
 * Reference call stack restated:
 *   rdc::Allreduce<OP,DType>          include/core/rdc-inl.h:125-135
 *   Communicator::TryAllreduce        src/comm/communicator_collective.cc:6-13
 *   Communicator::TryAllreduceRing    src/comm/communicator_collective.cc:183-203
 *   Communicator::TryReduceScatterRing src/comm/communicator_collective.cc:115-182
 *   Communicator::TryAllgatherRing    src/comm/communicator_collective.cc:79-114
 *   ring prev/next = (r-1+n)%n, (r+1)%n  src/utils/topo.cc:80-115
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rdc_oracle.h"

/* ------------------------------------------------------------------ */
/* dtype table: enum values are mpi::DataType (include/core/mpi.h:19-30) */
/* plus the MI355X build's additions kFloat16=10, kBFloat16=11.        */
/* ------------------------------------------------------------------ */
size_t rdc_oracle_dtype_size(int dtype) {
    switch (dtype) {
        case RDC_DT_INT8: case RDC_DT_UINT8: return 1;
        case RDC_DT_INT32: case RDC_DT_UINT32: case RDC_DT_FLOAT32: return 4;
        case RDC_DT_INT64: case RDC_DT_UINT64: case RDC_DT_FLOAT64:
        case RDC_DT_LONGLONG: case RDC_DT_ULONGLONG: return 8;
        case RDC_DT_FLOAT16: case RDC_DT_BFLOAT16: return 2;
        default: return 0;
    }
}

/* utils::Split (include/utils/utils.h:59-70): first len%n parts get one   */
/* extra element.  The reference computes in int; we use int64 and give   */
/* the same ranges for every count the reference can represent.          */
void rdc_oracle_split(int64_t begin, int64_t end, int nparts,
                      int64_t* out_begin, int64_t* out_end) {
    int64_t len = end - begin;
    int64_t k = len / nparts;
    int64_t m = len % nparts;
    for (int i = 0; i < nparts; ++i) {
        int64_t rb = begin + (int64_t)i * k + (i < m ? i : m);
        int64_t re = begin + (int64_t)(i + 1) * k + (i + 1 < m ? i + 1 : m);
        out_begin[i] = rb;
        out_end[i] = re;
    }
}

/* ---------------- binary16 / bfloat16 helpers (RNE) ---------------- */
float rdc_oracle_f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000) << 16;
    uint32_t exp = (h >> 10) & 0x1f;
    uint32_t mant = h & 0x3ff;
    uint32_t x;
    if (exp == 0) {
        if (mant == 0) {
            x = sign;
        } else { /* subnormal: normalise */
            int e = -1;
            do { mant <<= 1; ++e; } while ((mant & 0x400) == 0);
            mant &= 0x3ff;
            x = sign | ((uint32_t)(127 - 15 - e) << 23) | (mant << 13);
        }
    } else if (exp == 31) {
        x = sign | 0x7f800000u | (mant << 13);
    } else {
        x = sign | ((exp - 15 + 127) << 23) | (mant << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

uint16_t rdc_oracle_f32_to_f16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    uint16_t sign = (uint16_t)((x >> 16) & 0x8000);
    uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) {
        if (ax == 0x7f800000u) return sign | 0x7c00;
        return (uint16_t)(sign | 0x7e00 | ((ax >> 13) & 0x3ff)); /* quiet NaN */
    }
    if (ax >= 0x477ff000u) return sign | 0x7c00; /* >= 65520 -> inf */
    if (ax >= 0x38800000u) {                      /* normal half */
        uint32_t mant = ax & 0x7fffff;
        uint32_t e = (ax >> 23) - 127 + 15;
        uint32_t h = (e << 10) | (mant >> 13);
        uint32_t rem = mant & 0x1fff;
        if (rem > 0x1000 || (rem == 0x1000 && (h & 1))) h++;
        return (uint16_t)(sign | h);
    }
    if (ax <= 0x33000000u) return sign; /* <= 2^-25 rounds (ties-even) to 0 */
    {
        uint32_t E = ax >> 23;
        uint32_t m = (ax & 0x7fffff) | 0x800000;
        int s = 126 - (int)E; /* 14..24 */
        uint32_t h = m >> s;
        uint32_t rem = m & ((1u << s) - 1);
        uint32_t half = 1u << (s - 1);
        if (rem > half || (rem == half && (h & 1))) h++;
        return (uint16_t)(sign | h);
    }
}

float rdc_oracle_bf16_to_f32(uint16_t b) {
    uint32_t x = (uint32_t)b << 16;
    float f;
    memcpy(&f, &x, 4);
    return f;
}

uint16_t rdc_oracle_f32_to_bf16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    if ((x & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((x >> 16) | 0x40);
    x += 0x7fffu + ((x >> 16) & 1u);
    return (uint16_t)(x >> 16);
}

/* ------------------------------------------------------------------ */
/* op::Reducer<OP,DType> (include/core/mpi.h:113-120):                  */
/*   for i < len: OP::Reduce(dst[i], src[i])                            */
/* with OP::Reduce from include/core/mpi.h:85-112:                      */
/*   Max: if (dst < src) dst = src;   Min: if (dst > src) dst = src;    */
/*   Sum: dst += src;                 BitOR: dst |= src;                */
/* Signed integer Sum is computed in the unsigned type (two's-complement */
/* wrap, the bits g++ produces for the reference's overflowing adds).    */
/* f16/bf16 (no reference type): per-hop dst = round(f32(dst)+f32(src)), */
/* which equals the correctly rounded 16-bit add (f32 has >= 2p+2 bits). */
/* ------------------------------------------------------------------ */
#define REDUCE_LOOP(T, UT)                                                   \
    do {                                                                     \
        const T* s = (const T*)src;                                          \
        T* d = (T*)dst;                                                      \
        switch (op) {                                                        \
            case RDC_OP_MAX:                                                 \
                for (uint64_t i = 0; i < len; ++i) if (d[i] < s[i]) d[i] = s[i]; \
                return 0;                                                    \
            case RDC_OP_MIN:                                                 \
                for (uint64_t i = 0; i < len; ++i) if (d[i] > s[i]) d[i] = s[i]; \
                return 0;                                                    \
            case RDC_OP_SUM:                                                 \
                for (uint64_t i = 0; i < len; ++i)                           \
                    d[i] = (T)((UT)d[i] + (UT)s[i]);                         \
                return 0;                                                    \
            case RDC_OP_BITOR:                                               \
                for (uint64_t i = 0; i < len; ++i)                           \
                    d[i] = (T)((UT)d[i] | (UT)s[i]);                         \
                return 0;                                                    \
            default: return -1;                                              \
        }                                                                    \
    } while (0)

#define REDUCE_LOOP_FP(T)                                                    \
    do {                                                                     \
        const T* s = (const T*)src;                                          \
        T* d = (T*)dst;                                                      \
        switch (op) {                                                        \
            case RDC_OP_MAX:                                                 \
                for (uint64_t i = 0; i < len; ++i) if (d[i] < s[i]) d[i] = s[i]; \
                return 0;                                                    \
            case RDC_OP_MIN:                                                 \
                for (uint64_t i = 0; i < len; ++i) if (d[i] > s[i]) d[i] = s[i]; \
                return 0;                                                    \
            case RDC_OP_SUM:                                                 \
                for (uint64_t i = 0; i < len; ++i) d[i] += s[i];             \
                return 0;                                                    \
            default: return -1; /* BitOR on floating point does not compile  \
                                   in the reference (mpi.h:110) */           \
        }                                                                    \
    } while (0)

#define REDUCE_LOOP_16(TOF, FROMF)                                           \
    do {                                                                     \
        const uint16_t* s = (const uint16_t*)src;                            \
        uint16_t* d = (uint16_t*)dst;                                        \
        for (uint64_t i = 0; i < len; ++i) {                                 \
            float a = TOF(d[i]), b = TOF(s[i]);                              \
            switch (op) {                                                    \
                case RDC_OP_MAX: if (a < b) d[i] = s[i]; break;              \
                case RDC_OP_MIN: if (a > b) d[i] = s[i]; break;              \
                case RDC_OP_SUM: d[i] = FROMF(a + b); break;                 \
                default: return -1;                                          \
            }                                                                \
        }                                                                    \
        return 0;                                                            \
    } while (0)

int rdc_oracle_reducer(const void* src, void* dst, uint64_t len, int dtype, int op) {
    if (op < 0 || op > 3) return -1;
    switch (dtype) {
        case RDC_DT_INT8: REDUCE_LOOP(int8_t, uint8_t);
        case RDC_DT_UINT8: REDUCE_LOOP(uint8_t, uint8_t);
        case RDC_DT_INT32: REDUCE_LOOP(int32_t, uint32_t);
        case RDC_DT_UINT32: REDUCE_LOOP(uint32_t, uint32_t);
        case RDC_DT_INT64:
        case RDC_DT_LONGLONG: REDUCE_LOOP(int64_t, uint64_t);
        case RDC_DT_UINT64:
        case RDC_DT_ULONGLONG: REDUCE_LOOP(uint64_t, uint64_t);
        case RDC_DT_FLOAT32: REDUCE_LOOP_FP(float);
        case RDC_DT_FLOAT64: REDUCE_LOOP_FP(double);
        case RDC_DT_FLOAT16: REDUCE_LOOP_16(rdc_oracle_f16_to_f32, rdc_oracle_f32_to_f16);
        case RDC_DT_BFLOAT16: REDUCE_LOOP_16(rdc_oracle_bf16_to_f32, rdc_oracle_f32_to_bf16);
        default: return -1;
    }
}

/* ------------------------------------------------------------------ */
/* Ring schedule.  Every rank runs TryReduceScatterRing's index loop     */
/* (communicator_collective.cc:119-181); we derive, per rank and step,   */
/* which chunk it sends to prev and which it receives from next, using   */
/* the reference's own write_idx/read_idx/stop arithmetic, then execute  */
/* all ranks in lock-step (each ring step is a matched ISend/IRecv pair). */
/* ------------------------------------------------------------------ */
int rdc_oracle_ring_schedule(int n, int rank, int* rs_send, int* rs_recv,
                             int* ag_send, int* ag_recv) {
    /* TryReduceScatterRing (:119-143) */
    uint64_t next = (uint64_t)((rank + 1) % n);
    uint64_t write_idx = next;
    uint64_t read_idx = next + 1;
    uint64_t reduce_idx = read_idx;
    const uint64_t stop_read_idx = (uint64_t)n + next;
    uint64_t stop_write_idx = (uint64_t)n + (uint64_t)rank;
    int step = 0;
    if (stop_write_idx > stop_read_idx) stop_write_idx -= (uint64_t)n;
    for (;;) {
        int finished = (read_idx == stop_read_idx) && (write_idx == stop_write_idx);
        if (finished) break;
        if (step >= n) return -1;
        rs_send[step] = -1;
        rs_recv[step] = -1;
        if (write_idx < reduce_idx && write_idx != stop_write_idx) { /* :145-155 */
            rs_send[step] = (int)(write_idx % (uint64_t)n);
            write_idx++;
        }
        if (read_idx != stop_read_idx) { /* :156-178 */
            rs_recv[step] = (int)(read_idx % (uint64_t)n);
            if ((uint64_t)rs_recv[step] != reduce_idx % (uint64_t)n) return -2;
            read_idx++;
            reduce_idx++;
        }
        step++;
    }
    if (step != n - 1) return -3;
    /* TryAllgatherRing (:79-114) */
    {
        const uint64_t count_bufs = (uint64_t)n;
        const uint64_t stop_w = count_bufs + (uint64_t)rank - 1;
        const uint64_t stop_r = count_bufs + (uint64_t)rank;
        uint64_t w = (uint64_t)rank, r = (uint64_t)rank + 1;
        step = 0;
        for (;;) {
            if (r == stop_r && w == stop_w) break;
            if (step >= n) return -4;
            ag_send[step] = -1;
            ag_recv[step] = -1;
            if (w < r && w != stop_w) { ag_send[step] = (int)(w % count_bufs); w++; }
            if (r != stop_r) { ag_recv[step] = (int)(r % count_bufs); r++; }
            step++;
        }
        if (step != n - 1) return -5;
    }
    return 0;
}

int rdc_oracle_allreduce_ring(void** bufs, int n, uint64_t count, int dtype, int op) {
    size_t esz = rdc_oracle_dtype_size(dtype);
    int64_t cb[RDC_ORACLE_MAX_RANKS], ce[RDC_ORACLE_MAX_RANKS];
    int rs_send[RDC_ORACLE_MAX_RANKS][RDC_ORACLE_MAX_RANKS];
    int rs_recv[RDC_ORACLE_MAX_RANKS][RDC_ORACLE_MAX_RANKS];
    int ag_send[RDC_ORACLE_MAX_RANKS][RDC_ORACLE_MAX_RANKS];
    int ag_recv[RDC_ORACLE_MAX_RANKS][RDC_ORACLE_MAX_RANKS];
    if (esz == 0 || n < 1 || n > RDC_ORACLE_MAX_RANKS || op < 0 || op > 3) return -1;
    /* Communicator::Allreduce returns early at world size 1
       (include/comm/communicator_base.h:133-138) */
    if (n == 1 || count == 0) return 0;
    rdc_oracle_split(0, (int64_t)count, n, cb, ce);
    for (int r = 0; r < n; ++r) {
        int rc = rdc_oracle_ring_schedule(n, r, rs_send[r], rs_recv[r], ag_send[r], ag_recv[r]);
        if (rc) return rc;
    }
    /* Reduce-scatter: at step j rank r receives from next=(r+1)%n exactly the
       chunk next sends at step j, and reduces reducer(src=received,
       dst=own) (communicator_collective.cc:174-176). */
    for (int j = 0; j < n - 1; ++j) {
        for (int r = 0; r < n; ++r) {
            int nx = (r + 1) % n;
            int c = rs_recv[r][j];
            if (c < 0 || rs_send[nx][j] != c) return -6;
            uint64_t off = (uint64_t)cb[c] * esz, len = (uint64_t)(ce[c] - cb[c]);
            /* the chunk nx sends at step j is never the one nx reduces at
               step j, so in-place lock-step execution is exact. */
            int rc = rdc_oracle_reducer((const char*)bufs[nx] + off, (char*)bufs[r] + off,
                                        len, dtype, op);
            if (rc) return rc;
        }
    }
    /* Allgather: rank r copies chunk ag_recv[r][j] from next. */
    for (int j = 0; j < n - 1; ++j) {
        for (int r = 0; r < n; ++r) {
            int nx = (r + 1) % n;
            int c = ag_recv[r][j];
            if (c < 0 || ag_send[nx][j] != c) return -7;
            uint64_t off = (uint64_t)cb[c] * esz, len = (uint64_t)(ce[c] - cb[c]) * esz;
            memcpy((char*)bufs[r] + off, (const char*)bufs[nx] + off, len);
        }
    }
    return 0;
}

/* Closed form of the ring's per-chunk order (verified
   bit-exact against the running reference):
     chunk c: s = x[c-1]; s = OP(x[c-2], s); ...; s = OP(x[c], s)
   where OP(dst, src) is OP::Reduce and indices are mod n.  Result is
   written to out (one buffer); used to cross-check the lock-step ring. */
int rdc_oracle_allreduce_closed_form(const void* const* bufs, int n, uint64_t count,
                                     int dtype, int op, void* out) {
    size_t esz = rdc_oracle_dtype_size(dtype);
    int64_t cb[RDC_ORACLE_MAX_RANKS], ce[RDC_ORACLE_MAX_RANKS];
    if (esz == 0 || n < 1 || n > RDC_ORACLE_MAX_RANKS) return -1;
    if (count == 0) return 0;
    memcpy(out, bufs[0], count * esz);
    if (n == 1) return 0;
    rdc_oracle_split(0, (int64_t)count, n, cb, ce);
    {
        /* per chunk: acc = x[c-1]; then for k=2..n: acc = OP(x[c-k] as dst, acc as src) */
        size_t maxlen = (size_t)(ce[0] - cb[0]) * esz + 16;
        char* acc = (char*)malloc(maxlen);
        char* tmp = (char*)malloc(maxlen);
        if (!acc || !tmp) { free(acc); free(tmp); return -8; }
        for (int c = 0; c < n; ++c) {
            uint64_t off = (uint64_t)cb[c] * esz, len = (uint64_t)(ce[c] - cb[c]);
            int q = (c - 1 + n) % n;
            memcpy(acc, (const char*)bufs[q] + off, len * esz);
            for (int k = 2; k <= n; ++k) {
                q = ((c - k) % n + n) % n;
                memcpy(tmp, (const char*)bufs[q] + off, len * esz);
                int rc = rdc_oracle_reducer(acc, tmp, len, dtype, op);
                if (rc) { free(acc); free(tmp); return rc; }
                memcpy(acc, tmp, len * esz);
            }
            memcpy((char*)out + off, acc, len * esz);
        }
        free(acc);
        free(tmp);
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* Synthetic input generator, identical on device       */
/* (rdc_amd/csrc/rdc_fill.hip) and here:                                 */
/*   u = splitmix64(seed ^ (rank << 40) ^ i)                             */
/*   f32: (float)(int32)(u >> 32) * 2^-31   (full-mantissa values)       */
/*   f64: (double)(int64)u * 2^-63;  f16/bf16: RNE of the f32 value      */
/*   ints: low bytes of u                                                */
/* ------------------------------------------------------------------ */
uint64_t rdc_oracle_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

int rdc_oracle_fill(void* buf, uint64_t count, int dtype, uint64_t seed, int rank) {
    return rdc_oracle_fill_at(buf, 0, count, dtype, seed, rank);
}

/* elements [first, first+count) of the same stream (the generator is keyed
   by position, so a window of a huge buffer costs only its own length) */
int rdc_oracle_fill_at(void* buf, uint64_t first, uint64_t count, int dtype, uint64_t seed, int rank) {
    uint64_t key = seed ^ ((uint64_t)rank << 40);
    for (uint64_t i = 0; i < count; ++i) {
        uint64_t u = rdc_oracle_splitmix64(key ^ (first + i));
        switch (dtype) {
            case RDC_DT_INT8: case RDC_DT_UINT8: ((uint8_t*)buf)[i] = (uint8_t)u; break;
            case RDC_DT_INT32: case RDC_DT_UINT32: ((uint32_t*)buf)[i] = (uint32_t)u; break;
            case RDC_DT_INT64: case RDC_DT_UINT64: case RDC_DT_LONGLONG: case RDC_DT_ULONGLONG:
                ((uint64_t*)buf)[i] = u; break;
            case RDC_DT_FLOAT32:
                ((float*)buf)[i] = (float)(int32_t)(u >> 32) * 0x1p-31f; break;
            case RDC_DT_FLOAT64:
                ((double*)buf)[i] = (double)(int64_t)u * 0x1p-63; break;
            case RDC_DT_FLOAT16:
                ((uint16_t*)buf)[i] = rdc_oracle_f32_to_f16((float)(int32_t)(u >> 32) * 0x1p-31f); break;
            case RDC_DT_BFLOAT16:
                ((uint16_t*)buf)[i] = rdc_oracle_f32_to_bf16((float)(int32_t)(u >> 32) * 0x1p-31f); break;
            default: return -1;
        }
    }
    return 0;
}

/* The closed form above on a window of a buffer too large for the CPU check:
   wins[q] holds rank q's elements [first, first+m) of a `total`-element
   buffer; out receives the allreduce result of those positions, each folded
   in the ring order of its Split(0, total, n) chunk. */
int rdc_oracle_allreduce_window(const void* const* wins, int n, uint64_t total, uint64_t first, uint64_t m,
                                int dtype, int op, void* out) {
    size_t esz = rdc_oracle_dtype_size(dtype);
    int64_t cb[RDC_ORACLE_MAX_RANKS], ce[RDC_ORACLE_MAX_RANKS];
    if (esz == 0 || n < 1 || n > RDC_ORACLE_MAX_RANKS || first + m > total) return -1;
    if (m == 0) return 0;
    memcpy(out, wins[0], m * esz);
    if (n == 1) return 0;
    rdc_oracle_split(0, (int64_t)total, n, cb, ce);
    {
        char* acc = (char*)malloc(m * esz);
        char* tmp = (char*)malloc(m * esz);
        if (!acc || !tmp) { free(acc); free(tmp); return -8; }
        for (int c = 0; c < n; ++c) {
            uint64_t lo = (uint64_t)cb[c] > first ? (uint64_t)cb[c] : first;
            uint64_t hi = (uint64_t)ce[c] < first + m ? (uint64_t)ce[c] : first + m;
            if (lo >= hi) continue;
            uint64_t off = (lo - first) * esz, len = hi - lo;
            int q = (c - 1 + n) % n;
            memcpy(acc, (const char*)wins[q] + off, len * esz);
            for (int k = 2; k <= n; ++k) {
                q = ((c - k) % n + n) % n;
                memcpy(tmp, (const char*)wins[q] + off, len * esz);
                int rc = rdc_oracle_reducer(acc, tmp, len, dtype, op);
                if (rc) { free(acc); free(tmp); return rc; }
                memcpy(acc, tmp, len * esz);
            }
            memcpy((char*)out + off, acc, len * esz);
        }
        free(acc);
        free(tmp);
    }
    return 0;
}
