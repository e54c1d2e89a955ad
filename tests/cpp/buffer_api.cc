// The reference's Buffer-typed / custom-reducer / group C++ surface on the
// MI355X path (include/api.h:12-13,25-26,65-66,124-174;
// include/comm/communicator.h:56-134), as one program per rank.
//
//   buffer_api <outdir> [key=val ...]      (RDC_RANK / rdc_world_size / tracker keys)
//
// Checks what has a known answer itself (integers, copies); float results of
// the custom-reducer paths are written to <outdir>/<case>_rank<r>.bin for the
// Python test to compare with the oracle.  Inputs: splitmix64 floats, the
// oracle's generator (oracle/rdc_oracle.c rdc_oracle_fill).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "rdc.h"

static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static std::vector<float> fill(size_t n, uint64_t seed, int rank) {
    std::vector<float> v(n);
    const uint64_t key = seed ^ ((uint64_t)rank << 40);
    for (size_t i = 0; i < n; ++i) v[i] = (float)(int32_t)(splitmix64(key ^ i) >> 32) * (1.0f / 2147483648.0f);  // 2^-31, exact
    return v;
}

static std::string g_out;
static int g_rank = 0;
static void save(const char* name, const void* p, size_t bytes) {
    std::string path = g_out + "/" + name + "_rank" + std::to_string(g_rank) + ".bin";
    FILE* f = fopen(path.c_str(), "wb");
    if (!f || fwrite(p, 1, bytes, f) != bytes) {
        fprintf(stderr, "cannot write %s\n", path.c_str());
        abort();
    }
    fclose(f);
}
#define EXPECT(cond, ...)                                   \
    do {                                                    \
        if (!(cond)) {                                      \
            fprintf(stderr, "rank %d: FAILED %s: ", g_rank, #cond); \
            fprintf(stderr, __VA_ARGS__);                   \
            fprintf(stderr, "\n");                          \
            abort();                                        \
        }                                                   \
    } while (0)

static void fsum(float& dst, const float& src) { dst += src; }

struct Pair {  // trivially copyable item for Reducer<DType, freduce>
    int32_t count;
    float peak;
};
static void pair_reduce(Pair& dst, const Pair& src) {
    dst.count += src.count;
    if (dst.peak < src.peak) dst.peak = src.peak;
}

// SerializeReducer item: a variable-length list of (key, value) ints, merged by key
struct Bag {
    std::vector<std::pair<int32_t, int32_t>> kv;
    void Save(rdc::Stream& fo) const {
        const uint32_t n = (uint32_t)kv.size();
        fo.Write(n);
        for (const auto& e : kv) {
            fo.Write(e.first);
            fo.Write(e.second);
        }
    }
    void Load(rdc::Stream& fi) {
        uint32_t n = 0;
        fi.Read(&n);
        kv.resize(n);
        for (auto& e : kv) {
            fi.Read(&e.first);
            fi.Read(&e.second);
        }
    }
    void Reduce(const Bag& src, size_t) {
        for (const auto& e : src.kv) {
            bool found = false;
            for (auto& d : kv)
                if (d.first == e.first) {
                    d.second += e.second;
                    found = true;
                }
            if (!found) kv.push_back(e);
        }
    }
};

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    g_out = argv[1];
    rdc::Init(argc - 1, argv + 1);
    const int n = rdc::GetWorldSize(), r = rdc::GetRank();
    g_rank = r;

    // ---- Buffer as a view (buffer.h:15-257)
    {
        std::vector<int32_t> a(10);
        for (int i = 0; i < 10; ++i) a[(size_t)i] = i;
        rdc::Buffer b(a.data(), a.size() * 4);
        b.set_item_size(4);
        EXPECT(b.Count() == 10, "count %llu", (unsigned long long)b.Count());
        rdc::Buffer s = b.Slice(8, 24);
        EXPECT(s.Count() == 4 && *s.As<int32_t>() == 2 && *s.At<int32_t>(3) == 5 && s.start() == 8 && s.end() == 24,
               "slice");
        rdc::Buffer t(64);
        t.Alloc();
        memset(t.addr(), 7, 64);
        t.Free();
        EXPECT(t.addr() == nullptr, "free");
    }

    // ---- Allreduce<OP>(Buffer&) (api.h:65-66): typed Buffers
    {
        const size_t N = 1001;
        std::vector<int32_t> a(N);
        for (size_t i = 0; i < N; ++i) a[i] = r + (int32_t)N + (int32_t)i;  // test/allreduce.cc's values
        rdc::Buffer b(a.data(), N * 4);
        b.set_type<int32_t>();
        rdc::Allreduce<rdc::op::Max>(b);
        for (size_t i = 0; i < N; ++i) EXPECT(a[i] == (n - 1) + (int32_t)N + (int32_t)i, "max at %zu", i);
        std::vector<float> f = fill(N, 0x5EED3000, r);
        rdc::Buffer fb(f.data(), N * 4);
        fb.set_type<float>();
        rdc::Allreduce<rdc::op::Sum>(fb);
        save("typed_sum", f.data(), N * 4);
    }

    // ---- Broadcast(Buffer&, root) (api.h:25-26) and ICommunicator::Broadcast(Buffer, int)
    {
        std::vector<uint8_t> v(3001);
        for (size_t i = 0; i < v.size(); ++i) v[i] = (uint8_t)(i * 7 + r);
        rdc::Buffer b(v.data(), v.size());
        const int root = n - 1;
        rdc::Broadcast(b, root);
        for (size_t i = 0; i < v.size(); ++i) EXPECT(v[i] == (uint8_t)(i * 7 + root), "bcast at %zu", i);
        std::vector<uint8_t> w(17, (uint8_t)r);
        rdc::GetCommunicator()->Broadcast(rdc::Buffer(w.data(), w.size()), 0);
        for (uint8_t x : w) EXPECT(x == 0, "bcast(Buffer) value %d", (int)x);
    }

    // ---- Send / Recv on Buffers (rdc-inl.h:53-58, api.h:12-13): a ring shift
    {
        std::vector<int32_t> out(257), in(257, -1);
        for (size_t i = 0; i < out.size(); ++i) out[i] = r * 1000 + (int32_t)i;
        const int next = (r + 1) % n, prev = (r + n - 1) % n;
        rdc::Buffer ob(out.data(), out.size() * 4), ib(in.data(), in.size() * 4);
        if (r % 2 == 0) {
            rdc::Send(ob, next);
            rdc::Recv(ib, prev);
        } else {
            rdc::Recv(ib, prev);
            rdc::Send(ob, next);
        }
        for (size_t i = 0; i < in.size(); ++i) EXPECT(in[i] == prev * 1000 + (int32_t)i, "recv at %zu", i);
        std::vector<int32_t> in2(100, -1);
        rdc::Buffer ib2(in2.data(), in2.size() * 4);
        if (r % 2 == 0) {
            rdc::Send(ob, 100 * 4, next);
            rdc::Recv(ib2, 100 * 4, prev);
        } else {
            rdc::Recv(ib2, 100 * 4, prev);
            rdc::Send(ob, 100 * 4, next);
        }
        for (size_t i = 0; i < in2.size(); ++i) EXPECT(in2[i] == prev * 1000 + (int32_t)i, "recv(size) at %zu", i);
        rdc::comm::ICommunicator* c = rdc::GetCommunicator();
        rdc::WorkCompletion* ws = c->ISend(ob, next);
        rdc::WorkCompletion* wr = c->IRecv(ib, prev);
        EXPECT(ws->Wait() && wr->Wait(), "ISend/IRecv(Buffer)");
        delete ws;
        delete wr;
    }

    // ---- Allgather(std::vector<Buffer>&) (rdc-inl.h:106-110): buffer i has i + 5 int32
    {
        std::vector<std::vector<int32_t>> data((size_t)n);
        std::vector<rdc::Buffer> bufs;
        for (int i = 0; i < n; ++i) {
            data[(size_t)i].assign((size_t)(i + 5), -1);
            if (i == r)
                for (int j = 0; j < i + 5; ++j) data[(size_t)i][(size_t)j] = i * 100 + j;
            bufs.emplace_back(data[(size_t)i].data(), data[(size_t)i].size() * 4);
        }
        rdc::Allgather(bufs);
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < i + 5; ++j) EXPECT(data[(size_t)i][(size_t)j] == i * 100 + j, "allgather %d %d", i, j);
    }

    // ---- ICommunicator::Allreduce(Buffer, ReduceFunction) (communicator.h:92, virtual)
    {
        const size_t N = 1001;
        std::vector<float> f = fill(N, 0x5EED3100, r);
        rdc::Buffer b(f.data(), N * 4);
        b.set_item_size(4);
        int calls = 0;
        rdc::GetCommunicator()->Allreduce(b, [&calls](rdc::Buffer src, rdc::Buffer dst) {
            ++calls;
            float* d = dst.As<float>();
            const float* s = src.As<float>();
            for (uint64_t i = 0; i < dst.Count(); ++i) d[i] += s[i];
        });
        save("custom_sum", f.data(), N * 4);
        // chunks of zero length (count < ranks) and a count Split leaves ragged
        for (size_t M : {(size_t)1, (size_t)2, (size_t)3, ((size_t)1 << 18) + 3}) {
            std::vector<float> h = fill(M, 0x5EED3100 + (uint64_t)M, r);
            rdc::Buffer hb(h.data(), M * 4);
            hb.set_item_size(4);
            rdc::GetCommunicator()->Allreduce(hb, [](rdc::Buffer src, rdc::Buffer dst) {
                float* d = dst.As<float>();
                const float* s = src.As<float>();
                for (uint64_t i = 0; i < dst.Count(); ++i) d[i] += s[i];
            });
            save(("custom_sum_" + std::to_string(M)).c_str(), h.data(), M * 4);
        }
        std::vector<float> g = fill(N, 0x5EED3200, r);
        rdc::Reducer<float, fsum> red;
        red.Allreduce(g.data(), N);
        save("reducer_sum", g.data(), N * 4);
    }

    // ---- the reference's own reducer idiom (include/core/rdc-inl.h:125-135):
    // a typed Buffer, the lambda over op::Reducer<OP,DType> (mpi.h:113-120),
    // through the virtual ICommunicator::Allreduce(Buffer, ReduceFunction) and
    // through comm::Allreduce_ (src/comm/communicator.cc:24-28)
    {
        const size_t N = 1001;
        std::vector<float> f = fill(N, 0x5EED3400, r);
        rdc::Buffer sendrecvbuf(f.data(), N * sizeof(float));
        sendrecvbuf.set_item_size(sizeof(float));
        auto reducer = [](rdc::Buffer src, rdc::Buffer dst) {
            rdc::op::Reducer<rdc::op::Sum, float>(src.addr(), dst.addr(), src.Count());
        };
        rdc::GetCommunicator()->Allreduce(sendrecvbuf, reducer);
        save("op_reducer_sum", f.data(), N * 4);

        std::vector<float> m = fill(N, 0x5EED3500, r);
        rdc::Buffer mb(m.data(), N * sizeof(float));
        mb.set_item_size(sizeof(float));
        rdc::comm::Allreduce_(mb, [](rdc::Buffer src, rdc::Buffer dst) {
            rdc::op::Reducer<rdc::op::Max, float>(src.addr(), dst.addr(), src.Count());
        }, rdc::mpi::GetType<float>(), rdc::op::Max::kType, rdc::kMainCommName);
        save("op_reducer_max", m.data(), N * 4);

        // test/allreduce.cc's integer known answers through the same idiom
        std::vector<int32_t> a(N);
        for (size_t i = 0; i < N; ++i) a[i] = r + (int32_t)N + (int32_t)i;
        rdc::Buffer ab(a.data(), N * sizeof(int32_t));
        ab.set_item_size(sizeof(int32_t));
        rdc::comm::Allreduce_(ab, [](rdc::Buffer src, rdc::Buffer dst) {
            rdc::op::Reducer<rdc::op::Sum, int32_t>(src.addr(), dst.addr(), src.Count());
        }, rdc::mpi::kInt, rdc::mpi::kSum, rdc::kMainCommName);
        for (size_t i = 0; i < N; ++i) {
            int32_t want = 0;
            for (int q = 0; q < n; ++q) want += q + (int32_t)N + (int32_t)i;
            EXPECT(a[i] == want, "op::Reducer<Sum,int> at %zu: %d != %d", i, a[i], want);
        }
        std::vector<uint8_t> bits(N);
        for (size_t i = 0; i < N; ++i) bits[i] = (uint8_t)(1u << ((i + (size_t)r) % 8));
        rdc::Buffer bb(bits.data(), N);
        bb.set_item_size(1);
        rdc::GetCommunicator()->Allreduce(bb, [](rdc::Buffer src, rdc::Buffer dst) {
            rdc::op::Reducer<rdc::op::BitOR, uint8_t>(src.addr(), dst.addr(), src.Count());
        });
        for (size_t i = 0; i < N; ++i) {
            uint8_t want = 0;
            for (int q = 0; q < n; ++q) want |= (uint8_t)(1u << ((i + (size_t)q) % 8));
            EXPECT(bits[i] == want, "op::Reducer<BitOR,uint8_t> at %zu", i);
        }
    }

    // ---- Reducer<Pair, pair_reduce> (api.h:135-146): struct items, known answers
    {
        std::vector<Pair> p(33);
        for (size_t i = 0; i < p.size(); ++i) p[i] = Pair{r + 1, (float)(r * 10 + (int)i)};
        rdc::Reducer<Pair, pair_reduce> red;
        red.Allreduce(p.data(), p.size());
        for (size_t i = 0; i < p.size(); ++i)
            EXPECT(p[i].count == n * (n + 1) / 2 && p[i].peak == (float)((n - 1) * 10 + (int)i), "pair %zu", i);
    }

    // ---- SerializeReducer<Bag> (api.h:147-174): variable-length objects
    {
        std::vector<Bag> bags(5);
        for (size_t i = 0; i < bags.size(); ++i) {
            bags[i].kv.push_back(std::make_pair((int32_t)i, r + 1));        // shared key
            bags[i].kv.push_back(std::make_pair(100 + r, (int32_t)i));     // rank's own key
        }
        rdc::SerializeReducer<Bag> red;
        red.Allreduce(bags.data(), 4 + 8 * (2 + (size_t)n), bags.size());
        for (size_t i = 0; i < bags.size(); ++i) {
            EXPECT(bags[i].kv.size() == (size_t)(1 + n), "bag %zu size %zu", i, bags[i].kv.size());
            int32_t shared = -1, total_own = 0;
            for (const auto& e : bags[i].kv) {
                if (e.first == (int32_t)i) shared = e.second;
                else total_own += e.second;
            }
            EXPECT(shared == n * (n + 1) / 2 && total_own == n * (int32_t)i, "bag %zu values", i);
        }
    }

    // ---- CreateGroup (api.h:124-125): even ranks, reversed order
    {
        std::vector<int> members;
        for (int q = n - 1; q >= 0; --q)
            if (q % 2 == 0) members.push_back(q);
        std::unique_ptr<rdc::comm::ICommunicator> g = rdc::CreateGroup(members, "evens");
        if (r % 2 == 0) {
            EXPECT(g != nullptr, "member got no communicator");
            const int gs = (int)members.size();
            int me = -1;
            for (int i = 0; i < gs; ++i)
                if (members[(size_t)i] == r) me = i;
            EXPECT(g->GetWorldSize() == gs && g->GetRank() == me, "group rank %d size %d", g->GetRank(),
                   g->GetWorldSize());
            std::vector<int32_t> v(4099, r);
            g->Allreduce(v.data(), v.size(), rdc::mpi::kInt, rdc::mpi::kSum);
            int32_t want = 0;
            for (int q : members) want += q;
            for (int32_t x : v) EXPECT(x == want, "group sum %d != %d", x, want);
            std::vector<float> f = fill(1001, 0x5EED3300, me);
            g->Allreduce(f.data(), f.size(), rdc::mpi::kFloat, rdc::mpi::kSum);
            save("group_sum", f.data(), f.size() * 4);
            std::vector<char> s(11, (char)('a' + r));
            g->Broadcast(s.data(), s.size(), 0);
            for (char ch : s) EXPECT(ch == (char)('a' + members[0]), "group bcast");
        } else {
            EXPECT(g == nullptr, "non-member got a communicator");
        }
        g.reset();  // collective over the members
        std::vector<int32_t> all(8, 1);  // "main" still works after the group is gone
        rdc::Allreduce<rdc::op::Sum>(all.data(), all.size());
        for (int32_t x : all) EXPECT(x == n, "main after group");
    }

    printf("rank %d: buffer api OK\n", r);
    rdc::Finalize();
    return 0;
}
