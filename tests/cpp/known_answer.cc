// Known-answer program over include/rdc.h, following the checks of the
// reference's test/allreduce.cc:17-55, test/broadcast.cc and test/allgather.cc:
// every rank holds
// a[i] = rank + N + i; Allreduce<Max> must give (W-1)+N+i and Allreduce<Sum>
// sum_j (j+N+i); a broadcast string from rank 0 must arrive intact.
// Buffers live in host memory (the reference's own setting): the library
// stages them through HBM and runs the device allreduce.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "rdc.h"

static int fail(const char* what, int i, long got, long want) {
    fprintf(stderr, "rank %d: %s mismatch at %d: %ld != %ld\n", rdc::GetRank(), what, i, got, want);
    return 1;
}

int main(int argc, char* argv[]) {
    rdc::Init(argc, argv);
    rdc::NewCommunicator(rdc::kMainCommName);
    const int N = argc >= 2 ? atoi(argv[1]) : 3;
    const int W = rdc::GetWorldSize(), R = rdc::GetRank();
    std::vector<int> a(N);
    for (int i = 0; i < N; ++i) a[i] = R + N + i;
    rdc::Allreduce<rdc::op::Max>(&a[0], N);
    for (int i = 0; i < N; ++i)
        if (a[i] != (W - 1) + N + i) return fail("max", i, a[i], (W - 1) + N + i);
    for (int i = 0; i < N; ++i) a[i] = R + N + i;
    rdc::Allreduce<rdc::op::Sum>(&a[0], N);
    for (int i = 0; i < N; ++i) {
        long want = 0;
        for (int j = 0; j < W; ++j) want += j + N + i;
        if (a[i] != want) return fail("sum", i, a[i], want);
    }
    std::string s = R == 0 ? "hello world" : "";
    rdc::Broadcast(s, 0);
    if (s != "hello world") return fail("broadcast", 0, (long)s.size(), 11);
    std::vector<double> v;
    if (R == W - 1) v = {1.5, -2.25, 3.0};
    rdc::Broadcast(v, W - 1);
    if (v.size() != 3 || v[1] != -2.25) return fail("broadcast vector", 0, (long)v.size(), 3);
    // test/allgather.cc: a[i] has i+N items, rank i fills a[i][j] = i + j
    std::vector<std::vector<int>> g((size_t)W);
    for (int i = 0; i < W; ++i) {
        g[(size_t)i].resize((size_t)(i + N));
        if (i == R)
            for (int j = 0; j < i + N; ++j) g[(size_t)i][(size_t)j] = i + j;
    }
    rdc::Allgather(g);
    for (int i = 0; i < W; ++i)
        for (int j = 0; j < i + N; ++j)
            if (g[(size_t)i][(size_t)j] != i + j) return fail("allgather", j, g[(size_t)i][(size_t)j], i + j);
    // test/mallreduce.cc's rounds k = 0..iter-1 (a[i] = rank + N + k + i), all
    // rounds' buffers reduced by ONE coalesced call, then Max the same way
    const int iter = 5;
    std::vector<std::vector<int>> rounds((size_t)iter, std::vector<int>((size_t)N + 0));
    std::vector<int*> ptrs((size_t)iter);
    std::vector<uint64_t> counts((size_t)iter, (uint64_t)N);
    for (int op = 0; op < 2; ++op) {
        for (int k = 0; k < iter; ++k) {
            for (int i = 0; i < N; ++i) rounds[(size_t)k][(size_t)i] = R + N + k + i;
            ptrs[(size_t)k] = rounds[(size_t)k].data();
        }
        if (op == 0) rdc::AllreduceCoalesced<rdc::op::Sum>(ptrs.data(), counts.data(), iter);
        else rdc::AllreduceCoalesced<rdc::op::Max>(ptrs.data(), counts.data(), iter);
        for (int k = 0; k < iter; ++k)
            for (int i = 0; i < N; ++i) {
                long want = 0;
                for (int j = 0; j < W; ++j) want = op == 0 ? want + (j + N + k + i) : std::max<long>(want, j + N + k + i);
                if (rounds[(size_t)k][(size_t)i] != want)
                    return fail(op == 0 ? "coalesced sum" : "coalesced max", i, rounds[(size_t)k][(size_t)i], want);
            }
    }
    // test/sendrecv.cc: rank 0 sends "hello world %u " to rank 1, 20 times
    for (int i = 0; i < 20 && W > 1; ++i) {
        char str[32];
        const int len = snprintf(str, sizeof(str), "hello world %u ", (unsigned)i);
        if (R == 0) {
            rdc::Send(str, (uint64_t)len, 1);
        } else if (R == 1) {
            char s[32] = {0};
            rdc::Recv(s, (uint64_t)len, 0);
            if (strncmp(s, str, (size_t)len) != 0) return fail("sendrecv", i, s[0], str[0]);
        }
    }
    // ring of non-blocking exchanges (ISend to next, IRecv from prev)
    if (W > 1) {
        std::vector<int> out((size_t)N), in((size_t)N, -1);
        for (int i = 0; i < N; ++i) out[(size_t)i] = R * 1000003 + i;
        rdc::comm::ICommunicator* c = rdc::GetCommunicator();
        rdc::WorkCompletion* ws = c->ISend(out.data(), (uint64_t)N * sizeof(int), (R + 1) % W);
        rdc::WorkCompletion* wr = c->IRecv(in.data(), (uint64_t)N * sizeof(int), (R - 1 + W) % W);
        if (!ws->Wait() || !wr->Wait()) return fail("isend/irecv", 0, 0, 0);
        delete ws;
        delete wr;
        const int prev = (R - 1 + W) % W;
        for (int i = 0; i < N; ++i)
            if (in[(size_t)i] != prev * 1000003 + i) return fail("isend/irecv ring", i, in[(size_t)i], prev * 1000003 + i);
    }
    printf("rank %d: known-answer OK (world %d, N %d)\n", R, W, N);
    rdc::Finalize();
    return 0;
}
