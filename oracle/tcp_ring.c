/* ORACLE / CPU BASELINE — TEST INFRASTRUCTURE ONLY.
 *
 * A port of the reference's own CPU allreduce over loopback TCP, the
 * comparison point BASELINE.json's north star names ("the reference's own CPU
 * allreduce over loopback TCP timed on the same box's host cores").  The
 * reference itself does not build as shipped (SURVEY.md §0 finding 1) and
 * needs edits to its sources to run (liveness fix, virtual collectives), so
 * this restates its data path in plain C, step for step:
 *
 *   TryAllreduceRing (src/comm/communicator_collective.cc:183-203):
 *     malloc(S) scratch per call (:185-187), reduce-scatter, free, allgather.
 *   TryReduceScatterRing (:115-182): n-1 steps; each step ISend chunk
 *     write_idx%n to ring prev, IRecv chunk read_idx%n from ring next into
 *     scratch, wait for both (chain_wc->Wait()), then
 *     reducer(src = scratch chunk, dst = own chunk) (:174-176).
 *   TryAllgatherRing (:79-114): n-1 steps, send to prev / receive from next,
 *     in place.
 *   Chunk map utils::Split (include/utils/utils.h:59-70); per-step chunk
 *     indices from rdc_oracle_ring_schedule (the reference's write_idx /
 *     read_idx / stop arithmetic); op::Reducer = rdc_oracle_reducer.
 *   Transport: one TCP connection per ring link (rank r -> r-1), raw bytes,
 *     no framing (src/transport/tcp/tcp_channel.cc:99-208).  The reference
 *     drives the sockets from an epoll thread plus a thread pool; here one
 *     poll() loop per rank moves the send and the receive of a step
 *     concurrently (what the pool achieves), without the reference's
 *     liveness bug (SURVEY finding 4).
 *
 * Usage: tcp_ring -n N -c COUNT [-t DTYPE] [-o OP] [-i ITERS] [-w WARMUP]
 *                 [-p PORT] [-d OUTDIR]
 * Forks N rank processes on 127.0.0.1.  Inputs: rdc_oracle_fill(seed
 * 0x5EED0000, rank).  Rank 0 prints one JSON line with per-call times;
 * with -d every rank writes its result to OUTDIR/rank<r>.bin (parity tests).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>
#include <arpa/inet.h>

#include "rdc_oracle.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void die(const char* what) {
    perror(what);
    exit(2);
}

static void tune(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

/* Listeners are made by the parent before the ranks fork (kernel-chosen
 * ports unless -p is given), so every rank's listener exists before anyone
 * connects: no port collisions and no loopback self-connect (a connect to a
 * not-yet-listening port in the ephemeral range can open onto itself). */
static int make_listener(int port, int* bound) {
    int ls = socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) die("socket");
    int one = 1;
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    struct sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = htons((uint16_t)port);
    if (bind(ls, (struct sockaddr*)&a, sizeof(a)) < 0) die("bind");
    if (listen(ls, 4) < 0) die("listen");
    socklen_t al = sizeof(a);
    if (getsockname(ls, (struct sockaddr*)&a, &al) < 0) die("getsockname");
    *bound = ntohs(a.sin_port);
    return ls;
}

/* rank r connects to prev's listener (the r -> prev link) and accepts
 * next's connection on its own (the next -> r link) */
static void connect_ring(int rank, int n, int ls, const int* ports, int* to_prev, int* from_next) {
    const int prev = (rank - 1 + n) % n;
    struct sockaddr_in b;
    memset(&b, 0, sizeof(b));
    b.sin_family = AF_INET;
    b.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    b.sin_port = htons((uint16_t)ports[prev]);
    int s = socket(AF_INET, SOCK_STREAM, 0);
    if (s < 0) die("socket");
    if (connect(s, (struct sockaddr*)&b, sizeof(b)) != 0) die("connect");
    struct pollfd p = {ls, POLLIN, 0};
    if (poll(&p, 1, 60000) <= 0) die("accept wait");
    int c = accept(ls, NULL, NULL);
    if (c < 0) die("accept");
    close(ls);
    tune(s);
    tune(c);
    *to_prev = s;
    *from_next = c;
}

/* one ring step: send sbuf[0,slen) to prev while receiving rlen bytes from
 * next into rbuf (the ISend + IRecv + chain wait of one step) */
static void exchange(int to_prev, int from_next, const char* sbuf, size_t slen, char* rbuf, size_t rlen) {
    size_t sent = 0, got = 0;
    while (sent < slen || got < rlen) {
        struct pollfd p[2];
        int np = 0, is = -1, ir = -1;
        if (sent < slen) { p[np].fd = to_prev; p[np].events = POLLOUT; is = np++; }
        if (got < rlen) { p[np].fd = from_next; p[np].events = POLLIN; ir = np++; }
        if (poll(p, (nfds_t)np, 60000) <= 0) die("poll");
        if (is >= 0 && (p[is].revents & (POLLOUT | POLLERR | POLLHUP))) {
            ssize_t k = send(to_prev, sbuf + sent, slen - sent, MSG_DONTWAIT | MSG_NOSIGNAL);
            if (k > 0) sent += (size_t)k;
            else if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) die("send");
        }
        if (ir >= 0 && (p[ir].revents & (POLLIN | POLLERR | POLLHUP))) {
            ssize_t k = recv(from_next, rbuf + got, rlen - got, MSG_DONTWAIT);
            if (k > 0) got += (size_t)k;
            else if (k == 0) { fprintf(stderr, "peer closed\n"); exit(2); }
            else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) die("recv");
        }
    }
}

/* token twice around the ring: every rank has entered before anyone leaves */
static void ring_barrier(int rank, int n, int to_prev, int from_next) {
    char t = 1, r;
    for (int round = 0; round < 2; ++round) {
        if (rank == 0) {
            exchange(to_prev, from_next, &t, 1, &r, 0);
            exchange(to_prev, from_next, &t, 0, &r, 1);
        } else {
            exchange(to_prev, from_next, &t, 0, &r, 1);
            exchange(to_prev, from_next, &t, 1, &r, 0);
        }
    }
    (void)n;
}

typedef struct {
    int n, rank, dtype, op;
    uint64_t count;
    size_t esz;
    int64_t cb[RDC_ORACLE_MAX_RANKS], ce[RDC_ORACLE_MAX_RANKS];
    int rs_send[RDC_ORACLE_MAX_RANKS], rs_recv[RDC_ORACLE_MAX_RANKS];
    int ag_send[RDC_ORACLE_MAX_RANKS], ag_recv[RDC_ORACLE_MAX_RANKS];
    int to_prev, from_next;
} Ring;

static size_t coff(const Ring* R, int c) { return (size_t)R->cb[c] * R->esz; }
static size_t clen(const Ring* R, int c) { return c < 0 ? 0 : (size_t)(R->ce[c] - R->cb[c]) * R->esz; }

/* TryAllreduceRing (communicator_collective.cc:183-203) */
static void allreduce(const Ring* R, char* buf) {
    const size_t S = R->count * R->esz;
    char* scratch = (char*)malloc(S ? S : 1); /* :185-187, per call */
    if (!scratch) die("malloc");
    for (int j = 0; j < R->n - 1; ++j) {      /* TryReduceScatterRing */
        const int cs = R->rs_send[j], cr = R->rs_recv[j];
        exchange(R->to_prev, R->from_next, cs >= 0 ? buf + coff(R, cs) : NULL, clen(R, cs),
                 cr >= 0 ? scratch + coff(R, cr) : NULL, clen(R, cr));
        if (cr >= 0 && rdc_oracle_reducer(scratch + coff(R, cr), buf + coff(R, cr), (uint64_t)(R->ce[cr] - R->cb[cr]),
                                          R->dtype, R->op))
            die("reducer");
    }
    free(scratch);                             /* :189 */
    for (int j = 0; j < R->n - 1; ++j) {       /* TryAllgatherRing, in place */
        const int cs = R->ag_send[j], cr = R->ag_recv[j];
        exchange(R->to_prev, R->from_next, cs >= 0 ? buf + coff(R, cs) : NULL, clen(R, cs),
                 cr >= 0 ? buf + coff(R, cr) : NULL, clen(R, cr));
    }
}

static int cmp_d(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

static int run_rank(int rank, int n, uint64_t count, int dtype, int op, int iters, int warmup, int ls,
                    const int* ports, const char* outdir, int result_fd) {
    Ring R;
    memset(&R, 0, sizeof(R));
    R.n = n;
    R.rank = rank;
    R.count = count;
    R.dtype = dtype;
    R.op = op;
    R.esz = rdc_oracle_dtype_size(dtype);
    rdc_oracle_split(0, (int64_t)count, n, R.cb, R.ce);
    if (rdc_oracle_ring_schedule(n, rank, R.rs_send, R.rs_recv, R.ag_send, R.ag_recv)) die("schedule");
    connect_ring(rank, n, ls, ports, &R.to_prev, &R.from_next);
    const size_t S = count * R.esz;
    char* input = (char*)malloc(S ? S : 1);
    char* buf = (char*)malloc(S ? S : 1);
    if (!input || !buf) die("malloc");
    rdc_oracle_fill(input, count, dtype, 0x5EED0000ull, rank);
    double* t = (double*)calloc((size_t)(iters > 0 ? iters : 1), sizeof(double));
    for (int it = -warmup; it < iters; ++it) {
        memcpy(buf, input, S);                 /* fresh input every call */
        ring_barrier(rank, n, R.to_prev, R.from_next);
        const double t0 = now_s();
        allreduce(&R, buf);
        const double dt = now_s() - t0;
        if (it >= 0) t[it] = dt;
    }
    if (outdir) {
        char path[4096];
        snprintf(path, sizeof(path), "%s/rank%d.bin", outdir, rank);
        FILE* f = fopen(path, "wb");
        if (!f || fwrite(buf, 1, S, f) != S) die("write result");
        fclose(f);
    }
    if (rank == 0 && iters > 0) {
        /* rank 0's per-call times (the survey's convention, rank 0) */
        if (write(result_fd, t, sizeof(double) * (size_t)iters) < 0) die("pipe");
    }
    close(R.to_prev);
    close(R.from_next);
    free(t);
    free(buf);
    free(input);
    return 0;
}

int main(int argc, char** argv) {
    int n = 2, dtype = RDC_DT_FLOAT32, op = RDC_OP_SUM, iters = 5, warmup = 1, port = 0;
    uint64_t count = 1024;
    const char* outdir = NULL;
    int ch;
    while ((ch = getopt(argc, argv, "n:c:t:o:i:w:p:d:")) != -1) {
        switch (ch) {
            case 'n': n = atoi(optarg); break;
            case 'c': count = strtoull(optarg, NULL, 0); break;
            case 't': dtype = atoi(optarg); break;
            case 'o': op = atoi(optarg); break;
            case 'i': iters = atoi(optarg); break;
            case 'w': warmup = atoi(optarg); break;
            case 'p': port = atoi(optarg); break;
            case 'd': outdir = optarg; break;
            default: fprintf(stderr, "usage: tcp_ring -n N -c COUNT [-t dtype] [-o op] [-i iters] [-w warmup]\n"); return 2;
        }
    }
    if (n < 2 || n > RDC_ORACLE_MAX_RANKS || rdc_oracle_dtype_size(dtype) == 0 || iters < 0) {
        fprintf(stderr, "tcp_ring: bad arguments\n");
        return 2;
    }
    int ls[RDC_ORACLE_MAX_RANKS], ports[RDC_ORACLE_MAX_RANKS];
    for (int r = 0; r < n; ++r) ls[r] = make_listener(port ? port + r : 0, &ports[r]);
    int pfd[2];
    if (pipe(pfd) < 0) die("pipe");
    pid_t kids[RDC_ORACLE_MAX_RANKS];
    for (int r = 0; r < n; ++r) {
        kids[r] = fork();
        if (kids[r] < 0) die("fork");
        if (kids[r] == 0) {
            close(pfd[0]);
            for (int q = 0; q < n; ++q)
                if (q != r) close(ls[q]);
            _exit(run_rank(r, n, count, dtype, op, iters, warmup, ls[r], ports, outdir, pfd[1]));
        }
    }
    close(pfd[1]);
    for (int r = 0; r < n; ++r) close(ls[r]);
    double* t = (double*)calloc((size_t)(iters > 0 ? iters : 1), sizeof(double));
    size_t want = sizeof(double) * (size_t)iters, have = 0;
    while (have < want) {
        ssize_t k = read(pfd[0], (char*)t + have, want - have);
        if (k <= 0) break;
        have += (size_t)k;
    }
    int bad = 0;
    for (int r = 0; r < n; ++r) {
        int st = 0;
        waitpid(kids[r], &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad = 1;
    }
    if (bad || have < want) {
        fprintf(stderr, "tcp_ring: a rank failed\n");
        return 1;
    }
    if (iters > 0) {
        double sum = 0;
        for (int i = 0; i < iters; ++i) sum += t[i];
        double* s = (double*)malloc(sizeof(double) * (size_t)iters);
        memcpy(s, t, sizeof(double) * (size_t)iters);
        qsort(s, (size_t)iters, sizeof(double), cmp_d);
        const double med = s[iters / 2], S = (double)count * (double)rdc_oracle_dtype_size(dtype);
        const long cores = sysconf(_SC_NPROCESSORS_ONLN);
        printf("{\"cpu_tcp_ring\": true, \"n\": %d, \"bytes\": %.0f, \"dtype\": %d, \"iters\": %d, "
               "\"median_ms\": %.4f, \"mean_ms\": %.4f, \"best_ms\": %.4f, \"algbw_GBps\": %.4f, "
               "\"busbw_GBps\": %.4f, \"host_cpus\": %ld, \"threads_per_rank\": 1}\n",
               n, S, dtype, iters, med * 1e3, sum / iters * 1e3, s[0] * 1e3, S / med / 1e9,
               S / med / 1e9 * 2.0 * (n - 1) / n, cores);
        free(s);
    }
    free(t);
    return 0;
}
