// Probe: can a peer's hipMalloc allocation be imported at an address the
// importer chooses?  The direct schedule's refusals come from
// HIP IPC placing a new peer mapping partly over address ranges the process
// unmapped; the fault that rule avoids needs that placement.  If the importer
// maps peers' memory inside its own reserved arena, at addresses no mapping
// used before (or exactly where one of the same size was), the placement never
// happens and no call has to fall back.
//
//   exporter: hipMalloc X1, X2 (16 MiB), fill, hsa_amd_portable_export_dmabuf
//             -> the fds over a unix socket (SCM_RIGHTS; pidfd_getfd is not
//             permitted on the box), offsets in shared memory ............ stage 1
//   importer: receive the fds, hsa_amd_vmem_import_shareable_handle,
//             hsa_amd_vmem_map into a reserved arena at +0 and +16 MiB,
//             set_access, read-check in a kernel, unmap, release ...... stage 1
//   exporter: hipFree X1, X2, hipMalloc Y (64 MiB), fill, export ........ stage 2
//   importer: import Y at arena +64 MiB (fresh), read-check, rewrite;
//             then unmap and map Y again exactly there, read-check ...... stage 2
//   exporter: read-check the importer's rewrite; free memory returned? . stage 3
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/vmem_import_probe tools/vmem_import_probe.hip -lhsa-runtime64 -lrt
//   tools/vmem_import_probe exporter NAME & tools/vmem_import_probe importer NAME
// Every step's status is printed; the importer launches a kernel on a mapping
// only after import, map and set_access all succeeded.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <sys/un.h>
#include <unistd.h>

#include <chrono>
#include <string>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

constexpr size_t kMiB = 1 << 20;

struct Ctl {
    int stage_e, stage_i;
    int pid;
    int fd[3];
    uint64_t off[3];
    size_t size[3];
    uint32_t pat[3];
    long long free_mib[3];
};

__global__ void k_fill(uint32_t* p, size_t n, uint32_t pat) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = pat ^ (uint32_t)i;
}

__global__ void k_check(const uint32_t* p, size_t n, uint32_t pat, unsigned long long* bad) {
    unsigned long long b = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += p[i] != (pat ^ (uint32_t)i);
    if (b) atomicAdd(bad, b);
}

static Ctl* map_ctl(const std::string& name, bool create) {
    const std::string path = "/rdc_vmem_" + name;
    int fd = shm_open(path.c_str(), O_RDWR | (create ? O_CREAT : 0), 0600);
    for (int i = 0; fd < 0 && i < 200; ++i) {
        usleep(50000);
        fd = shm_open(path.c_str(), O_RDWR, 0600);
    }
    if (fd < 0) {
        perror("shm_open");
        exit(1);
    }
    if (create && ftruncate(fd, sizeof(Ctl)) != 0) exit(1);
    void* p = mmap(nullptr, sizeof(Ctl), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    return static_cast<Ctl*>(p);
}

static void wait_for(volatile int* v, int want, const char* what) {
    for (int i = 0; i < 1200 && __atomic_load_n(v, __ATOMIC_ACQUIRE) < want; ++i) usleep(50000);
    if (__atomic_load_n(v, __ATOMIC_ACQUIRE) < want) {
        fprintf(stderr, "timed out waiting for %s\n", what);
        exit(2);
    }
}

static long long free_mib() {
    size_t f = 0, t = 0;
    CK(hipMemGetInfo(&f, &t));
    return (long long)(f / kMiB);
}

static unsigned long long check(const void* p, size_t bytes, uint32_t pat, unsigned long long* dbad) {
    CK(hipMemset(dbad, 0, sizeof(*dbad)));
    k_check<<<1024, 256>>>(static_cast<const uint32_t*>(p), bytes / 4, pat, dbad);
    CK(hipDeviceSynchronize());
    unsigned long long b = 0;
    CK(hipMemcpy(&b, dbad, sizeof(b), hipMemcpyDeviceToHost));
    return b;
}

// SCM_RIGHTS over an abstract unix socket: the exporter listens, the importer connects
static void sock_addr(const std::string& name, sockaddr_un* a, socklen_t* len) {
    memset(a, 0, sizeof(*a));
    a->sun_family = AF_UNIX;
    const std::string n = "rdc_vmem_" + name;
    memcpy(a->sun_path + 1, n.data(), n.size());
    *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n.size());
}

static bool send_fd(int sock, int fd) {
    char byte = 'f';
    iovec iov{&byte, 1};
    char ctl[CMSG_SPACE(sizeof(int))];
    memset(ctl, 0, sizeof(ctl));
    msghdr m{};
    m.msg_iov = &iov;
    m.msg_iovlen = 1;
    m.msg_control = ctl;
    m.msg_controllen = sizeof(ctl);
    cmsghdr* c = CMSG_FIRSTHDR(&m);
    c->cmsg_level = SOL_SOCKET;
    c->cmsg_type = SCM_RIGHTS;
    c->cmsg_len = CMSG_LEN(sizeof(int));
    memcpy(CMSG_DATA(c), &fd, sizeof(int));
    return sendmsg(sock, &m, 0) == 1;
}

static int recv_fd(int sock) {
    char byte;
    iovec iov{&byte, 1};
    char ctl[CMSG_SPACE(sizeof(int))];
    msghdr m{};
    m.msg_iov = &iov;
    m.msg_iovlen = 1;
    m.msg_control = ctl;
    m.msg_controllen = sizeof(ctl);
    if (recvmsg(sock, &m, 0) != 1) return -1;
    cmsghdr* c = CMSG_FIRSTHDR(&m);
    if (!c || c->cmsg_type != SCM_RIGHTS) return -1;
    int fd;
    memcpy(&fd, CMSG_DATA(c), sizeof(int));
    return fd;
}

static hsa_agent_t g_agent;
static hsa_status_t find_gpu(hsa_agent_t a, void*) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU) {
        g_agent = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

// one import: the received fd, import, map at va, set_access; *h and the local fd
// returned for the unmap; false (and a printed reason) on any failure
struct Import {
    void* va = nullptr;
    size_t size = 0;
    hsa_amd_vmem_alloc_handle_t h{};
    int fd = -1;
    double us = 0;
};

static bool import_at(int fd, void* va, Import* im, std::string* why) {
    const auto t0 = std::chrono::steady_clock::now();
    im->fd = dup(fd);
    if (im->fd < 0) {
        *why = "no fd received";
        return false;
    }
    const off_t sz = lseek(im->fd, 0, SEEK_END);
    if (sz <= 0) {
        *why = "lseek on the dma-buf";
        return false;
    }
    im->size = (size_t)sz;
    hsa_status_t s = hsa_amd_vmem_import_shareable_handle(im->fd, &im->h);
    if (s != HSA_STATUS_SUCCESS) {
        *why = "vmem_import_shareable_handle " + std::to_string((int)s);
        return false;
    }
    s = hsa_amd_vmem_map(va, im->size, 0, im->h, 0);
    if (s != HSA_STATUS_SUCCESS) {
        *why = "vmem_map " + std::to_string((int)s);
        hsa_amd_vmem_handle_release(im->h);
        return false;
    }
    hsa_amd_memory_access_desc_t d;
    d.permissions = HSA_ACCESS_PERMISSION_RW;
    d.agent_handle = g_agent;
    s = hsa_amd_vmem_set_access(va, im->size, &d, 1);
    if (s != HSA_STATUS_SUCCESS) {
        *why = "vmem_set_access " + std::to_string((int)s);
        hsa_amd_vmem_unmap(va, im->size);
        hsa_amd_vmem_handle_release(im->h);
        return false;
    }
    im->va = va;
    im->us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    return true;
}

static double unmap(Import* im) {
    const auto t0 = std::chrono::steady_clock::now();
    hsa_amd_vmem_unmap(im->va, im->size);
    hsa_amd_vmem_handle_release(im->h);
    close(im->fd);
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

static int exporter(const std::string& name) {
    Ctl* c = map_ctl(name, true);
    memset(c, 0, sizeof(*c));
    c->pid = getpid();
    const int ls = socket(AF_UNIX, SOCK_STREAM, 0);
    sockaddr_un sa;
    socklen_t sl;
    sock_addr(name, &sa, &sl);
    if (ls < 0 || bind(ls, (sockaddr*)&sa, sl) != 0 || listen(ls, 1) != 0) {
        perror("listen");
        return 1;
    }
    CK(hipSetDevice(0));
    void* x[2];
    for (int i = 0; i < 2; ++i) {
        c->size[i] = 16 * kMiB;
        c->pat[i] = 0x1000u * (i + 1);
        CK(hipMalloc(&x[i], c->size[i]));
        k_fill<<<1024, 256>>>(static_cast<uint32_t*>(x[i]), c->size[i] / 4, c->pat[i]);
    }
    CK(hipDeviceSynchronize());
    for (int i = 0; i < 2; ++i) {
        hsa_status_t s = hsa_amd_portable_export_dmabuf(x[i], c->size[i], &c->fd[i], &c->off[i]);
        if (s != HSA_STATUS_SUCCESS) {
            printf("{\"role\": \"exporter\", \"error\": \"portable_export_dmabuf %d\"}\n", (int)s);
            c->stage_e = -1;
            return 1;
        }
    }
    const int sock = accept(ls, nullptr, nullptr);
    if (sock < 0 || !send_fd(sock, c->fd[0]) || !send_fd(sock, c->fd[1])) {
        perror("send_fd");
        return 1;
    }
    __atomic_store_n(&c->stage_e, 1, __ATOMIC_RELEASE);
    wait_for(&c->stage_i, 1, "importer stage 1");
    for (int i = 0; i < 2; ++i) {
        hsa_amd_portable_close_dmabuf(c->fd[i]);
        CK(hipFree(x[i]));
    }
    void* y;
    c->size[2] = 64 * kMiB;
    c->pat[2] = 0x3000u;
    CK(hipMalloc(&y, c->size[2]));
    k_fill<<<1024, 256>>>(static_cast<uint32_t*>(y), c->size[2] / 4, c->pat[2]);
    CK(hipDeviceSynchronize());
    if (hsa_amd_portable_export_dmabuf(y, c->size[2], &c->fd[2], &c->off[2]) != HSA_STATUS_SUCCESS ||
        !send_fd(sock, c->fd[2])) {
        c->stage_e = -1;
        return 1;
    }
    __atomic_store_n(&c->stage_e, 2, __ATOMIC_RELEASE);
    wait_for(&c->stage_i, 2, "importer stage 2");
    unsigned long long* dbad;
    CK(hipMalloc(&dbad, sizeof(*dbad)));
    const unsigned long long bad = check(y, c->size[2], ~c->pat[2], dbad);  // the importer's rewrite
    c->free_mib[0] = free_mib();
    hsa_amd_portable_close_dmabuf(c->fd[2]);
    CK(hipFree(y));
    c->free_mib[1] = free_mib();
    __atomic_store_n(&c->stage_e, 3, __ATOMIC_RELEASE);
    wait_for(&c->stage_i, 3, "importer stage 3");
    c->free_mib[2] = free_mib();
    printf("{\"role\": \"exporter\", \"offsets\": [%llu, %llu, %llu], \"rewrite_bad\": %llu, "
           "\"free_mib_before_free\": %lld, \"after_free\": %lld, \"after_importer_unmap\": %lld}\n",
           (unsigned long long)c->off[0], (unsigned long long)c->off[1], (unsigned long long)c->off[2], bad,
           c->free_mib[0], c->free_mib[1], c->free_mib[2]);
    return bad == 0 ? 0 : 1;
}

static int importer(const std::string& name) {
    Ctl* c = map_ctl(name, false);
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    if (hsa_init() != HSA_STATUS_SUCCESS) return 1;
    hsa_iterate_agents(find_gpu, nullptr);
    unsigned long long* dbad;
    CK(hipMalloc(&dbad, sizeof(*dbad)));
    void* own;  // the rank's own buffer, freed before stage 2 (the round-5 pattern)
    CK(hipMalloc(&own, 16 * kMiB));
    const int sock = socket(AF_UNIX, SOCK_STREAM, 0);
    sockaddr_un sa;
    socklen_t sl;
    sock_addr(name, &sa, &sl);
    int cr = -1;
    for (int i = 0; i < 200 && cr != 0; ++i) {
        cr = connect(sock, (sockaddr*)&sa, sl);
        if (cr != 0) usleep(50000);
    }
    if (cr != 0) {
        printf("{\"role\": \"importer\", \"error\": \"connect: %s\"}\n", strerror(errno));
        return 1;
    }
    wait_for(&c->stage_e, 1, "exporter stage 1");
    int rfd[3] = {recv_fd(sock), recv_fd(sock), -1};
    void* arena = nullptr;
    const size_t arena_bytes = 1024 * kMiB;
    hsa_status_t s = hsa_amd_vmem_address_reserve_align(&arena, arena_bytes, 0, 2 * kMiB, 0);
    if (s != HSA_STATUS_SUCCESS) {
        printf("{\"role\": \"importer\", \"error\": \"address_reserve %d\"}\n", (int)s);
        return 1;
    }
    std::string why;
    Import im[2];
    unsigned long long bad1[2] = {~0ull, ~0ull};
    double us_map[2] = {0, 0}, us_unmap[2] = {0, 0};
    for (int i = 0; i < 2; ++i) {
        if (!import_at(rfd[i], (char*)arena + i * 16 * kMiB, &im[i], &why)) {
            printf("{\"role\": \"importer\", \"stage\": 1, \"buffer\": %d, \"error\": \"%s\"}\n", i, why.c_str());
            __atomic_store_n(&c->stage_i, 3, __ATOMIC_RELEASE);
            return 1;
        }
        us_map[i] = im[i].us;
        bad1[i] = check((char*)im[i].va + c->off[i], c->size[i], c->pat[i], dbad);
    }
    for (int i = 0; i < 2; ++i) us_unmap[i] = unmap(&im[i]);
    CK(hipFree(own));
    __atomic_store_n(&c->stage_i, 1, __ATOMIC_RELEASE);
    wait_for(&c->stage_e, 2, "exporter stage 2");
    rfd[2] = recv_fd(sock);
    Import y;
    if (!import_at(rfd[2], (char*)arena + 64 * kMiB, &y, &why)) {
        printf("{\"role\": \"importer\", \"stage\": 2, \"error\": \"%s\"}\n", why.c_str());
        __atomic_store_n(&c->stage_i, 3, __ATOMIC_RELEASE);
        return 1;
    }
    const unsigned long long bad2 = check((char*)y.va + c->off[2], c->size[2], c->pat[2], dbad);
    // the same allocation mapped again exactly where it was
    const double us_unmap_y = unmap(&y);
    Import y2;
    unsigned long long bad3 = ~0ull;
    if (import_at(rfd[2], (char*)arena + 64 * kMiB, &y2, &why)) {
        bad3 = check((char*)y2.va + c->off[2], c->size[2], c->pat[2], dbad);
        k_fill<<<1024, 256>>>(reinterpret_cast<uint32_t*>((char*)y2.va + c->off[2]), c->size[2] / 4, ~c->pat[2]);
        CK(hipDeviceSynchronize());
    }
    __atomic_store_n(&c->stage_i, 2, __ATOMIC_RELEASE);
    wait_for(&c->stage_e, 3, "exporter stage 3");
    if (y2.va) unmap(&y2);
    hsa_amd_vmem_address_free(arena, arena_bytes);
    for (int fd : rfd) if (fd >= 0) close(fd);
    close(sock);
    printf("{\"role\": \"importer\", \"arena\": \"%p\", \"dmabuf_sizes\": [%zu, %zu, %zu], \"bad_x\": [%llu, %llu], "
           "\"bad_y\": %llu, \"bad_y_remapped\": %llu, \"map_us\": [%.1f, %.1f, %.1f, %.1f], "
           "\"unmap_us\": [%.1f, %.1f, %.1f], \"remap_error\": \"%s\"}\n",
           arena, im[0].size, im[1].size, y.size, bad1[0], bad1[1], bad2, bad3, us_map[0], us_map[1], y.us, y2.us,
           us_unmap[0], us_unmap[1], us_unmap_y, y2.va ? "" : why.c_str());
    __atomic_store_n(&c->stage_i, 3, __ATOMIC_RELEASE);
    return bad1[0] == 0 && bad1[1] == 0 && bad2 == 0 && bad3 == 0 ? 0 : 1;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s exporter|importer NAME\n", argv[0]);
        return 2;
    }
    const std::string role = argv[1], name = argv[2];
    return role == "exporter" ? exporter(name) : importer(name);
}
