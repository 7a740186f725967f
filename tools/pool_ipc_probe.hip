// Registration probe: hipMemPool shareable handles vs hipIpc memory handles.
//
// Two processes (fork before any HIP call). The exporter allocates N buffers
// both ways, the importer maps them and writes a pattern the exporter checks.
// Reports per-step wall time, so the runtime's registration choice (ocmd
// exports 4 GiB slabs with hipIpcGetMemHandle) rests on a measurement.
//
//   hipcc --offload-arch=gfx950 -O2 tools/pool_ipc_probe.hip -o build/bin/pool_ipc_probe
//   build/bin/pool_ipc_probe [count] [bytes]
#include <hip/hip_runtime.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(3);                                                                       \
        }                                                                                       \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void send_fd(int sock, int fd) {
    char c = 0;
    iovec iov{&c, 1};
    char ctl[CMSG_SPACE(sizeof(int))] = {};
    msghdr m{};
    m.msg_iov = &iov;
    m.msg_iovlen = 1;
    m.msg_control = ctl;
    m.msg_controllen = sizeof(ctl);
    cmsghdr *h = CMSG_FIRSTHDR(&m);
    h->cmsg_level = SOL_SOCKET;
    h->cmsg_type = SCM_RIGHTS;
    h->cmsg_len = CMSG_LEN(sizeof(int));
    std::memcpy(CMSG_DATA(h), &fd, sizeof(int));
    if (sendmsg(sock, &m, 0) != 1) std::exit(4);
}

static int recv_fd(int sock) {
    char c;
    iovec iov{&c, 1};
    char ctl[CMSG_SPACE(sizeof(int))] = {};
    msghdr m{};
    m.msg_iov = &iov;
    m.msg_iovlen = 1;
    m.msg_control = ctl;
    m.msg_controllen = sizeof(ctl);
    if (recvmsg(sock, &m, 0) != 1) std::exit(5);
    int fd = -1;
    std::memcpy(&fd, CMSG_DATA(CMSG_FIRSTHDR(&m)), sizeof(int));
    return fd;
}

static void xsend(int s, const void *p, size_t n) {
    if (send(s, p, n, 0) != (ssize_t)n) std::exit(6);
}
static void xrecv(int s, void *p, size_t n) {
    size_t got = 0;
    while (got < n) {
        ssize_t r = recv(s, (char *)p + got, n - got, 0);
        if (r <= 0) std::exit(7);
        got += r;
    }
}

__global__ void fill(uint32_t *p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)i * 2654435761u ^ seed;
}

__global__ void check(const uint32_t *p, size_t n, uint32_t seed, unsigned long long *bad) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (p[i] != ((uint32_t)i * 2654435761u ^ seed)) atomicAdd(bad, 1ull);
}

int main(int argc, char **argv) {
    const int count = argc > 1 ? std::atoi(argv[1]) : 16;
    const size_t bytes = argc > 2 ? std::strtoull(argv[2], nullptr, 0) : (64ull << 20);
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 2;
    pid_t pid = fork();
    if (pid == 0) {
        // ---------------- importer ----------------
        close(sv[0]);
        int s = sv[1];
        CK(hipSetDevice(0));
        CK(hipFree(nullptr));
        int pfd = recv_fd(s);
        double t0 = now_us();
        hipMemPool_t pool;
        CK(hipMemPoolImportFromShareableHandle(&pool, (void *)(intptr_t)pfd, hipMemHandleTypePosixFileDescriptor, 0));
        double t_pool = now_us() - t0;
        std::vector<hipMemPoolPtrExportData> pexp(count);
        std::vector<hipIpcMemHandle_t> ih(count);
        xrecv(s, pexp.data(), sizeof(hipMemPoolPtrExportData) * count);
        xrecv(s, ih.data(), sizeof(hipIpcMemHandle_t) * count);
        std::vector<void *> pp(count), ip(count);
        t0 = now_us();
        for (int i = 0; i < count; i++) CK(hipMemPoolImportPointer(&pp[i], pool, &pexp[i]));
        double t_pimp = (now_us() - t0) / count;
        t0 = now_us();
        for (int i = 0; i < count; i++) CK(hipIpcOpenMemHandle(&ip[i], ih[i], hipIpcMemLazyEnablePeerAccess));
        double t_iimp = (now_us() - t0) / count;
        const size_t n = bytes / 4;
        for (int i = 0; i < count; i++) {
            hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, (uint32_t *)pp[i], n, 100u + i);
            hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, (uint32_t *)ip[i], n, 200u + i);
        }
        CK(hipDeviceSynchronize());
        t0 = now_us();
        for (int i = 0; i < count; i++) CK(hipFree(pp[i]));  // pool-imported pointers are released with hipFree
        double t_pfree = (now_us() - t0) / count;
        t0 = now_us();
        for (int i = 0; i < count; i++) CK(hipIpcCloseMemHandle(ip[i]));
        double t_iclose = (now_us() - t0) / count;
        double r[5] = {t_pool, t_pimp, t_iimp, t_pfree, t_iclose};
        xsend(s, r, sizeof(r));
        CK(hipMemPoolDestroy(pool));
        return 0;
    }
    // ---------------- exporter ----------------
    close(sv[1]);
    int s = sv[0];
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipMemPoolProps props;
    std::memset(&props, 0, sizeof(props));
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypePosixFileDescriptor;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = 0;
    double t0 = now_us();
    hipMemPool_t pool;
    CK(hipMemPoolCreate(&pool, &props));
    uint64_t keep = ~0ull;
    CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep));
    int pfd = -1;
    CK(hipMemPoolExportToShareableHandle(&pfd, pool, hipMemHandleTypePosixFileDescriptor, 0));
    double t_pexp_pool = now_us() - t0;
    std::vector<void *> pp(count), ip(count);
    std::vector<hipMemPoolPtrExportData> pexp(count);
    std::vector<hipIpcMemHandle_t> ih(count);
    t0 = now_us();
    for (int i = 0; i < count; i++) CK(hipMallocFromPoolAsync(&pp[i], bytes, pool, st));
    CK(hipStreamSynchronize(st));
    double t_palloc = (now_us() - t0) / count;
    t0 = now_us();
    for (int i = 0; i < count; i++) CK(hipMemPoolExportPointer(&pexp[i], pp[i]));
    double t_pexp = (now_us() - t0) / count;
    t0 = now_us();
    for (int i = 0; i < count; i++) CK(hipMalloc(&ip[i], bytes));
    double t_ialloc = (now_us() - t0) / count;
    t0 = now_us();
    for (int i = 0; i < count; i++) CK(hipIpcGetMemHandle(&ih[i], ip[i]));
    double t_iexp = (now_us() - t0) / count;
    send_fd(s, pfd);
    xsend(s, pexp.data(), sizeof(hipMemPoolPtrExportData) * count);
    xsend(s, ih.data(), sizeof(hipIpcMemHandle_t) * count);
    double r[5];
    xrecv(s, r, sizeof(r));
    int status = 0;
    waitpid(pid, &status, 0);
    unsigned long long *bad;
    CK(hipHostMalloc((void **)&bad, sizeof(*bad), hipHostMallocCoherent));
    *bad = 0;
    const size_t n = bytes / 4;
    for (int i = 0; i < count; i++) {
        hipLaunchKernelGGL(check, dim3(1024), dim3(256), 0, 0, (const uint32_t *)pp[i], n, 100u + i, bad);
        hipLaunchKernelGGL(check, dim3(1024), dim3(256), 0, 0, (const uint32_t *)ip[i], n, 200u + i, bad);
    }
    CK(hipDeviceSynchronize());
    std::printf("{\"count\": %d, \"bytes\": %zu, \"child_status\": %d, \"bad_words\": %llu,\n", count, bytes, status,
                *bad);
    std::printf(" \"pool\": {\"create_export_fd_us\": %.1f, \"alloc_us\": %.2f, \"export_ptr_us\": %.2f, "
                "\"import_pool_us\": %.1f, \"import_ptr_us\": %.2f, \"importer_free_us\": %.2f},\n",
                t_pexp_pool, t_palloc, t_pexp, r[0], r[1], r[3]);
    std::printf(" \"ipc\": {\"alloc_us\": %.2f, \"get_handle_us\": %.2f, \"open_us\": %.2f, \"close_us\": %.2f}}\n",
                t_ialloc, t_iexp, r[2], r[4]);
    return (status == 0 && *bad == 0) ? 0 : 1;
}
