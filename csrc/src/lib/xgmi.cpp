// Raw xGMI backend (see ocm/xgmi.h). Exported from libocm.so.
// Reference parity: the ib_* API of inc/io/rdma.h:36-45 (src/rdma.c:46-302,
// src/rdma_server.c:40-236, src/rdma_client.c:39-252) and the extoll_* API of
// inc/io/extoll.h:50-59 (src/extoll*.c): new / connect / read / write /
// disconnect over IPC-mapped peer HBM instead of verbs QPs or RMA2 ports.
#include "ocm/xgmi.h"

#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "ocm/log.h"
#include "ocm/pmsg.h"
#include "ocm/xfer.h"

using namespace ocm;

namespace {

constexpr uint32_t kMagic = 0x4f434d58;  // "OCMX"

struct Reg {  // the registration both sides exchange (RDMA-CM private data analogue)
    uint32_t magic;
    uint32_t host;  // 1: host memfd slab, 0: HBM
    uint64_t len;
    int32_t gpu;
    int32_t pid;
    uint8_t handle[64];
};

enum : uint8_t { K_REG = 'R', K_CTRL = 'C', K_BYE = 'B' };

int dev_count() {
    int n = 0;
    if (std::getenv("OCM_NO_GPU") || hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

}  // namespace

struct xgmi_alloc {
    std::string endpoint;
    int gpu = -1;        // where the local buffer lives (-1 host)
    int device = -1;     // device used to run copies (-1: CPU memcpy)
    char *buf = nullptr;
    char *dbuf = nullptr;  // device-usable address of buf
    size_t len = 0;
    bool own = false;
    int memfd = -1;
    bool registered = false;
    Reg mine{};
    // remote
    char *rbuf = nullptr;   // device-usable (or host) address of the peer buffer
    char *rhost = nullptr;  // host mapping when the peer buffer is a host slab
    size_t rlen = 0;
    bool rhost_registered = false;
    bool rgpu = false;
    int listen_fd = -1, fd = -1;
    hipStream_t stream = nullptr;
    bool pending = false;
};

namespace {

int send_kind(int fd, uint8_t kind, const void *p, size_t n) {
    char buf[512];
    if (n + 1 > sizeof(buf)) return -1;
    buf[0] = (char)kind;
    if (n) std::memcpy(buf + 1, p, n);
    return send(fd, buf, n + 1, MSG_NOSIGNAL) == (ssize_t)(n + 1) ? 0 : -1;
}

// Receive one record; returns its payload length or -1.
int recv_kind(int fd, uint8_t *kind, void *p, size_t cap, int timeout_ms) {
    struct pollfd q = {fd, POLLIN, 0};
    int rc = poll(&q, 1, timeout_ms);
    if (rc <= 0) return -1;
    char buf[512];
    ssize_t n = recv(fd, buf, sizeof(buf), 0);
    if (n <= 0) return -1;
    *kind = (uint8_t)buf[0];
    size_t m = std::min((size_t)n - 1, cap);
    std::memcpy(p, buf + 1, m);
    return (int)m;
}

int export_local(xgmi_t x) {
    std::memset(&x->mine, 0, sizeof(x->mine));
    x->mine.magic = kMagic;
    x->mine.len = x->len;
    x->mine.gpu = x->gpu;
    x->mine.pid = (int32_t)getpid();
    if (x->gpu >= 0) {
        hipIpcMemHandle_t h;
        if (hipIpcGetMemHandle(&h, x->buf) != hipSuccess) OCM_FAIL(-1, "hipIpcGetMemHandle failed");
        std::memcpy(x->mine.handle, &h, sizeof(h));
        x->mine.host = 0;
    } else {
        if (x->memfd < 0) OCM_FAIL(-1, "host buffers passed by the caller cannot be exported; let xgmi_new allocate");
        x->mine.host = 1;  // the memfd rides along with the record
    }
    return 0;
}

// Takes ownership of `passed` (the peer's memfd for a host buffer, or -1).
int import_remote(xgmi_t x, const Reg &r, int passed) {
    if (r.magic != kMagic || (r.host && passed < 0)) {
        if (passed >= 0) close(passed);
        OCM_FAIL(-1, "bad registration record");
    }
    x->rlen = r.len;
    if (!r.host) {
        if (passed >= 0) close(passed);
        if (x->device < 0) OCM_FAIL(-1, "peer buffer is HBM but this process has no GPU");
        hipIpcMemHandle_t h;
        std::memcpy(&h, r.handle, sizeof(h));
        void *p = nullptr;
        if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
            OCM_FAIL(-1, "hipIpcOpenMemHandle of the peer buffer failed");
        x->rbuf = static_cast<char *>(p);
        x->rgpu = true;
        return 0;
    }
    const int fd = passed;
    size_t maplen = (r.len + 4095) & ~size_t(4095);
    void *p = mmap(nullptr, maplen, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) OCM_FAIL(-1, "mmap peer host buffer: %s", strerror(errno));
    x->rhost = static_cast<char *>(p);
    x->rbuf = x->rhost;
    if (x->device >= 0 && hipHostRegister(p, maplen, hipHostRegisterMapped) == hipSuccess) {
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, p, 0) == hipSuccess) x->rbuf = static_cast<char *>(dp);
        x->rhost_registered = true;
    } else {
        (void)hipGetLastError();
    }
    return 0;
}

// Registration records travel with the host buffer's memfd attached
// (SCM_RIGHTS): the peer maps it even if this process has exited by then,
// which a /proc/<pid>/fd path would not survive.
int exchange(xgmi_t x) {
    if (export_local(x) != 0) return -1;
    char out[1 + sizeof(Reg)];
    out[0] = (char)K_REG;
    std::memcpy(out + 1, &x->mine, sizeof(Reg));
    if (mbox_send_fd(x->fd, out, sizeof(out), x->mine.host ? x->memfd : -1, 10000) != 1)
        OCM_FAIL(-1, "registration send failed");
    char in[1 + sizeof(Reg)];
    int passed = -1;
    struct pollfd q = {x->fd, POLLIN, 0};
    if (poll(&q, 1, 10000) <= 0 || mbox_recv_fd(x->fd, in, sizeof(in), &passed, 10000) != 1 || in[0] != (char)K_REG) {
        if (passed >= 0) close(passed);
        OCM_FAIL(-1, "registration receive failed");
    }
    Reg r;
    std::memcpy(&r, in + 1, sizeof(r));
    return import_remote(x, r, passed);
}

int copy(xgmi_t x, bool write, size_t loff, size_t roff, size_t n) {
    if (loff + n > x->len) OCM_FAIL(-1, "local range [%zu,+%zu) exceeds %zu", loff, n, x->len);
    if (roff + n > x->rlen) OCM_FAIL(-1, "remote range [%zu,+%zu) exceeds %zu", roff, n, x->rlen);
    if (n == 0) return 0;
    char *l = x->buf + loff;
    if (x->device < 0) {
        char *r = x->rhost + roff;
        std::memcpy(write ? r : l, write ? l : r, n);
        return 0;
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(x->device);
    hipError_t e;
    if (x->gpu >= 0 || x->rgpu) {
        XferArgs a;
        std::memset(&a, 0, sizeof(a));
        a.lin = x->dbuf + loff;
        a.ext[0] = x->rbuf;
        a.n_ext = 1;
        a.rem_off = roff;
        a.len = n;
        a.put = write ? 1 : 0;
        e = xfer_launch(a, xfer_tuning_from_env(), x->stream);
    } else {
        char *r = x->rhost + roff;
        std::memcpy(write ? r : l, write ? l : r, n);
        e = hipSuccess;
    }
    (void)hipSetDevice(prev);
    if (e != hipSuccess) OCM_FAIL(-1, "transfer launch: %s", hipGetErrorString(e));
    x->pending = true;
    return 0;
}

}  // namespace

extern "C" {

int xgmi_init(void) { return 0; }

xgmi_t xgmi_new(const struct xgmi_params *p) {
    if (!p || !p->endpoint || !p->buf_len) OCM_FAIL(nullptr, "xgmi_new: endpoint and buf_len required");
    auto *x = new xgmi_alloc();
    x->endpoint = std::string("ocm_xgmi_") + p->endpoint;
    x->len = p->buf_len;
    const int ndev = dev_count();
    x->gpu = (p->gpu >= 0 && p->gpu < ndev) ? p->gpu : -1;
    x->device = x->gpu >= 0 ? x->gpu : (ndev > 0 ? 0 : -1);
    if (x->device >= 0) {
        (void)hipSetDevice(x->device);
        if (hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess) x->stream = nullptr;
    }
    if (p->buf) {
        x->buf = static_cast<char *>(p->buf);
    } else if (x->gpu >= 0) {
        if (hipMalloc(reinterpret_cast<void **>(&x->buf), x->len) != hipSuccess) {
            delete x;
            OCM_FAIL(nullptr, "hipMalloc(%zu) failed", p->buf_len);
        }
        x->own = true;
    } else {
        size_t maplen = (x->len + 4095) & ~size_t(4095);
        x->memfd = memfd_create("ocm_xgmi", MFD_CLOEXEC);
        void *m = MAP_FAILED;
        if (x->memfd >= 0 && ftruncate(x->memfd, (off_t)maplen) == 0)
            m = mmap(nullptr, maplen, PROT_READ | PROT_WRITE, MAP_SHARED, x->memfd, 0);
        if (m == MAP_FAILED) {
            if (x->memfd >= 0) close(x->memfd);
            delete x;
            OCM_FAIL(nullptr, "host buffer of %zu bytes failed", p->buf_len);
        }
        x->buf = static_cast<char *>(m);
        x->own = true;
        if (x->device >= 0 && hipHostRegister(m, maplen, hipHostRegisterMapped) == hipSuccess)
            x->registered = true;
        else
            (void)hipGetLastError();
    }
    x->dbuf = x->buf;
    if (x->gpu < 0 && x->device >= 0) {
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, x->buf, 0) == hipSuccess)
            x->dbuf = static_cast<char *>(dp);
        else
            (void)hipGetLastError();
    }
    return x;
}

int xgmi_connect(xgmi_t x, bool is_server) {
    if (!x) return -1;
    if (is_server) {
        x->listen_fd = mbox_listen(x->endpoint, 1);
        if (x->listen_fd < 0) return -1;
        struct pollfd q = {x->listen_fd, POLLIN, 0};
        if (poll(&q, 1, 600000) <= 0) OCM_FAIL(-1, "no client connected to %s", x->endpoint.c_str());
        x->fd = mbox_accept(x->listen_fd, nullptr);
        if (x->fd < 0) OCM_FAIL(-1, "accept failed");
        // blocking from here on
        fcntl(x->fd, F_SETFL, fcntl(x->fd, F_GETFL, 0) & ~O_NONBLOCK);
    } else {
        x->fd = mbox_connect(x->endpoint, 10000);
        if (x->fd < 0) return -1;
        fcntl(x->fd, F_SETFL, fcntl(x->fd, F_GETFL, 0) & ~O_NONBLOCK);
    }
    return exchange(x);
}

int xgmi_read(xgmi_t x, size_t src_offset, size_t dest_offset, size_t len) {
    return x ? copy(x, false, src_offset, dest_offset, len) : -1;
}

int xgmi_write(xgmi_t x, size_t src_offset, size_t dest_offset, size_t len) {
    return x ? copy(x, true, src_offset, dest_offset, len) : -1;
}

int xgmi_poll(xgmi_t x) {
    if (!x) return -1;
    if (!x->pending || !x->stream) return 0;
    x->pending = false;
    return hipStreamSynchronize(x->stream) == hipSuccess ? 0 : -1;
}

void *xgmi_localbuf(xgmi_t x, size_t *len) {
    if (!x) return nullptr;
    if (len) *len = x->len;
    return x->buf;
}

size_t xgmi_remote_len(xgmi_t x) { return x ? x->rlen : 0; }

int xgmi_send_ctrl(xgmi_t x, const char *text) {
    if (!x || x->fd < 0) return -1;
    return send_kind(x->fd, K_CTRL, text, std::strlen(text) + 1);
}

int xgmi_recv_ctrl(xgmi_t x, char *text, size_t cap, int timeout_ms) {
    if (!x || x->fd < 0 || cap == 0) return -1;
    uint8_t k = 0;
    int n = recv_kind(x->fd, &k, text, cap - 1, timeout_ms);
    if (n < 0) return -1;
    text[n] = 0;
    if (k == K_BYE) return 0;
    return k == K_CTRL ? n : -1;
}

int xgmi_disconnect(xgmi_t x, bool is_server) {
    if (!x) return -1;
    xgmi_poll(x);
    if (x->fd >= 0) {
        send_kind(x->fd, K_BYE, nullptr, 0);
        close(x->fd);
        x->fd = -1;
    }
    if (x->listen_fd >= 0) close(x->listen_fd);
    x->listen_fd = -1;
    if (x->rgpu && x->rbuf) (void)hipIpcCloseMemHandle(x->rbuf);
    if (x->rhost) {
        if (x->rhost_registered) (void)hipHostUnregister(x->rhost);
        munmap(x->rhost, (x->rlen + 4095) & ~size_t(4095));
    }
    x->rbuf = x->rhost = nullptr;
    x->rlen = 0;
    (void)is_server;
    return 0;
}

int xgmi_free(xgmi_t x) {
    if (!x) return -1;
    if (x->fd >= 0 || x->rbuf) xgmi_disconnect(x, false);
    if (x->own) {
        if (x->gpu >= 0) {
            (void)hipFree(x->buf);
        } else {
            if (x->registered) (void)hipHostUnregister(x->buf);
            munmap(x->buf, (x->len + 4095) & ~size_t(4095));
            close(x->memfd);
        }
    }
    if (x->stream) (void)hipStreamDestroy(x->stream);
    delete x;
    return 0;
}

}  // extern "C"
