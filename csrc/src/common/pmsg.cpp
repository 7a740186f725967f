#include "ocm/pmsg.h"

#include <fcntl.h>
#include <poll.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>

#include "ocm/log.h"
#include "ocm/msg.h"

namespace ocm {

std::string pmsg_namespace() {
    const char *ns = std::getenv("OCM_NS");
    std::string s = (ns && *ns) ? ns : "default";
    for (char &c : s)
        if (c == '/' || c == ' ' || c == '\0') c = '_';
    return s;
}

std::string daemon_mailbox_name(int rank, const std::string &ns) { return "ocm_" + ns + "_d" + std::to_string(rank); }

std::string app_mailbox_name(pid_t pid, const std::string &ns) { return "ocm_" + ns + "_p" + std::to_string((long)pid); }

namespace {

socklen_t make_addr(const std::string &name, struct sockaddr_un *a) {
    std::memset(a, 0, sizeof(*a));
    a->sun_family = AF_UNIX;
    // Abstract namespace: leading NUL, no filesystem entry.
    const size_t n = std::min(name.size(), sizeof(a->sun_path) - 2);
    std::memcpy(a->sun_path + 1, name.data(), n);
    return (socklen_t)(offsetof(struct sockaddr_un, sun_path) + 1 + n);
}

long mono_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1000L + ts.tv_nsec / 1000000L;
}

// Wait for `events` on fd. Returns 1 ready, 0 timeout, -1 error.
int wait_fd(int fd, short events, int timeout_ms) {
    struct pollfd p;
    p.fd = fd;
    p.events = events;
    p.revents = 0;
    for (;;) {
        int rc = poll(&p, 1, timeout_ms);
        if (rc > 0) return 1;
        if (rc == 0) return 0;
        if (errno != EINTR) return -1;
    }
}

}  // namespace

int mbox_listen(const std::string &name, int backlog) {
    int fd = socket(AF_UNIX, SOCK_SEQPACKET | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (fd < 0) OCM_FAIL(-1, "socket(AF_UNIX): %s", strerror(errno));
    struct sockaddr_un a;
    socklen_t len = make_addr(name, &a);
    if (bind(fd, (struct sockaddr *)&a, len) != 0) {
        int e = errno;
        close(fd);
        OCM_FAIL(-1, "bind mailbox @%s: %s", name.c_str(), strerror(e));
    }
    if (listen(fd, backlog) != 0) {
        int e = errno;
        close(fd);
        OCM_FAIL(-1, "listen mailbox @%s: %s", name.c_str(), strerror(e));
    }
    return fd;
}

pid_t mbox_peer_pid(int fd) {
    struct ucred cr;
    socklen_t l = sizeof(cr);
    if (getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cr, &l) != 0) return -1;
    return cr.pid;
}

int mbox_peer_uid(int fd) {
    struct ucred cr;
    socklen_t l = sizeof(cr);
    if (getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cr, &l) != 0) return -1;
    return (int)cr.uid;
}

int mbox_accept(int listen_fd, pid_t *peer_pid) {
    for (;;) {
        int fd = accept4(listen_fd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
        if (fd >= 0) {
            if (peer_pid) *peer_pid = mbox_peer_pid(fd);
            return fd;
        }
        if (errno == EINTR) continue;
        return -1;
    }
}

int mbox_connect(const std::string &name, int timeout_ms) {
    struct sockaddr_un a;
    socklen_t len = make_addr(name, &a);
    const long deadline = mono_ms() + timeout_ms;
    for (;;) {
        int fd = socket(AF_UNIX, SOCK_SEQPACKET | SOCK_CLOEXEC, 0);
        if (fd < 0) OCM_FAIL(-1, "socket(AF_UNIX): %s", strerror(errno));
        if (connect(fd, (struct sockaddr *)&a, len) == 0) {
            // Non-blocking; send/recv apply their own timeouts with poll().
            fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK);
            return fd;
        }
        int e = errno;
        close(fd);
        if (mono_ms() >= deadline) OCM_FAIL(-1, "connect mailbox @%s: %s", name.c_str(), strerror(e));
        usleep(5000);
    }
}

int mbox_send(int fd, const void *msg, size_t size, int timeout_ms) {
    if (fd < 0) OCM_FAIL(-1, "send on closed mailbox");
    for (;;) {
        ssize_t n = send(fd, msg, size, MSG_NOSIGNAL);
        if (n == (ssize_t)size) return 1;
        if (n >= 0) OCM_FAIL(-1, "short mailbox send (%zd)", n);
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) {
            if (timeout_ms == 0) return 0;
            int w = wait_fd(fd, POLLOUT, timeout_ms);
            if (w == 0) return 0;
            if (w < 0) return -1;
            continue;
        }
        OCM_FAIL(-1, "mailbox send: %s", strerror(errno));
    }
}

int mbox_recv(int fd, void *msg, size_t size, int timeout_ms) {
    if (fd < 0) OCM_FAIL(-1, "recv on closed mailbox");
    for (;;) {
        ssize_t n = recv(fd, msg, size, 0);
        if (n == (ssize_t)size) return 1;
        if (n == 0) OCM_FAIL(-1, "mailbox peer closed");
        if (n > 0) OCM_FAIL(-1, "short mailbox record (%zd bytes)", n);
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) {
            if (timeout_ms == 0) return 0;
            int w = wait_fd(fd, POLLIN, timeout_ms);
            if (w == 0) return 0;
            if (w < 0) return -1;
            continue;
        }
        OCM_FAIL(-1, "mailbox recv: %s", strerror(errno));
    }
}

int mbox_send_fd(int fd, const void *msg, size_t size, int pass_fd, int timeout_ms) {
    if (fd < 0) OCM_FAIL(-1, "send on closed mailbox");
    struct iovec iov = {const_cast<void *>(msg), size};
    union {
        char buf[CMSG_SPACE(sizeof(int))];
        struct cmsghdr align;
    } ctl;
    std::memset(&ctl, 0, sizeof(ctl));
    struct msghdr mh;
    std::memset(&mh, 0, sizeof(mh));
    mh.msg_iov = &iov;
    mh.msg_iovlen = 1;
    if (pass_fd >= 0) {
        mh.msg_control = ctl.buf;
        mh.msg_controllen = sizeof(ctl.buf);
        struct cmsghdr *c = CMSG_FIRSTHDR(&mh);
        c->cmsg_level = SOL_SOCKET;
        c->cmsg_type = SCM_RIGHTS;
        c->cmsg_len = CMSG_LEN(sizeof(int));
        std::memcpy(CMSG_DATA(c), &pass_fd, sizeof(int));
    }
    for (;;) {
        ssize_t n = sendmsg(fd, &mh, MSG_NOSIGNAL);
        if (n == (ssize_t)size) return 1;
        if (n >= 0) OCM_FAIL(-1, "short mailbox send (%zd)", n);
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) {
            if (timeout_ms == 0) return 0;
            int w = wait_fd(fd, POLLOUT, timeout_ms);
            if (w <= 0) return w;
            continue;
        }
        OCM_FAIL(-1, "mailbox send: %s", strerror(errno));
    }
}

int mbox_recv_fd(int fd, void *msg, size_t size, int *passed, int timeout_ms) {
    *passed = -1;
    if (fd < 0) OCM_FAIL(-1, "recv on closed mailbox");
    for (;;) {
        struct iovec iov = {msg, size};
        union {
            char buf[CMSG_SPACE(sizeof(int))];
            struct cmsghdr align;
        } ctl;
        struct msghdr mh;
        std::memset(&mh, 0, sizeof(mh));
        mh.msg_iov = &iov;
        mh.msg_iovlen = 1;
        mh.msg_control = ctl.buf;
        mh.msg_controllen = sizeof(ctl.buf);
        ssize_t n = recvmsg(fd, &mh, MSG_CMSG_CLOEXEC);
        if (n > 0) {
            for (struct cmsghdr *c = CMSG_FIRSTHDR(&mh); c; c = CMSG_NXTHDR(&mh, c))
                if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_RIGHTS && c->cmsg_len >= CMSG_LEN(sizeof(int)))
                    std::memcpy(passed, CMSG_DATA(c), sizeof(int));
        }
        if (n == (ssize_t)size) return 1;
        if (*passed >= 0) {
            ::close(*passed);
            *passed = -1;
        }
        if (n == 0) OCM_FAIL(-1, "mailbox peer closed");
        if (n > 0) OCM_FAIL(-1, "short mailbox record (%zd bytes)", n);
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) {
            if (timeout_ms == 0) return 0;
            int w = wait_fd(fd, POLLIN, timeout_ms);
            if (w <= 0) return w;
            continue;
        }
        OCM_FAIL(-1, "mailbox recv: %s", strerror(errno));
    }
}

int Channel::connect(const std::string &name, int timeout_ms) {
    close();
    fd_ = mbox_connect(name, timeout_ms);
    return fd_ >= 0 ? 0 : -1;
}

void Channel::close() {
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
}

bool mbox_alive(const std::string &name) {
    int fd = mbox_connect(name, 0);
    if (fd < 0) return false;
    ::close(fd);
    return true;
}

int pmsg_cleanup(const std::string &) { return 0; }

}  // namespace ocm

// ---------------- reference-shaped C interface ----------------
// One process-wide mailbox: a listening endpoint for ourselves plus the
// connections we initiated (attach) or accepted. Records from any of them are
// delivered by pmsg_recv; pmsg_send(to) uses the connection to/from `to`.
namespace {

struct PmsgState {
    size_t size = ocm::kMsgBytes;
    int listen_fd = -1;
    std::map<pid_t, int> peers;  // peer id (pid, or PMSG_DAEMON_PID) -> fd
    std::vector<int> accepted;
} g;

std::string endpoint(pid_t id) {
    const std::string ns = ocm::pmsg_namespace();
    return id < 0 ? ocm::daemon_mailbox_name(-1 - id, ns) : ocm::app_mailbox_name(id, ns);
}

void accept_pending() {
    if (g.listen_fd < 0) return;
    pid_t pp = -1;
    int fd;
    while ((fd = ocm::mbox_accept(g.listen_fd, &pp)) >= 0) {
        g.accepted.push_back(fd);
        if (pp > 0 && !g.peers.count(pp)) g.peers[pp] = fd;  // replies to this app go back on its connection
    }
}

}  // namespace

extern "C" {
int pmsg_init(size_t pmsg_size) {
    g.size = pmsg_size;
    return 0;
}
int pmsg_open(pid_t self_pid) {
    g.listen_fd = ocm::mbox_listen(endpoint(self_pid));
    return g.listen_fd >= 0 ? 0 : -1;
}
int pmsg_close(void) {
    for (int fd : g.accepted) close(fd);
    g.accepted.clear();
    for (auto &kv : g.peers) close(kv.second);
    g.peers.clear();
    if (g.listen_fd >= 0) close(g.listen_fd);
    g.listen_fd = -1;
    return 0;
}
int pmsg_attach(pid_t to) {
    if (g.peers.count(to)) return 0;
    int fd = ocm::mbox_connect(endpoint(to), 1000);
    if (fd < 0) return -1;
    g.peers[to] = fd;
    g.accepted.push_back(fd);  // replies arrive on it
    return 0;
}
int pmsg_detach(pid_t to) {
    g.peers.erase(to);
    return 0;
}
int pmsg_send(pid_t to, void *msg) {
    accept_pending();
    auto it = g.peers.find(to);
    if (it == g.peers.end()) return -1;
    return ocm::mbox_send(it->second, msg, g.size, -1) == 1 ? 0 : -1;
}
int pmsg_recv(void *msg, bool block) {
    for (;;) {
        accept_pending();
        std::vector<struct pollfd> p;
        if (g.listen_fd >= 0) p.push_back({g.listen_fd, POLLIN, 0});
        for (int fd : g.accepted) p.push_back({fd, POLLIN, 0});
        if (p.empty()) return -1;
        int rc = poll(p.data(), p.size(), block ? -1 : 0);
        if (rc <= 0) {
            if (rc < 0 && errno == EINTR) continue;
            return -1;
        }
        for (auto &q : p) {
            if (q.fd == g.listen_fd || !(q.revents & (POLLIN | POLLHUP))) continue;
            int r = ocm::mbox_recv(q.fd, msg, g.size, 0);
            if (r == 1) return 0;
            if (r < 0) {  // peer gone
                close(q.fd);
                for (auto it = g.accepted.begin(); it != g.accepted.end(); ++it)
                    if (*it == q.fd) {
                        g.accepted.erase(it);
                        break;
                    }
                for (auto it = g.peers.begin(); it != g.peers.end(); ++it)
                    if (it->second == q.fd) {
                        g.peers.erase(it);
                        break;
                    }
            }
        }
        if (!block) return -1;
    }
}
int pmsg_cleanup_all(void) { return ocm::pmsg_cleanup(ocm::pmsg_namespace()); }
int pmsg_pending(void) {
    int total = 0;
    for (int fd : g.accepted) {
        int n = 0;
        if (ioctl(fd, FIONREAD, &n) == 0 && n > 0) total += n / (int)g.size;
    }
    return total;
}
}
