// TCP helpers for the mesh links and the network-tier data server.
// Reference parity: conn_connect / localbind / accept / put / get of
// src/sock.c:18-261 (inc/sock.h:30-47), with connect timeouts and non-blocking
// record framing added.
#include "ocm/sock.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>

#include "ocm/log.h"

namespace ocm {

static long now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1000L + ts.tv_nsec / 1000000L;
}

void tune_socket(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    setsockopt(fd, SOL_SOCKET, SO_KEEPALIVE, &one, sizeof(one));
}

int set_nonblocking(int fd, bool on) {
    int fl = fcntl(fd, F_GETFL, 0);
    if (fl < 0) return -1;
    fl = on ? (fl | O_NONBLOCK) : (fl & ~O_NONBLOCK);
    return fcntl(fd, F_SETFL, fl);
}

int tcp_listen(const std::string &bind_ip, int port, int backlog) {
    struct addrinfo hints, *res = nullptr;
    std::memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_flags = AI_PASSIVE;
    std::string p = std::to_string(port);
    int rc = getaddrinfo(bind_ip.empty() ? nullptr : bind_ip.c_str(), p.c_str(), &hints, &res);
    if (rc != 0) OCM_FAIL(-1, "getaddrinfo(%s:%d): %s", bind_ip.c_str(), port, gai_strerror(rc));
    int fd = -1;
    for (auto *ai = res; ai; ai = ai->ai_next) {
        fd = socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
        if (fd < 0) continue;
        int one = 1;
        setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        if (bind(fd, ai->ai_addr, ai->ai_addrlen) == 0 && listen(fd, backlog) == 0) break;
        close(fd);
        fd = -1;
    }
    freeaddrinfo(res);
    if (fd < 0) OCM_FAIL(-1, "cannot listen on %s:%d: %s", bind_ip.c_str(), port, strerror(errno));
    return fd;
}

int tcp_connect(const std::string &host, int port, int timeout_ms) {
    const long deadline = now_ms() + timeout_ms;
    std::string p = std::to_string(port);
    for (;;) {
        struct addrinfo hints, *res = nullptr;
        std::memset(&hints, 0, sizeof(hints));
        hints.ai_family = AF_INET;
        hints.ai_socktype = SOCK_STREAM;
        int rc = getaddrinfo(host.c_str(), p.c_str(), &hints, &res);
        if (rc == 0) {
            for (auto *ai = res; ai; ai = ai->ai_next) {
                int fd = socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
                if (fd < 0) continue;
                if (connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) {
                    freeaddrinfo(res);
                    tune_socket(fd);
                    return fd;
                }
                close(fd);
            }
            freeaddrinfo(res);
        }
        if (now_ms() >= deadline) break;
        usleep(20000);
    }
    OCM_FAIL(-1, "connect %s:%d timed out after %d ms", host.c_str(), port, timeout_ms);
}

int tcp_accept(int listen_fd) {
    for (;;) {
        int fd = accept4(listen_fd, nullptr, nullptr, SOCK_CLOEXEC);
        if (fd >= 0) {
            tune_socket(fd);
            return fd;
        }
        if (errno == EINTR) continue;
        return -1;
    }
}

int send_all(int fd, const void *buf, size_t len) {
    const char *p = static_cast<const char *>(buf);
    while (len > 0) {
        ssize_t n = send(fd, p, len, MSG_NOSIGNAL);
        if (n > 0) {
            p += n;
            len -= (size_t)n;
        } else if (n < 0 && errno == EINTR) {
            continue;
        } else if (n < 0 && (errno == EPIPE || errno == ECONNRESET)) {
            return 0;
        } else {
            return -1;
        }
    }
    return 1;
}

int recv_all(int fd, void *buf, size_t len) {
    char *p = static_cast<char *>(buf);
    while (len > 0) {
        ssize_t n = recv(fd, p, len, 0);
        if (n > 0) {
            p += n;
            len -= (size_t)n;
        } else if (n == 0) {
            return 0;
        } else if (errno == EINTR) {
            continue;
        } else {
            return -1;
        }
    }
    return 1;
}

int conn_read_records(Conn &c, size_t rec, std::vector<std::vector<uint8_t>> &out) {
    uint8_t buf[16384];
    for (;;) {
        ssize_t n = recv(c.fd, buf, sizeof(buf), 0);
        if (n > 0) {
            c.rx.insert(c.rx.end(), buf, buf + n);
            size_t off = 0;
            while (c.rx.size() - off >= rec) {
                out.emplace_back(c.rx.begin() + (long)off, c.rx.begin() + (long)(off + rec));
                off += rec;
            }
            if (off) c.rx.erase(c.rx.begin(), c.rx.begin() + (long)off);
            continue;
        }
        if (n == 0) return -1;  // EOF
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) return 0;
        return -1;
    }
}

int conn_flush(Conn &c) {
    while (c.tx_off < c.tx.size()) {
        ssize_t n = send(c.fd, c.tx.data() + c.tx_off, c.tx.size() - c.tx_off, MSG_NOSIGNAL);
        if (n > 0) {
            c.tx_off += (size_t)n;
            continue;
        }
        if (n < 0 && errno == EINTR) continue;
        if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
        return -1;
    }
    if (c.tx_off == c.tx.size()) {
        c.tx.clear();
        c.tx_off = 0;
        c.want_write = false;
    } else {
        c.want_write = true;
    }
    return 0;
}

int conn_write(Conn &c, const void *buf, size_t len) {
    const uint8_t *p = static_cast<const uint8_t *>(buf);
    c.tx.insert(c.tx.end(), p, p + len);
    return conn_flush(c);
}

}  // namespace ocm
