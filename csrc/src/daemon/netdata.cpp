#include "ocm/netdata.h"

#include <hip/hip_runtime_api.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstring>

#include "ocm/arena.h"
#include "ocm/log.h"
#include "ocm/sock.h"

// Requests on different connections (an app's parallel streams, or its next op
// on another stream) touch the same slab bytes from different server threads.
// Their order is set by the app, which waits for each response before it sends
// a request that depends on it; TSan cannot see that through the sockets, so
// every request acquires, and every completed one releases, a per-server token.
#if defined(__has_feature)
#if __has_feature(thread_sanitizer)
#define OCM_TSAN 1
extern "C" void __tsan_acquire(void *addr);
extern "C" void __tsan_release(void *addr);
#endif
#endif
#ifndef OCM_TSAN
#define OCM_TSAN 0
#endif

namespace ocm {

namespace {
inline void hb_acquire([[maybe_unused]] void *tok) {
#if OCM_TSAN
    __tsan_acquire(tok);
#endif
}
inline void hb_release([[maybe_unused]] void *tok) {
#if OCM_TSAN
    __tsan_release(tok);
#endif
}
}  // namespace

bool parse_net_handle(const uint8_t *handle, std::string *ip, int *port, uint64_t *token) {
    char buf[65] = {0};
    std::memcpy(buf, handle, 64);
    char host[64] = {0};
    int p = 0;
    unsigned long long t = 0;
    if (std::sscanf(buf, "net:%63[^:]:%d:%llx", host, &p, &t) != 3 || p <= 0) return false;
    *ip = host;
    *port = p;
    *token = t;
    return true;
}

DataServer::DataServer(Arena *arena, int gpu, uint64_t token) : arena_(arena), gpu_(gpu), token_(token) {}

DataServer::~DataServer() { stop(); }

int DataServer::start(const std::string &bind_ip) {
    listen_fd_ = tcp_listen(bind_ip, 0, 64);
    if (listen_fd_ < 0) return -1;
    struct sockaddr_in a;
    socklen_t l = sizeof(a);
    if (getsockname(listen_fd_, (struct sockaddr *)&a, &l) != 0) return -1;
    port_ = ntohs(a.sin_port);
    acceptor_ = std::thread([this] { accept_loop(); });
    return 0;
}

void DataServer::stop() {
    if (!acceptor_.joinable()) return;
    stop_ = true;
    shutdown(listen_fd_, SHUT_RDWR);
    acceptor_.join();
    {
        std::lock_guard<std::mutex> lk(mu_);
        for (int fd : conns_) shutdown(fd, SHUT_RDWR);
    }
    for (auto &w : workers_)
        if (w.th.joinable()) w.th.join();
    workers_.clear();
    close(listen_fd_);
    listen_fd_ = -1;
}

void DataServer::accept_loop() {
    while (!stop_) {
        struct pollfd p = {listen_fd_, POLLIN, 0};
        int rc = poll(&p, 1, 200);
        if (rc <= 0) continue;
        int fd = tcp_accept(listen_fd_);
        if (fd < 0) continue;
        std::lock_guard<std::mutex> lk(mu_);
        reap();
        if (conns_.size() >= kMaxConns) {
            OCM_WARN("data server: %zu connections open, refusing another", conns_.size());
            close(fd);
            continue;
        }
        conns_.push_back(fd);
        auto done = std::make_shared<std::atomic<bool>>(false);
        workers_.push_back(Worker{std::thread([this, fd, done] {
                                      serve(fd);
                                      done->store(true);
                                  }),
                                  done});
    }
}

void DataServer::reap() {
    for (auto it = workers_.begin(); it != workers_.end();) {
        if (it->done->load()) {
            it->th.join();
            it = workers_.erase(it);
        } else {
            ++it;
        }
    }
}

void DataServer::serve(int fd) {
    void *stage = nullptr;
    if (gpu_ >= 0) {
        (void)hipSetDevice(gpu_);
        if (hipHostMalloc(&stage, kNetChunk, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            stage = nullptr;
        }
    }
    std::vector<char> sink;
    NetReq q;
    uint64_t tok = 0;
    const bool authed = recv_all(fd, &tok, sizeof(tok)) == 1 && tok == token_;
    if (!authed) OCM_WARN("data server: dropping a connection without the owner's token");
    while (authed && !stop_ && recv_all(fd, &q, sizeof(q)) == 1) {
        NetResp r{kNetMagic, 0, q.len};
        if (q.magic != kNetMagic) break;
        hb_acquire(&token_);
        void *mem = nullptr;
        uint32_t tier = 0;
        if (q.op == NET_PING) {
            r.len = 0;
            if (send_all(fd, &r, sizeof(r)) != 1) break;
            continue;
        }
        if (!arena_->locate(q.slab_id, q.offset, q.len, &mem, &tier)) r.err = EFAULT;
        if (tier == TIER_GPU && !stage) r.err = r.err ? r.err : ENOMEM;
        bool ok = true;
        if (q.op == NET_PUT) {
            for (uint64_t done = 0; ok && done < q.len;) {
                const size_t n = (size_t)std::min<uint64_t>(kNetChunk, q.len - done);
                if (r.err) {
                    sink.resize(n);
                    ok = recv_all(fd, sink.data(), n) == 1;  // keep the stream in sync
                } else if (tier == TIER_HOST) {
                    ok = recv_all(fd, static_cast<char *>(mem) + done, n) == 1;
                } else {
                    ok = recv_all(fd, stage, n) == 1 &&
                         hipMemcpy(static_cast<char *>(mem) + done, stage, n, hipMemcpyHostToDevice) == hipSuccess;
                }
                done += n;
            }
            hb_release(&token_);
            if (!ok || send_all(fd, &r, sizeof(r)) != 1) break;
        } else if (q.op == NET_GET) {
            if (r.err) r.len = 0;
            if (send_all(fd, &r, sizeof(r)) != 1) break;
            for (uint64_t done = 0; ok && !r.err && done < q.len;) {
                const size_t n = (size_t)std::min<uint64_t>(kNetChunk, q.len - done);
                if (tier == TIER_HOST) {
                    ok = send_all(fd, static_cast<char *>(mem) + done, n) == 1;
                } else {
                    ok = hipMemcpy(stage, static_cast<char *>(mem) + done, n, hipMemcpyDeviceToHost) == hipSuccess &&
                         send_all(fd, stage, n) == 1;
                }
                done += n;
            }
            hb_release(&token_);
            if (!ok) break;
        } else {
            break;
        }
    }
    if (stage) (void)hipHostFree(stage);
    std::lock_guard<std::mutex> lk(mu_);
    for (auto it = conns_.begin(); it != conns_.end(); ++it)
        if (*it == fd) {
            conns_.erase(it);
            break;
        }
    close(fd);
}

}  // namespace ocm
