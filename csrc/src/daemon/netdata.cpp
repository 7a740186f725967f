#include "ocm/netdata.h"

#include <hip/hip_runtime_api.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <random>

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

DataServer::DataServer(Arena *arena, int gpu, uint64_t token) : arena_(arena), gpu_(gpu), token_(token) {}

DataServer::~DataServer() { stop(); }

int DataServer::start(const std::string &bind_ip, int port) {
    listen_fd_ = tcp_listen(bind_ip, port, 64);
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

uint64_t DataServer::grant(uint32_t slab_id, uint64_t offset, uint64_t bytes) {
    static thread_local std::mt19937_64 rng(std::random_device{}() ^ ((uint64_t)std::random_device{}() << 32));
    std::lock_guard<std::mutex> lk(mu_);
    uint64_t g = 0;
    while (g == 0 || grants_.count(g)) g = rng();
    Grant &e = grants_[g];
    e.slab_id = slab_id;
    e.offset = offset;
    e.bytes = bytes;
    return g;
}

bool DataServer::revoke(uint64_t g) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = grants_.find(g);
    if (it == grants_.end()) return true;
    if (it->second.busy > 0) {
        it->second.revoked = true;  // release() frees the extent
        return false;
    }
    grants_.erase(it);
    return true;
}

size_t DataServer::grants() const {
    std::lock_guard<std::mutex> lk(mu_);
    return grants_.size();
}

bool DataServer::acquire(const NetReq &q, void **mem, uint32_t *tier, int *err) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = grants_.find(q.grant);
    if (it == grants_.end() || it->second.revoked) {
        *err = EACCES;
        return false;
    }
    Grant &g = it->second;
    if (q.offset > g.bytes || q.len > g.bytes - q.offset) {
        *err = EFAULT;
        return false;
    }
    // The extent cannot be freed while busy > 0, so its slab stays mapped.
    if (!arena_->locate(g.slab_id, g.offset + q.offset, q.len, mem, tier)) {
        *err = EFAULT;
        return false;
    }
    g.busy++;
    return true;
}

void DataServer::release(uint64_t g) {
    uint32_t slab = 0;
    uint64_t off = 0;
    {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = grants_.find(g);
        if (it == grants_.end()) return;
        if (--it->second.busy > 0 || !it->second.revoked) return;
        slab = it->second.slab_id;
        off = it->second.offset;
        grants_.erase(it);
    }
    arena_->free(slab, off);  // the owner freed it while we were copying
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
        if (q.op == NET_PING) {
            r.len = 0;
            if (send_all(fd, &r, sizeof(r)) != 1) break;
            continue;
        }
        if (q.op != NET_PUT && q.op != NET_GET) break;
        hb_acquire(&token_);
        void *mem = nullptr;
        uint32_t tier = 0;
        int err = 0;
        const bool held = acquire(q, &mem, &tier, &err);
        if (!held) r.err = err;
        if (held && tier == TIER_GPU && !stage) r.err = ENOMEM;
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
            if (held) release(q.grant);
            if (!ok || send_all(fd, &r, sizeof(r)) != 1) break;
        } else {
            if (r.err) r.len = 0;
            ok = send_all(fd, &r, sizeof(r)) == 1;
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
            if (held) release(q.grant);
            if (!ok) break;
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
