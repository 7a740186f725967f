// ocmd app protocol: CONNECT/DISCONNECT (crash reclaim), REQ_ALLOC, REQ_FREE, STATS.
// Reference parity: the app registry and process_msg dispatch of src/main.c:46-104
// and mem_new_request src/mem.c:514-530; crash reclaim was a TODO there
// (src/main.c:6-7, README:68-69).
#include "ocm/daemon.h"

#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/signalfd.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

#include "../../include/oncillamem.h"
#include "ocm/log.h"
#include "ocm/trace.h"
#include "util.h"

namespace ocm {
using namespace dm;

// ---------------------------------------------------------------- app messages

void Daemon::handle_app_msg(Msg &m) {
    TraceRange tr(msg_type_str(m.type));
    OCM_LOG("rank %d <- app %d: %s", rank_, m.pid, msg_type_str(m.type));
    if (m.type != MSG_CONNECT && m.type != MSG_SHUTDOWN && !apps_.count(m.pid)) {
        OCM_WARN("rank %d: %s from unknown app %d ignored", rank_, msg_type_str(m.type), m.pid);
        return;
    }
    switch (m.type) {
    case MSG_WAKE: break;  // the app posted on its shared-memory link while we slept: the loop looks there
    case MSG_DISCONNECT: app_disconnect(m.pid, false); break;
    case MSG_REQ_ALLOC: app_req_alloc(m); break;
    case MSG_REQ_FREE: app_req_free(m); break;
    case MSG_STATS: app_stats(m); break;
    case MSG_TICK_STATS: app_tick_stats(m); break;
    case MSG_PING: {
        Msg r = m;
        r.status = MSG_RESPONSE;
        r.type = MSG_RELEASE_APP;
        send_app(m.pid, r);
        break;
    }
    case MSG_SHUTDOWN: stop_ = true; break;
    default: OCM_WARN("rank %d: unexpected app message %s", rank_, msg_type_str(m.type)); break;
    }
}

void Daemon::app_connect(const Msg &m, int fd) {
    pid_t pid = m.pid;
    if (apps_.count(pid)) {
        auto &old = apps_[pid];
        if (old.fd != fd) {
            app_disconnect(pid, false);
        } else if (old.pidfd >= 0) {
            // A CONNECT retried on the same socket (the mesh was still joining):
            // the entry is replaced below with a pidfd of its own (the
            // old one leaked, with its epoll registration, on every retry).
            ep_del(old.pidfd);
            close(old.pidfd);
            old.pidfd = -1;
        }
    }
    App a;
    a.pid = pid;
    a.fd = fd;
    // OCM_SHM_LINK_ACCEPT=0: take no links (apps then keep to the socket).
    static const bool accept_links = [] {
        const char *v = std::getenv("OCM_SHM_LINK_ACCEPT");
        return !(v && std::strcmp(v, "0") == 0);
    }();
    if (pending_link_fd_ >= 0 && !accept_links) {
        close(pending_link_fd_);
        pending_link_fd_ = -1;
    }
    if (pending_link_fd_ >= 0) {
        // The app offered a shared-memory link with its CONNECT (SCM_RIGHTS).
        auto link = std::make_shared<ShmLink>();
        const int lfd = pending_link_fd_;
        pending_link_fd_ = -1;
        if (link->attach(lfd) == 0) {
            link->set_daemon_polling(links_polling_);
            a.link = std::move(link);
        } else {
            OCM_WARN("rank %d: app %d offered an unusable shared-memory link; using its mailbox", rank_, (int)pid);
        }
    }
    a.pidfd = pidfd_open_compat(pid);
    if (a.pidfd >= 0) ep_add(a.pidfd, EPOLLIN, tag(T_PIDFD, (uint64_t)pid));
    apps_[pid] = std::move(a);
    Msg r;
    std::memset(&r, 0, sizeof(r));
    r.type = MSG_CONNECT_CONFIRM;
    r.status = MSG_RESPONSE;
    r.pid = pid;
    r.rank = rank_;
    r.seq = m.seq;
    r.u.node = my_config();
    r.err = ready_ ? 0 : EAGAIN;
    send_app(pid, r);
}

void Daemon::app_disconnect(pid_t pid, bool crashed) {
    auto it = apps_.find(pid);
    if (it == apps_.end()) return;
    // Reclaim whatever the app still holds (reference README:68-69 left this a TODO).
    std::vector<uint64_t> mine;
    for (auto &kv : origin_allocs_)
        if (kv.second.pid == pid) mine.push_back(kv.first);
    for (uint64_t id : mine) {
        start_free(id, 0, 0);
        n_reclaimed_++;
    }
    for (auto &kv : pending_)
        if (kv.second.pid == pid) kv.second.pid = 0;  // finish silently, then reclaim
    App &a = it->second;
    if (a.watching_out && a.fd >= 0) ep_mod(a.fd, EPOLLIN, tag(T_APPCONN, (uint64_t)a.fd));
    if (a.pidfd >= 0) {
        ep_del(a.pidfd);
        close(a.pidfd);
    }
    auto ac = app_conns_.find(a.fd);
    if (ac != app_conns_.end()) ac->second.app_pid = 0;  // connection may be reused by a new CONNECT
    apps_.erase(it);
    (void)crashed;
    OCM_LOG("rank %d: app %d detached (%zu allocations reclaimed)", rank_, (int)pid, mine.size());
}

void Daemon::app_req_alloc(Msg &m) {
    const AllocReq &req = m.u.req;
    if (req.bytes == 0) {
        Msg r = m;
        r.type = MSG_RELEASE_APP;
        r.status = MSG_RESPONSE;
        r.err = EINVAL;
        send_app(m.pid, r);
        return;
    }
    if (!is_remote_kind(req.kind)) {
        // Local kinds: the app allocates the memory itself (malloc / hipMalloc);
        // the daemon only records it. No rank0 round trip on this path.
        uint64_t id = (1ull << 63) | ((uint64_t)rank_ << 40) | (++local_ids_);
        OriginAlloc oa;
        oa.pid = m.pid;
        oa.remote = false;
        oa.bytes = req.bytes;
        origin_allocs_[id] = oa;
        n_alloc_++;
        Msg r;
        std::memset(&r, 0, sizeof(r));
        r.type = MSG_RELEASE_APP;
        r.status = MSG_RESPONSE;
        r.pid = m.pid;
        r.rank = rank_;
        r.seq = m.seq;
        r.u.region.alloc_id = id;
        r.u.region.bytes = req.bytes;
        r.u.region.tier = (uint16_t)(req.kind == OCM_LOCAL_GPU ? TIER_GPU : TIER_HOST);
        r.u.region.owner_rank = rank_;
        r.u.region.orig_rank = rank_;
        r.u.region.owner_gpu = gpu_;
        r.u.region.n_extents = 0;
        send_app(m.pid, r);
        return;
    }
    if (try_lease_alloc(m)) return;
    Pending p;
    p.seq = next_seq();
    p.pid = m.pid;
    p.type = MSG_REQ_ALLOC;
    p.kind = req.kind;
    p.total_bytes = req.bytes;
    p.awaiting.insert(0);
    p.app_seq = m.seq;
    p.t0_ms = now_ms();
    pending_[p.seq] = p;
    Msg f = m;
    f.type = MSG_REQ_ALLOC;
    f.status = MSG_REQUEST;
    f.rank = rank_;
    f.seq = p.seq;
    f.u.req.orig_rank = rank_;
    f.u.req.app_pid = m.pid;
    send_rank(0, f);
}

void Daemon::app_req_free(Msg &m) {
    const uint64_t id = m.u.req.alloc_id;
    auto it = origin_allocs_.find(id);
    if (it == origin_allocs_.end() || it->second.pid != m.pid) {
        Msg r = m;
        r.type = MSG_RELEASE_APP;
        r.status = MSG_RESPONSE;
        r.err = ENOENT;
        send_app(m.pid, r);
        return;
    }
    if (!it->second.remote) {
        origin_allocs_.erase(it);
        n_free_++;
        Msg r = m;
        r.type = MSG_RELEASE_APP;
        r.status = MSG_RESPONSE;
        r.err = 0;
        send_app(m.pid, r);
        return;
    }
    start_free(id, m.pid, m.seq);
}

void Daemon::app_stats(Msg &m) {
    const int target = m.u.req.remote_rank;
    if (target >= 0 && target != rank_) {
        Pending p;
        p.seq = next_seq();
        p.pid = m.pid;
        p.type = MSG_STATS;
        p.app_seq = m.seq;
        p.t0_ms = now_ms();
        p.awaiting.insert(target);
        pending_[p.seq] = p;
        Msg f = m;
        f.status = MSG_REQUEST;
        f.rank = rank_;
        f.seq = p.seq;
        send_rank(target, f);
        return;
    }
    Msg r;
    std::memset(&r, 0, sizeof(r));
    r.type = MSG_RELEASE_APP;
    r.status = MSG_RESPONSE;
    r.pid = m.pid;
    r.rank = rank_;
    r.seq = m.seq;
    r.u.node = my_config();
    send_app(m.pid, r);
}


// The tick control transport's statistics (this daemon only; zeros without one).
void Daemon::app_tick_stats(Msg &m) {
    Msg r;
    std::memset(&r, 0, sizeof(r));
    r.type = MSG_RELEASE_APP;
    r.status = MSG_RESPONSE;
    r.pid = m.pid;
    r.rank = rank_;
    r.seq = m.seq;
    TickStatsWire st;
    std::memset(&st, 0, sizeof(st));
    if (tick_) tick_->stats(&st);
    st.transport = my_config().ctrl;
    st.tcp_wakes = tcp_wakes_;
    std::memcpy(r.u.raw, &st, sizeof(st));
    send_app(m.pid, r);
}

}  // namespace ocm
