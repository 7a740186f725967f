// ocmd core: init (GPU discovery, arena, data server, mailbox, mesh links),
// the epoll event loop, event sources and message routing. Protocol handlers
// live in apps.cpp (app <-> daemon), mesh.cpp (daemon <-> daemon), lease.cpp
// (capacity leases) and resume.cpp (rank0 checkpoint / rejoin).
// Reference parity: daemon main and mailbox poller src/main.c:106-224 (a
// 500 us usleep poll there, src/main.c:112-126; epoll here), daemon core
// src/mem.c:485-535 (mem_init / mem_new_request / mem_fin, inc/mem.h:29-33).
#include "ocm/daemon.h"

#include "ocm/affinity.h"

#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/prctl.h>
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

void Daemon::ep_add(int fd, uint32_t events, uint64_t t) {
    struct epoll_event ev;
    std::memset(&ev, 0, sizeof(ev));
    ev.events = events;
    ev.data.u64 = t;
    if (epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev) != 0) OCM_WARN("epoll add fd %d: %s", fd, strerror(errno));
}

void Daemon::ep_mod(int fd, uint32_t events, uint64_t t) {
    struct epoll_event ev;
    std::memset(&ev, 0, sizeof(ev));
    ev.events = events;
    ev.data.u64 = t;
    epoll_ctl(ep_, EPOLL_CTL_MOD, fd, &ev);
}

void Daemon::ep_del(int fd) { epoll_ctl(ep_, EPOLL_CTL_DEL, fd, nullptr); }

NodeConfig Daemon::my_config() const {
    NodeConfig c;
    std::memset(&c, 0, sizeof(c));
    if (!cfg_.host_alias.empty())
        std::snprintf(c.host, sizeof(c.host), "%s", cfg_.host_alias.c_str());
    else
        gethostname(c.host, sizeof(c.host) - 1);
    c.rank = rank_;
    c.gpu = gpu_;
    c.num_gpu = num_gpu_;
    c.pid = (int32_t)getpid();
    c.gpu_total = gpu_total_;
    c.gpu_capacity = arena_ ? arena_->capacity(TIER_GPU) : 0;
    c.host_capacity = arena_ ? arena_->capacity(TIER_HOST) : 0;
    c.gpu_used = arena_ ? arena_->used(TIER_GPU) : 0;
    c.host_used = arena_ ? arena_->used(TIER_HOST) : 0;
    c.num_nodes = (uint16_t)n_;
    c.num_apps = (uint16_t)std::min<size_t>(apps_.size(), 65535);
    for (uint32_t p = 0; p < links_.n && p < (uint32_t)kMaxLinkGpus; p++) {
        const uint8_t h = links_.hops[p];
        if ((int)p == gpu_ || h == kHopsUnknown) continue;
        c.xgmi_peers++;
        c.min_hops = c.min_hops ? std::min(c.min_hops, h) : h;
        c.max_hops = std::max(c.max_hops, h);
    }
    c.n_alloc = (uint32_t)n_alloc_;
    c.n_free = (uint32_t)n_free_;
    c.n_reclaimed = (uint32_t)n_reclaimed_;
    c.n_spilled = (uint32_t)(gov_ ? gov_->spilled_count() : n_spilled_);
    c.n_slabs = (uint32_t)(arena_ ? arena_->num_slabs() : 0);
    c.ticks = (uint32_t)(tick_ ? tick_->ticks() : 0);
    c.ctrl = !tick_ ? 0 : tick_left_ || tick_->failed() ? 3 : !tick_->up() ? 4 : std::strcmp(tick_->collective_name(), "rccl") == 0 ? 2 : 1;
    for (auto &l : leases_) c.n_leases += l != nullptr;
    c.lease_allocs = (uint32_t)n_lease_allocs_;
    return c;
}

int Daemon::init() {
    std::string err;
    if (const char *nd = std::getenv("OCM_NONDUMPABLE"); nd && std::strcmp(nd, "1") == 0) {
        // Hardening: no ptrace / core dumps, and /proc/<pid>/fd becomes root-only.
        // Apps still map host-tier slabs: they receive the memfds (MSG_SLAB_FD).
        if (prctl(PR_SET_DUMPABLE, 0, 0, 0, 0) != 0) OCM_WARN("prctl(PR_SET_DUMPABLE): %s", strerror(errno));
    }
    if (parse_nodefile(cfg_.nodefile, &nf_, &err) != 0) {
        OCM_ERR("%s", err.c_str());
        return -1;
    }
    rank_ = resolve_rank(nf_, cfg_.rank, &err);
    if (rank_ < 0) {
        OCM_ERR("%s", err.c_str());
        return -1;
    }
    n_ = nf_.size();
    ns_ = cfg_.ns;
    parse_faults();
    const NodeEntry &me = nf_.nodes[rank_];

    // ---- GPU discovery ----
    int ndev = 0;
    if (cfg_.gpu != -1) {
        if (hipGetDeviceCount(&ndev) != hipSuccess) {
            (void)hipGetLastError();
            ndev = 0;
        }
    }
    num_gpu_ = ndev;
    if (cfg_.gpu >= 0)
        gpu_ = cfg_.gpu;
    else if (cfg_.gpu == -2 && me.gpu >= 0)
        gpu_ = me.gpu;
    else if (cfg_.gpu == -2 && ndev > 0)
        gpu_ = rank_ % ndev;
    else
        gpu_ = -1;
    if (gpu_ >= ndev) {
        OCM_ERR("gpu %d requested but only %d visible", gpu_, ndev);
        return -1;
    }
    ArenaConfig ac;
    ac.gpu = gpu_;
    ac.numa_node = gpu_numa_node(gpu_);
    if (const char *v = std::getenv("OCM_HOST_NUMA")) ac.numa_node = std::atoi(v);  // -1: no policy
    ac.slab_bytes = cfg_.slab_bytes;
    ac.zero_on_alloc = cfg_.zero_on_alloc;
    if (gpu_ >= 0) {
        size_t free_b = 0, total_b = 0;
        (void)hipSetDevice(gpu_);
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
            OCM_ERR("hipMemGetInfo failed on gpu %d", gpu_);
            return -1;
        }
        gpu_total_ = total_b;
        ac.gpu_capacity = cfg_.gpu_capacity ? cfg_.gpu_capacity : (uint64_t)((double)free_b * cfg_.gpu_fraction);
    }
    int local_daemons = 0;
    for (auto &e : nf_.nodes) local_daemons += (e.dns == me.dns);
    ac.host_capacity = cfg_.host_capacity
                           ? cfg_.host_capacity
                           : (uint64_t)((double)mem_available() * cfg_.host_fraction / std::max(1, local_daemons));
    arena_ = std::make_unique<Arena>(ac);
    {
        uint64_t tok = 0;
        std::ifstream ur("/dev/urandom", std::ios::binary);
        ur.read(reinterpret_cast<char *>(&tok), sizeof(tok));
        data_token_ = tok ? tok : ((uint64_t)getpid() << 20) ^ (uint64_t)now_ms();
    }
    data_ = std::make_unique<DataServer>(arena_.get(), gpu_, data_token_);
    // The nodefile's 5th column (the reference's rdmacm port) fixes the data
    // server's port, for firewalled clusters; 0 or out of range: ephemeral.
    const int want_port = nf_.nodes[rank_].data_port > 0 && nf_.nodes[rank_].data_port <= 65535
                              ? nf_.nodes[rank_].data_port
                              : 0;
    const std::string data_bind = cfg_.bind_ip.empty() ? "0.0.0.0" : cfg_.bind_ip;
    if (want_port && data_->start(data_bind, want_port) != 0) {
        OCM_WARN("rank %d: data port %d unavailable; using an ephemeral port", rank_, want_port);
        data_ = std::make_unique<DataServer>(arena_.get(), gpu_, data_token_);
        if (data_->start(data_bind) != 0) data_.reset();
    } else if (!want_port && data_->start(data_bind) != 0) {
        data_.reset();
    }
    if (!data_) {
        OCM_WARN("rank %d: network data server unavailable; cross-node placement disabled here", rank_);
        data_.reset();
    }
    if (gpu_ >= 0) {
        // The event loop next to its GPU, on the L3 complex its apps use (ocm/affinity.h);
        // the data server's threads (started above) keep the full mask.
        char bus[64] = {0};
        orig_cpus_ = thread_cpus();
        if (hipDeviceGetPCIBusId(bus, sizeof(bus), gpu_) == hipSuccess) {
            pinned_cpus_ = pin_near_gpu(bus, gpu_, PinRole::Daemon, rank_).size();
            if (pinned_cpus_) near_cpus_ = near_gpu_cpus(bus, gpu_, PinRole::App, rank_);
        }
        else
            (void)hipGetLastError();
    }
    {
        std::ifstream ur("/dev/urandom", std::ios::binary);
        ur.read(reinterpret_cast<char *>(&boot_id_), sizeof(boot_id_));
        if (!boot_id_) boot_id_ = ((uint64_t)getpid() << 32) ^ (uint64_t)now_ms();
    }
    {
        const std::string bind = cfg_.bind_ip.empty() ? "0.0.0.0" : cfg_.bind_ip;
        const bool loopback = bind.compare(0, 4, "127.") == 0 || bind == "::1" || bind == "localhost";
        if (cfg_.mesh_key.empty() && n_ == 1) {
            // No peer has to agree on it: a random secret keeps the port closed.
            uint64_t k = 0;
            std::ifstream ur("/dev/urandom", std::ios::binary);
            ur.read(reinterpret_cast<char *>(&k), sizeof(k));
            char hex[17];
            std::snprintf(hex, sizeof(hex), "%016llx", (unsigned long long)(k ^ boot_id_));
            cfg_.mesh_key = hex;
        } else if (cfg_.mesh_key.empty() && !loopback) {
            const char *insecure = std::getenv("OCM_MESH_INSECURE");
            if (!insecure || std::strcmp(insecure, "1") != 0) {
                OCM_ERR("rank %d: the mesh port binds %s but OCM_MESH_KEY is not set: anyone reaching it could "
                        "free or allocate memory. Set the same OCM_MESH_KEY on every daemon (or OCM_MESH_INSECURE=1 "
                        "on a trusted network)", rank_, bind.c_str());
                return -1;
            }
            OCM_WARN("rank %d: UNAUTHENTICATED mesh on %s (OCM_MESH_INSECURE=1, no OCM_MESH_KEY)", rank_, bind.c_str());
        }
        // HELLOs are signed with a key derived from namespace + shared key:
        // strangers on the mesh port cannot join, and a recorded HELLO cannot be replayed.
        mesh_key_ = sip_derive_key(ns_ + '\x1f' + cfg_.mesh_key);
    }
    if (rank_ == 0) {
        gov_ = std::make_unique<Governor>(n_, cfg_.policy, cfg_.stripe_unit);
        std::ifstream sf(cfg_.state_file.empty() ? std::string() : cfg_.state_file);
        if (sf) {
            // Resume: reload the directory; survivors rejoin and confirm what they hold.
            std::stringstream buf;
            buf << sf.rdbuf();
            std::string err;
            int n = gov_->restore(buf.str(), &err);
            if (n < 0) {
                OCM_WARN("rank 0: ignoring directory checkpoint %s: %s", cfg_.state_file.c_str(), err.c_str());
            } else {
                resumed_ = true;
                OCM_INFO("rank 0: resuming directory from %s (%d allocations, awaiting owner reports)",
                         cfg_.state_file.c_str(), n);
            }
        }
        saved_version_ = gov_->version();
    }
    table_.assign(n_, NodeConfig{});
    joined_.assign(n_, false);
    peer_fd_.assign(n_, -1);

    // ---- event loop plumbing ----
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    sigset_t mask;
    sigemptyset(&mask);
    sigaddset(&mask, SIGINT);
    sigaddset(&mask, SIGTERM);
    sigprocmask(SIG_BLOCK, &mask, nullptr);
    signal(SIGPIPE, SIG_IGN);
    sig_fd_ = signalfd(-1, &mask, SFD_CLOEXEC | SFD_NONBLOCK);
    ep_add(sig_fd_, EPOLLIN, tag(T_SIGNAL, 0));
    if (cfg_.watch_pid > 0) {
        int wfd = pidfd_open_compat(cfg_.watch_pid);
        if (wfd < 0) {
            OCM_ERR("--watch-pid %d: process not found", cfg_.watch_pid);
            return -1;
        }
        ep_add(wfd, EPOLLIN, tag(T_WATCH, 0));
    }

    if (mbox_alive(daemon_mailbox_name(rank_, ns_))) {
        OCM_ERR("another ocmd already serves rank %d in namespace %s", rank_, ns_.c_str());
        return -1;
    }
    mbox_fd_ = mbox_listen(daemon_mailbox_name(rank_, ns_));
    if (mbox_fd_ < 0) {
        OCM_ERR("cannot open daemon mailbox: %s", last_error());
        return -1;
    }
    ep_add(mbox_fd_, EPOLLIN, tag(T_MBOX, 0));

    listen_fd_ = tcp_listen(cfg_.bind_ip.empty() ? "0.0.0.0" : cfg_.bind_ip, me.ocm_port, 64);
    if (listen_fd_ < 0) {
        OCM_ERR("%s", last_error());
        return -1;
    }
    set_nonblocking(listen_fd_, true);
    ep_add(listen_fd_, EPOLLIN, tag(T_LISTEN, 0));

    // Mesh: connect to every lower rank; higher ranks connect to us.
    for (int r = 0; r < rank_; r++) {
        const NodeEntry &ne = nf_.nodes[r];
        int fd = tcp_connect(ne.ip, ne.ocm_port, cfg_.join_timeout_ms);
        if (fd < 0) {
            if (r == 0) {
                OCM_ERR("cannot reach rank0 at %s:%d (start the master first)", ne.ip.c_str(), ne.ocm_port);
                return -1;
            }
            OCM_WARN("rank %d unreachable; continuing without it", r);
            continue;
        }
        send_hello(fd, r);
        set_nonblocking(fd, true);
        auto c = std::make_unique<Conn>();
        c->fd = fd;
        c->peer_rank = r;
        peer_fd_[r] = fd;
        ep_add(fd, EPOLLIN, tag(T_CONN, (uint64_t)fd));
        conns_[fd] = std::move(c);
    }
    probe_links();
    if (const char *v = std::getenv("OCM_TICK_UP_MS"); v && *v) tick_up_ms_ = std::max(1, std::atoi(v));
    if (const char *v = std::getenv("OCM_TICK_IDLE_US"); v && *v) tick_idle_us_ = (uint32_t)std::max(0, std::min(std::atoi(v), 20000));
    if (rank_ == 0) resolve_ctrl();
    // Join: report our configuration to rank0 (reference notify_rank0, src/main.c:143-160).
    // With a tick transport possible, a peer first waits for rank0's decision so that
    // the join is the transport's first traffic (bounded by OCM_TICK_UP_MS).
    if (n_ > 1 && rank_ != 0 && cfg_.ctrl != "tcp") {
        join_deferred_ = true;
        tick_deadline_ms_ = now_ms() + tick_up_ms_;
    } else {
        join_rank0();
    }
    OCM_INFO("ocmd rank %d/%d up: gpu %d (%d visible, host tier on NUMA node %d), hbm capacity %.1f GiB, host tier %.1f GiB, policy %s, ns %s",
             rank_, n_, gpu_, num_gpu_, arena_->config().numa_node, (double)arena_->capacity(TIER_GPU) / (1 << 30),
             (double)arena_->capacity(TIER_HOST) / (1 << 30), policy_name(cfg_.policy), ns_.c_str());
    return 0;
}

void Daemon::check_ready() {
    if (ready_) return;
    for (int r = 0; r < n_; r++)
        if (!joined_[r]) return;
    ready_ = true;
    OCM_LOG("rank %d: mesh complete (%d nodes)", rank_, n_);
    if (rank_ == 0 && n_ == 1 && (cfg_.ctrl == "rccl" || cfg_.ctrl == "socket") && !resumed_) {
        // A single daemon only ticks when asked to (OCM_TICK_SELF tests: its own
        // records through a 1-rank communicator); meshes bootstrap at link-up.
        uint8_t uid[128] = {};
        std::string err;
        if (cfg_.ctrl == "rccl" && rccl_unique_id(uid, &err) != 0)
            OCM_WARN("rccl control plane unavailable (%s); staying on TCP", err.c_str());
        else
            start_tick(uid, cfg_.ctrl == "rccl", tick_idle_us_);
    }
    if (!cfg_.ready_file.empty()) {
        std::string tmp = cfg_.ready_file + ".tmp";
        std::ofstream f(tmp);
        f << "{\"rank\": " << rank_ << ", \"gpu\": " << gpu_ << ", \"pid\": " << getpid() << ", \"nodes\": " << n_
          << ", \"data_port\": " << (data_ ? data_->port() : 0) << "}\n";
        f.close();
        rename(tmp.c_str(), cfg_.ready_file.c_str());
    }
}

void Daemon::shutdown() {
    if (ep_ < 0) return;
    save_checkpoint(true);
    if (tick_) {
        tick_->stop();
        tick_.reset();
    }
    if (tick_bell_) {  // after the tick thread (and the collective that mapped it) is gone
        tick_bell_close(tick_bell_, ns_);
        tick_bell_ = nullptr;
    }
    if (data_) {
        data_->stop();
        data_.reset();
    }
    for (auto &kv : apps_) {
        if (kv.second.pidfd >= 0) close(kv.second.pidfd);
    }
    apps_.clear();
    for (auto &kv : app_conns_) close(kv.first);
    app_conns_.clear();
    if (mbox_fd_ >= 0) close(mbox_fd_);
    mbox_fd_ = -1;
    for (auto &kv : conns_) close(kv.first);
    conns_.clear();
    if (listen_fd_ >= 0) close(listen_fd_);
    listen_fd_ = -1;
    arena_.reset();
    if (sig_fd_ >= 0) close(sig_fd_);
    sig_fd_ = -1;
    close(ep_);
    ep_ = -1;
    if (!cfg_.ready_file.empty()) unlink(cfg_.ready_file.c_str());
}

int Daemon::run() {
    if (init() != 0) {
        shutdown();
        return 1;
    }
    int rc = loop();
    OCM_INFO("ocmd rank %d exiting (allocs %llu, frees %llu, reclaimed %llu)", rank_,
             (unsigned long long)n_alloc_, (unsigned long long)n_free_, (unsigned long long)n_reclaimed_);
    shutdown();
    return rc;
}

int Daemon::loop() {
    struct epoll_event evs[64];
    // Bounded post-activity polling: for spin_us after the last event the loop
    // polls epoll without sleeping, so the next record of a burst (an app's
    // alloc/free sequence, the owner's reply) skips the scheduler wake-up. Idle
    // daemons block as before; nothing spins without recent traffic.
    const uint64_t spin_ns = cfg_.spin_us > 0 ? (uint64_t)cfg_.spin_us * 1000 : 0;
    uint64_t last_event_ns = 0;
    while (!stop_) {
        while (!self_q_.empty() && !stop_) {
            Msg m = self_q_.front();
            self_q_.pop_front();
            handle_mesh_msg(m, -1);
        }
        if (stop_) break;
        save_checkpoint(false);
        if (r0_lost_) try_rejoin_rank0();
        int timeout = 1000;
        if (r0_lost_) timeout = 100;
        if (gov_ && !cfg_.state_file.empty() && gov_->version() != saved_version_) timeout = cfg_.state_interval_ms;
        // Apps' shared-memory links are looked at on every pass: while the loop
        // is awake (its post-activity spin) their requests need no wake-up.
        if (poll_links() > 0) last_event_ns = now_ns();
        if (tick_ && tick_->has_input()) {  // delivered by the tick thread: no epoll round
            on_tick();
            last_event_ns = now_ns();
        }
        if (!overflowed_apps_.empty()) reap_overflowed_apps();
        const bool spinning = spin_ns && now_ns() - last_event_ns < spin_ns;
        int wait_ms = (self_q_.empty() && !spinning) ? timeout : 0;
        // Replies waiting for room in an app's ring: the app frees slots
        // without waking us, so look again within a millisecond instead of sleeping
        // up to the loop timeout while it sleeps waiting for them.
        if (links_backlogged_ && wait_ms > 1) wait_ms = 1;
        if (wait_ms > 0) {
            // About to sleep: from here on an app that posts must wake us; look once more.
            links_polling(false);
            if (poll_links() > 0) {
                last_event_ns = now_ns();
                wait_ms = 0;
            } else if (links_backlogged_) {
                wait_ms = 1;
            }
        }
        int n = epoll_wait(ep_, evs, 64, wait_ms);
        links_polling(true);
        if (n > 0 && spin_ns) last_event_ns = now_ns();
        sweep_timeouts();
        check_tick_bootstrap();
        return_idle_leases();
        if (n < 0) {
            if (errno == EINTR) continue;
            OCM_ERR("epoll_wait: %s", strerror(errno));
            return 1;
        }
        for (int i = 0; i < n && !stop_; i++) {
            const uint64_t t = evs[i].data.u64;
            const uint32_t e = evs[i].events;
            switch (tag_kind(t)) {
            case T_MBOX: on_mailbox(); break;
            case T_LISTEN: on_accept(); break;
            case T_CONN:
                if (e & (EPOLLIN | EPOLLHUP | EPOLLERR)) on_conn_readable((int)tag_id(t));
                if ((e & EPOLLOUT) && conns_.count((int)tag_id(t))) on_conn_writable((int)tag_id(t));
                break;
            case T_PIDFD: on_pidfd((pid_t)tag_id(t)); break;
            case T_APPCONN: on_app_conn((int)tag_id(t), e); break;
            case T_SIGNAL: on_signal(); break;
            case T_TICK: on_tick(); break;
            case T_WATCH:
                OCM_INFO("rank %d: launcher %d exited; shutting down", rank_, cfg_.watch_pid);
                stop_ = true;
                break;
            default: break;
            }
        }
    }
    return 0;
}

// ---------------------------------------------------------------- sources

void Daemon::on_signal() {
    struct signalfd_siginfo si;
    while (read(sig_fd_, &si, sizeof(si)) == (ssize_t)sizeof(si)) {
        OCM_INFO("rank %d: signal %u, shutting down", rank_, si.ssi_signo);
        stop_ = true;
    }
}

void Daemon::on_mailbox() {
    for (;;) {
        pid_t peer = -1;
        int fd = mbox_accept(mbox_fd_, &peer);
        if (fd < 0) break;
        // Abstract sockets carry no file permissions: only our own user (or root)
        // may attach, allocate, free or stop us (OCM_ALLOW_ANY_UID=1 lifts this).
        static const bool any_uid = std::getenv("OCM_ALLOW_ANY_UID") != nullptr;
        const int uid = mbox_peer_uid(fd);
        if (!any_uid && uid != (int)geteuid() && uid != 0) {
            OCM_WARN("rank %d: refusing mailbox connection from uid %d (pid %d)", rank_, uid, (int)peer);
            close(fd);
            continue;
        }
        AppConn c;
        c.fd = fd;
        c.peer_pid = peer;
        c.same_user = uid == (int)geteuid() || uid == 0;
        app_conns_[fd] = c;
        ep_add(fd, EPOLLIN, tag(T_APPCONN, (uint64_t)fd));
    }
}

void Daemon::close_app_conn(int fd) {
    auto it = app_conns_.find(fd);
    if (it == app_conns_.end()) return;
    const pid_t pid = it->second.app_pid;
    ep_del(fd);
    close(fd);
    app_conns_.erase(it);
    auto ap = apps_.find(pid);
    if (pid && ap != apps_.end() && ap->second.fd == fd) {
        // The connection died with the app (or the app closed it without
        // MSG_DISCONNECT): reclaim exactly as for a crash.
        ap->second.fd = -1;
        OCM_INFO("rank %d: app %d went away without ocm_tini; reclaiming its memory", rank_, (int)pid);
        app_disconnect(pid, true);
    }
}

void Daemon::on_app_conn(int fd, uint32_t events) {
    auto it = app_conns_.find(fd);
    if (it == app_conns_.end()) return;
    if (events & EPOLLOUT) {
        auto ap = apps_.find(it->second.app_pid);
        if (ap != apps_.end()) {
            App &a = ap->second;
            while (!a.backlog.empty()) {
                int rc = mbox_send(fd, &a.backlog.front(), kMsgBytes, 0);
                if (rc != 1) break;
                a.backlog.pop_front();
            }
            if (a.backlog.empty() && a.watching_out) {
                ep_mod(fd, EPOLLIN, tag(T_APPCONN, (uint64_t)fd));
                a.watching_out = false;
            }
        }
    }
    if (!(events & (EPOLLIN | EPOLLHUP | EPOLLERR))) return;
    Msg m;
    for (int i = 0; i < 64; i++) {
        int passed = -1;
        int rc = mbox_recv_fd(fd, &m, kMsgBytes, &passed, 0);
        if (rc == 0) return;
        if (rc < 0) {
            if (passed >= 0) close(passed);
            close_app_conn(fd);
            return;
        }
        // Trust the kernel's view of who is talking, not the record.
        if (it->second.peer_pid > 0) m.pid = it->second.peer_pid;
        if (m.type == MSG_CONNECT) {
            it->second.app_pid = m.pid;
            pending_link_fd_ = passed;  // a shared-memory link, if the app offered one
            app_connect(m, fd);
            if (pending_link_fd_ >= 0) close(pending_link_fd_);
            pending_link_fd_ = -1;
            continue;
        }
        if (passed >= 0) close(passed);  // descriptors ride only with CONNECT
        if (m.type == MSG_SLAB_FD) {
            // Capability transfer of a host-tier slab to an app of our uid (checked at
            // accept): the memfd itself, so no /proc path (ptrace rules, hidepid) is needed.
            // Another user (OCM_ALLOW_ANY_UID) gets a slab only if one of its own
            // allocations lives there: a memfd opens the whole slab.
            bool allowed = it->second.same_user;
            for (auto oit = owned_.begin(); !allowed && oit != owned_.end(); ++oit)
                allowed = oit->second.slab_id == m.u.region.slab_id && oit->second.tier == TIER_HOST &&
                          oit->second.app_pid == m.pid;
            Msg r = m;
            r.status = MSG_RESPONSE;
            const int sfd = allowed && arena_ ? arena_->dup_slab_fd(m.u.region.slab_id) : -1;
            r.err = !allowed ? EACCES : sfd >= 0 ? 0 : ENOENT;
            // Never block the event loop: the app waits for this reply, so its queue has room;
            // if not, it times out and falls back to the /proc path.
            if (mbox_send_fd(fd, &r, kMsgBytes, sfd, 0) != 1) OCM_WARN("rank %d: slab fd reply to pid %d failed", rank_, (int)m.pid);
            if (sfd >= 0) close(sfd);
            continue;
        }
        handle_app_msg(m);
        it = app_conns_.find(fd);
        if (it == app_conns_.end()) return;
    }
}

void Daemon::on_accept() {
    for (;;) {
        int fd = tcp_accept(listen_fd_);
        if (fd < 0) break;
        set_nonblocking(fd, true);
        auto c = std::make_unique<Conn>();
        c->fd = fd;
        ep_add(fd, EPOLLIN, tag(T_CONN, (uint64_t)fd));
        conns_[fd] = std::move(c);
    }
}

void Daemon::drop_conn(int fd) {
    auto it = conns_.find(fd);
    if (it == conns_.end()) return;
    int r = it->second->peer_rank;
    ep_del(fd);
    close(fd);
    conns_.erase(it);
    if (r >= 0 && r < n_ && peer_fd_[r] == fd) {
        peer_fd_[r] = -1;
        peer_lost(r);
    }
}

void Daemon::on_conn_readable(int fd) {
    auto it = conns_.find(fd);
    if (it == conns_.end()) return;
    std::vector<std::vector<uint8_t>> recs;
    int rc = conn_read_records(*it->second, kMsgBytes, recs);
    for (auto &r : recs) {
        if (!conns_.count(fd)) return;  // dropped while handling an earlier record
        Msg m;
        std::memcpy(&m, r.data(), kMsgBytes);
        handle_mesh_msg(m, fd);
    }
    if (rc != 0) drop_conn(fd);
}

void Daemon::on_conn_writable(int fd) {
    auto it = conns_.find(fd);
    if (it == conns_.end()) return;
    if (conn_flush(*it->second) != 0) {
        drop_conn(fd);
        return;
    }
    if (!it->second->want_write) ep_mod(fd, EPOLLIN, tag(T_CONN, (uint64_t)fd));
}

void Daemon::on_pidfd(pid_t pid) {
    OCM_INFO("rank %d: app %d exited without ocm_tini; reclaiming its memory", rank_, (int)pid);
    app_disconnect(pid, true);
}

// ---------------------------------------------------------------- routing

void Daemon::send_rank(int r, Msg &m) {
    m.src_rank = rank_;
    // OCM_TICK_SELF=1 (tests): self-addressed records also ride the tick
    // transport, so a 1-GPU box exercises the real ncclAllGather path.
    static const bool tick_self = std::getenv("OCM_TICK_SELF") != nullptr;
    if (r == rank_ && !(tick_self && tick_ && tick_->up())) {
        self_q_.push_back(m);
        return;
    }
    if (tick_ && tick_->up() && r >= 0 && r < n_ && tick_->post(r, m)) return;
    if (r == rank_) {
        self_q_.push_back(m);
        return;
    }
    send_tcp(r, m);
}

void Daemon::send_tcp(int r, Msg &m) {
    m.src_rank = rank_;
    if (r < 0 || r >= n_ || peer_fd_[r] < 0) {
        OCM_WARN("rank %d: no link to rank %d for %s", rank_, r, msg_type_str(m.type));
        // Bounce the request back as a local failure so the origin can answer the app.
        if ((m.status & ~kMsgResent) == MSG_REQUEST &&
            (m.type == MSG_REQ_ALLOC || m.type == MSG_DO_ALLOC || m.type == MSG_DO_FREE || m.type == MSG_STATS)) {
            Msg f = m;
            f.status = MSG_RESPONSE;
            f.err = EHOSTDOWN;
            f.src_rank = r;
            if (f.type == MSG_DO_ALLOC && rank_ == 0 && f.rank != rank_) {
                send_rank(f.rank, f);
                return;
            }
            if (f.type == MSG_REQ_ALLOC) f.type = MSG_DO_ALLOC;
            self_q_.push_back(f);
        }
        return;
    }
    int fd = peer_fd_[r];
    Conn &c = *conns_[fd];
    if (conn_write(c, &m, sizeof(m)) != 0) {
        drop_conn(fd);
        return;
    }
    if (c.want_write) ep_mod(fd, EPOLLIN | EPOLLOUT, tag(T_CONN, (uint64_t)fd));
}

void Daemon::app_overflowed(App &a) {
    if (a.overflowed) return;
    a.overflowed = true;
    OCM_WARN("rank %d: app %d does not take its replies (%zu queued); disconnecting it", rank_, (int)a.pid,
             kAppBacklogMax);
    overflowed_apps_.push_back(a.pid);
}

void Daemon::reap_overflowed_apps() {
    // Outside any handler: closing the connection reclaims the app's memory.
    std::vector<pid_t> pids;
    pids.swap(overflowed_apps_);
    for (pid_t pid : pids) {
        auto it = apps_.find(pid);
        if (it == apps_.end() || !it->second.overflowed) continue;
        if (it->second.fd >= 0) close_app_conn(it->second.fd);
        else app_disconnect(pid, true);
    }
}

int Daemon::poll_links() {
    int n = 0;
    links_backlogged_ = 0;
    link_pids_.clear();
    for (auto &kv : apps_)
        if (kv.second.link) link_pids_.push_back(kv.first);
    for (pid_t pid : link_pids_) {
        auto it = apps_.find(pid);
        if (it == apps_.end() || !it->second.link) continue;
        std::shared_ptr<ShmLink> link = it->second.link;  // stays mapped if the app goes away meanwhile
        App &a = it->second;
        bool wake = false;
        while (!a.link_backlog.empty() && link->post_reply(a.link_backlog.front())) {
            a.link_backlog.pop_front();
            wake = true;
        }
        if (wake && link->reply_needs_wake()) {
            Msg w;
            std::memset(&w, 0, sizeof(w));
            w.type = MSG_WAKE;
            w.pid = pid;
            w.rank = rank_;
            send_app(pid, w);
        }
        if (!a.link_backlog.empty()) links_backlogged_++;
        Msg m;
        for (int i = 0; i < 64 && link->take_request(&m); i++) {
            m.pid = pid;  // the connection's SO_PEERCRED pid, never the record's
            n++;
            if (m.type == MSG_CONNECT || m.type == MSG_SLAB_FD || m.type == MSG_WAKE) continue;  // socket-only records
            handle_app_msg(m);
            if (!apps_.count(pid)) break;  // it disconnected
        }
    }
    return n;
}

void Daemon::links_polling(bool on) {
    if (links_polling_ == on) return;
    links_polling_ = on;
    for (auto &kv : apps_)
        if (kv.second.link) kv.second.link->set_daemon_polling(on);
}

void Daemon::send_app(pid_t pid, const Msg &m) {
    auto it = apps_.find(pid);
    if (it == apps_.end() || it->second.fd < 0) return;
    App &a = it->second;
    if (a.link && m.type != MSG_WAKE) {
        // Replies ride the app's shared-memory link, in order; the socket only wakes it.
        if (a.link_backlog.empty() && a.link->post_reply(m)) {
            if (a.link->reply_needs_wake()) {
                Msg w;
                std::memset(&w, 0, sizeof(w));
                w.type = MSG_WAKE;
                w.pid = pid;
                w.rank = rank_;
                send_app(pid, w);
            }
        } else if (a.link_backlog.size() < kAppBacklogMax) {
            a.link_backlog.push_back(m);  // drained by poll_links
        } else {
            app_overflowed(a);
        }
        return;
    }
    if (a.backlog.size() >= kAppBacklogMax) {
        app_overflowed(a);
        return;
    }
    if (a.backlog.empty()) {
        int rc = mbox_send(a.fd, &m, kMsgBytes, 0);
        if (rc == 1) return;
        if (rc < 0) {
            OCM_WARN("send to app %d failed: %s", (int)pid, last_error());
            return;
        }
    }
    a.backlog.push_back(m);
    if (!a.watching_out) {
        ep_mod(a.fd, EPOLLIN | EPOLLOUT, tag(T_APPCONN, (uint64_t)a.fd));
        a.watching_out = true;
    }
}


}  // namespace ocm
