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

namespace ocm {

namespace {

enum Tag : uint64_t { T_MBOX = 1, T_LISTEN, T_CONN, T_PIDFD, T_APPCONN, T_SIGNAL, T_TICK, T_WATCH };
inline uint64_t tag(Tag k, uint64_t id) { return (static_cast<uint64_t>(k) << 56) | (id & 0x00ffffffffffffffull); }
inline Tag tag_kind(uint64_t t) { return static_cast<Tag>(t >> 56); }
inline uint64_t tag_id(uint64_t t) { return t & 0x00ffffffffffffffull; }

long now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1000L + ts.tv_nsec / 1000000L;
}

int pidfd_open_compat(pid_t pid) { return (int)syscall(SYS_pidfd_open, pid, 0); }

bool is_remote_kind(uint32_t kind) {
    return kind == OCM_REMOTE_GPU || kind == OCM_REMOTE_RDMA || kind == OCM_REMOTE_RMA;
}

uint64_t parse_bytes(const std::string &s) {
    char *end = nullptr;
    double v = std::strtod(s.c_str(), &end);
    std::string suf = end ? end : "";
    uint64_t mul = 1;
    if (suf == "K" || suf == "KiB" || suf == "k") mul = 1ull << 10;
    else if (suf == "M" || suf == "MiB") mul = 1ull << 20;
    else if (suf == "G" || suf == "GiB") mul = 1ull << 30;
    else if (suf == "T" || suf == "TiB") mul = 1ull << 40;
    return (uint64_t)(v * (double)mul);
}

uint64_t mem_available() {
    std::ifstream f("/proc/meminfo");
    std::string k;
    uint64_t v;
    std::string unit;
    while (f >> k >> v >> unit)
        if (k == "MemAvailable:") return v * 1024ull;
    return 0;
}

}  // namespace

int parse_daemon_args(int argc, char **argv, DaemonConfig *cfg, std::string *err) {
    auto env = [](const char *k) -> const char * {
        const char *v = std::getenv(k);
        return (v && *v) ? v : nullptr;
    };
    if (const char *v = env("OCM_NODEFILE")) cfg->nodefile = v;
    if (const char *v = env("OCM_PLACEMENT")) cfg->policy = parse_policy(v, cfg->policy);
    if (const char *v = env("OCM_STRIPE_UNIT")) cfg->stripe_unit = parse_bytes(v);
    if (const char *v = env("OCM_SLAB_BYTES")) cfg->slab_bytes = parse_bytes(v);
    if (const char *v = env("OCM_GPU_CAPACITY")) cfg->gpu_capacity = parse_bytes(v);
    if (const char *v = env("OCM_HOST_CAPACITY")) cfg->host_capacity = parse_bytes(v);
    if (const char *v = env("OCM_GPU_FRACTION")) cfg->gpu_fraction = std::atof(v);
    if (const char *v = env("OCM_HOST_FRACTION")) cfg->host_fraction = std::atof(v);
    if (env("OCM_ZERO_ON_ALLOC")) cfg->zero_on_alloc = true;
    if (env("OCM_NO_GPU")) cfg->gpu = -1;
    if (const char *v = env("OCM_CTRL")) cfg->ctrl = v;
    if (const char *v = env("OCM_LEASE_BYTES")) cfg->lease_bytes = parse_bytes(v);
    if (const char *v = env("OCM_LEASE_AFTER")) cfg->lease_after = std::atoi(v);
    if (env("OCM_LEASE_HOST")) cfg->lease_host = true;
    if (const char *v = env("OCM_LEASE_IDLE_MS")) cfg->lease_idle_ms = std::atoi(v);
    if (const char *v = env("OCM_HOST_ALIAS")) cfg->host_alias = v;
    if (const char *v = env("OCM_STATE_FILE")) cfg->state_file = v;
    if (const char *v = env("OCM_MESH_KEY")) cfg->mesh_key = v;
    if (const char *v = env("OCM_STATE_INTERVAL_MS")) cfg->state_interval_ms = std::atoi(v);
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto val = [&](std::string *out) {
            if (i + 1 >= argc) {
                *err = "missing value for " + a;
                return false;
            }
            *out = argv[++i];
            return true;
        };
        std::string v;
        if (a == "--rank") {
            if (!val(&v)) return -1;
            cfg->rank = std::atoi(v.c_str());
        } else if (a == "--gpu") {
            if (!val(&v)) return -1;
            cfg->gpu = (v == "none" || v == "cpu") ? -1 : std::atoi(v.c_str());
        } else if (a == "--ns") {
            if (!val(&cfg->ns)) return -1;
        } else if (a == "--policy") {
            if (!val(&v)) return -1;
            cfg->policy = parse_policy(v, cfg->policy);
        } else if (a == "--stripe-unit") {
            if (!val(&v)) return -1;
            cfg->stripe_unit = parse_bytes(v);
        } else if (a == "--slab-bytes") {
            if (!val(&v)) return -1;
            cfg->slab_bytes = parse_bytes(v);
        } else if (a == "--gpu-capacity") {
            if (!val(&v)) return -1;
            cfg->gpu_capacity = parse_bytes(v);
        } else if (a == "--host-capacity") {
            if (!val(&v)) return -1;
            cfg->host_capacity = parse_bytes(v);
        } else if (a == "--join-timeout-ms") {
            if (!val(&v)) return -1;
            cfg->join_timeout_ms = std::atoi(v.c_str());
        } else if (a == "--ready-file") {
            if (!val(&cfg->ready_file)) return -1;
        } else if (a == "--bind") {
            if (!val(&cfg->bind_ip)) return -1;
        } else if (a == "--ctrl") {
            if (!val(&cfg->ctrl)) return -1;
            if (cfg->ctrl != "tcp" && cfg->ctrl != "rccl" && cfg->ctrl != "socket") {
                *err = "--ctrl must be tcp, rccl or socket";
                return -1;
            }
        } else if (a == "--host-alias") {
            if (!val(&cfg->host_alias)) return -1;
        } else if (a == "--state-file") {
            if (!val(&cfg->state_file)) return -1;
        } else if (a == "--lease-bytes") {
            if (!val(&v)) return -1;
            cfg->lease_bytes = parse_bytes(v);
        } else if (a == "--watch-pid") {
            if (!val(&v)) return -1;
            cfg->watch_pid = std::atoi(v.c_str());
        } else if (a == "--zero") {
            cfg->zero_on_alloc = true;
        } else if (!a.empty() && a[0] == '-') {
            *err = "unknown option " + a;
            return -1;
        } else {
            cfg->nodefile = a;
        }
    }
    if (cfg->nodefile.empty()) {
        *err = "usage: ocmd <nodefile> [--rank R] [--gpu G|none] [--ns NS] [--policy ring|least_loaded|stripe|loopback]";
        return -1;
    }
    if (cfg->ns.empty()) cfg->ns = pmsg_namespace();
    return 0;
}

Daemon::Daemon(const DaemonConfig &cfg) : cfg_(cfg) {}

Daemon::~Daemon() { shutdown(); }

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
    c.num_nodes = (uint32_t)n_;
    c.num_apps = (uint32_t)apps_.size();
    c.n_alloc = (uint32_t)n_alloc_;
    c.n_free = (uint32_t)n_free_;
    c.n_reclaimed = (uint32_t)n_reclaimed_;
    c.n_spilled = (uint32_t)(gov_ ? gov_->spilled_count() : n_spilled_);
    c.n_slabs = (uint32_t)(arena_ ? arena_->num_slabs() : 0);
    c.ticks = (uint32_t)(tick_ ? tick_->ticks() : 0);
    for (auto &l : leases_) c.n_leases += l != nullptr;
    c.lease_allocs = (uint32_t)n_lease_allocs_;
    return c;
}

int Daemon::init() {
    std::string err;
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
    if (data_->start(cfg_.bind_ip.empty() ? "0.0.0.0" : cfg_.bind_ip) != 0) {
        OCM_WARN("rank %d: network data server unavailable; cross-node placement disabled here", rank_);
        data_.reset();
    }
    {
        std::ifstream ur("/dev/urandom", std::ios::binary);
        ur.read(reinterpret_cast<char *>(&boot_id_), sizeof(boot_id_));
        if (!boot_id_) boot_id_ = ((uint64_t)getpid() << 32) ^ (uint64_t)now_ms();
    }
    {
        // FNV-1a over namespace + shared key: strangers on the mesh port cannot join.
        uint64_t h = 1469598103934665603ull;
        for (char ch : ns_ + '\x1f' + cfg_.mesh_key) h = (h ^ (uint8_t)ch) * 1099511628211ull;
        mesh_token_ = h ? h : 1;
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
        send_hello(fd);
        set_nonblocking(fd, true);
        auto c = std::make_unique<Conn>();
        c->fd = fd;
        c->peer_rank = r;
        peer_fd_[r] = fd;
        ep_add(fd, EPOLLIN, tag(T_CONN, (uint64_t)fd));
        conns_[fd] = std::move(c);
    }
    // Join: report our configuration to rank0 (reference notify_rank0, src/main.c:143-160).
    join_rank0();
    OCM_INFO("ocmd rank %d/%d up: gpu %d (%d visible), hbm capacity %.1f GiB, host tier %.1f GiB, policy %s, ns %s",
             rank_, n_, gpu_, num_gpu_, (double)arena_->capacity(TIER_GPU) / (1 << 30),
             (double)arena_->capacity(TIER_HOST) / (1 << 30), policy_name(cfg_.policy), ns_.c_str());
    return 0;
}

void Daemon::send_hello(int fd) {
    Msg hello;
    std::memset(&hello, 0, sizeof(hello));
    hello.type = MSG_HELLO;
    hello.src_rank = rank_;
    hello.rank = rank_;
    hello.seq = mesh_token_;
    send_all(fd, &hello, sizeof(hello));
}

void Daemon::join_rank0() {
    Msg add;
    std::memset(&add, 0, sizeof(add));
    add.type = MSG_ADD_NODE;
    add.status = MSG_REQUEST;
    add.rank = rank_;
    add.seq = boot_id_;
    add.u.node = my_config();
    send_rank(0, add);
    // What we hold (empty on first boot): lets a restarted rank0 rebuild its directory.
    for (auto &kv : owned_) {
        const OwnedExtent &oe = kv.second;
        Msg o;
        std::memset(&o, 0, sizeof(o));
        o.type = MSG_OWNED;
        o.status = MSG_REQUEST;
        o.rank = rank_;
        o.pid = oe.app_pid;
        Region &rg = o.u.region;
        rg.alloc_id = kv.first.first;
        rg.extent_idx = (uint16_t)kv.first.second;
        rg.n_extents = oe.n_extents;
        rg.bytes = oe.bytes;
        rg.offset = oe.offset;
        rg.slab_id = oe.slab_id;
        rg.stripe_unit = oe.stripe_unit;
        rg.owner_rank = rank_;
        rg.orig_rank = oe.orig_rank;
        rg.tier = (uint16_t)oe.tier;
        rg.flags = oe.flags;
        send_rank(0, o);
    }
    Msg done;
    std::memset(&done, 0, sizeof(done));
    done.type = MSG_OWNED_DONE;
    done.status = MSG_REQUEST;
    done.rank = rank_;
    done.seq = owned_.size();
    send_rank(0, done);
}

void Daemon::try_rejoin_rank0() {
    const long now = now_ms();
    if (now < next_rejoin_ms_) return;
    next_rejoin_ms_ = now + 100;
    const NodeEntry &ne = nf_.nodes[0];
    int fd = tcp_connect(ne.ip, ne.ocm_port, 50);
    if (fd < 0) return;
    send_hello(fd);
    set_nonblocking(fd, true);
    auto c = std::make_unique<Conn>();
    c->fd = fd;
    c->peer_rank = 0;
    peer_fd_[0] = fd;
    ep_add(fd, EPOLLIN, tag(T_CONN, (uint64_t)fd));
    conns_[fd] = std::move(c);
    r0_lost_ = false;
    OCM_INFO("rank %d: reconnected to rank 0; reporting %zu owned extents", rank_, owned_.size());
    join_rank0();
}

void Daemon::save_checkpoint(bool force) {
    if (!gov_ || cfg_.state_file.empty()) return;
    const uint64_t v = gov_->version();
    if (v == saved_version_) return;
    const long now = now_ms();
    if (!force && now - last_save_ms_ < cfg_.state_interval_ms) return;
    const std::string tmp = cfg_.state_file + ".tmp";
    {
        std::ofstream f(tmp, std::ios::trunc);
        f << gov_->checkpoint();
        if (!f) {
            OCM_WARN("rank 0: cannot write directory checkpoint %s", tmp.c_str());
            return;
        }
    }
    if (rename(tmp.c_str(), cfg_.state_file.c_str()) != 0) {
        OCM_WARN("rank 0: cannot publish directory checkpoint %s: %s", cfg_.state_file.c_str(), strerror(errno));
        return;
    }
    saved_version_ = v;
    last_save_ms_ = now;
}

void Daemon::check_ready() {
    if (ready_) return;
    for (int r = 0; r < n_; r++)
        if (!joined_[r]) return;
    ready_ = true;
    OCM_LOG("rank %d: mesh complete (%d nodes)", rank_, n_);
    if (rank_ == 0 && cfg_.ctrl != "tcp" && !resumed_) {
        // Bootstrap the tick transport (not after a resume: survivors stay on TCP): rank0 picks the RCCL id and tells everybody over TCP.
        Msg t;
        std::memset(&t, 0, sizeof(t));
        t.type = MSG_TICK_START;
        t.status = MSG_REQUEST;
        t.rank = 0;
        std::string err;
        if (cfg_.ctrl == "rccl" && rccl_unique_id(t.u.raw, &err) != 0) {
            OCM_WARN("rccl control plane unavailable (%s); staying on TCP", err.c_str());
        } else {
            for (int r = 1; r < n_; r++) send_tcp(r, t);
            start_tick(t.u.raw);
        }
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
        int n = epoll_wait(ep_, evs, 64, self_q_.empty() ? timeout : 0);
        sweep_timeouts();
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
        int rc = mbox_recv(fd, &m, kMsgBytes, 0);
        if (rc == 0) return;
        if (rc < 0) {
            close_app_conn(fd);
            return;
        }
        // Trust the kernel's view of who is talking, not the record.
        if (it->second.peer_pid > 0) m.pid = it->second.peer_pid;
        if (m.type == MSG_CONNECT) {
            it->second.app_pid = m.pid;
            app_connect(m, fd);
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
        if (m.status == MSG_REQUEST && (m.type == MSG_REQ_ALLOC || m.type == MSG_DO_ALLOC || m.type == MSG_DO_FREE ||
                                        m.type == MSG_STATS)) {
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

void Daemon::send_app(pid_t pid, const Msg &m) {
    auto it = apps_.find(pid);
    if (it == apps_.end() || it->second.fd < 0) return;
    App &a = it->second;
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

// ---------------------------------------------------------------- app messages

void Daemon::handle_app_msg(Msg &m) {
    TraceRange tr(msg_type_str(m.type));
    OCM_LOG("rank %d <- app %d: %s", rank_, m.pid, msg_type_str(m.type));
    if (m.type != MSG_CONNECT && m.type != MSG_SHUTDOWN && !apps_.count(m.pid)) {
        OCM_WARN("rank %d: %s from unknown app %d ignored", rank_, msg_type_str(m.type), m.pid);
        return;
    }
    switch (m.type) {
    case MSG_DISCONNECT: app_disconnect(m.pid, false); break;
    case MSG_REQ_ALLOC: app_req_alloc(m); break;
    case MSG_REQ_FREE: app_req_free(m); break;
    case MSG_STATS: app_stats(m); break;
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
        if (old.fd != fd) app_disconnect(pid, false);
    }
    App a;
    a.pid = pid;
    a.fd = fd;
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

// ---------------------------------------------------------------- mesh messages

void Daemon::handle_mesh_msg(Msg &m, int from_fd) {
    if (from_fd >= 0) {
        // An inbound link is anonymous until its HELLO carries our mesh token.
        auto it = conns_.find(from_fd);
        if (it == conns_.end()) return;
        if (it->second->peer_rank < 0 &&
            (m.type != MSG_HELLO || m.seq != mesh_token_ || m.src_rank < 0 || m.src_rank >= n_ || m.src_rank == rank_)) {
            OCM_WARN("rank %d: dropping unauthenticated mesh link (%s)", rank_, msg_type_str(m.type));
            drop_conn(from_fd);
            return;
        }
    }
    TraceRange tr(msg_type_str(m.type));
    OCM_LOG("rank %d <- rank %d: %s/%s seq %llu", rank_, m.src_rank, msg_type_str(m.type), msg_status_str(m.status),
            (unsigned long long)m.seq);
    switch (m.type) {
    case MSG_HELLO: {
        auto it = conns_.find(from_fd);
        if (it != conns_.end() && m.src_rank >= 0 && m.src_rank < n_) {
            it->second->peer_rank = m.src_rank;
            if (peer_fd_[m.src_rank] >= 0 && peer_fd_[m.src_rank] != from_fd) drop_conn(peer_fd_[m.src_rank]);
            peer_fd_[m.src_rank] = from_fd;
        }
        break;
    }
    case MSG_ADD_NODE:
        if (rank_ == 0) r0_add_node(m.u.node, m.seq);
        break;
    case MSG_OWNED:
        if (rank_ == 0 && gov_) gov_->confirm_extent(m.src_rank, m.u.region, m.pid);
        break;
    case MSG_OWNED_DONE:
        if (rank_ == 0 && gov_) {
            int dropped = gov_->end_reconcile(m.src_rank);
            if (m.seq || dropped)
                OCM_INFO("rank 0: rank %d confirmed %llu extents (%d stale entries dropped)", m.src_rank,
                         (unsigned long long)m.seq, dropped);
        }
        break;
    case MSG_NODE_TABLE: {
        const NodeConfig &c = m.u.node;
        if (c.rank >= 0 && c.rank < n_) {
            table_[c.rank] = c;
            joined_[c.rank] = true;
            check_ready();
        }
        break;
    }
    case MSG_REQ_ALLOC:
        if (rank_ == 0) r0_req_alloc(m);
        break;
    case MSG_PLACE_FAIL:
        if (rank_ == 0) r0_place_fail(m);
        break;
    case MSG_DO_ALLOC:
        if (m.status == MSG_REQUEST)
            owner_do_alloc(m);
        else
            origin_do_alloc_resp(m);
        break;
    case MSG_DO_FREE:
        if (m.status == MSG_REQUEST)
            owner_do_free(m);
        else
            origin_do_free_resp(m);
        break;
    case MSG_FREED:
        if (rank_ == 0 && gov_) gov_->release(m.u.region.alloc_id);
        break;
    case MSG_STATS:
        if (m.status == MSG_REQUEST) {
            Msg r = m;
            r.status = MSG_RESPONSE;
            r.u.node = my_config();
            send_rank(m.rank, r);
        } else {
            auto it = pending_.find(m.seq);
            if (it == pending_.end()) break;
            Msg r = m;
            r.type = MSG_RELEASE_APP;
            r.status = MSG_RESPONSE;
            r.pid = it->second.pid;
            r.seq = it->second.app_seq;
            if (it->second.pid) send_app(it->second.pid, r);
            pending_.erase(it);
        }
        break;
    case MSG_TICK_START:
        if (!tick_ && cfg_.ctrl != "tcp") start_tick(m.u.raw);
        break;
    case MSG_TICK_WAKE:
        if (tick_) tick_->wake_at(m.u.req.bytes);
        break;
    case MSG_SHUTDOWN: stop_ = true; break;
    case MSG_PING:
        if (m.status == MSG_REQUEST) {
            Msg r = m;
            r.status = MSG_RESPONSE;
            send_rank(m.src_rank, r);
        }
        break;
    default: OCM_WARN("rank %d: unexpected mesh message %s", rank_, msg_type_str(m.type)); break;
    }
}

void Daemon::r0_add_node(const NodeConfig &cfg, uint64_t boot_id) {
    if (cfg.rank < 0 || cfg.rank >= n_) return;
    gov_->add_node(cfg, boot_id);
    table_[cfg.rank] = cfg;
    joined_[cfg.rank] = true;
    // Fan the directory out: the newcomer gets the whole table, everybody else the newcomer.
    for (int r = 0; r < n_; r++) {
        if (!joined_[r]) continue;
        Msg t;
        std::memset(&t, 0, sizeof(t));
        t.type = MSG_NODE_TABLE;
        t.status = MSG_RESPONSE;
        t.rank = 0;
        if (r == cfg.rank) {
            for (int k = 0; k < n_; k++) {
                if (!joined_[k] || k == 0) continue;  // rank0 learns from itself below
                t.u.node = table_[k];
                if (r != 0) send_rank(r, t);
            }
            if (r != 0) {
                t.u.node = my_config();
                send_rank(r, t);
            }
        } else if (r != 0) {
            t.u.node = cfg;
            send_rank(r, t);
        }
    }
    if (cfg.rank == 0) table_[0] = my_config();
    check_ready();
}

void Daemon::r0_req_alloc(Msg &m) {
    PlaceRequest pr;
    pr.orig_rank = m.u.req.orig_rank;
    pr.remote_rank = m.u.req.remote_rank;
    pr.bytes = m.u.req.bytes;
    pr.flags = m.u.req.flags;
    pr.stripe_width = m.u.req.stripe_width;
    pr.stripe_unit = m.u.req.stripe_unit;
    pr.remote = true;
    pr.app_pid = m.u.req.app_pid;
    Placement p = gov_->place(pr);
    if (p.err) {
        Msg r;
        std::memset(&r, 0, sizeof(r));
        r.type = MSG_DO_ALLOC;
        r.status = MSG_RESPONSE;
        r.rank = m.rank;
        r.seq = m.seq;
        r.err = p.err;
        r.u.region.n_extents = 0;
        send_rank(m.rank, r);
        return;
    }
    for (size_t i = 0; i < p.extents.size(); i++) {
        const PlacedExtent &e = p.extents[i];
        Msg d;
        std::memset(&d, 0, sizeof(d));
        d.type = MSG_DO_ALLOC;
        d.status = MSG_REQUEST;
        d.pid = m.pid;
        d.rank = m.rank;  // origin daemon: responses go there
        d.seq = m.seq;
        Region &rg = d.u.region;
        rg.alloc_id = p.alloc_id;
        rg.bytes = e.bytes;
        rg.stripe_unit = p.stripe_unit;
        rg.owner_rank = e.owner;
        rg.orig_rank = m.rank;
        rg.tier = (uint16_t)e.tier;
        rg.flags = (uint16_t)((e.spilled ? REGION_SPILLED : 0) | (cross_host(m.rank, e.owner) ? REGION_NET : 0));
        rg.extent_idx = (uint16_t)i;
        rg.n_extents = (uint16_t)p.extents.size();
        send_rank(e.owner, d);
    }
}

void Daemon::r0_place_fail(Msg &m) {
    Region rg = m.u.region;
    PlacedExtent e;
    if (gov_->replace_extent(rg.alloc_id, rg.extent_idx, rg.owner_rank, &e)) {
        Msg d = m;
        d.type = MSG_DO_ALLOC;
        d.status = MSG_REQUEST;
        d.err = 0;
        d.u.region.owner_rank = e.owner;
        d.u.region.tier = (uint16_t)e.tier;
        d.u.region.flags =
            (uint16_t)((e.spilled ? REGION_SPILLED : 0) | (cross_host(m.rank, e.owner) ? REGION_NET : 0));
        OCM_LOG("re-placing alloc %llu extent %d on rank %d tier %u", (unsigned long long)rg.alloc_id,
                rg.extent_idx, e.owner, e.tier);
        send_rank(e.owner, d);
        return;
    }
    Msg r = m;
    r.type = MSG_DO_ALLOC;
    r.status = MSG_RESPONSE;
    r.err = ENOMEM;
    send_rank(m.rank, r);
}

void Daemon::parse_faults() {
    const char *f = std::getenv("OCM_FAULT");
    if (const char *t = std::getenv("OCM_REQUEST_TIMEOUT_MS")) request_timeout_ms_ = std::atoi(t);
    if (!f || !*f) return;
    std::string spec = f;
    size_t pos = 0;
    while (pos < spec.size()) {
        size_t end = spec.find(',', pos);
        std::string item = spec.substr(pos, end == std::string::npos ? std::string::npos : end - pos);
        size_t eq = item.find('=');
        std::string k = item.substr(0, eq);
        int v = eq == std::string::npos ? 1 : std::atoi(item.c_str() + eq + 1);
        if (k == "do_alloc_fail") fault_alloc_fail_ = v;
        else if (k == "drop_do_alloc") fault_drop_alloc_ = v;
        else if (k == "crash_after_allocs") fault_crash_after_ = v;
        else OCM_WARN("unknown OCM_FAULT item '%s'", item.c_str());
        if (end == std::string::npos) break;
        pos = end + 1;
    }
    OCM_INFO("rank %d: fault injection: do_alloc_fail=%d drop_do_alloc=%d crash_after_allocs=%d", rank_,
             fault_alloc_fail_, fault_drop_alloc_, fault_crash_after_);
}

void Daemon::owner_do_alloc(Msg &m) {
    Region rg = m.u.region;
    if (fault_drop_alloc_ > 0) {
        fault_drop_alloc_--;
        OCM_WARN("rank %d: fault injection: dropping DO_ALLOC for alloc %llu", rank_, (unsigned long long)rg.alloc_id);
        return;
    }
    if (fault_crash_after_ == 0) {
        OCM_WARN("rank %d: fault injection: crashing", rank_);
        _exit(3);
    }
    if (fault_crash_after_ > 0) fault_crash_after_--;
    int err = fault_alloc_fail_ > 0 ? (fault_alloc_fail_--, ENOMEM) : arena_->alloc(rg.tier, rg.bytes, &rg);
    if (err) {
        OCM_LOG("rank %d: DO_ALLOC %llu bytes tier %u failed (%d)", rank_, (unsigned long long)rg.bytes, rg.tier, err);
        Msg f = m;
        f.type = MSG_PLACE_FAIL;
        f.status = MSG_REQUEST;
        f.err = err;
        f.u.region.owner_rank = rank_;
        send_rank(0, f);
        return;
    }
    rg.owner_rank = rank_;
    if (rg.flags & REGION_NET) {
        if (!data_) {
            arena_->free(rg.slab_id, rg.offset);
            Msg f = m;
            f.type = MSG_PLACE_FAIL;
            f.status = MSG_REQUEST;
            f.err = ENETUNREACH;
            f.u.region.owner_rank = rank_;
            send_rank(0, f);
            return;
        }
        // Other node: the app streams through our data server instead of mapping the slab.
        std::memset(rg.handle, 0, sizeof(rg.handle));
        std::snprintf(reinterpret_cast<char *>(rg.handle), sizeof(rg.handle), "net:%s:%d:%llx",
                      nf_.nodes[rank_].ip.c_str(), data_->port(), (unsigned long long)data_token_);
        rg.flags = (uint16_t)(rg.flags & ~REGION_DEDICATED);
    }
    OwnedExtent oe;
    oe.slab_id = rg.slab_id;
    oe.offset = rg.offset;
    oe.tier = rg.tier;
    oe.orig_rank = rg.orig_rank;
    oe.bytes = rg.bytes;
    oe.app_pid = m.pid;
    oe.flags = rg.flags;
    oe.n_extents = rg.n_extents ? rg.n_extents : 1;
    oe.stripe_unit = rg.stripe_unit;
    owned_[{rg.alloc_id, (int)rg.extent_idx}] = oe;
    if (rg.flags & REGION_SPILLED) n_spilled_++;
    Msg r = m;
    r.status = MSG_RESPONSE;
    r.err = 0;
    r.u.region = rg;
    send_rank(m.rank, r);
}

void Daemon::owner_do_free(Msg &m) {
    const Region &rg = m.u.region;
    auto it = owned_.find({rg.alloc_id, (int)rg.extent_idx});
    int err = ENOENT;
    if (it != owned_.end()) {
        err = arena_->free(it->second.slab_id, it->second.offset);
        owned_.erase(it);
    }
    Msg r = m;
    r.status = MSG_RESPONSE;
    r.err = err;
    send_rank(m.rank, r);
}

void Daemon::origin_do_alloc_resp(Msg &m) {
    auto it = pending_.find(m.seq);
    if (it == pending_.end()) {
        // Origin gave up (e.g. peer loss) but the owner allocated: give it back.
        if (!m.err && m.u.region.alloc_id) {
            Msg f;
            std::memset(&f, 0, sizeof(f));
            f.type = MSG_DO_FREE;
            f.status = MSG_REQUEST;
            f.rank = rank_;
            f.seq = 0;
            f.u.region = m.u.region;
            send_rank(m.u.region.owner_rank, f);
        }
        return;
    }
    Pending &p = it->second;
    const Region &rg = m.u.region;
    if (p.expect == 0) {
        // First response fixes the extent count (0 when rank0 refused the request).
        p.expect = rg.n_extents ? rg.n_extents : 1;
        p.extents.assign(p.expect, Region{});
        p.have.assign(p.expect, false);
        p.awaiting.clear();
    }
    if (m.err) p.err = p.err ? p.err : m.err;
    if (rg.n_extents == 0) {
        // rank0 refused: nothing was placed.
        p.got = p.expect;
    } else if (rg.extent_idx < p.expect && !p.have[rg.extent_idx]) {
        p.have[rg.extent_idx] = true;
        p.got++;
        if (!m.err) p.extents[rg.extent_idx] = rg;
        p.alloc_id = rg.alloc_id;
    }
    if (p.got >= p.expect) finish_alloc(p);
}

void Daemon::finish_alloc(Pending &p) {
    const uint64_t seq = p.seq;
    const uint64_t app_seq = p.app_seq;
    const pid_t pid = p.pid;
    if (p.lease_owner >= 0) {
        const int owner = p.lease_owner;
        lease_inflight_.erase(owner);
        if (!p.err && p.expect == 1 && p.have[0] && p.extents[0].tier == p.lease_tier) {
            auto l = std::make_unique<Lease>();
            l->owner = owner;
            l->tier = p.lease_tier;
            l->base = p.extents[0];
            l->ra.reset(l->base.bytes);
            l->idle_since_ms = now_ms();
            OCM_LOG("rank %d: leased %llu bytes of rank %d HBM", rank_, (unsigned long long)l->base.bytes, owner);
            leases_.push_back(std::move(l));
        } else if (p.err) {
            // Refused (no capacity): need much more demand before asking again.
            lease_demand_[owner] = -16 * std::max(1, cfg_.lease_after);
        } else if (p.expect >= 1) {
            // Not what we asked for (e.g. spilled): give it back.
            for (int i = 0; i < p.expect; i++) {
                if (!p.have[i]) continue;
                Msg f;
                std::memset(&f, 0, sizeof(f));
                f.type = MSG_DO_FREE;
                f.status = MSG_REQUEST;
                f.rank = rank_;
                f.u.region = p.extents[i];
                send_rank(p.extents[i].owner_rank, f);
            }
            Msg fr;
            std::memset(&fr, 0, sizeof(fr));
            fr.type = MSG_FREED;
            fr.u.region.alloc_id = p.alloc_id;
            send_rank(0, fr);
        }
        pending_.erase(seq);
        return;
    }
    if (p.err) {
        // Roll back the extents that did get memory.
        for (int i = 0; i < p.expect; i++) {
            if (!p.have[i] || p.extents[i].alloc_id == 0) continue;
            Msg f;
            std::memset(&f, 0, sizeof(f));
            f.type = MSG_DO_FREE;
            f.status = MSG_REQUEST;
            f.rank = rank_;
            f.seq = 0;
            f.u.region = p.extents[i];
            send_rank(p.extents[i].owner_rank, f);
        }
        if (p.alloc_id) {
            Msg fr;
            std::memset(&fr, 0, sizeof(fr));
            fr.type = MSG_FREED;
            fr.u.region.alloc_id = p.alloc_id;
            send_rank(0, fr);
        }
        if (pid && apps_.count(pid)) {
            Msg r;
            std::memset(&r, 0, sizeof(r));
            r.type = MSG_RELEASE_APP;
            r.status = MSG_RESPONSE;
            r.pid = pid;
            r.rank = rank_;
            r.seq = app_seq;
            r.err = p.err;
            send_app(pid, r);
        }
        pending_.erase(seq);
        return;
    }
    OriginAlloc oa;
    oa.pid = pid;
    oa.remote = true;
    oa.bytes = p.total_bytes;
    oa.extents = p.extents;
    const uint64_t id = p.alloc_id;
    if (oa.extents.size() == 1 && cfg_.lease_bytes && oa.extents[0].owner_rank != rank_ &&
        (oa.extents[0].tier == TIER_GPU || (cfg_.lease_host && oa.extents[0].tier == TIER_HOST)) &&
        !(oa.extents[0].flags & (REGION_SPILLED | REGION_NET)) &&
        ++lease_demand_[oa.extents[0].owner_rank] >= cfg_.lease_after)
        request_lease(oa.extents[0].owner_rank, oa.extents[0].tier);
    origin_allocs_[id] = oa;
    n_alloc_++;
    pending_.erase(seq);
    if (!pid || !apps_.count(pid)) {
        // The app vanished while we were allocating.
        start_free(id, 0, 0);
        n_reclaimed_++;
        return;
    }
    // Header + one EXTENT record per extent (a 160-byte record holds one region).
    Msg h;
    std::memset(&h, 0, sizeof(h));
    h.type = MSG_RELEASE_APP;
    h.status = MSG_RESPONSE;
    h.pid = pid;
    h.rank = rank_;
    h.seq = app_seq;
    h.u.region = oa.extents[0];
    h.u.region.bytes = oa.bytes;  // header carries the total
    send_app(pid, h);
    for (size_t i = 0; i < oa.extents.size(); i++) {
        Msg e;
        std::memset(&e, 0, sizeof(e));
        e.type = MSG_EXTENT;
        e.status = MSG_RESPONSE;
        e.pid = pid;
        e.rank = rank_;
        e.seq = app_seq;
        e.u.region = oa.extents[i];
        send_app(pid, e);
    }
}

void Daemon::start_free(uint64_t alloc_id, pid_t reply_pid, uint64_t reply_seq) {
    auto it = origin_allocs_.find(alloc_id);
    if (it == origin_allocs_.end()) return;
    OriginAlloc oa = it->second;
    origin_allocs_.erase(it);
    if (!oa.remote) {
        n_free_++;
        return;
    }
    if (oa.lease >= 0 && oa.lease < (int)leases_.size() && leases_[oa.lease]) {
        Lease &l = *leases_[oa.lease];
        l.ra.free(oa.extents[0].offset - l.base.offset);
        if (l.ra.used() == 0) l.idle_since_ms = now_ms();
        n_free_++;
        if (reply_pid && apps_.count(reply_pid)) {
            Msg r;
            std::memset(&r, 0, sizeof(r));
            r.type = MSG_RELEASE_APP;
            r.status = MSG_RESPONSE;
            r.pid = reply_pid;
            r.rank = rank_;
            r.seq = reply_seq;
            send_app(reply_pid, r);
        }
        return;
    }
    Pending p;
    p.seq = next_seq();
    p.pid = reply_pid;
    p.type = MSG_REQ_FREE;
    p.alloc_id = alloc_id;
    p.app_seq = reply_seq;
    p.t0_ms = now_ms();
    p.expect = (int)oa.extents.size();
    for (auto &e : oa.extents) p.awaiting.insert(e.owner_rank);
    pending_[p.seq] = p;
    for (auto &e : oa.extents) {
        Msg f;
        std::memset(&f, 0, sizeof(f));
        f.type = MSG_DO_FREE;
        f.status = MSG_REQUEST;
        f.rank = rank_;
        f.seq = p.seq;
        f.u.region = e;
        send_rank(e.owner_rank, f);
    }
}

void Daemon::origin_do_free_resp(Msg &m) {
    if (m.seq == 0) return;  // rollback frees need no answer
    auto it = pending_.find(m.seq);
    if (it == pending_.end()) return;
    Pending &p = it->second;
    p.got++;
    // A dead owner's memory is gone already: count it as freed.
    if (m.err && m.err != ENOENT && m.err != EHOSTDOWN) p.err = m.err;
    if (p.got < p.expect) return;
    n_free_++;
    Msg fr;
    std::memset(&fr, 0, sizeof(fr));
    fr.type = MSG_FREED;
    fr.u.region.alloc_id = p.alloc_id;
    send_rank(0, fr);
    if (p.pid && apps_.count(p.pid)) {
        Msg r;
        std::memset(&r, 0, sizeof(r));
        r.type = MSG_RELEASE_APP;
        r.status = MSG_RESPONSE;
        r.pid = p.pid;
        r.rank = rank_;
        r.seq = p.app_seq;
        r.err = p.err;
        send_app(p.pid, r);
    }
    pending_.erase(it);
}

void Daemon::fail_pending_on(int rank) {
    std::vector<uint64_t> dead;
    for (auto &kv : pending_) {
        const Pending &p = kv.second;
        // Owners of not-yet-answered extents are unknown to the origin (rank0
        // picked them), so an unfinished allocation may wait on the dead rank:
        // fail it now; late successes are freed by origin_do_alloc_resp.
        const bool open_alloc = p.type == MSG_REQ_ALLOC && (p.expect == 0 || p.got < p.expect);
        if (p.awaiting.count(rank) || open_alloc) dead.push_back(kv.first);
    }
    for (uint64_t s : dead) {
        auto it = pending_.find(s);
        if (it == pending_.end()) continue;
        Pending &p = it->second;
        if (p.type == MSG_REQ_ALLOC) {
            p.err = EHOSTDOWN;
            if (p.expect == 0) {
                p.expect = 1;
                p.have.assign(1, false);
                p.extents.assign(1, Region{});
            }
            finish_alloc(p);
        } else {
            if (p.pid && apps_.count(p.pid)) {
                Msg r;
                std::memset(&r, 0, sizeof(r));
                r.type = MSG_RELEASE_APP;
                r.status = MSG_RESPONSE;
                r.pid = p.pid;
                r.rank = rank_;
                r.seq = p.app_seq;
                r.err = EHOSTDOWN;
                send_app(p.pid, r);
            }
            pending_.erase(it);
        }
    }
}

void Daemon::peer_lost(int rank) {
    OCM_WARN("rank %d: lost link to rank %d", rank_, rank);
    if (rank == 0 && rank_ != 0) {
        // Keep serving (data plane, leases, frees to owners) and wait for a restarted rank0.
        r0_lost_ = true;
        next_rejoin_ms_ = now_ms() + 50;
    }
    for (auto &l : leases_)
        if (l && l->owner == rank) l.reset();  // its memory died with it
    lease_inflight_.erase(rank);
    if (tick_) tick_->abort();  // the dead rank will never join another tick
    if (gov_) gov_->mark_dead(rank);
    fail_pending_on(rank);
    // Extents we own for allocations that originated at the dead daemon stay
    // mapped by its apps; keep them until those apps' reclaim would have
    // happened, i.e. reclaim now only when no app can still reach them.
    std::vector<std::pair<uint64_t, int>> orphan;
    for (auto &kv : owned_)
        if (kv.second.orig_rank == rank) orphan.push_back(kv.first);
    for (auto &k : orphan) {
        arena_->free(owned_[k].slab_id, owned_[k].offset);
        owned_.erase(k);
        n_reclaimed_++;
    }
}

void Daemon::sweep_timeouts() {
    if (pending_.empty()) return;
    const long now = now_ms();
    std::vector<uint64_t> late;
    for (auto &kv : pending_)
        if (kv.second.t0_ms && now - kv.second.t0_ms > request_timeout_ms_) late.push_back(kv.first);
    for (uint64_t s : late) {
        auto it = pending_.find(s);
        if (it == pending_.end()) continue;
        Pending &p = it->second;
        OCM_WARN("rank %d: request seq %llu (%s) timed out", rank_, (unsigned long long)s, msg_type_str(p.type));
        if (p.type == MSG_REQ_ALLOC) {
            p.err = ETIMEDOUT;
            if (p.expect == 0) {
                p.expect = 1;
                p.have.assign(1, false);
                p.extents.assign(1, Region{});
            }
            finish_alloc(p);
        } else {
            if (p.pid && apps_.count(p.pid)) {
                Msg r;
                std::memset(&r, 0, sizeof(r));
                r.type = MSG_RELEASE_APP;
                r.status = MSG_RESPONSE;
                r.pid = p.pid;
                r.rank = rank_;
                r.seq = p.app_seq;
                r.err = ETIMEDOUT;
                send_app(p.pid, r);
            }
            pending_.erase(it);
        }
    }
}

void Daemon::start_tick(const uint8_t *id) {
    if (tick_) return;
    CollectiveFactory f;
    if (cfg_.ctrl == "rccl") {
        if (gpu_ < 0) {
            OCM_WARN("rank %d: --ctrl rccl needs a GPU; staying on TCP", rank_);
            return;
        }
        std::vector<uint8_t> uid(id, id + 128);
        const int gpu = gpu_, rank = rank_, n = n_;
        f = [uid, gpu, rank, n](std::string *err, const std::atomic<bool> *cancel) {
            return make_rccl_collective(gpu, rank, n, uid.data(), err, cancel);
        };
    } else {
        const std::string ns = ns_;
        const int rank = rank_, n = n_;
        f = [ns, rank, n](std::string *err, const std::atomic<bool> *cancel) {
            return make_socket_collective(ns, rank, n, err, cancel);
        };
    }
    tick_ = std::make_unique<TickTransport>(rank_, n_, f);
    ep_add(tick_->event_fd(), EPOLLIN, tag(T_TICK, 0));
    tick_->start();
    OCM_INFO("rank %d: control records will ride the %s tick transport", rank_, cfg_.ctrl.c_str());
}

void Daemon::on_tick() {
    if (!tick_) return;
    for (Msg &m : tick_->drain()) handle_mesh_msg(m, -1);
    uint64_t t = 0;
    if (tick_->take_announce(&t)) {
        // Wake the peers for the tick this rank is starting from idle.
        Msg w;
        std::memset(&w, 0, sizeof(w));
        w.type = MSG_TICK_WAKE;
        w.status = MSG_REQUEST;
        w.rank = rank_;
        w.u.req.bytes = t;
        for (int r = 0; r < n_; r++)
            if (r != rank_) send_tcp(r, w);
    }
    if (tick_->failed()) {
        for (TickRecord &rec : tick_->take_unsent()) send_tcp(rec.dest, rec.msg);
    }
}

int Daemon::preferred_owner() const {
    // The governor's first choice for a single-extent remote allocation:
    // the next live same-host peer in ring order, (rank + d) % N.
    for (int d = 1; d < n_; d++) {
        const int k = (rank_ + d) % n_;
        if (!joined_[k] || peer_fd_[k] < 0) continue;
        if (std::strncmp(table_[k].host, table_[rank_].host, sizeof(table_[k].host)) != 0) continue;
        return k;
    }
    return -1;
}

void Daemon::return_idle_leases() {
    if (leases_.empty() || cfg_.lease_idle_ms < 0) return;
    const long now = now_ms();
    for (auto &lp : leases_) {
        if (!lp || lp->ra.used() != 0 || now - lp->idle_since_ms < cfg_.lease_idle_ms) continue;
        // Nothing carved from it for a while: the owner gets the chunk back.
        Msg f;
        std::memset(&f, 0, sizeof(f));
        f.type = MSG_DO_FREE;
        f.status = MSG_REQUEST;
        f.rank = rank_;
        f.seq = 0;  // no answer needed
        f.u.region = lp->base;
        send_rank(lp->owner, f);
        Msg fr;
        std::memset(&fr, 0, sizeof(fr));
        fr.type = MSG_FREED;
        fr.u.region.alloc_id = lp->base.alloc_id;
        send_rank(0, fr);
        OCM_LOG("rank %d: returned idle lease of %llu bytes on rank %d", rank_, (unsigned long long)lp->base.bytes,
                lp->owner);
        lease_demand_[lp->owner] = 0;
        lp.reset();  // slot stays: OriginAlloc::lease indices remain valid
    }
}

void Daemon::request_lease(int owner, uint32_t tier) {
    if (!cfg_.lease_bytes || lease_inflight_.count(owner)) return;
    lease_inflight_.insert(owner);
    Pending p;
    p.seq = next_seq();
    p.pid = 0;
    p.type = MSG_REQ_ALLOC;
    p.kind = OCM_REMOTE_GPU;
    p.total_bytes = cfg_.lease_bytes;
    p.lease_owner = owner;
    p.lease_tier = tier;
    p.t0_ms = now_ms();
    p.awaiting.insert(0);
    pending_[p.seq] = p;
    Msg f;
    std::memset(&f, 0, sizeof(f));
    f.type = MSG_REQ_ALLOC;
    f.status = MSG_REQUEST;
    f.rank = rank_;
    f.seq = p.seq;
    f.u.req.orig_rank = rank_;
    f.u.req.remote_rank = owner;
    f.u.req.bytes = cfg_.lease_bytes;
    f.u.req.kind = OCM_REMOTE_GPU;
    f.u.req.flags = OCM_ALLOC_NO_SPILL | (tier == TIER_HOST ? OCM_ALLOC_HOST_TIER : 0);
    f.u.req.app_pid = 0;
    send_rank(0, f);
}

bool Daemon::try_lease_alloc(Msg &m) {
    const AllocReq &req = m.u.req;
    if (!cfg_.lease_bytes || leases_.empty()) return false;
    if (req.flags & (OCM_ALLOC_LOOPBACK | OCM_ALLOC_STRIPE | OCM_ALLOC_ZERO)) return false;
    const uint32_t want_tier = (req.flags & OCM_ALLOC_HOST_TIER) ? TIER_HOST : TIER_GPU;
    if (req.bytes > cfg_.lease_bytes / 4) return false;
    // Policy-faithful: only requests the governor would place as ONE extent on
    // the ring successor (ring, or stripe with bytes <= stripe unit).
    if (cfg_.policy == Policy::LeastLoaded || cfg_.policy == Policy::Loopback) return false;
    const uint64_t unit = req.stripe_unit ? req.stripe_unit : cfg_.stripe_unit;
    if (cfg_.policy == Policy::Stripe && req.bytes > unit) return false;
    const int owner = preferred_owner();
    if (owner < 0 || (req.remote_rank >= 0 && req.remote_rank != owner)) return false;
    for (size_t i = 0; i < leases_.size(); i++) {
        Lease *l = leases_[i].get();
        if (!l || l->owner != owner || l->tier != want_tier) continue;
        uint64_t off = 0;
        if (!l->ra.alloc(req.bytes, 4096, &off)) continue;
        Region rg = l->base;
        rg.alloc_id = (1ull << 62) | ((uint64_t)rank_ << 40) | (++lease_ids_);
        rg.offset = l->base.offset + off;
        rg.bytes = req.bytes;
        rg.stripe_unit = 0;
        rg.extent_idx = 0;
        rg.n_extents = 1;
        rg.orig_rank = rank_;
        rg.flags = (uint16_t)(rg.flags & ~REGION_DEDICATED);  // importers keep the chunk mapped
        OriginAlloc oa;
        oa.pid = m.pid;
        oa.remote = true;
        oa.bytes = req.bytes;
        oa.lease = (int)i;
        oa.extents.push_back(rg);
        origin_allocs_[rg.alloc_id] = oa;
        n_alloc_++;
        n_lease_allocs_++;
        // Top up before the chunk runs dry.
        if (l->ra.largest_free() < cfg_.lease_bytes / 4) request_lease(owner, want_tier);
        Msg h;
        std::memset(&h, 0, sizeof(h));
        h.type = MSG_RELEASE_APP;
        h.status = MSG_RESPONSE;
        h.pid = m.pid;
        h.rank = rank_;
        h.seq = m.seq;
        h.u.region = rg;
        send_app(m.pid, h);
        Msg e = h;
        e.type = MSG_EXTENT;
        send_app(m.pid, e);
        return true;
    }
    return false;
}

bool Daemon::cross_host(int a, int b) const {
    if (a < 0 || b < 0 || a >= n_ || b >= n_) return false;
    return std::strncmp(table_[a].host, table_[b].host, sizeof(table_[a].host)) != 0;
}

}  // namespace ocm
