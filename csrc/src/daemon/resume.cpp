// ocmd checkpoint / resume: mesh HELLO, the join report (ADD_NODE + OWNED
// extents), survivors reconnecting to a restarted rank0, and rank0's
// directory checkpoint.
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

namespace {

uint64_t realtime_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (uint64_t)ts.tv_sec * 1000ull + (uint64_t)ts.tv_nsec / 1000000ull;
}

constexpr uint64_t kHelloWindowMs = 10ull * 60 * 1000;  // clock skew tolerated between daemons

uint64_t hello_mac(const SipKey &k, const Hello &h) {
    const uint64_t w[4] = {(uint64_t)(uint32_t)h.src_rank | ((uint64_t)(uint32_t)h.dst_rank << 32), h.ts_ms, h.nonce,
                           (uint64_t)MSG_HELLO};
    return siphash24(k, w, sizeof(w));
}

}  // namespace

void Daemon::send_hello(int fd, int dst_rank) {
    Msg hello;
    std::memset(&hello, 0, sizeof(hello));
    hello.type = MSG_HELLO;
    hello.src_rank = rank_;
    hello.rank = rank_;
    Hello &h = hello.u.hello;
    h.src_rank = rank_;
    h.dst_rank = dst_rank;
    h.ts_ms = realtime_ms();
    std::ifstream ur("/dev/urandom", std::ios::binary);
    ur.read(reinterpret_cast<char *>(&h.nonce), sizeof(h.nonce));
    if (!ur) h.nonce ^= boot_id_ ^ (h.ts_ms << 20) ^ (uint64_t)fd;
    h.mac = hello_mac(mesh_key_, h);
    send_all(fd, &hello, sizeof(hello));
}

// First record of an inbound mesh link: a HELLO signed for us, fresh, never seen.
bool Daemon::hello_ok(const Msg &m) {
    const Hello &h = m.u.hello;
    if (m.type != MSG_HELLO || m.src_rank < 0 || m.src_rank >= n_ || m.src_rank == rank_ || h.src_rank != m.src_rank ||
        h.dst_rank != rank_ || hello_mac(mesh_key_, h) != h.mac)
        return false;
    const uint64_t now = realtime_ms();
    const uint64_t skew = now > h.ts_ms ? now - h.ts_ms : h.ts_ms - now;
    if (skew > kHelloWindowMs) {
        OCM_WARN("rank %d: HELLO from rank %d is %llu ms off our clock", rank_, m.src_rank, (unsigned long long)skew);
        return false;
    }
    for (auto it = hello_seen_.begin(); it != hello_seen_.end();) {  // forget what the window no longer admits
        const uint64_t age = now > it->second ? now - it->second : it->second - now;
        it = age > 2 * kHelloWindowMs ? hello_seen_.erase(it) : std::next(it);
    }
    return hello_seen_.emplace(h.nonce, h.ts_ms).second;  // a replay repeats its nonce
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
    if (links_.gpu >= 0) {
        Msg l;
        std::memset(&l, 0, sizeof(l));
        l.type = MSG_NODE_LINKS;
        l.status = MSG_REQUEST;
        l.rank = rank_;
        l.u.links = links_;
        send_rank(0, l);
    }
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

// hipExtGetLinkTypeAndHopCount from our GPU to every other ordinal on the node.
// OCM_LINK_HOPS="h0,h1,..." overrides the hop counts (tests: synthetic topologies).
void Daemon::probe_links() {
    std::memset(&links_, 0, sizeof(links_));
    links_.rank = rank_;
    links_.gpu = gpu_;
    std::memset(links_.hops, kHopsUnknown, sizeof(links_.hops));
    if (gpu_ < 0) return;
    links_.n = (uint32_t)std::min(num_gpu_, kMaxLinkGpus);
    for (int p = 0; p < (int)links_.n; p++) {
        if (p == gpu_) continue;
        uint32_t type = 0, hops = 0;
        if (hipExtGetLinkTypeAndHopCount(gpu_, p, &type, &hops) == hipSuccess && hops < kHopsUnknown) {
            links_.hops[p] = (uint8_t)hops;
            links_.type[p] = (uint8_t)type;
        } else {
            (void)hipGetLastError();
        }
    }
    if (const char *o = std::getenv("OCM_LINK_HOPS")) {
        std::stringstream ss(o);
        std::string tok;
        for (int p = 0; p < kMaxLinkGpus && std::getline(ss, tok, ','); p++)
            if (!tok.empty()) links_.hops[p] = (uint8_t)std::min(254, std::atoi(tok.c_str()));
        links_.n = (uint32_t)kMaxLinkGpus;
    }
}

void Daemon::try_rejoin_rank0() {
    const long now = now_ms();
    if (now < next_rejoin_ms_) return;
    next_rejoin_ms_ = now + 100;
    const NodeEntry &ne = nf_.nodes[0];
    int fd = tcp_connect(ne.ip, ne.ocm_port, 50);
    if (fd < 0) return;
    send_hello(fd, 0);
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


}  // namespace ocm
