// ocmd mesh protocol: rank0 placement (ADD_NODE, REQ_ALLOC, PLACE_FAIL),
// owner DO_ALLOC/DO_FREE, origin completion, peer loss, timeouts and the
// tick control transport.
// Reference parity: the inter-daemon protocol of src/mem.c:53-535 (a TCP
// connection and a thread per RPC there; persistent links and one event loop
// here), alloc_find placement src/alloc.c:76-140 (Governor::place),
// alloc_ate / dealloc_ate src/alloc.c:150-282 (owner_do_alloc / owner_do_free),
// message states inc/msg.h:24-45.
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

// ---------------------------------------------------------------- mesh messages

namespace {
uint64_t record_hash(const Msg &m) {
    // FNV-1a over the whole 160-byte record
    const unsigned char *p = reinterpret_cast<const unsigned char *>(&m);
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(Msg); i++) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}
constexpr size_t kMeshSeenMax = 8192;  // > every rank's unsent window (kTickRing records) together
}  // namespace

void Daemon::SeenWindow::add(uint64_t h) {
    set.insert(h);
    order.push_back(h);
    if (order.size() > kMeshSeenMax) {
        auto it = set.find(order.front());
        if (it != set.end()) set.erase(it);
        order.pop_front();
    }
}

bool Daemon::SeenWindow::take(uint64_t h) {
    auto it = set.find(h);
    if (it == set.end()) return false;
    set.erase(it);  // its entry in `order` ages out harmlessly
    return true;
}

bool Daemon::mesh_duplicate(const Msg &m, bool via_tick, bool resent) {
    if (!via_tick && !resent) return false;  // ordinary TCP and local traffic
    switch (m.type) {
    case MSG_REQ_ALLOC:
    case MSG_DO_ALLOC:
    case MSG_DO_FREE:
    case MSG_PLACE_FAIL:
    case MSG_FREED:
    case MSG_STATS:
        break;
    default:
        return false;
    }
    const uint64_t h = record_hash(m);
    SeenWindow &mine = via_tick ? seen_tick_ : seen_resent_;
    SeenWindow &other = via_tick ? seen_resent_ : seen_tick_;
    if (other.take(h)) {
        mesh_dups_dropped_++;
        OCM_WARN("rank %d: dropping a second copy of %s/%s seq %llu from rank %d (tick fallback re-send)", rank_,
                 msg_type_str(m.type), msg_status_str(m.status), (unsigned long long)m.seq, m.src_rank);
        return true;
    }
    mine.add(h);
    return false;
}

void Daemon::handle_mesh_msg(Msg &m, int from_fd, bool via_tick) {
    const bool resent = (m.status & kMsgResent) != 0;
    m.status &= ~kMsgResent;
    if (mesh_duplicate(m, via_tick, resent)) return;
    if (from_fd >= 0) {
        // An inbound link is anonymous until its HELLO carries a valid MAC.
        auto it = conns_.find(from_fd);
        if (it == conns_.end()) return;
        if (it->second->peer_rank < 0 && !hello_ok(m)) {
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
            if (rank_ == 0 && m.src_rank != 0) send_ctrl_decision(m.src_rank);
        }
        break;
    }
    case MSG_ADD_NODE:
        if (rank_ == 0) r0_add_node(m.u.node, m.seq);
        break;
    case MSG_OWNED:
        if (rank_ == 0 && gov_) gov_->confirm_extent(m.src_rank, m.u.region, m.pid);
        break;
    case MSG_NODE_LINKS:
        if (rank_ == 0 && gov_) {
            m.u.links.rank = m.rank;
            gov_->set_links(m.u.links);
        }
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
        if (!tick_ && !tick_left_ && cfg_.ctrl != "tcp") {
            start_tick(m.u.raw, m.seq == 1, (uint32_t)std::max(0, m.pid));  // rank0's idle-tick setting
            if (!tick_ && join_deferred_) join_now("this rank cannot run the chosen tick transport");
        }
        break;
    case MSG_TICK_WAKE:
        if (tick_ && !tick_left_) tick_->wake_at(m.u.req.bytes);
        break;
    case MSG_TICK_STOP:
        if (tick_) {
            leave_tick("a peer left it");
        } else {
            tick_left_ = true;  // rank0 chose TCP: ignore any later start
            if (join_deferred_) join_now("rank0 chose TCP");
        }
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
    uint64_t grant = 0;
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
        // Other node: the app streams through our data server instead of mapping the
        // slab, with a capability for this extent alone.
        grant = data_->grant(rg.slab_id, rg.offset, rg.bytes);
        if (!format_net_handle(rg.handle, nf_.nodes[rank_].ip, data_->port(), data_token_, grant)) {
            OCM_ERR("rank %d: net handle for %s does not fit %zu bytes", rank_, nf_.nodes[rank_].ip.c_str(),
                    kHandleBytes);
            data_->revoke(grant);
            arena_->free(rg.slab_id, rg.offset);
            Msg f = m;
            f.type = MSG_PLACE_FAIL;
            f.status = MSG_REQUEST;
            f.err = ENAMETOOLONG;
            f.u.region.owner_rank = rank_;
            send_rank(0, f);
            return;
        }
        rg.flags = (uint16_t)(rg.flags & ~REGION_DEDICATED);
    }
    OwnedExtent oe;
    oe.grant = grant;
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

// Give an owned extent back to the arena. A network-tier extent first loses its
// grant; when a data-server request is still copying it, that request frees it.
int Daemon::free_owned(const OwnedExtent &oe) {
    if (oe.grant && data_ && !data_->revoke(oe.grant)) return 0;
    return arena_->free(oe.slab_id, oe.offset);
}

void Daemon::owner_do_free(Msg &m) {
    const Region &rg = m.u.region;
    auto it = owned_.find({rg.alloc_id, (int)rg.extent_idx});
    int err = ENOENT;
    if (it != owned_.end()) {
        err = free_owned(it->second);
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
    if (tick_) leave_tick("a peer died");  // the dead rank will never join another tick
    if (gov_) gov_->mark_dead(rank);
    fail_pending_on(rank);
    // Extents we own for allocations that originated at the dead daemon stay
    // mapped by its apps; keep them until those apps' reclaim would have
    // happened, i.e. reclaim now only when no app can still reach them.
    std::vector<std::pair<uint64_t, int>> orphan;
    for (auto &kv : owned_)
        if (kv.second.orig_rank == rank) orphan.push_back(kv.first);
    for (auto &k : orphan) {
        free_owned(owned_[k]);
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

void Daemon::resolve_ctrl() {
    ctrl_mode_ = "tcp";
    if (n_ <= 1 || resumed_ || cfg_.ctrl == "tcp") {
        if (resumed_ && cfg_.ctrl != "tcp") OCM_INFO("rank 0: resumed directory: control records stay on TCP");
        return;
    }
    if (cfg_.ctrl == "rccl" || cfg_.ctrl == "socket") {
        ctrl_mode_ = cfg_.ctrl;
    } else {
        // auto: RCCL when every rank has a GPU of its own (one rank per GPU, the
        // layout RCCL requires). GPUs come from the nodefile's gpu= column; a
        // rank without one on this host uses rank % visible GPUs, as it will.
        std::set<std::pair<std::string, int>> seen;
        bool own = gpu_ >= 0;
        const std::string &my_ip = nf_.nodes[rank_].ip;
        for (const NodeEntry &ne : nf_.nodes) {
            int g = ne.gpu;
            if (g < 0 && ne.ip == my_ip && num_gpu_ > 0) g = ne.rank % num_gpu_;
            if (g < 0 || !seen.insert({ne.ip, g}).second) {
                own = false;
                break;
            }
        }
        const char *sock = std::getenv("OCM_CTRL_AUTO_SOCKET");  // CPU meshes in tests: the socket ring instead
        ctrl_mode_ = own ? "rccl" : (sock && std::strcmp(sock, "1") == 0) ? "socket" : "tcp";
    }
    if (ctrl_mode_ == "rccl") {
        std::string err;
        if (rccl_unique_id(tick_uid_, &err) != 0) {
            OCM_WARN("rank 0: rccl control plane unavailable (%s); control records stay on TCP", err.c_str());
            ctrl_mode_ = "tcp";
        }
    }
    if (ctrl_mode_ != "tcp") tick_deadline_ms_ = now_ms() + tick_up_ms_;
    OCM_INFO("rank 0: daemon<->daemon records: %s (--ctrl %s)", ctrl_mode_.c_str(), cfg_.ctrl.c_str());
}

void Daemon::send_ctrl_decision(int r) {
    if (r <= 0 || r >= n_) return;
    Msg t;
    std::memset(&t, 0, sizeof(t));
    t.status = MSG_REQUEST;
    t.rank = 0;
    if (ctrl_mode_ == "tcp" || tick_left_) {
        t.type = MSG_TICK_STOP;
    } else {
        t.type = MSG_TICK_START;
        t.seq = ctrl_mode_ == "rccl" ? 1 : 2;
        t.pid = (int32_t)tick_idle_us_;  // every rank must run the same ticks: rank0's setting
        std::memcpy(t.u.raw, tick_uid_, sizeof(tick_uid_));
    }
    send_tcp(r, t);
    if (t.type == MSG_TICK_START && !tick_) start_tick(tick_uid_, ctrl_mode_ == "rccl", tick_idle_us_);
}

void Daemon::join_now(const char *why) {
    if (!join_deferred_) return;
    join_deferred_ = false;
    OCM_INFO("rank %d: joining rank0 (%s)", rank_, why);
    join_rank0();
}

void Daemon::check_tick_bootstrap() {
    if (!tick_deadline_ms_ || now_ms() < tick_deadline_ms_) return;
    tick_deadline_ms_ = 0;
    char why[96];
    std::snprintf(why, sizeof(why), "not up within OCM_TICK_UP_MS=%d ms", tick_up_ms_);
    if (tick_ && !tick_->up() && !tick_left_) {
        leave_tick(why);  // the whole mesh falls back to TCP (MSG_TICK_STOP); a deferred join follows
    } else if (!tick_ && join_deferred_) {
        tick_left_ = true;  // no decision from rank0 in time: join over TCP, ignore a late start
        join_now("no control-plane decision from rank0 in time");
    }
}

void Daemon::start_tick(const uint8_t *id, bool rccl, uint32_t idle_us) {
    if (tick_) return;
    tick_idle_us_ = idle_us;
    CollectiveFactory f;
    if (rccl) {
        if (gpu_ < 0) {
            OCM_WARN("rank %d: the RCCL control plane needs a GPU; staying on TCP", rank_);
            return;
        }
        std::vector<uint8_t> uid(id, id + 128);
        const int gpu = gpu_, rank = rank_, n = n_;
        f = [uid, gpu, rank, n](std::string *err, const std::atomic<bool> *cancel) {
            return make_rccl_collective(gpu, rank, n, uid.data(), sizeof(TickSlot), err, cancel);
        };
    } else {
        const std::string ns = ns_;
        const int rank = rank_, n = n_;
        f = [ns, rank, n](std::string *err, const std::atomic<bool> *cancel) {
            return make_socket_collective(ns, rank, n, sizeof(TickSlot), err, cancel);
        };
    }
    tick_ = std::make_unique<TickTransport>(rank_, n_, f);
    // The tick thread busy-polls its collective during traffic, and RCCL's proxy
    // threads inherit its mask: keep them off the event loop's pinned core, on the
    // rest of the GPU's L3 complex (OCM_TICK_CPUS=ccd, default), the process's whole
    // mask (=all), or sharing the event loop's core as before round 3 (=loop).
    if (pinned_cpus_) {
        const char *tc = std::getenv("OCM_TICK_CPUS");
        const std::string mode = tc && *tc ? tc : "ccd";
        if (mode == "all")
            tick_->set_cpus(orig_cpus_);
        else if (mode != "loop")
            tick_->set_cpus(near_cpus_.empty() ? orig_cpus_ : near_cpus_);
    }
    if (idle_us) {
        // Idle ticks instead of TCP wake-ups; the doorbell is shared by the daemons of
        // this host (a peer on another host simply waits out its idle tick).
        if (!tick_bell_) tick_bell_ = tick_bell_open(ns_);
        if (!tick_bell_) OCM_WARN("rank %d: no tick doorbell (shared memory); idle ticks run their full length", rank_);
        tick_->set_idle(idle_us, tick_bell_);
    }
    ep_add(tick_->event_fd(), EPOLLIN, tag(T_TICK, 0));
    tick_->start();
    OCM_INFO("rank %d: control records will ride the %s tick transport (%s)", rank_, rccl ? "rccl" : "socket",
             idle_us ? "idle ticks, no TCP wake-ups" : "idle mesh woken over TCP");
}

void Daemon::on_tick() {
    if (!tick_) return;
    for (Msg &m : tick_->drain()) handle_mesh_msg(m, -1, true);
    if (tick_->up() && tick_deadline_ms_) {
        tick_deadline_ms_ = 0;
        if (join_deferred_) join_now("tick transport up: the join is its first traffic");
    }
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
            if (r != rank_) {
                send_tcp(r, w);
                tcp_wakes_++;
            }
    }
    if (tick_->failed()) leave_tick("the collective failed here");
}

void Daemon::leave_tick(const char *why) {
    if (!tick_) return;
    if (!tick_->failed()) tick_->abort();
    // send_rank: records to ourselves (OCM_TICK_SELF) go back to the local queue
    for (TickRecord &rec : tick_->take_unsent()) {
        rec.msg.status |= kMsgResent;  // the receiver compares it with what the ticks delivered
        send_rank(rec.dest, rec.msg);
    }
    tick_deadline_ms_ = 0;
    if (join_deferred_) join_now(why);
    if (tick_left_) return;
    tick_left_ = true;
    OCM_WARN("rank %d: leaving the %s tick transport (%s); control records ride TCP", rank_,
             tick_->collective_name(), why);
    Msg s;
    std::memset(&s, 0, sizeof(s));
    s.type = MSG_TICK_STOP;
    s.status = MSG_REQUEST;
    s.rank = rank_;
    for (int r = 0; r < n_; r++)
        if (r != rank_ && peer_fd_[r] >= 0) send_tcp(r, s);
}

bool Daemon::cross_host(int a, int b) const {
    if (a < 0 || b < 0 || a >= n_ || b >= n_) return false;
    return std::strncmp(table_[a].host, table_[b].host, sizeof(table_[a].host)) != 0;
}


}  // namespace ocm
