// ocmd capacity leases: origins carve small remote allocations from chunks
// leased on owners (no rank0 / owner round trip), and give idle chunks back.
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


}  // namespace ocm
