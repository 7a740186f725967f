#include "ocm/governor.h"

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <iterator>
#include <map>
#include <sstream>

#include "../../include/oncillamem.h"
#include "ocm/log.h"

namespace ocm {

Policy parse_policy(const std::string &s, Policy dflt) {
    if (s == "ring") return Policy::Ring;
    if (s == "least_loaded" || s == "least-loaded") return Policy::LeastLoaded;
    if (s == "stripe") return Policy::Stripe;
    if (s == "loopback" || s == "local") return Policy::Loopback;
    return dflt;
}

const char *policy_name(Policy p) {
    switch (p) {
    case Policy::Ring: return "ring";
    case Policy::LeastLoaded: return "least_loaded";
    case Policy::Stripe: return "stripe";
    case Policy::Loopback: return "loopback";
    }
    return "?";
}

uint64_t stripe_extent_bytes(uint64_t total, uint64_t unit, int n, int idx) {
    if (n <= 1 || unit == 0) return idx == 0 ? total : 0;
    const uint64_t units = (total + unit - 1) / unit;
    if ((uint64_t)idx >= units) return 0;
    const uint64_t cnt = (units - (uint64_t)idx + (uint64_t)n - 1) / (uint64_t)n;
    const uint64_t last = units - 1;
    if (last % (uint64_t)n == (uint64_t)idx) return (cnt - 1) * unit + (total - last * unit);
    return cnt * unit;
}

Governor::Governor(int num_nodes, Policy policy, uint64_t default_stripe_unit)
    : nodes_(num_nodes), policy_(policy), default_stripe_unit_(default_stripe_unit ? default_stripe_unit : (1ull << 20)) {
    for (int i = 0; i < num_nodes; i++) nodes_[i].rank = i;
}

void Governor::add_node(const NodeConfig &cfg, uint64_t boot_id) {
    if (cfg.rank < 0 || cfg.rank >= (int)nodes_.size()) {
        OCM_WARN("ADD_NODE for rank %d outside nodefile (%zu nodes)", cfg.rank, nodes_.size());
        return;
    }
    version_++;
    NodeState &n = nodes_[cfg.rank];
    const bool same = boot_id != 0 && n.boot_id == boot_id;
    if (same) {
        // The same process reconnected (link loss, or rank0 restarted): its memory is
        // intact. Un-reserve its extents until its OWNED report confirms them.
        for (auto &kv : table_)
            for (auto &e : kv.second.placement.extents)
                if (e.owner == cfg.rank && e.held) {
                    reserve(e.owner, e.tier, e.bytes, -1);
                    e.held = false;
                }
    } else {
        // A new process (or an unknown one) lost whatever the directory says it owned.
        size_t dropped = 0;
        for (auto it = table_.begin(); it != table_.end();) {
            bool owned = false;
            for (auto &e : it->second.placement.extents) owned |= e.owner == cfg.rank;
            if (owned) {
                for (auto &e : it->second.placement.extents)
                    if (e.owner != cfg.rank && e.held) reserve(e.owner, e.tier, e.bytes, -1);
                it = table_.erase(it);
                dropped++;
            } else {
                ++it;
            }
        }
        if (dropped) OCM_WARN("rank %d re-joined as a new process; dropped %zu allocations it owned", cfg.rank, dropped);
        n.gpu_reserved = n.host_reserved = 0;
    }
    n.boot_id = boot_id;
    n.joined = true;
    n.alive = true;
    n.gpu = cfg.gpu;
    n.gpu_capacity = cfg.gpu_capacity;
    n.host_capacity = cfg.host_capacity;
    n.host = std::string(cfg.host, strnlen(cfg.host, sizeof(cfg.host)));
}

void Governor::confirm_extent(int owner, const Region &r, int app_pid) {
    if (owner < 0 || owner >= (int)nodes_.size()) return;
    version_++;
    const int n_ext = std::max<int>(1, r.n_extents);
    auto it = table_.find(r.alloc_id);
    if (it == table_.end()) {
        // Placed after the last checkpoint: rebuild the entry from the owners' reports.
        Entry ent{r.orig_rank, app_pid, Placement{}, {}, 0};
        ent.placement.alloc_id = r.alloc_id;
        ent.placement.stripe_unit = r.stripe_unit;
        ent.placement.extents.assign(n_ext, PlacedExtent{-1, TIER_NONE, 0, false, false, false});
        it = table_.emplace(r.alloc_id, ent).first;
    }
    auto &ext = it->second.placement.extents;
    if ((int)ext.size() <= r.extent_idx) ext.resize(r.extent_idx + 1, PlacedExtent{-1, TIER_NONE, 0, false, false, false});
    PlacedExtent &e = ext[r.extent_idx];
    if (e.held) reserve(e.owner, e.tier, e.bytes, -1);
    e.owner = owner;
    e.tier = r.tier;
    e.bytes = r.bytes;
    e.spilled = (r.flags & REGION_SPILLED) != 0;
    e.net = (r.flags & REGION_NET) != 0;
    e.held = true;
    reserve(owner, e.tier, e.bytes, +1);
    if (r.alloc_id < (1ull << 62)) next_id_ = std::max(next_id_, r.alloc_id + 1);  // rank0-issued ids only
}

int Governor::end_reconcile(int owner) {
    int dropped = 0;
    for (auto it = table_.begin(); it != table_.end();) {
        bool any = false;
        for (auto &e : it->second.placement.extents) {
            if (e.owner == owner && !e.held) {
                e = PlacedExtent{-1, TIER_NONE, 0, false, false, false};
                dropped++;
            }
            any |= e.owner >= 0;
        }
        it = any ? std::next(it) : table_.erase(it);
    }
    if (dropped) version_++;
    return dropped;
}

std::string Governor::checkpoint() const {
    std::ostringstream o;
    o << "ocm-directory 1\n" << "next_id " << next_id_ << "\n" << "spilled " << n_spilled_ << "\n";
    for (auto &n : nodes_)
        if (n.boot_id) o << "node " << n.rank << " " << n.boot_id << "\n";
    for (auto &kv : table_) {
        const Entry &e = kv.second;
        o << "entry " << kv.first << " " << e.orig_rank << " " << e.pid << " " << e.placement.stripe_unit << " "
          << e.placement.extents.size() << "\n";
        for (auto &x : e.placement.extents)
            o << "ext " << x.owner << " " << x.tier << " " << x.bytes << " " << (int)x.spilled << " " << (int)x.net
              << "\n";
    }
    o << "end\n";
    return o.str();
}

int Governor::restore(const std::string &text, std::string *err) {
    std::istringstream in(text);
    std::string tag;
    int version = 0;
    if (!(in >> tag >> version) || tag != "ocm-directory" || version != 1) {
        *err = "not an ocm directory checkpoint";
        return -1;
    }
    std::map<uint64_t, Entry> table;
    uint64_t next_id = 1, spilled = 0;
    std::vector<uint64_t> boots(nodes_.size(), 0);
    Entry *cur = nullptr;
    bool complete = false;
    while (in >> tag) {
        if (tag == "next_id") {
            in >> next_id;
        } else if (tag == "spilled") {
            in >> spilled;
        } else if (tag == "node") {
            int r = -1;
            uint64_t b = 0;
            in >> r >> b;
            if (r >= 0 && r < (int)boots.size()) boots[r] = b;
        } else if (tag == "entry") {
            uint64_t id = 0, unit = 0;
            int orig = 0, pid = 0;
            size_t n_ext = 0;
            in >> id >> orig >> pid >> unit >> n_ext;
            Entry e{orig, pid, Placement{}, {}, 0};
            e.placement.alloc_id = id;
            e.placement.stripe_unit = unit;
            cur = &(table[id] = e);
        } else if (tag == "ext") {
            PlacedExtent x;
            int sp = 0, net = 0;
            in >> x.owner >> x.tier >> x.bytes >> sp >> net;
            x.spilled = sp;
            x.net = net;
            x.held = false;  // reserved again once the owner confirms it
            if (cur) cur->placement.extents.push_back(x);
        } else if (tag == "end") {
            complete = true;
            break;
        } else {
            *err = "unexpected token '" + tag + "'";
            return -1;
        }
        if (!in) {
            *err = "truncated checkpoint";
            return -1;
        }
    }
    if (!complete) {
        *err = "truncated checkpoint";
        return -1;
    }
    table_ = std::move(table);
    next_id_ = std::max(next_id_, next_id);
    n_spilled_ = spilled;
    for (size_t r = 0; r < nodes_.size(); r++) nodes_[r].boot_id = boots[r];
    version_++;
    return (int)table_.size();
}

void Governor::set_links(const NodeLinks &l) {
    if (l.rank < 0 || l.rank >= (int)nodes_.size()) return;
    const uint32_t n = std::min<uint32_t>(l.n, (uint32_t)kMaxLinkGpus);
    nodes_[l.rank].hops.assign(l.hops, l.hops + n);
    version_++;
}

int Governor::hops(int a, int b) const {
    if (a < 0 || b < 0 || a >= (int)nodes_.size() || b >= (int)nodes_.size()) return kHopsUnknown;
    const NodeState &x = nodes_[a], &y = nodes_[b];
    if (x.host != y.host || x.gpu < 0 || y.gpu < 0 || y.gpu >= (int)x.hops.size()) return kHopsUnknown;
    return x.hops[(size_t)y.gpu];
}

void Governor::mark_dead(int rank) {
    if (rank >= 0 && rank < (int)nodes_.size()) nodes_[rank].alive = false;
    version_++;
}

int Governor::num_alive() const {
    int c = 0;
    for (auto &n : nodes_) c += n.alive && n.joined;
    return c;
}

bool Governor::fits(const NodeState &n, uint32_t tier, uint64_t bytes) const {
    if (!n.alive || !n.joined) return false;
    // Overflow-safe: `reserved + bytes` would wrap for absurd requests.
    auto room = [&](uint64_t used, uint64_t cap) { return bytes <= cap && used <= cap - bytes; };
    if (tier == TIER_GPU) return n.gpu >= 0 && room(n.gpu_reserved, n.gpu_capacity);
    if (tier == TIER_HOST) return room(n.host_reserved, n.host_capacity);
    return false;
}

void Governor::reserve(int rank, uint32_t tier, uint64_t bytes, int sign) {
    if (rank < 0 || rank >= (int)nodes_.size()) return;
    NodeState &n = nodes_[rank];
    uint64_t &slot = tier == TIER_GPU ? n.gpu_reserved : n.host_reserved;
    if (sign > 0)
        slot += bytes;
    else
        slot = slot >= bytes ? slot - bytes : 0;
}

std::vector<int> Governor::remote_candidates(const PlaceRequest &r) const {
    std::vector<int> out;
    const int n = (int)nodes_.size();
    const std::string &home = nodes_[r.orig_rank].host;
    for (int d = 1; d < n; d++) {
        int k = (r.orig_rank + d) % n;
        if (nodes_[k].alive && nodes_[k].joined && nodes_[k].host != home) out.push_back(k);
    }
    return out;
}

std::vector<int> Governor::candidates(const PlaceRequest &r) const {
    // Peers on the origin's host: the data plane maps their memory into the
    // app (IPC over xGMI for HBM, /proc/<pid>/fd for host slabs).
    std::vector<int> out;
    const int n = (int)nodes_.size();
    const std::string &home = nodes_[r.orig_rank].host;
    for (int d = 1; d < n; d++) {
        int k = (r.orig_rank + d) % n;
        if (nodes_[k].alive && nodes_[k].joined && nodes_[k].host == home) out.push_back(k);
    }
    // Nearest GPUs first (xGMI hop count from the origin's GPU), ring order among equals.
    std::stable_sort(out.begin(), out.end(), [&](int a, int b) { return hops(r.orig_rank, a) < hops(r.orig_rank, b); });
    return out;
}

bool Governor::place_one(int preferred, uint64_t bytes, uint32_t want_tier, bool allow_spill,
                         const std::vector<int> &fallback, const std::vector<int> &spill_to, PlacedExtent *out) {
    auto take = [&](int rank, uint32_t tier, bool spilled) {
        reserve(rank, tier, bytes, +1);
        out->owner = rank;
        out->tier = tier;
        out->bytes = bytes;
        out->spilled = spilled;
        if (spilled) n_spilled_++;
        return true;
    };
    if (fits(nodes_[preferred], want_tier, bytes)) return take(preferred, want_tier, false);
    for (int k : fallback)
        if (k != preferred && fits(nodes_[k], want_tier, bytes)) return take(k, want_tier, false);
    if (allow_spill && want_tier == TIER_GPU) {
        if (fits(nodes_[preferred], TIER_HOST, bytes)) return take(preferred, TIER_HOST, true);
        for (int k : spill_to)
            if (k != preferred && fits(nodes_[k], TIER_HOST, bytes)) return take(k, TIER_HOST, true);
    }
    return false;
}

Placement Governor::place(const PlaceRequest &r) {
    Placement p;
    const int n = (int)nodes_.size();
    if (r.bytes == 0 || r.orig_rank < 0 || r.orig_rank >= n) {
        p.err = EINVAL;
        return p;
    }
    // The data plane addresses stripes with shifts: a unit must be a power of two >= 16.
    if (r.stripe_unit && (r.stripe_unit < 16 || (r.stripe_unit & (r.stripe_unit - 1)))) {
        p.err = EINVAL;
        return p;
    }
    if (!r.remote) {
        // Local kinds: the app allocates the memory itself; rank0 only records it.
        PlacedExtent e;
        e.owner = r.orig_rank;
        e.tier = r.local_tier;
        e.bytes = r.bytes;
        p.extents.push_back(e);
        p.alloc_id = next_id_++;
        table_[p.alloc_id] = Entry{r.orig_rank, r.app_pid, p, {}, 0};
        table_[p.alloc_id].placement.extents[0].tier = TIER_NONE;  // nothing reserved
        return p;
    }
    uint32_t want_tier = (r.flags & OCM_ALLOC_HOST_TIER) ? TIER_HOST : TIER_GPU;
    const bool allow_spill = !(r.flags & OCM_ALLOC_NO_SPILL);
    std::vector<int> peers = candidates(r);
    std::vector<int> owners;
    bool explicit_owner = false;
    if (r.remote_rank >= 0) {
        if (r.remote_rank >= n || !nodes_[r.remote_rank].alive) {
            p.err = r.remote_rank >= n ? EINVAL : EHOSTDOWN;
            return p;
        }
        owners.push_back(r.remote_rank);
        explicit_owner = true;
    } else if ((r.flags & OCM_ALLOC_LOOPBACK) || policy_ == Policy::Loopback) {
        owners.push_back(r.orig_rank);
        explicit_owner = true;
    } else if (peers.empty() && !remote_candidates(r).empty()) {
        // One daemon on this host, others elsewhere (the reference's layout):
        // ring to the next node, through the network tier.
        owners.push_back(remote_candidates(r)[0]);
    } else if (peers.empty()) {
        // Single daemon: no peer HBM exists, the remote half lives in the host tier
        // (the reference coerced every request to host memory here, src/alloc.c:82-83).
        owners.push_back(r.orig_rank);
        want_tier = TIER_HOST;
    } else if ((r.flags & OCM_ALLOC_STRIPE) || policy_ == Policy::Stripe) {
        owners = peers;
        size_t width = r.stripe_width ? r.stripe_width : owners.size();
        width = std::min<size_t>({width, owners.size(), (size_t)kMaxExtents});
        owners.resize(width);
    } else if (policy_ == Policy::LeastLoaded) {
        int best = peers[0];
        uint64_t best_free = 0;
        for (int k : peers) {
            const NodeState &s = nodes_[k];
            uint64_t f = s.gpu_capacity > s.gpu_reserved ? s.gpu_capacity - s.gpu_reserved : 0;
            if (f > best_free) {
                best_free = f;
                best = k;
            }
        }
        owners.push_back(best);
    } else {
        owners.push_back(peers[0]);  // ring: (orig + 1) % N, skipping dead nodes
    }

    uint64_t unit = r.stripe_unit ? r.stripe_unit : default_stripe_unit_;
    int nx = (int)owners.size();
    if (nx > 1) {
        const uint64_t units = (r.bytes + unit - 1) / unit;
        if (units < (uint64_t)nx) nx = (int)units;
    }
    if (nx <= 1) unit = 0;

    std::vector<int> fallback = explicit_owner ? std::vector<int>{} : peers;
    if (!explicit_owner && want_tier == TIER_HOST) fallback.push_back(r.orig_rank);
    // HBM exhausted: spill to a host tier, peers first, then the origin node's own.
    std::vector<int> spill_to = explicit_owner ? std::vector<int>{} : peers;
    if (!explicit_owner) spill_to.push_back(r.orig_rank);
    for (int i = 0; i < nx; i++) {
        PlacedExtent e;
        const uint64_t b = stripe_extent_bytes(r.bytes, unit, nx, i);
        if (!place_one(owners[i], b, want_tier, allow_spill, fallback, spill_to, &e)) {
            for (auto &done : p.extents) reserve(done.owner, done.tier, done.bytes, -1);
            p.extents.clear();
            p.err = ENOMEM;
            return p;
        }
        e.net = nodes_[e.owner].host != nodes_[r.orig_rank].host;
        p.extents.push_back(e);
    }
    p.stripe_unit = unit;
    p.alloc_id = next_id_++;
    table_[p.alloc_id] = Entry{r.orig_rank, r.app_pid, p, {}, 0};
    version_++;
    return p;
}

bool Governor::replace_extent(uint64_t alloc_id, int idx, int failed_owner, PlacedExtent *out) {
    auto it = table_.find(alloc_id);
    if (it == table_.end() || idx < 0 || idx >= (int)it->second.placement.extents.size()) return false;
    Entry &ent = it->second;
    PlacedExtent &old = ent.placement.extents[idx];
    version_++;
    if (old.held) reserve(old.owner, old.tier, old.bytes, -1);
    old.held = false;
    // Never retry an (owner, tier) that already refused this allocation, and
    // bound the retries: the directory's view can be wrong (HBM used by other
    // processes, fragmentation), the owner's arena is authoritative.
    ent.failed.emplace_back(failed_owner, old.tier);
    const int n = (int)nodes_.size();
    if (++ent.replacements > 2 * n) {
        old.owner = -1;
        return false;
    }
    auto refused = [&](int k, uint32_t t) {
        for (auto &f : ent.failed)
            if (f.first == k && f.second == t) return true;
        return false;
    };
    std::vector<int> order;
    for (int d = 1; d <= n; d++) order.push_back((failed_owner + d) % n);  // failed owner last
    PlacedExtent e;
    bool ok = false;
    if (old.tier == TIER_GPU) {
        for (int k : order)
            if (!ok && !refused(k, TIER_GPU) && fits(nodes_[k], TIER_GPU, old.bytes)) {
                e = PlacedExtent{k, TIER_GPU, old.bytes, false};
                ok = true;
            }
    }
    if (!ok) {
        // Host tier: the failed owner's own host tier first (same node), then the others.
        std::vector<int> horder{failed_owner};
        for (int k : order)
            if (k != failed_owner) horder.push_back(k);
        for (int k : horder)
            if (!ok && !refused(k, TIER_HOST) && fits(nodes_[k], TIER_HOST, old.bytes)) {
                e = PlacedExtent{k, TIER_HOST, old.bytes, old.tier == TIER_GPU};
                ok = true;
            }
    }
    if (!ok) {
        old.owner = -1;
        return false;
    }
    reserve(e.owner, e.tier, e.bytes, +1);
    if (e.spilled) n_spilled_++;
    old = e;
    *out = e;
    return true;
}

bool Governor::release(uint64_t alloc_id) {
    auto it = table_.find(alloc_id);
    if (it == table_.end()) return false;
    for (auto &e : it->second.placement.extents)
        if (e.owner >= 0 && e.held) reserve(e.owner, e.tier, e.bytes, -1);
    table_.erase(it);
    version_++;
    return true;
}

std::vector<uint64_t> Governor::allocations_of_app(int orig_rank, int pid) const {
    std::vector<uint64_t> v;
    for (auto &kv : table_)
        if (kv.second.orig_rank == orig_rank && kv.second.pid == pid) v.push_back(kv.first);
    return v;
}

std::vector<uint64_t> Governor::allocations_from(int orig_rank) const {
    std::vector<uint64_t> v;
    for (auto &kv : table_)
        if (kv.second.orig_rank == orig_rank) v.push_back(kv.first);
    return v;
}

const Governor::Entry *Governor::find(uint64_t id) const {
    auto it = table_.find(id);
    return it == table_.end() ? nullptr : &it->second;
}

}  // namespace ocm
