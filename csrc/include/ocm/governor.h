// Allocation governor: rank0's directory and placement policy.
//
// Parity with reference src/alloc.c:59-140 (alloc_add_node, alloc_find): rank0
// records joining nodes and decides where a request lands; HOST/GPU kinds stay
// on the origin, remote kinds go to (orig_rank + 1) % N. Extended MI355X-first:
//   * capacity accounting per daemon for HBM and the pinned host tier, fed by
//     hipMemGetInfo at join (the reference's get_free_mem check was commented out);
//   * an explicit remote_rank is honoured (reference field "not yet used");
//   * policies: ring (reference), least_loaded, stripe (one allocation spread
//     over several peers so put/get use several xGMI links), loopback;
//   * spill to the host tier when HBM is exhausted, ENOMEM when both are;
//   * an allocation table keyed by alloc_id for free/crash reclaim;
//   * peers on the origin's host first; other hosts only when the origin's
//     host has none (or one is named), through the network tier (netdata.h).
// Pure logic (no I/O) so it is unit-tested on CPU.
#pragma once
#include <cstdint>
#include <map>
#include <utility>
#include <string>
#include <vector>

#include "ocm/msg.h"

namespace ocm {

enum class Policy { Ring, LeastLoaded, Stripe, Loopback };
Policy parse_policy(const std::string &s, Policy dflt);
const char *policy_name(Policy p);

struct NodeState {
    int rank = -1;
    bool joined = false;
    bool alive = false;
    int gpu = -1;
    uint64_t gpu_capacity = 0, gpu_reserved = 0;
    uint64_t host_capacity = 0, host_reserved = 0;
    std::string host;
    uint64_t boot_id = 0;      // identifies one ocmd process lifetime (resume: same id = memory survived)
    std::vector<uint8_t> hops; // by GPU ordinal on its host: xGMI hops from this node's GPU (MSG_NODE_LINKS)
};

struct PlacedExtent {
    int owner = -1;
    uint32_t tier = TIER_NONE;
    uint64_t bytes = 0;
    bool spilled = false;
    bool net = false;      // owner on another host: reached through the network tier
    bool held = true;      // capacity reserved in the directory (false while unconfirmed after a resume)
};

struct PlaceRequest {
    int orig_rank = 0;
    int remote_rank = -1;
    uint64_t bytes = 0;
    uint32_t flags = 0;         // ocm_alloc_flags
    uint32_t stripe_width = 0;  // 0 = all peers
    uint64_t stripe_unit = 0;
    bool remote = true;         // false: local kind (owner = orig)
    uint32_t local_tier = TIER_HOST;
    int app_pid = 0;
};

struct Placement {
    uint64_t alloc_id = 0;
    uint64_t stripe_unit = 0;   // 0: single extent
    std::vector<PlacedExtent> extents;
    int err = 0;                // errno (ENOMEM, EINVAL, EHOSTDOWN)
};

class Governor {
public:
    Governor(int num_nodes, Policy policy, uint64_t default_stripe_unit);
    // ADD_NODE. A node that comes back with the same boot id kept its memory:
    // its extents stay in the directory, unconfirmed until it reports them
    // (confirm_extent ... end_reconcile). Any other (re)join drops what the
    // directory thought it owned.
    void add_node(const NodeConfig &cfg, uint64_t boot_id = 0);
    void mark_dead(int rank);
    // A node's xGMI table (MSG_NODE_LINKS): same-host peers are then tried
    // nearest first (ring order among equals), so ring / least_loaded / stripe
    // prefer 1-hop GPUs. Without tables every peer is equally near.
    void set_links(const NodeLinks &l);
    // xGMI hops from rank a's GPU to rank b's GPU; kHopsUnknown when not on one host / unknown.
    int hops(int a, int b) const;
    const NodeState &node(int rank) const { return nodes_.at(rank); }
    int num_nodes() const { return static_cast<int>(nodes_.size()); }
    int num_alive() const;
    Policy policy() const { return policy_; }

    // Decide owners for a request, reserve capacity, assign an alloc_id.
    Placement place(const PlaceRequest &r);
    // Re-place one extent of a live allocation after its owner failed DO_ALLOC.
    // Returns false when nothing fits.
    bool replace_extent(uint64_t alloc_id, int extent_idx, int failed_owner, PlacedExtent *out);
    // Release an allocation (all extents). Returns false when unknown.
    bool release(uint64_t alloc_id);
    // Drop every allocation of an app (crash reclaim) or whose origin died.
    std::vector<uint64_t> allocations_of_app(int orig_rank, int pid) const;
    std::vector<uint64_t> allocations_from(int orig_rank) const;
    size_t live_allocations() const { return table_.size(); }
    uint64_t spilled_count() const { return n_spilled_; }

    // ---- checkpoint / resume (persist the rank0 directory) ----
    // An owner's report of one extent it holds (OWNED): confirms a restored
    // entry or adds one placed after the last checkpoint; re-reserves capacity.
    void confirm_extent(int owner, const Region &r, int app_pid);
    // End of that owner's report (OWNED_DONE): extents still unconfirmed on it
    // were freed while rank0 was away. Returns how many were dropped.
    int end_reconcile(int owner);
    // Text snapshot of the directory (entries, id counter, node boot ids).
    std::string checkpoint() const;
    // Load a snapshot into an empty governor: entries start unconfirmed and
    // reserve nothing until their owners rejoin. Returns entries or -1.
    int restore(const std::string &text, std::string *err);
    // Bumped by every directory mutation (the daemon checkpoints when it moves).
    uint64_t version() const { return version_; }

    struct Entry {
        int orig_rank;
        int pid;
        Placement placement;
        std::vector<std::pair<int, uint32_t>> failed;  // (owner, tier) that refused DO_ALLOC
        int replacements = 0;
    };
    const Entry *find(uint64_t id) const;

private:
    bool fits(const NodeState &n, uint32_t tier, uint64_t bytes) const;
    void reserve(int rank, uint32_t tier, uint64_t bytes, int sign);
    std::vector<int> candidates(const PlaceRequest &r) const;         // same-host peers, ring order
    std::vector<int> remote_candidates(const PlaceRequest &r) const;  // other hosts, ring order
    bool place_one(int preferred, uint64_t bytes, uint32_t want_tier, bool allow_spill,
                   const std::vector<int> &fallback, const std::vector<int> &spill_to, PlacedExtent *out);

    std::vector<NodeState> nodes_;
    Policy policy_;
    uint64_t default_stripe_unit_;
    uint64_t next_id_ = 1;
    uint64_t n_spilled_ = 0;
    uint64_t version_ = 0;
    std::map<uint64_t, Entry> table_;
};

// Stripe geometry shared by the governor, daemon and data plane: an allocation
// of `total` bytes striped over `n` extents in units of `unit` bytes puts unit
// u on extent u % n at extent offset (u / n) * unit.
uint64_t stripe_extent_bytes(uint64_t total, uint64_t unit, int n, int idx);

}  // namespace ocm
