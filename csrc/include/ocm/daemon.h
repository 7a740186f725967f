// ocmd: one daemon per MI355X (or per host when CPU-only).
//
// Parity with reference src/main.c + src/mem.c (daemon entry, app registry,
// mailbox poller, inter-daemon protocol, listener/inbound/request threads) and
// src/alloc.c (owner-side alloc/free). Re-designed as ONE epoll event loop:
//   * app mailbox (POSIX mqueue fd), mesh sockets, app pidfds (crash reclaim),
//     signalfd — no thread per request, no usleep(500) poll, no busy spin;
//   * persistent mesh links instead of a TCP connection per RPC;
//   * rank0 owns the Governor (directory + placement);
//   * owners serve DO_ALLOC from a registered Arena (HBM slabs exported with
//     hipIpcGetMemHandle, pinned host-tier slabs);
//   * requests are asynchronous state machines keyed by a sequence number.
#pragma once
#include <sys/types.h>

#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "ocm/arena.h"
#include "ocm/governor.h"
#include "ocm/msg.h"
#include "ocm/netdata.h"
#include "ocm/nodefile.h"
#include "ocm/pmsg.h"
#include "ocm/siphash.h"
#include "ocm/sock.h"
#include "ocm/shmlink.h"
#include "ocm/tick.h"

namespace ocm {

struct DaemonConfig {
    std::string nodefile;
    int rank = -1;
    int gpu = -2;                    // -2 auto, -1 CPU-only, >=0 explicit
    std::string ns;
    Policy policy = Policy::Ring;
    uint64_t stripe_unit = 1ull << 20;
    uint64_t slab_bytes = 4ull << 30;  // HBM slab: requests < 2 GiB carve from resident slabs
    uint64_t gpu_capacity = 0;       // 0: fraction of free HBM
    double gpu_fraction = 0.75;
    uint64_t host_capacity = 0;      // 0: fraction of MemAvailable
    double host_fraction = 0.25;
    int join_timeout_ms = 60000;
    bool zero_on_alloc = false;
    std::string ready_file;
    std::string bind_ip;             // default: 0.0.0.0
    std::string ctrl = "auto";       // daemon<->daemon records: auto | tcp | rccl | socket (tick transports)
    int watch_pid = 0;               // exit when this process (the launcher) exits
    uint64_t lease_bytes = 1ull << 30;  // HBM leased per owner for local sub-allocation (0 = off)
    int lease_after = 2;             // normal placements on an owner before leasing there
    int lease_idle_ms = 2000;        // give an empty lease back after this long (capacity is not stranded)
    bool lease_host = false;         // also lease host-tier capacity (tests; OCM_LEASE_HOST=1)
    std::string host_alias;          // report this host name (tests: pretend daemons are on other nodes)
    std::string mesh_key;            // OCM_MESH_KEY: shared secret mixed into the mesh HELLO token
    std::string state_file;          // rank0: directory checkpoint (resume after a rank0 restart)
    int state_interval_ms = 20;      // max staleness of that checkpoint while the directory changes
    int spin_us = 50;                // after activity, poll without sleeping this long (0: always block)
};

int parse_daemon_args(int argc, char **argv, DaemonConfig *cfg, std::string *err);

class Daemon {
public:
    explicit Daemon(const DaemonConfig &cfg);
    ~Daemon();
    int run();           // blocks until shutdown; returns exit code
    void request_stop() { stop_ = true; }

private:
    struct App {
        pid_t pid = 0;
        int fd = -1;               // mailbox connection the app CONNECTed on
        int pidfd = -1;
        std::deque<Msg> backlog;
        bool watching_out = false;
        std::shared_ptr<ShmLink> link;  // shared-memory fast path (ocm/shmlink.h), if the app offered one
        std::deque<Msg> link_backlog;   // replies waiting for room in the link's ring
        bool overflowed = false;        // its replies piled up past kAppBacklogMax: being dropped
    };
    struct AppConn {
        int fd = -1;
        pid_t peer_pid = -1;       // SO_PEERCRED
        pid_t app_pid = 0;         // set by MSG_CONNECT
        bool same_user = true;     // SO_PEERCRED uid is ours or root (others: OCM_ALLOW_ANY_UID)
    };
    struct Pending {
        uint64_t seq = 0;
        uint64_t app_seq = 0;     // the app's correlation id, echoed in the reply
        long t0_ms = 0;           // for the request timeout sweep
        pid_t pid = 0;            // 0: internal (reclaim), no app reply
        uint32_t type = 0;        // MSG_REQ_ALLOC / MSG_REQ_FREE / MSG_STATS
        int expect = 0, got = 0;
        int err = 0;
        uint64_t alloc_id = 0;
        uint64_t stripe_unit = 0;
        uint64_t total_bytes = 0;
        uint32_t kind = 0;
        std::vector<Region> extents;
        std::vector<bool> have;
        std::set<int> awaiting;   // ranks we wait on (peer death fails the request)
        int lease_owner = -1;     // >= 0: this is a lease request for that owner
        uint32_t lease_tier = 0;
    };
    // A chunk of an owner's HBM leased to this (origin) daemon: small remote
    // allocations on that owner are carved from it and freed locally, with no
    // mesh round trip (rank0 reserved the whole chunk when granting it).
    struct Lease {
        int owner = -1;
        uint32_t tier = TIER_GPU;
        Region base;               // the chunk as the owner exported it
        RangeAllocator ra;
        long idle_since_ms = 0;    // last time it became empty
    };
    struct OriginAlloc {
        pid_t pid = 0;
        bool remote = false;
        int lease = -1;            // index into leases_ when carved from a lease
        uint64_t bytes = 0;
        std::vector<Region> extents;
    };
    struct OwnedExtent {
        uint32_t slab_id = 0;
        uint64_t offset = 0;
        uint32_t tier = 0;
        int orig_rank = -1;
        uint64_t bytes = 0;
        // what rank0 needs to rebuild its directory entry after a restart
        int app_pid = 0;
        uint16_t flags = 0;
        uint16_t n_extents = 1;
        uint64_t stripe_unit = 0;
        uint64_t grant = 0;        // network tier: the data-server capability of this extent
    };

    int init();
    void shutdown();
    int loop();
    void ep_add(int fd, uint32_t events, uint64_t tag);
    void ep_mod(int fd, uint32_t events, uint64_t tag);
    void ep_del(int fd);

    // sources
    void on_mailbox();
    void on_app_conn(int fd, uint32_t events);
    void close_app_conn(int fd);
    void on_accept();
    void on_conn_readable(int fd);
    void on_conn_writable(int fd);
    void on_pidfd(pid_t pid);
    void on_signal();
    void drop_conn(int fd);

    // dispatch
    void handle_app_msg(Msg &m);
    // via_tick: delivered by the tick transport (from_fd -1); the local queue passes false.
    void handle_mesh_msg(Msg &m, int from_fd, bool via_tick = false);
    // Shared-memory links of the apps: take their requests (returns how many),
    // and the daemon_polling flag around the event loop's sleeps.
    int poll_links();
    void links_polling(bool on);
    bool links_polling_ = true;
    int pending_link_fd_ = -1;  // a link memfd that arrived with MSG_CONNECT, for app_connect
    // An app that never takes its replies (socket or link) must not grow the
    // daemon without bound: past this many queued replies it is disconnected
    // and its memory reclaimed, as if it had died.
    static constexpr size_t kAppBacklogMax = 4096;
    std::vector<pid_t> overflowed_apps_;
    std::vector<pid_t> link_pids_;  // poll_links scratch
    int links_backlogged_ = 0;      // apps whose replies wait for ring room (after the last poll_links)
    void reap_overflowed_apps();
    void app_overflowed(App &a);
    // Once a tick transport exists, the allocation protocol's records are
    // remembered by content: when the transport fails, a sender re-sends over TCP
    // every record it cannot prove delivered (TickTransport::take_unsent), and a
    // copy of one that did arrive (by the tick, or by TCP first) is dropped here
    // instead of being handled twice (a second DO_ALLOC would leak the first
    // extent; a second DO_ALLOC response would free a live one). Those records
    // are unique by construction (seq, alloc_id, extent index), so a repeat is
    // always such a copy.
    // A record that reached us both through a tick and as a kMsgResent TCP copy
    // (the tick fallback): the second arrival is dropped. Only those two paths are
    // compared; plain TCP records are never de-duplicated.
    bool mesh_duplicate(const Msg &m, bool via_tick, bool resent);
    struct SeenWindow {  // content hashes, bounded, oldest first
        std::unordered_multiset<uint64_t> set;
        std::deque<uint64_t> order;
        void add(uint64_t h);
        bool take(uint64_t h);  // true (and forgotten) if present
    };
    SeenWindow seen_tick_, seen_resent_;
    uint64_t mesh_dups_dropped_ = 0;
    void send_rank(int r, Msg &m);      // to a daemon (self = local queue)
    void send_app(pid_t pid, const Msg &m);

    // protocol steps
    void app_connect(const Msg &m, int fd);
    void app_disconnect(pid_t pid, bool crashed);
    void app_req_alloc(Msg &m);
    void app_req_free(Msg &m);
    void app_stats(Msg &m);
    void app_tick_stats(Msg &m);
    void r0_add_node(const NodeConfig &cfg, uint64_t boot_id);
    void join_rank0();                   // ADD_NODE + OWNED report (boot and rejoin)
    void try_rejoin_rank0();             // survivors: reconnect to a restarted rank0
    void save_checkpoint(bool force);
    void r0_req_alloc(Msg &m);
    void r0_place_fail(Msg &m);
    void owner_do_alloc(Msg &m);
    void owner_do_free(Msg &m);
    int free_owned(const OwnedExtent &oe);
    void origin_do_alloc_resp(Msg &m);
    void origin_do_free_resp(Msg &m);
    void finish_alloc(Pending &p);
    void start_free(uint64_t alloc_id, pid_t reply_pid, uint64_t reply_seq);
    void fail_pending_on(int rank);
    void peer_lost(int rank);
    void sweep_timeouts();
    bool try_lease_alloc(Msg &m);
    void request_lease(int owner, uint32_t tier);
    void return_idle_leases();
    int preferred_owner() const;
    bool cross_host(int a, int b) const;
    void start_tick(const uint8_t *id, bool rccl, uint32_t idle_us);
    // Leave the tick transport (it failed here, a peer died, or a peer left it):
    // abort it, re-send over TCP every record it cannot prove delivered, and tell
    // the peers once (MSG_TICK_STOP) so the whole mesh leaves it together instead
    // of an idle rank posting into a collective nobody else runs any more.
    void leave_tick(const char *why);
    bool tick_left_ = false;
    // Control-plane bootstrap (n > 1). rank0 resolves --ctrl (auto: RCCL when the
    // nodefile gives every rank a GPU of its own, else TCP) and tells each peer as
    // soon as its link is up: MSG_TICK_START (u.raw = the ncclUniqueId, seq = the
    // collective: 1 RCCL, 2 socket) or MSG_TICK_STOP (TCP). A peer defers its join
    // (ADD_NODE, NODE_LINKS, OWNED) until its tick transport is up, so the join is
    // the transport's first traffic, or until it is told TCP / gives up after
    // OCM_TICK_UP_MS: then the join rides TCP.
    std::string ctrl_mode_ = "tcp";     // rank0's resolved transport: tcp | rccl | socket
    uint8_t tick_uid_[128] = {};
    bool join_deferred_ = false;        // our join waits for the transport decision / the tick
    long tick_deadline_ms_ = 0;         // bootstrap bound (0: none pending)
    int tick_up_ms_ = 20000;            // OCM_TICK_UP_MS
    // Idle ticks (OCM_TICK_IDLE_US, default 1000; 0: the round-3 protocol, where an
    // idle mesh stops and a rank starting a burst wakes its peers over TCP). rank0's
    // value travels in MSG_TICK_START (pid field) so every rank runs the same ticks.
    uint32_t tick_idle_us_ = 1000;
    uint32_t *tick_bell_ = nullptr;     // the host-wide tick doorbell (shared memory), idle ticks only
    uint64_t tcp_wakes_ = 0;            // MSG_TICK_WAKE records sent (TickStatsWire::tcp_wakes)
    void resolve_ctrl();                // rank0, at init
    void send_ctrl_decision(int r);     // rank0 -> rank r, once its link is up
    void join_now(const char *why);     // the deferred join, over whatever transport is up
    void check_tick_bootstrap();        // deadlines, from the event loop
    void on_tick();
    void send_tcp(int r, Msg &m);

    NodeConfig my_config() const;
    void check_ready();
    uint64_t next_seq() { return ++seq_; }

    DaemonConfig cfg_;
    NodeFile nf_;
    int rank_ = -1, n_ = 0, gpu_ = -1, num_gpu_ = 0;
    uint64_t gpu_total_ = 0;
    std::string ns_;
    int mbox_fd_ = -1;                             // listening app mailbox
    std::map<int, AppConn> app_conns_;             // fd -> connection
    int ep_ = -1, listen_fd_ = -1, sig_fd_ = -1;
    bool stop_ = false, ready_ = false;
    std::unique_ptr<Arena> arena_;
    std::unique_ptr<Governor> gov_;
    std::map<int, std::unique_ptr<Conn>> conns_;   // fd -> connection
    std::vector<int> peer_fd_;                     // rank -> fd (-1 none)
    std::vector<NodeConfig> table_;
    std::vector<bool> joined_;
    std::deque<Msg> self_q_;
    std::map<pid_t, App> apps_;
    std::map<uint64_t, Pending> pending_;
    std::map<uint64_t, OriginAlloc> origin_allocs_;
    std::map<std::pair<uint64_t, int>, OwnedExtent> owned_;
    uint64_t seq_ = 0, local_ids_ = 0;
    int request_timeout_ms_ = 30000;
    std::unique_ptr<TickTransport> tick_;
    std::unique_ptr<DataServer> data_;  // network tier: serves PUT/GET from other nodes
    std::vector<std::unique_ptr<Lease>> leases_;
    std::map<int, int> lease_demand_;   // owner -> normal placements seen
    std::set<int> lease_inflight_;      // owners with an outstanding lease request
    uint64_t lease_ids_ = 0, n_lease_allocs_ = 0;
    // Fault injection (OCM_FAULT="do_alloc_fail=N,drop_do_alloc=N,crash_after_allocs=N"):
    int fault_alloc_fail_ = 0, fault_drop_alloc_ = 0, fault_crash_after_ = -1;
    void parse_faults();
    uint64_t n_alloc_ = 0, n_free_ = 0, n_reclaimed_ = 0, n_spilled_ = 0;
    // checkpoint / resume
    uint64_t boot_id_ = 0;               // this process lifetime
    std::vector<int> orig_cpus_;         // the process's mask before the event loop was pinned
    std::vector<int> near_cpus_;         // the GPU's L3 complex minus the event loop's core (tick thread)
    size_t pinned_cpus_ = 0;             // event loop restricted to this many CPUs near the GPU (0: not pinned)
    SipKey mesh_key_{};                  // HELLO MAC key (namespace + OCM_MESH_KEY)
    std::unordered_map<uint64_t, uint64_t> hello_seen_;  // nonce -> ts_ms of HELLOs accepted in the window
    bool hello_ok(const Msg &m);
    uint64_t data_token_ = 0;            // network-tier data server: random per boot
    NodeLinks links_{};                  // xGMI link table of our GPU (sent to rank0 after ADD_NODE)
    void probe_links();
    void send_hello(int fd, int dst_rank);
    bool resumed_ = false;               // rank0 restored its directory from state_file
    uint64_t saved_version_ = 0;
    long last_save_ms_ = 0;
    bool r0_lost_ = false;               // survivors: link to rank0 down, retrying
    long next_rejoin_ms_ = 0;
};

}  // namespace ocm
