// libocm internals shared by the library's translation units (not installed).
//
// runtime.cpp  process state, mailbox RPC, IPC/memfd import cache, local halves
// transfer.cpp copy engine: segments, lanes/events, copy service, xfer, local copies
// net.cpp      network-tier client (owners on other nodes)
// batch.cpp    batched one-sided ops, stream interop, transfer plans (hipGraph)
// libocm.cpp   the C ABI (oncillamem.h)
#pragma once
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "oncillamem.h"
#include "ocm/log.h"
#include "ocm/msg.h"
#include "ocm/netdata.h"
#include "ocm/pmsg.h"
#include "ocm/range_alloc.h"
#include "ocm/shmlink.h"
#include "ocm/sock.h"
#include "ocm/trace.h"
#include "ocm/aql.h"
#include "ocm/xfer.h"


namespace ocmlib {
using namespace ocm;
#pragma GCC visibility push(hidden)


enum Loc { LOC_HOST = 0, LOC_PINNED = 1, LOC_DEVICE = 2 };

// Resident copy service defaults (OCM_SERVICE_MAX / _BLOCKS / _SOLO_TILES).
// Measured (profiles/svc_probe_r01.json): a 32-workgroup gang beats a kernel
// launch + sync (13.7-14.9 us) up to 4 MiB on HBM pairs: 8.8 us at 128 KiB-1 MiB,
// 11.8 us at 4 MiB; requests of <= 2 tiles (64 KiB) stay on workgroup 0 (4.6 us at 4 KiB).
constexpr uint64_t kServiceMaxDefault = 4ull << 20;
// Pairs whose remote half is all host tier: the gang stays ahead of the DMA
// engines up to 16 MiB (8 MiB 152/155 us against 164/164, 16 MiB 300/303 against
// 312/312 put/get; profiles/svc_max_ab_r02.json). OCM_SERVICE_MAX_HOST.
constexpr uint64_t kServiceMaxHostDefault = 16ull << 20;
// 128 workgroups: with the direct gang record only 16 of them poll host memory,
// so the width costs small ops nothing, and HBM gangs of 4-64 MiB run 1.5-7 us
// faster than 32 (or a launch); host-tier gangs stay at 32, since wider ones
// lose at 8-16 MiB (188 vs 153 us; profiles/svc_blocks_r02.json).
constexpr int kServiceBlocksDefault = 128;
constexpr unsigned kServiceGangHostDefault = 32;
// Pairs wholly in this GPU's HBM keep blocking ops up to 64 MiB on the service
// (64 MiB: 23.5-24 vs 30.5 us for launch + completion); peer HBM over xGMI
// keeps kServiceMaxDefault, above which the autotuned launches take over.
constexpr uint64_t kServiceMaxLocalDefault = 64ull << 20;
constexpr int kServiceSoloTilesDefault = 2;
constexpr int kServiceIdleUsDefault = 50;
constexpr int kServiceLoneUsDefault = 2000;
// Write-through hand-offs, the records in write-combined memory, and gang
// requests polled directly by the first 16 workgroups: small ops -0.1/-0.2 us,
// host-tier 128 KiB-4 MiB and HBM 256 KiB-1 MiB gangs 1-1.5 us faster than the
// relay (profiles/svc_direct_gang_ab_r02.json, svc_direct_hybrid_r02.json).
// Round 3: gangs complete through per-workgroup done words (WGDONE) instead of a
// device-scope counter: host-tier 64-128 KiB ops 0.2-0.3 us faster, 256 KiB-4 MiB
// 0.1 us, small ops unchanged (profiles/svc_wgdone_ab_r03.json).
constexpr unsigned kServiceProtoDefault =
    kServiceProtoWT | kServiceProtoGangRec | kServiceProtoWCReq | kServiceProtoWgDone;
constexpr int kServiceDirectDefault = 16;
// Direct gangs (at most kServiceDirectDefault workgroups) for ops up to these
// sizes; wider relayed gangs above, where 16 workgroups copy too slowly
// (host-tier 16 MiB get 310-320 vs 302 us; HBM 4 MiB 10.9 vs 9.1 us).
constexpr uint64_t kServiceDirectMaxHost = 4ull << 20;
constexpr uint64_t kServiceDirectMaxHbm = 1ull << 20;
// Kernel-published completion of blocking launches (XferDone) up to this size.
// Measured on HBM pairs (profiles/launch_flag_r01.json): 9.1-13.4 us against
// 13.0-14.6 us with the runtime event up to 4 MiB; above that the per-workgroup
// system-scope writeback costs more than it saves (16 MiB: 30.9 against 15.8 us).
constexpr uint64_t kLaunchFlagMaxDefault = 4ull << 20;

// One data-server connection of the network tier, with its own pinned staging
// buffer for device-side local halves (allocated on first device use).
struct NetConn {
    int fd = -1;
    void *stage = nullptr;
};

struct Extent {
    Region r;
    char *dptr = nullptr;  // device-usable address of the extent start (nullptr: none)
    char *hptr = nullptr;  // host address (host tier only)
    bool dev_ok = false;   // a kernel on this process's GPU can access dptr
    bool net = false;      // owner on another node: streamed through its data server
    std::string ep;        // "ip:port" of that data server
    uint64_t net_token = 0;  // presented first on each connection to it
    uint64_t net_grant = 0;  // this extent's capability, named by every request
};


}  // namespace ocmlib

// lib_alloc is the public opaque handle (oncillamem.h), so it keeps default visibility
// while the ocmlib types it holds are hidden; g++ warns about that (-Wattributes), clang
// does not. Hiding lib_alloc instead would hide every C entry point taking it.
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wattributes"
struct lib_alloc {
    enum ocm_kind kind;
    uint64_t alloc_id = 0;
    void *local = nullptr;
    size_t local_bytes = 0;
    ocmlib::Loc loc = ocmlib::LOC_HOST;
    bool remote = false;
    size_t remote_bytes = 0;
    uint64_t stripe_unit = 0;
    std::vector<ocmlib::Extent> ext;
    bool all_gpu = false;
    bool any_gpu = false;
    bool all_dev_ok = false;  // every extent reachable by a kernel on this GPU
    bool any_net = false;     // some extent lives on another node
    bool same_gpu = false;    // every extent in this process's own GPU's HBM (another daemon on it, via IPC)
    bool any_peer = false;    // some extent in ANOTHER GPU's HBM (xGMI): the copy service's fenced hand-off
    bool async_pending = false;
    bool pooled = false;      // local half from the stream-ordered pool
    int lane = -1;            // async ops: index into State::lanes (per-allocation ordering)
    hipEvent_t ev = nullptr;  // completion of the last async op (ocm_wait)
    void *batch_dev = nullptr;  // device copy of large batch descriptor lists
    void *batch_host = nullptr; // pinned staging for their upload
    size_t batch_cap = 0;
    hipEvent_t batch_up = nullptr;  // the last upload out of batch_host finished
    hipEvent_t dep_ev = nullptr;    // ocm_stream_wait: external work the next op depends on
    bool dep_pending = false;
    int plans = 0;                  // ocm_plan stages that reference this allocation
};
#pragma GCC diagnostic pop

struct ocm_plan {
    struct Stage {
        lib_alloc *a = nullptr;
        ocm::XferBatchArgs args;
        void *dev = nullptr;  // descriptors + wave table (large lists)
    };
    std::vector<Stage> stages;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    uint64_t bytes = 0, n_ops = 0;
};


namespace ocmlib {

struct SlabKey {
    int owner;
    uint32_t tier;
    uint32_t slab;
    bool operator<(const SlabKey &o) const {
        return owner != o.owner ? owner < o.owner : tier != o.tier ? tier < o.tier : slab < o.slab;
    }
};

struct Mapping {
    char *dbase = nullptr;
    char *hbase = nullptr;
    uint64_t bytes = 0;
    uint8_t handle[kHandleBytes] = {};
    int refs = 0;
    bool dedicated = false;
    bool registered = false;
    // HBM slabs: the same slab opened on OTHER devices of this process (push-based
    // gets launch on the owner's GPU and need an address valid there).
    std::map<int, char *> dev_views;
};

// Push-based gets: one stream per owner device this process launches on.
struct PushDev {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    bool ready = false;
};

struct State {
    std::recursive_mutex mu;
    bool inited = false;
    pid_t pid = 0;
    std::string ns, daemon_mbox;
    Channel chan;
    ShmLink link;
    bool last_via_link = false;  // the last record recv_record returned came over the link  // shared-memory fast path to the daemon (OCM_SHM_LINK=0: the mailbox alone)
    NodeConfig daemon{};
    int daemon_rank = 0;
    int device = -1;
    // xGMI self-diagnosis (ocm_x_xgmi_diag): peers this device got access to at
    // init, and slabs of OTHER GPUs' HBM imported / refused by hipIpcOpenMemHandle.
    int peers_enabled = 0;
    uint64_t ipc_peer_imports = 0, ipc_peer_failures = 0;
    hipStream_t stream = nullptr;
    uint64_t seq = 0;
    std::map<SlabKey, Mapping> imports;
    std::set<lib_alloc *> allocs;
    XferTuning tuning;
    // Per-direction override ([0] get, [1] put) for one-sided kernel ops,
    // set by an autotune (variant XFER_AUTO: use `tuning`).
    XferTuning dir_tuning[2];
    // Host-tier pairs: the PCIe streaming kernel (default), or with OCM_HOST_ENGINE=sdma
    // the runtime's copy engines above host_kernel_max (the measured baseline).
    bool host_engine_kernel = true;
    uint64_t host_kernel_max = 0;
    int sync_mode = 0;             // 0 stream sync, 1 spin on an event, 2 blocking event sync
    OpCounters ctr;
    // persistent copy service (small blocking one-sided ops)
    ServiceSlot *svc = nullptr;
    ServiceReq *svc_req = nullptr;   // request record (&svc->req)
    ServiceReq *svc_greq = nullptr;  // GANGREC: gang requests' record, a page of its own
    unsigned svc_greq_copies = 1;    // COPIES: one gang record per direct poller on that page
    char *svc_rec_pages = nullptr;   // separately allocated record pages (GANGREC / WCREQ), freed at stop
    ServiceBox *svc_box = nullptr;   // device-memory mailbox of the gang (the current lane's)
    unsigned long long *pattern_bad = nullptr;  // device counter of ocm_x_pattern checks
    hipStream_t svc_stream = nullptr;  // the current lane's stream
    // Lanes of the service: a stream and a gang box each. An instance whose lead has
    // left may still have workgroups that never got a CU (another process holds
    // them); the next instance starts on a lane whose stream has drained, a new lane
    // (up to OCM_SERVICE_STREAMS, default 4), or waits for one. Requests carry the
    // instance's epoch (ocm/xfer.h), so such a late workgroup never takes one.
    struct SvcLane {
        bool aql = false;                   // an AQL queue of the library's own (else `stream`)
        AqlLane q;
        hipStream_t stream = nullptr;
        ServiceBox *box = nullptr;
        bool dirty = true;                  // clear the box before its next launch
        unsigned long long checkins = 0;    // the box's check-in counter once its instances drained
        unsigned long long gang_total = 0;  // the box's gang completion counter (mirror)
    };
    std::vector<SvcLane> svc_lanes;
    // OCM_SERVICE_QUEUE=aql (default): lanes are AQL queues when the embedded code
    // object loads (svc_aql), =hip: HIP streams.
    bool svc_queue_aql = true, svc_aql = false;
    AqlKernel svc_kernel;
    AqlKernel svc_clear_kernel;     // ocm_service_box_clear (object 0: clear with a host memset)
    // Lone lead (ocm/xfer.h): the lead stays resident alone this long after the
    // members left (OCM_SERVICE_LONE_US; AQL lanes only, 100 MHz ticks). 2 ms: a
    // 4 KiB op after a 1 ms pause stays hot (6.4-6.8 us against 17 us through a
    // relaunch), while any resident workgroup delays a full-GPU GEMM launched
    // meanwhile by ~45% (bf16 8192^3: 0.93 -> 1.38 ms: the CU it holds runs its
    // tile late), so the window stays short (profiles/lone_sweep_r04.json).
    unsigned long long svc_lone_ticks = 100ull * kServiceLoneUsDefault;
    uint64_t svc_promotions = 0;  // gang ops that replaced a lone lead with a full instance
    uint64_t svc_overlaps = 0;    // instances dispatched on a lane whose previous lead had not left yet
    uint64_t svc_drain_max_ns = 0;   // the longest wait for a lane to drain (health)
    unsigned svc_drain_max_site = 0; // where: 1 start, 2 park, 3 stop, 4 abort, 5 re-post
    int svc_lane = -1;
    unsigned svc_lanes_max = 4;
    unsigned svc_epoch = 0;
    int svc_stream_prio = 0;
    bool svc_prio_ok = false;
    uint64_t svc_degraded_idle_ticks = 100ull * 5000;  // OCM_SERVICE_DEGRADED_IDLE_US (5 ms)
    unsigned svc_blocks = kServiceBlocksDefault;          // gang size (OCM_SERVICE_BLOCKS)
    unsigned svc_solo_tiles = kServiceSoloTilesDefault;  // requests of <= this many tiles stay on workgroup 0
    unsigned svc_solo_tiles_host_get = 1;  // ... for gets from the host tier (OCM_SERVICE_SOLO_TILES_HOST_GET)
    unsigned svc_proto = kServiceProtoDefault;           // hand-off protocol bits (OCM_SERVICE_PROTO)
    bool svc_force_strict = false;                       // OCM_SERVICE_STRICT: every request STRICT
    unsigned svc_direct = kServiceDirectDefault;          // GANGREC direct pollers (OCM_SERVICE_DIRECT)
    uint64_t svc_direct_max_host = kServiceDirectMaxHost;  // OCM_SERVICE_DIRECT_MAX_HOST
    uint64_t svc_direct_max_hbm = kServiceDirectMaxHbm;    // OCM_SERVICE_DIRECT_MAX_HBM
    // Smaller tiles for host-tier ops of svc_host_tile_min..max bytes (0: the 32 KiB
    // default), so a direct gang spreads them over more CUs' miss queues. Gets use
    // 16 KiB tiles there: 64/128/256 KiB 6.9/7.75/9.86 vs 7.6/8.3/10.4 us; 8 and 4 KiB
    // tiles lose, and so do puts and a 32 KiB get as a gang of two
    // (profiles/svc_host_tile_ab_r02.json). Puts take 16 KiB tiles there too since round 4:
    // with WGDONE completion and the roster a 64 KiB put as a gang of four beats it solo,
    // 64/128/256 KiB 6.2-6.4/6.9-7.3/9.2-9.3 vs 7.5-7.6/7.2-7.5/9.6-9.7 us in six interleaved
    // runs (profiles/host_mid_ab_r04p.json, profiles/host_put_ab_r04q.json).
    unsigned svc_host_tile_shift_get = 14, svc_host_tile_shift_put = 14;  // OCM_SERVICE_HOST_TILE_SHIFT_GET/_PUT
    uint64_t svc_host_tile_min = 64ull << 10;                             // OCM_SERVICE_HOST_TILE_MIN
    uint64_t svc_host_tile_max = 256ull << 10;                            // OCM_SERVICE_HOST_TILE_MAX
    // Host-tier gets of at least svc_host_get_narrow_min bytes go to at most
    // svc_host_get_width members: fewer reads in flight over PCIe end closer together.
    // 1/2/4 MiB gets 24.5-24.6/43.3/79.9 us with 12 members against 25.8-26.1/44.7-45.1/
    // 81.8-82.1 with 16; 512 KiB keeps 16 (14.9-15.0 against 15.2-15.4 with 12), and 8 or
    // 4 members lose (profiles/host_wide_ab_r04q.json).
    uint64_t svc_host_get_narrow_min = 1ull << 20;  // OCM_SERVICE_HOST_GET_NARROW_MIN
    unsigned svc_host_get_width = 12;               // OCM_SERVICE_HOST_GET_WIDTH
    bool svc_running = false;
    bool svc_shared_queue = false;  // no priority stream for the service: it may share a launch stream's hardware queue
    bool svc_park_kernel = false;  // park the service during kernel transfers above svc_max (OCM_SERVICE_PARK_KERNEL)
    unsigned long long svc_seq = 0;
    uint64_t svc_ops = 0, svc_ns_post = 0, svc_ns_wait = 0;  // service diagnostics (ocm_x_service_stats)
    uint64_t svc_gpu_ticks_done = 0;  // GPU ticks of the instances before the current one
    uint64_t svc_max = kServiceMaxDefault;           // 0: the service is off (or failed)
    uint64_t svc_max_host = kServiceMaxHostDefault;  // the same bound for host-tier-only pairs
    // Largest blocking op the service takes for a pair with (`hbm`) or without HBM extents.
    uint64_t svc_max_local = kServiceMaxLocalDefault;  // ... for pairs wholly in this GPU's HBM (OCM_SERVICE_MAX_LOCAL)
    unsigned svc_gang_host = kServiceGangHostDefault;  // widest gang for host-tier ops (OCM_SERVICE_GANG_HOST)
    uint64_t svc_limit(const lib_alloc *a) const {
        if (svc_max == 0) return 0;
        if (!a->any_gpu) return svc_max_host;
        return a->same_gpu ? std::max(svc_max, svc_max_local) : svc_max;
    }
    // Idle exit after OCM_SERVICE_IDLE_US (50 us; 100 MHz ticks): long enough to
    // stay resident through a burst of blocking ops, short enough that a
    // device-wide synchronize right after one (torch.cuda.synchronize) does not
    // wait long for the persistent kernel to leave.
    unsigned long long svc_idle_ticks = 100ull * kServiceIdleUsDefault;
    uint64_t svc_relaunches = 0;    // instances started after an idle exit (ocm_x_service_stats)
    uint64_t svc_ns_relaunch = 0;   // host time of those restarts (reap + launch), ocm_x_service_health
    uint64_t svc_ns_pick = 0, svc_ns_launch = 0, svc_epoch_starts = 0;  // every start: choosing a lane, the launch call
    bool svc_relaunch_query = false;  // OCM_SERVICE_RELAUNCH_QUERY=1: always ask the runtime which lane drained
    // Roster (ocm/xfer.h): gangs are sized to the members already running. Right
    // after a launch a gang op waits up to svc_roster_wait_ns for the grid to check
    // in before it settles for fewer members (OCM_SERVICE_ROSTER_WAIT_US).
    uint64_t svc_launch_ns = 0;
    // A lane's gang box is zeroed only when it must be (ocm/xfer.h): at its first
    // launch, after an instance left a request unfinished, or always with
    // OCM_SERVICE_BOX_RESET=1. Otherwise the next instance's check-in tickets start
    // at the lane's `checkins` (every workgroup of every earlier instance took one).
    bool svc_box_reset_always = false;
    uint64_t svc_roster_wait_ns = 200000;
    // Health counters (ocm_x_service_health): gang ops sized below the width they
    // wanted because fewer members were resident, instances that left with the
    // posted op unfinished (re-posted), ops abandoned after OCM_SERVICE_TIMEOUT_MS
    // (drained, then redone by a launch), and whether an instance could not even
    // be drained (the service is then off for good and the op fails).
    uint64_t svc_degraded = 0, svc_incomplete_exits = 0, svc_aborts = 0;
    unsigned long long svc_roster_min = ~0ull;  // smallest roster a gang op was sized to
    bool svc_wedged = false;
    uint64_t svc_timeout_ns = 10ull * 1000000000ull;  // OCM_SERVICE_TIMEOUT_MS
    uint64_t svc_drain_ns = 10ull * 1000000000ull;    // OCM_SERVICE_DRAIN_MS: bound on the STOP drain after a timeout
    // network tier
    std::map<std::string, NetConn> net_conns;  // "ip:port#stream" -> connection
    std::map<int, int> fd_chans;               // owner rank -> mailbox connection for slab fds (MSG_SLAB_FD)
    int net_streams = 4;                       // OCM_NET_STREAMS: parallel connections per owner
    uint64_t net_split_min = 1ull << 20;       // OCM_NET_SPLIT_MIN: smallest part worth its own stream
    // Local GPU halves: stream-ordered pool (no device-wide sync in free, freed
    // blocks reused without a new VA mapping). Reference K8: cudaMalloc/cudaFree.
    hipMemPool_t pool = nullptr;
    // Async one-sided ops run on lane streams, one lane per allocation (round
    // robin), so ops on different allocations (different peers / links) overlap.
    std::vector<hipStream_t> lanes;
    int n_lanes = 4, next_lane = 0;
    // Kernel-published completion of blocking launch-path ops (XferDone), one
    // slot per lane: a host-coherent flag line and a device counter line.
    unsigned long long *lane_flags = nullptr;  // 16 words per lane
    unsigned int *lane_cnt = nullptr;          // 32 words per lane
    std::vector<unsigned long long> lane_flag_seq;
    bool launch_flags = true;                  // OCM_LAUNCH_FLAG=0 waits on the runtime event instead
    uint64_t launch_flag_max = kLaunchFlagMaxDefault;  // OCM_LAUNCH_FLAG_MAX
    bool pool_tried = false;
    uint64_t pool_keep = 8ull << 30;       // bytes kept reserved across frees
    // Freed pool blocks kept for an exact-size reuse (OCM_LOCAL_CACHE bytes, 0 = off):
    // a reuse needs no HIP call at all, where a pool allocation right after a
    // stream-ordered free must wait for that free on the stream.
    std::multimap<size_t, void *> dev_cache;
    uint64_t dev_cache_bytes = 0;
    uint64_t dev_cache_cap = 1ull << 30;
    hipEvent_t done = nullptr;
    int rpc_timeout_ms = 60000;
    uint64_t rpc_spin_ns = 50000;          // OCM_RPC_SPIN_US: poll for a reply this long before sleeping
    uint64_t pinned_keep = 2ull << 30;     // idle pinned chunks kept for reuse
    class PinnedArena *pinned = nullptr;   // created on first use
    std::map<int, PushDev> push;           // XFER_PUSH: owner device -> its stream
    hipEvent_t push_order = nullptr;       // the app stream's position the push launches wait for
    uint64_t push_launches = 0;
};

State &S();
int env_int(const char *k, int dflt);
long now_ms();
Msg new_msg(uint32_t type);
// Send a request and wait for the reply carrying the same seq.
int rpc(Msg &req, Msg *reply, int timeout_ms);
int recv_seq(Msg *m, uint64_t seq, uint32_t type, int timeout_ms);
bool is_pair(enum ocm_kind k);

struct DeviceGuard {
    int prev = -1;
    bool active = false;
    explicit DeviceGuard(int dev) {
        if (dev < 0) return;
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) {
            (void)hipSetDevice(dev);
            active = true;
        }
    }
    ~DeviceGuard() {
        if (active) (void)hipSetDevice(prev);
    }
};

inline int log2_exact(uint64_t v) {
    if (v == 0 || (v & (v - 1))) return -1;
    return __builtin_ctzll(v);
}

// ---- import cache (runtime.cpp)
int import_extent(Extent &e);
int slab_fd_from_owner(int owner, uint32_t slab_id);
void close_fd_chans();
void release_extent(const Extent &e, bool force);

// ---- pinned host arena for local halves (runtime.cpp)
// hipHostMalloc pins pages (64 MiB ~ 10 ms) and hipHostFree synchronizes the
// device (~230 us even for 4 KiB), so pinned local halves come from chunks
// pinned once: small requests are best-fit ranges of shared 64 MiB chunks,
// large ones get a dedicated chunk that is cached for reuse after free. Idle
// chunks beyond OCM_PINNED_KEEP bytes (default 2 GiB) are unpinned.
class PinnedArena {
public:
    void *alloc(size_t bytes);
    bool free(void *p);  // false: not from this arena
    void release_all();
    uint64_t pinned() const { return pinned_; }

private:
    struct Chunk {
        char *base = nullptr;
        uint64_t bytes = 0;
        bool dedicated = false;
        RangeAllocator ra;
    };
    void trim();
    std::map<uintptr_t, Chunk> chunks_;  // base -> chunk
    uint64_t pinned_ = 0;
};

// ---- local halves (runtime.cpp)
Loc pointer_loc(const void *p);
void release_dev_cache();
hipMemPool_t local_pool();
int free_local_half(lib_alloc *a);
int alloc_local_half(lib_alloc *a, size_t bytes, Loc want);

// ---- copy engine (transfer.cpp)
struct Seg {
    int ext;
    uint64_t ext_off;
    uint64_t lin_off;
    uint64_t len;
};
void segments(const lib_alloc *a, uint64_t rem_off, uint64_t len, std::vector<Seg> &out);
int wait_event(hipEvent_t ev);
int honor_dep(lib_alloc *a, hipStream_t st, bool host_wait);
int wait_alloc(lib_alloc *a);
hipStream_t lane_stream(lib_alloc *a);
int sync_stream();
int service_start(unsigned long long first_seq);
void service_park();
void service_stop();
// strict: an extent is in another GPU's HBM (kServiceGangStrict).
// 0: done; -1: failed, and no instance holds the request any more (a launch may
// redo the op); -2: failed and the instance could not be drained (no fallback).
int service_xfer(XferArgs x, unsigned solo_tiles, bool hbm, bool strict);
// Before a library launch: park the service when it may share the launch's hardware queue.
void before_launch();
// `done` (optional, async launches on a lane): receives the kernel-published
// completion flag of the launch, or flag == nullptr when the op has none.
int xfer(lib_alloc *a, bool put, char *lin, Loc lloc, uint64_t rem_off, uint64_t len, bool async,
         XferDone *done = nullptr);
// Wait for a kernel-published flag (>= val), with the runtime event as the backstop.
int wait_done(const XferDone &d, hipEvent_t ev);
int copy_local(void *dst, Loc dl, const void *src, Loc sl, size_t n);
// Push-based get (XFER_PUSH): launches on every owner's GPU, ordered after the work
// queued on `st`; blocking ops wait on the host, async ones make `st` wait.
int push_get(lib_alloc *a, char *lin, uint64_t rem_off, uint64_t len, hipStream_t st, bool async);
void push_release();
// An address of extent e valid on device `dev` (its owner's GPU), opening its slab there once.
char *extent_view(const Extent &e, int dev);

// ---- batches (batch.cpp)
int run_batch(lib_alloc *a, XferBatchArgs &args, std::vector<XferBatchOp> &v, bool async);
// Copy absolute device ranges (op.lin_off = address) into dst's remote half, one launch.
int batch_put_abs(lib_alloc *dst, std::vector<XferBatchOp> &v);

// ---- network tier (net.cpp)
void net_drop(const std::string &ep);
void net_close_all();
int net_piece(const Extent &e, bool put, char *lin, Loc lloc, uint64_t ext_off, uint64_t len);

#pragma GCC visibility pop
}  // namespace ocmlib
