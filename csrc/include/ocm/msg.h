// Wire record shared by app<->daemon (mailbox) and daemon<->daemon (mesh).
//
// Parity: reference inc/msg.h:24-73 defines one fixed 160-byte `struct message`
// with {type, status, pid, rank, union{request, allocation, node config}} and the
// CONNECT/ADD_NODE/REQ_ALLOC/DO_ALLOC/REQ_FREE/DO_FREE/RELEASE_APP states. This
// record keeps that size and those states, and adds what an asynchronous
// event-loop daemon needs: a correlation sequence number, an explicit sender
// rank and an error code. The allocation body carries the peer-memory export
// handle (hipIpcMemHandle_t, 64 B) where the reference carried ib_ip[64].
#pragma once
#include <cstddef>
#include <cstdint>

namespace ocm {

constexpr size_t kMsgBytes = 160;
constexpr size_t kHandleBytes = 64;  // == sizeof(hipIpcMemHandle_t)
constexpr int kMaxExtents = 8;       // == OCM_MAX_EXTENTS

enum MsgType : uint32_t {
    MSG_INVALID = 0,
    MSG_CONNECT,          // app -> daemon
    MSG_CONNECT_CONFIRM,  // daemon -> app (carries node config of the daemon)
    MSG_DISCONNECT,       // app -> daemon
    MSG_ADD_NODE,         // daemon -> rank0 on boot / rejoin (node config; seq = boot id)
    MSG_REQ_ALLOC,        // app -> daemon -> rank0
    MSG_DO_ALLOC,         // rank0 -> owner; owner -> origin daemon (response)
    MSG_REQ_FREE,         // app -> daemon
    MSG_DO_FREE,          // origin daemon -> owner; owner -> origin (response)
    MSG_RELEASE_APP,      // daemon -> app: request finished (header of a reply)
    // --- additions ---
    MSG_EXTENT,           // daemon -> app: one extent of a multi-extent reply
    MSG_HELLO,            // mesh link handshake
    MSG_NODE_TABLE,       // rank0 -> all: one node config per message
    MSG_PLACE_FAIL,       // owner -> rank0: DO_ALLOC failed, re-place
    MSG_FREED,            // owner -> rank0: capacity returned
    MSG_STATS,            // app -> daemon (-> peer): statistics query
    MSG_APP_DEAD,         // origin daemon -> rank0: app crashed, drop its directory entries
    MSG_SHUTDOWN,         // any -> daemon: orderly exit
    MSG_PING,             // liveness / latency probe
    MSG_TICK_START,       // rank0 -> all (TCP): start the tick transport; u.raw = ncclUniqueId
    MSG_TICK_WAKE,        // any -> all (TCP): join tick number u.req.bytes
    MSG_OWNED,            // daemon -> rank0 after ADD_NODE: one extent it holds (u.region, pid = app)
    MSG_OWNED_DONE,       // daemon -> rank0: end of that report
    MSG_NODE_LINKS,       // daemon -> rank0 after ADD_NODE: xGMI link type / hops from its GPU (u.links)
    MSG_SLAB_FD,          // app -> owner daemon: a host-tier slab's memfd (u.region.slab_id), reply carries it (SCM_RIGHTS)
    MSG_TICK_STOP,        // any -> all (TCP): the sender left the tick transport; leave it too (records ride TCP)
    MSG_WAKE,             // app <-> daemon (mailbox socket): look at the shared-memory link (ocm/shmlink.h)
    MSG_TICK_STATS,       // app -> its daemon: the tick transport's statistics (u.raw = TickStatsWire)
    MSG_MAX
};

enum MsgStatus : uint32_t { MSG_NO_STATUS = 0, MSG_REQUEST, MSG_RESPONSE };
// Status bit of a mesh record re-sent over TCP after the tick transport failed
// (TickTransport::take_unsent): the receiver drops it if the same record already
// came through a tick, and a later tick copy if it came first. Cleared on receipt.
constexpr uint32_t kMsgResent = 0x80000000u;

enum Tier : uint32_t { TIER_NONE = 0, TIER_HOST = 1, TIER_GPU = 2 };

// Request body (REQ_ALLOC / REQ_FREE / STATS).
struct AllocReq {
    int32_t orig_rank;     // daemon the app is attached to
    int32_t remote_rank;   // requested owner, -1 = rank0 decides
    uint64_t bytes;        // remote bytes (pairs) or local bytes (local kinds)
    uint32_t kind;         // enum ocm_kind of the app request
    uint32_t flags;        // enum ocm_alloc_flags
    uint32_t stripe_width;
    uint32_t tier;         // requested tier (TIER_GPU unless HOST_TIER flag)
    uint64_t stripe_unit;
    uint64_t alloc_id;     // REQ_FREE: the allocation to free
    int32_t app_pid;
    int32_t n_extents;     // REQ_FREE: extents the app holds
    uint8_t pad[72];
};

// One placed extent (DO_ALLOC response, EXTENT, DO_FREE).
enum RegionFlags : uint16_t {
    REGION_DEDICATED = 1u << 0,  // slab holds only this extent: importer unmaps it on free
    REGION_SPILLED = 1u << 1,    // placed in the host tier because HBM was exhausted
    REGION_NET = 1u << 2,        // owner on another node: handle = "net:<ip>:<port>" (netdata.h)
};

struct Region {
    uint64_t alloc_id;
    uint64_t bytes;        // bytes of this extent
    uint64_t offset;       // offset of the extent inside its slab
    uint64_t slab_bytes;
    uint64_t stripe_unit;  // 0 when the allocation is a single extent
    uint32_t slab_id;
    int32_t owner_rank;
    int32_t orig_rank;
    int32_t owner_gpu;     // node-local device ordinal, -1 for host tier
    uint16_t tier;         // enum Tier
    uint16_t flags;        // enum RegionFlags
    uint16_t extent_idx;
    uint16_t n_extents;
    uint8_t handle[kHandleBytes];  // hipIpcMemHandle_t (GPU) or "/proc/<pid>/fd/<n>" (host)
};

// Node description (ADD_NODE / NODE_TABLE / CONNECT_CONFIRM / STATS reply).
struct NodeConfig {
    char host[32];
    int32_t rank;
    int32_t gpu;           // device ordinal, -1 = CPU-only daemon
    int32_t num_gpu;       // GPUs visible on the node
    int32_t pid;
    uint64_t gpu_total;    // bytes of HBM on `gpu`
    uint64_t gpu_capacity; // bytes this daemon may hand out
    uint64_t host_capacity;
    uint64_t gpu_used;
    uint64_t host_used;
    uint16_t num_nodes;
    uint16_t num_apps;
    uint8_t xgmi_peers;    // GPUs on the node this daemon's GPU reaches over xGMI
    uint8_t min_hops, max_hops;  // over those links (0 when none)
    uint8_t ctrl;          // control transport (ocm_daemon_stats.ctrl_transport)
    uint32_t n_alloc, n_free, n_reclaimed, n_spilled, n_slabs;
    uint32_t ticks;        // allgather ticks of the control transport (0 on TCP)
    uint32_t n_leases;     // capacity leases this daemon holds on peers
    uint32_t lease_allocs; // allocations served from them (no mesh round trip)
};

// Statistics of a daemon's tick control transport (MSG_TICK_STATS reply, in u.raw):
// this rank's own records from post to delivery in a gathered tick, the gaps
// between completed ticks, and the host time the tick thread spends queueing them.
struct TickStatsWire {
    uint64_t ticks;           // ticks completed
    uint64_t own_records;     // own records seen delivered
    uint64_t lat_sum_ns, lat_max_ns;
    uint64_t periods, period_sum_ns;
    uint64_t starts, start_sum_ns, start_max_ns;  // Collective::start calls and their host time
    uint32_t transport;       // ocm_daemon_stats.ctrl_transport
    uint32_t ticks_per_start; // > 1: ticks queued as captured graphs (OCM_TICK_GRAPH)
    // Hop breakdown of the own records above (round 4): post -> the carrying tick
    // queued (wait; 0 when a tick was already queued), its queueing -> completion seen
    // by the tick thread (exec), and completion -> the event loop took the records
    // (deliver, over every delivered batch, deliver_n of them).
    uint64_t wait_sum_ns, exec_sum_ns, deliver_sum_ns, deliver_n;
    uint64_t lazy_ticks;      // idle ticks (OCM_TICK_IDLE_US): the mesh keeps ticking, no TCP wake-ups
    uint64_t tcp_wakes;       // MSG_TICK_WAKE records this daemon sent over TCP (0 with idle ticks)
};

// Topology of one daemon's GPU (hipExtGetLinkTypeAndHopCount to every other
// GPU ordinal on its node), fed to rank0's placement (nearest peer first).
constexpr int kMaxLinkGpus = 32;
constexpr uint8_t kHopsUnknown = 0xFF;
struct NodeLinks {
    int32_t rank;
    int32_t gpu;           // -1: CPU-only daemon (no table)
    uint32_t n;            // entries used (GPU ordinals 0..n-1)
    uint32_t pad;
    uint8_t hops[kMaxLinkGpus];  // kHopsUnknown: no link / self
    uint8_t type[kMaxLinkGpus];  // hipExtLinkType* value
};

static_assert(sizeof(NodeLinks) <= 128, "NodeLinks fits the message union");
static_assert(sizeof(TickStatsWire) <= 128, "TickStatsWire fits the message union");

// MSG_HELLO body: the first record on a mesh link. mac = SipHash-2-4 under the
// key derived from namespace + OCM_MESH_KEY over (src, dst, ts_ms, nonce); the
// acceptor checks dst, a +-10 min clock window and that the nonce is new, so a
// recorded HELLO cannot be replayed.
struct Hello {
    int32_t src_rank;
    int32_t dst_rank;
    uint64_t ts_ms;   // CLOCK_REALTIME of the sender
    uint64_t nonce;   // random per HELLO
    uint64_t mac;
    uint8_t pad[96];
};
static_assert(sizeof(Hello) == 128, "Hello fills the message union");

struct Msg {
    uint32_t type;     // MsgType
    uint32_t status;   // MsgStatus
    int32_t pid;       // app which made the request
    int32_t rank;      // rank of the daemon that originated the request
    uint64_t seq;      // correlation id (origin daemon scope)
    int32_t src_rank;  // rank of the sender of this record (-1 = app)
    int32_t err;       // 0 or a positive errno
    union {
        AllocReq req;
        Region region;
        NodeConfig node;
        NodeLinks links;
        Hello hello;
        uint8_t raw[128];
    } u;
};

static_assert(sizeof(AllocReq) == 128, "AllocReq must be 128 bytes");
static_assert(sizeof(Region) == 128, "Region must be 128 bytes");
static_assert(sizeof(NodeConfig) == 128, "NodeConfig must be 128 bytes");
static_assert(sizeof(Msg) == kMsgBytes, "wire record must stay 160 bytes");
static_assert(offsetof(Msg, u) == 32, "union must start at byte 32");

const char *msg_type_str(uint32_t t);
const char *msg_status_str(uint32_t s);

}  // namespace ocm
