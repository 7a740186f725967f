// Data-plane transfer engine: one-sided put/get between a linear buffer and a
// (possibly striped) remote buffer, as hand-written gfx950 kernels.
//
// Replaces the reference's one-sided fabric operations:
//   ib_write/ib_read  (RDMA WRITE/READ, src/rdma.c:46-85,240-263)
//   extoll_write/read (RMA2 put/get in 8 MiB chunks x 2 in flight, src/extoll.c:40-173)
// On MI355X the "NIC" is the GPU itself: a kernel on the initiating GPU streams
// 16-byte vectors between its HBM and peer HBM mapped over xGMI (IPC import).
// A put pushes (local loads, remote stores); a get pulls (remote loads).
// A remote buffer can be striped over several owners: unit u of the striped
// address space lives on extent u % n at extent offset (u / n) * unit, so one
// launch drives several xGMI links at once.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace ocm {

constexpr int kXferMaxExtents = 8;

struct XferArgs {
    char *lin;                       // linear side, already offset to the first byte
    char *ext[kXferMaxExtents];      // extent bases of the striped side
    uint64_t rem_off;                // first byte in striped coordinates
    uint64_t len;                    // bytes
    uint32_t unit_shift;             // log2(stripe unit); ignored when n_ext == 1
    uint32_t n_ext;                  // 1..8
    uint32_t tile_shift;             // log2(tile bytes), tile <= unit
    uint32_t put;                    // 1: lin -> striped, 0: striped -> lin
};

enum XferVariant : int {
    XFER_AUTO = 0,
    XFER_REG = 1,    // register-staged, 8 x 16 B loads in flight per lane
    XFER_LDS = 2,    // LDS-DMA (global_load_lds_dwordx4) staged, wave-private double buffer
    XFER_DMA = 3,    // no kernel: the runtime's copy engines, one hipMemcpyAsync per stripe segment
                     // (a measured baseline: autotune reports it, never installs it)
    XFER_PCIE = 4,   // PCIe streaming: 8 KiB tiles on a small grid (128), write-through stores to the
                     // host tier; the default for pairs whose remote half is in the pinned host tier
    XFER_PUSH = 5,   // gets only: a kernel on each OWNER's GPU reads its extents (local HBM) and
                     // writes the app's local half over xGMI (remote writes instead of remote reads)
};

struct XferTuning {
    int variant = XFER_AUTO;
    int max_blocks = 0;      // 0: per-path default
    bool nontemporal = true; // nt stores on the destination
    bool write_through = false;  // register kernel: sc1 (write-through) loads and stores instead
                                 // (autotune candidate over xGMI; what won PCIe puts)
};

// Completion published by the kernel itself (blocking ops): every workgroup
// drains and releases its bytes system-wide and counts itself in `cnt`
// (device memory, zero between launches); the last one re-zeroes `cnt` and
// stores `val` to `flag` (host-coherent memory, release). The host spins on
// the flag instead of the runtime's end-of-kernel signal, which costs ~6 us
// more per op (tools/launch_probe.hip: 5.3 us flag vs 11.1 us event).
struct XferDone {
    unsigned long long *flag = nullptr;  // nullptr: no flag
    unsigned int *cnt = nullptr;
    unsigned long long val = 0;
};

// Validate and fill tile_shift (xfer_launch does this itself; the service needs it up front).
hipError_t xfer_normalize(XferArgs &a);

// Launch one transfer on `stream`. Returns hipSuccess or the launch error.
hipError_t xfer_launch(const XferArgs &a, const XferTuning &t, hipStream_t stream, const XferDone *done = nullptr);

// Push-based get: the tiles of the extents in `ext_mask` (bit i: extent i), launched on
// the current device (the owner of those extents); a.ext[i] must be addresses valid
// there for the masked extents, a.lin an address of the app's buffer valid there too.
hipError_t xfer_push_launch(const XferArgs &a, uint32_t ext_mask, int max_blocks, hipStream_t stream);

// Plain device copy dst <- src (both device-accessible), via the same kernel.
hipError_t xfer_copy(void *dst, const void *src, uint64_t bytes, const XferTuning &t, hipStream_t stream);

// Default tuning from the environment (OCM_XFER_VARIANT, OCM_XFER_BLOCKS, OCM_XFER_NT).
XferTuning xfer_tuning_from_env();

// ---- batched one-sided ops (scatter/gather lists) ----
// Many ops on one remote pair in ONE launch. The batch is cut into 4 KiB
// wave-tiles (smaller when the stripe unit is): the host prefix-sums each op's
// tile count into `first_tile`, sizes the grid, and gives every wave a
// contiguous tile range plus the op its first tile belongs to (`wave_op`), so
// waves never search; they walk forward through the ops they cover. Small
// batches travel in the kernel arguments, large ones in a device buffer.
struct XferBatchOp {
    uint64_t lin_off;     // offset in the linear buffer
    uint64_t rem_off;     // offset in striped coordinates
    uint64_t len;
    uint64_t first_tile;  // exclusive prefix sum of the ops' tile counts
    uint32_t put;         // 1: lin -> striped, 0: striped -> lin
    uint32_t pad;
};
static_assert(sizeof(XferBatchOp) == 40, "batch op layout");

constexpr int kXferInlineOps = 48;  // ops carried in the kernarg segment

struct XferBatchArgs {
    char *lin;
    char *ext[kXferMaxExtents];
    uint32_t unit_shift;
    uint32_t n_ext;
    uint32_t tile_shift;
    uint32_t n_ops;
    uint64_t total_tiles;
    uint32_t grid;                        // workgroups (4 waves each)
    uint32_t abs_lin;                     // 1: op.lin_off is an absolute device address (lin unused)
    uint32_t host_tier;                   // 1: every extent is pinned host memory (PCIe launch shape, sc1 puts)
    uint32_t pad0;
    const XferBatchOp *ops;               // device copy when n_ops > kXferInlineOps
    const uint32_t *wave_op;              // device: first op of each wave (n_ops > kXferInlineOps)
    XferBatchOp inline_ops[kXferInlineOps];
};

// Host-side plan. Fills first_tile, returns total tiles.
uint64_t xfer_batch_plan(XferBatchOp *ops, uint32_t n, uint32_t tile_shift);
// Workgroups for `total_tiles` (4 waves each, capped for residency; host-tier
// batches are capped lower, OCM_BATCH_HOST_GRID: PCIe wants fewer streams).
uint32_t xfer_batch_grid(uint64_t total_tiles, bool host_tier = false);
// wave_op[w] for every wave of `grid` workgroups (4 * grid entries).
void xfer_batch_wave_ops(const XferBatchOp *ops, uint32_t n, uint64_t total_tiles, uint32_t grid, uint32_t *out);
// tile shift for a remote layout: 4 KiB wave-tiles, or the stripe unit when smaller.
uint32_t xfer_batch_tile_shift(uint32_t n_ext, uint32_t unit_shift);
hipError_t xfer_batch_launch(const XferBatchArgs &a, const XferTuning &t, hipStream_t stream);
// The same launch as a kernel node of `graph` after `dep` (nullptr: a root node);
// *node is the new node (an empty node when there is nothing to copy). `a` must
// stay alive as long as the graph.
hipError_t xfer_batch_graph_node(hipGraph_t graph, hipGraphNode_t dep, const XferBatchArgs &a, const XferTuning &t,
                                 hipGraphNode_t *node);

// ---- persistent copy service (low-latency blocking one-sided ops) ----
// A resident gang of `blocks` workgroups. Workgroup 0 polls one 128-byte
// request record {args, gang, sum, seq} in host-pinned memory (ServiceReq),
// 16 lanes in one load instruction; `sum` (a hash of seq and the other words)
// proves that a snapshot is whole, so a torn or reordered write of the record
// (write-combining may reorder the host's stores) is simply read again. The
// host sizes each request: `gang` = active | target << 16, where `active`
// workgroups (1 for small requests, up to `blocks`) copy tiles i, i + active, ...
// and `target` is the running total of gang completions that finishes this
// request (the device counter only grows, so it is never reset between
// requests). Workgroup 0 relays a gang request, exactly as read, into the
// device box with one write-through store; the other workgroups poll that copy
// and check the same hash. Completion: every taking-part workgroup drains its
// write-through stores (no release fence) and counts itself in; the one that
// reaches `target` (or the only one) stores `done = seq` in the host slot.
// Bounded: workgroup 0 leaves on kServiceStop or after `idle_ticks` of
// s_memrealtime (100 MHz) without work; on leaving it stores STOP as the relayed
// seq (the gang leaves on it) and `exited` = the first seq it did not serve.
// Roster (round 4): nothing guarantees that all `blocks` workgroups of the
// launch are resident at once (other processes' kernels hold CUs; a queue can be
// preempted). Completion must never wait for a workgroup that has not started:
// a gang member's id is its check-in order (every workgroup takes a ticket from
// ServiceBox::checkin when it starts; the first one is member 0, the lead called
// workgroup 0 above), the lead publishes the number of checked-in members as
// ServiceSlot::roster, and the host
// sizes every gang to at most that roster, so each member a request names is
// already running. A member that checks in later only gets requests posted after
// it was counted. Workgroup 0 also takes its idle exit only once the last gang
// request is complete (every member it named has finished), so a member that was
// slow to see a request is never told to leave before serving it.
// Measured history: profiles/svc_trace_r02.json (a relay that re-hashed and
// fenced first cost the gang ~2 us), profiles/svc_v3_direct_r02.json (every
// workgroup polling the host record cost every op 3-4 us), profiles/
// svc_doorbell_r01.json (a BAR-mapped HBM record was slower than host memory).
constexpr unsigned long long kServiceStop = ~0ull;
constexpr int kServiceArgWords = (int)((sizeof(XferArgs) + 7) / 8);
constexpr int kServiceReqGang = 13;  // record word: active | target << 16 | STRICT
// Gang word bit 63 (STRICT): some extent is in another GPU's HBM, so this request
// takes the fenced hand-off (system acquire before the copy, release before
// `done`) whatever the protocol bits say.
constexpr unsigned long long kServiceGangStrict = 1ull << 63;
constexpr unsigned long long kServiceGangTargetMask = (1ull << 31) - 1;  // bits 16..46
// Bits 47..62: the epoch of the instance the request is for (its launch number,
// mod 2^16). Instances run on a small pool of streams, so a relaunch need not wait
// for workgroups of an earlier instance that never got a CU (another process holds
// them): such a workgroup that starts late polls the same host gang record, and
// must leave a newer instance's request alone.
constexpr int kServiceGangEpochShift = 47;
constexpr unsigned long long kServiceGangEpochMask = 0xFFFFull;
static_assert(kServiceArgWords <= kServiceReqGang, "service request record holds 13 argument words");

struct alignas(128) ServiceReq {
    unsigned long long args[14];      // XferArgs (words 0..12), gang word (13), host -> device
    unsigned long long sum;           // hash of seq and words 0..13 (word 14)
    unsigned long long seq;           // host -> device, written last (word 15, second cache line)
};
static_assert(sizeof(ServiceReq) == 128, "service request layout");
static_assert(__builtin_offsetof(ServiceReq, seq) == 120 && __builtin_offsetof(ServiceReq, sum) == 112,
              "the kernel reads seq/sum as words 15/14");

// Lone lead (round 4, OCM_SERVICE_LONE_US): after the idle window the members
// leave and the lead stays alone for lone_ticks more, polling only the small-op
// record at a slower rate, and serves solo requests at hot latency. It never takes
// a gang request: the host sees `lone` and starts a full instance (a new epoch),
// whereupon the lone lead leaves without touching the slot. Only an instance on
// the library's own AQL queue runs lone: HIP does not know that queue, so a
// device-wide synchronize never waits for it (on a HIP stream it would).
//
// Device -> host status words (exited, roster, lone) carry the epoch of the
// instance that wrote them in bits 48..63, so a word left by an earlier instance
// is never read as the current one's.
constexpr int kServiceTagShift = 48;
constexpr unsigned long long kServiceTagValueMask = (1ull << kServiceTagShift) - 1;
constexpr unsigned long long service_tag(unsigned epoch, unsigned long long v) {
    return ((unsigned long long)(epoch & 0xFFFFu) << kServiceTagShift) | (v & kServiceTagValueMask);
}
// The value of a tagged word if instance `epoch` wrote it, else 0.
constexpr unsigned long long service_untag(unsigned epoch, unsigned long long w) {
    return (w >> kServiceTagShift) == (epoch & 0xFFFFu) ? (w & kServiceTagValueMask) : 0ull;
}

constexpr int kServiceWgDoneMax = 128;  // WGDONE: gangs of at most this many workgroups
struct alignas(128) ServiceSlot {
    ServiceReq req;                   // the request record
    unsigned long long done;          // device -> host (own cache line)
    unsigned long long exited;        // device -> host, tagged: first seq NOT served when it left
    // device -> host, tagged: gang members resident so far (workgroup 0 included);
    // the host sizes every gang to at most this many.
    unsigned long long roster;
    unsigned long long lone;          // device -> host, tagged: first seq after which the members left
    unsigned long long epoch_now;     // host -> device: the current instance's epoch (a lone lead of another leaves)
    unsigned long long lead_xcd;      // device -> host, tagged: 1 + the XCD the current lead runs on (diagnostic)
    unsigned long long pad0[2];
    // device -> host: this instance's sum of request-seen -> done ticks of its lead (100 MHz).
    // Written after every op, so it sits on the next cache line, away from `done`, which the
    // host spins on.
    unsigned long long gpu_ticks;
    unsigned long long pad[7];
    // WGDONE: gang member i stores the seq it finished here (device -> host)
    unsigned long long wg_done[kServiceWgDoneMax];
};
static_assert(sizeof(ServiceSlot) == 256 + 8 * kServiceWgDoneMax, "service slot layout");
static_assert(__builtin_offsetof(ServiceSlot, gpu_ticks) / 64 != __builtin_offsetof(ServiceSlot, done) / 64,
              "gpu_ticks on a cache line of its own");

constexpr int kServiceTraceWgs = 64;
// Device-memory state of the gang. Zeroed only at the first launch and after an
// instance left with a request unfinished: a relaunch after a clean idle exit
// reuses it as it is (the check-in counter and the gang counter keep growing,
// the host passes the check-in base; a stale relayed record carries a seq below
// the new instance's first, and `stop` names the instance that left).
struct alignas(128) ServiceBox {
    unsigned long long rec[16];       // relayed request record (ServiceReq words), STOP as seq to leave
    unsigned long long cnt;           // gang completions, over all requests (only grows)
    unsigned long long pad1[15];
    unsigned long long checkin;       // workgroups that have started, over every instance (id = ticket - base)
    unsigned long long pad2[15];
    unsigned long long stop;          // first seq of the instance whose lead has left (its members leave too)
    unsigned long long pad3[15];
    // OCM_SERVICE_PROTO bit 16 (TRACE): per workgroup, GPU clock (100 MHz) of its
    // last request: seen, copy start, copy drained, counted in / done published.
    unsigned long long trace[kServiceTraceWgs][4];
};

// Workgroups that copy a (normalized) request: 1 when it has at most
// `solo_tiles` tiles or the gang has one workgroup, else min(tiles, blocks).
// `blocks` is the host's wanted width, already capped at the roster.
uint32_t service_gang_size(const XferArgs &a, unsigned blocks, unsigned solo_tiles);
// Post one request (words, sum, then seq with release) to `copies` adjacent records
// and flush the CPU's write-combining buffers. gang = active | target << 16.
void service_post(ServiceReq *req, const XferArgs &a, unsigned long long gang, unsigned long long seq,
                  unsigned copies = 1);
// Store one word of the record(s) (seq: 0 to re-arm, kServiceStop) and flush.
void service_store_seq(ServiceReq *req, unsigned long long seq, unsigned copies = 1);

// Hand-off protocol bits of the service (OCM_SERVICE_PROTO):
//   WT        copied bytes are loaded sc1 and stored write-through (sc1), and
//             every wave drains its stores: neither an acquire after the
//             doorbell nor a system-scope release (buffer_wbl2) before `done`.
//             Without WT: plain loads and stores, system acquire and release.
//             STRICT requests (peer HBM) always take the fenced path.
//   GANGREC   gang requests go to a second host record on a page of their own
//             (`gang_req`), which the first `direct_wgs` workgroups poll
//             themselves: no relay through device memory (1.3 us across XCD
//             L2s) for gangs that fit them; wider gangs are relayed to the
//             rest as before. Workgroup 0's small-op record is read by
//             workgroup 0 alone, which reads both records with one load
//             instruction; direct pollers also watch the box's STOP word, so
//             they leave with workgroup 0.
//   WCREQ     the request record(s) in write-combined host memory (uncached on
//             the CPU side, so GPU polls need no snoop of the CPU's caches; the
//             host only ever writes them), `done` stays in coherent memory
//   WGDONE    gang completion without the device-scope counter: every member
//             stores the seq it finished into its own ServiceSlot::wg_done word
//             and the host waits for all `active` of them (gangs of at most
//             kServiceWgDoneMax); the counter's atomic round trip is then off the
//             last workgroup's path to `done`
//   TRACE     diagnostics: stamp each workgroup's phases into ServiceBox::trace
//   STRICTWT  STRICT requests (an extent in another GPU's HBM) keep the system
//             acquire before the copy (this GPU's L2 may hold stale lines of
//             peer memory from an earlier request: sc1 loads are L2-served) but
//             copy write-through (sc1 stores drop their lines from L2 and write
//             through) and drain, instead of a plain copy and a system release
//             (an L2 writeback) before `done`
//   COPIES    (with GANGREC) the gang record is written once per direct poller,
//             128-byte copies side by side on the gang page, and member i polls
//             copy i (the lead copy 0): GPU reads of one host line from many
//             workgroups at once are served one after another (16 pollers: 2.8 us
//             per read against 1.2 us with a line each; 64: 10.4 us,
//             profiles/host_mem_latency_r04.json)
constexpr unsigned kServiceProtoWT = 1u, kServiceProtoGangRec = 2u, kServiceProtoWCReq = 4u, kServiceProtoWgDone = 8u,
                   kServiceProtoTrace = 16u, kServiceProtoStrictWT = 32u, kServiceProtoCopies = 64u;
constexpr unsigned kServiceProtoMask = 127u;
constexpr int kServiceGangCopiesMax = 4096 / 128;  // copies on the gang page
// Whether a gang of `active` workgroups completes through ServiceSlot::wg_done.
constexpr bool service_wg_done(unsigned proto, unsigned long long active) {
    return (proto & kServiceProtoWgDone) && active > 1 && active <= (unsigned long long)kServiceWgDoneMax;
}

// first_seq >= 1: the first request this instance serves. gang_req: the
// GANGREC record (nullptr: gang requests are relayed by workgroup 0).
// direct_wgs: with gang_req, workgroups 0..direct_wgs-1 poll it themselves.
// checkin_base: ServiceBox::checkin when this instance starts (0 after a reset);
// reset_box: zero the box first (stream-ordered memset).
// epoch: this instance's launch number (mod 2^16, see kServiceGangEpochShift).
// degraded_idle_ticks: the idle exit while part of the grid has not started yet.
// lone_ticks: how long the lead stays alone after the members left (0: it leaves with them).
struct ServiceKernelArgs {
    const ServiceReq *req;
    const ServiceReq *gang_req;
    ServiceSlot *slot;
    ServiceBox *box;
    unsigned long long first_seq;
    unsigned long long idle_ticks;
    unsigned proto;
    unsigned direct_wgs;
    unsigned long long checkin_base;
    unsigned epoch;
    unsigned blocks;  // the grid (the kernel never reads gridDim: a hidden argument it would reload in its loops)
    unsigned long long degraded_idle_ticks;
    unsigned long long lone_ticks;
};
// The kernel takes ServiceKernelArgs as its explicit kernel arguments, in this
// order (an AQL dispatch copies the struct into the kernarg segment as is).
static_assert(sizeof(ServiceKernelArgs) == 88, "service kernel argument layout");
hipError_t service_launch(const ServiceKernelArgs &args, unsigned blocks, bool reset_box, hipStream_t stream);
// The service kernel's symbol in the device code object embedded in libocm (AQL dispatch).
constexpr const char *kServiceKernelSymbol = "ocm_service_kernel";
// ... and the kernel that zeroes a gang box (one workgroup, ServiceBox * argument).
constexpr const char *kServiceBoxClearSymbol = "ocm_service_box_clear";

// Deterministic 32-bit word pattern (word i of a buffer) for data verification.
hipError_t pattern_fill(void *p, uint64_t words, uint64_t first_word, uint32_t seed, hipStream_t stream);
// Adds the number of mismatching words to *bad_dev (device memory).
hipError_t pattern_check(const void *p, uint64_t words, uint64_t first_word, uint32_t seed, unsigned long long *bad_dev,
                         hipStream_t stream);
uint32_t pattern_word_host(uint64_t i, uint32_t seed);

}  // namespace ocm
