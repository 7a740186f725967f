// Tick transport: daemon<->daemon control records carried by a collective.
//
// the reference's control plane was one TCP connection per
// RPC (src/mem.c:62-111) plus "start the master first"; the MI355X design
// carries the 160-byte records over RCCL on xGMI. RCCL operations must be
// matched on every rank, so records move in *ticks*: every daemon contributes
// one fixed slot (up to kTickMsgs addressed records) to an allgather, then
// keeps the records addressed to it. An idle mesh does not tick; a daemon that
// posts into an idle mesh nudges its peers awake (a 1-byte doorbell on the
// existing mesh sockets) and everybody ticks back-to-back while traffic lasts.
//
// Ticks can be pipelined: up to depth() ticks queued on the GPU at once (a
// launch-and-wait costs ~12-16 us on MI355X, a queued collective ~3.5 us,
// profiles/rccl_tick_floor_r02.json). Whether tick k is issued is decided from
// the gathered contents of ticks that every rank has already completed, so all
// ranks issue the same sequence. With device-sealed slots (the default) a record
// rides the next tick to execute, not the next one queued, so the RCCL default
// depth is 2 (OCM_TICK_DEPTH; host-filled slots: 1, where a queued record would
// wait behind empty ticks). OCM_TICK_GRAPH=K queues ticks K at a time as replays
// of captured graphs.
//
// The collective is pluggable: RcclCollective (ncclAllGather on the daemon's
// MI355X) in production, SocketCollective (ring allgather over abstract unix
// sockets) so the tick protocol itself is exercised multi-rank on CPU. Any
// collective error disables the transport; the daemon falls back to TCP links.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "ocm/msg.h"

namespace ocm {

constexpr int kTickMsgs = 8;

struct TickRecord {
    int32_t dest;      // destination rank
    int32_t pad;
    Msg msg;
};

struct TickSlot {
    uint32_t count;    // records used in this slot
    uint32_t busy;     // sender still has queued records (keep ticking)
    uint64_t first;    // device-sealed slots: ring index of rec[0] (the sender's progress)
    uint64_t tick;     // device-sealed slots: the tick number the seal ran for
    uint64_t tag;      // device-sealed slots: tick_slot_tag() of this slot, so a receiver that
                       // reads the gathered slots in place can tell a whole copy from one in flight
    TickRecord rec[kTickMsgs];
};
static_assert(sizeof(TickRecord) == 168, "tick record layout");

// Outbox of a device-sealed collective: pinned, device-mapped host memory the
// tick transport appends records to (then releases `published`). A small
// kernel queued in front of each collective ("seal", csrc/src/kernels/tick.hip)
// moves up to kTickMsgs unsent records into that tick's send slot WHEN THE
// TICK RUNS, so a record posted while ticks are queued rides the next tick to
// execute instead of waiting behind them.
constexpr uint32_t kTickRing = 256;  // power of two
struct TickRing {
    uint64_t published;               // records appended so far (host, release)
    uint64_t pad[15];
    TickRecord rec[kTickRing];        // record j lives at rec[j % kTickRing]
    uint64_t tag[kTickRing];          // tick_record_tag(rec j, j), stored after the record
};
constexpr int kTickRecordWords = (int)(sizeof(TickRecord) / sizeof(uint64_t));  // 21
static_assert(sizeof(TickRecord) % sizeof(uint64_t) == 0, "tick records are whole words");

// Hash of record j's words and its ring index. The seal kernel loads `published`,
// the next records and their tags in ONE round trip over PCIe; a record read
// before the host finished writing it (or left from an earlier lap of the ring)
// fails this check, and the kernel reads it again once `published` is known.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint64_t tick_record_tag(const uint64_t *w, uint64_t j) {
    uint64_t h = (j + 1) * 0x9E3779B97F4A7C15ull;
    for (int k = 0; k < kTickRecordWords; k++) {
        h ^= w[k] + 0x632BE59BD9B4E019ull * (uint64_t)(k + 1);
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 29;
    }
    return h;
}

// Tag of a sealed slot: its header, its tick number, and the XOR of its records'
// tick_record_tag()s (record r at ring index first + r). Whoever reads the
// gathered slots while the collective may still be writing them (the tick
// thread polls them in mapped host memory instead of waiting for a done kernel)
// takes a slot only when its tick and tag match.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint64_t tick_slot_tag(uint32_t count, uint32_t busy, uint64_t first, uint64_t tick, uint64_t rec_xor) {
    uint64_t h = (tick + 0x51ull) * 0x9E3779B97F4A7C15ull;
    h ^= (((uint64_t)count << 32) | busy) * 0xBF58476D1CE4E5B9ull;
    h ^= h >> 31;
    h ^= first * 0x94D049BB133111EBull;
    h ^= h >> 29;
    h ^= rec_xor;
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 32);
}
// Host: `s` (a private copy) is the whole slot sealed for tick `tick`.
bool tick_slot_whole(const TickSlot &s, uint64_t tick);
// Host: what tick_seal_kernel stores into a slot's tick/tag fields.
void tick_slot_seal_tag(TickSlot *s, uint64_t tick);

// Queue the seal of one tick on `stream`: *consumed (device memory, only this
// stream touches it) -> slot->first, up to kTickMsgs records of `ring` -> slot.
// `tick`: the tick's number (stored with the slot's tag). `wait_us`: when the
// ring holds nothing unsent, the seal polls it for up to this long before it
// seals an empty slot, so a record the host posts right after the previous
// tick completed still rides this one (OCM_TICK_SEAL_WAIT_US). `tick_ctr`
// (device memory, graph-captured ticks): the seal numbers the tick itself,
// *tick_ctr + 1, and stores that back; `tick` is then ignored.
// `bell` / `bell_seen` (idle ticks, device pointers): the host-wide tick doorbell
// and this stream's last view of it; the wait also ends when the bell moved (any
// daemon of the host posted into the idle mesh), and the seal stores what it saw.
hipError_t tick_seal_launch(const TickRing *ring, uint64_t *consumed, TickSlot *slot, uint64_t tick, uint32_t wait_us,
                            hipStream_t stream, uint64_t *tick_ctr = nullptr, const uint32_t *bell = nullptr,
                            uint32_t *bell_seen = nullptr);
// Queue a one-lane kernel that stores `seq` to `flag` (pinned, device-mapped
// host memory) at system scope: the host sees a tick end ~6 us sooner than
// through an event query (tools/launch_probe.hip, profiles/launch_flag_r01.json).
hipError_t tick_done_launch(uint64_t *flag, uint64_t seq, hipStream_t stream);

class Collective {
public:
    virtual ~Collective() = default;
    // Ring of depth() tick slots: fill send_slot(i), start(i) gathers every
    // rank's slot i into recv_slots(i) (rank-major), test(i) reports it done.
    // Ticks on different slots may be in flight together (stream-ordered).
    virtual int depth() const { return 1; }
    // Ticks one start() queues: start(i) runs slots i .. i + K - 1 (i a multiple
    // of K; depth() a multiple of 2K). K > 1: a graph of K captured ticks.
    virtual int ticks_per_start() const { return 1; }
    // Every rank rounds its tick target up to a multiple of this (the configured
    // K, the same on every rank), so a rank whose graphs could not be captured
    // and queues ticks one at a time still joins exactly the same collectives.
    virtual int tick_quantum() const { return ticks_per_start(); }
    // Device-sealed collectives expose their outbox ring; the transport then
    // appends records there instead of filling send slots (host-filled: null).
    virtual TickRing *ring() { return nullptr; }
    virtual void *send_slot(int i) = 0;
    virtual const void *recv_slots(int i) = 0;
    virtual int start(int i) = 0;   // 0 ok
    // Idle tick (OCM_TICK_IDLE_US): collectives that can wait on the device
    // (device_idle_wait) queue a tick whose seal waits up to `wait_us` for a record
    // of ours or a ring of the host-wide bell (set_bell); the others start at once
    // (the tick thread has waited on the bell on the host already).
    virtual bool device_idle_wait() const { return false; }
    virtual int start_idle(int i, uint32_t wait_us) { return start(i); }
    // The host-wide tick doorbell (a 32-bit word in shared, pinned-able memory).
    virtual void set_bell(uint32_t *bell) {}
    virtual int test(int i) = 0;    // 1 done, 0 in flight, -1 failed
    virtual void abort() {}
    virtual const char *name() const = 0;
    virtual std::string error() const { return std::string(); }  // why start/test failed, if known
};

// Collective constructors block until every rank joined; `cancel` aborts them.
// RCCL over xGMI. `id` is the ncclUniqueId (128 bytes) chosen by rank0.
// `slot_bytes`: size of one rank's slot (sizeof(TickSlot)).
std::unique_ptr<Collective> make_rccl_collective(int gpu, int rank, int nranks, const uint8_t *id, size_t slot_bytes,
                                                 std::string *err, const std::atomic<bool> *cancel);
// Fill a fresh ncclUniqueId (rank0). Returns 0 on success.
int rccl_unique_id(uint8_t out[128], std::string *err);
// Ring allgather over abstract unix sockets (same host), for CPU meshes/tests.
std::unique_ptr<Collective> make_socket_collective(const std::string &ns, int rank, int nranks, size_t slot_bytes,
                                                   std::string *err, const std::atomic<bool> *cancel);

using CollectiveFactory = std::function<std::unique_ptr<Collective>(std::string *err, const std::atomic<bool> *cancel)>;

// The host-wide tick doorbell of namespace `ns`: one page of POSIX shared memory
// ("/ocm_<ns>_tickbell") every daemon of the host maps; word 0 is the bell (a
// futex word). nullptr on failure. Close unmaps it and removes the name (the
// daemons that still map it keep their mapping).
uint32_t *tick_bell_open(const std::string &ns);
void tick_bell_close(uint32_t *bell, const std::string &ns);

class TickTransport {
public:
    // The collective is created on the tick thread (its construction blocks
    // until every rank joined).
    TickTransport(int rank, int nranks, CollectiveFactory factory);
    ~TickTransport();
    // CPUs the tick thread runs on (set before start(); empty: inherit the caller's).
    void set_cpus(std::vector<int> cpus) { cpus_ = std::move(cpus); }
    // Idle ticks (set before start()): with `idle_us` > 0 an idle mesh keeps ticking,
    // one tick per idle_us at most, instead of stopping and waking its peers over TCP
    // (take_announce never fires). `bell`: the host-wide doorbell every daemon of the
    // host rings (futex word, shared memory) when it posts into an idle mesh, so the
    // idle tick ends at once on every rank; nullptr: idle ticks run their full length.
    // An RCCL idle tick's seal waits for the bell on the GPU, which keeps one workgroup
    // resident; that delays a full-GPU GEMM by ~45 % (profiles/resident_cost_r04.json).
    // So the seal waits on the GPU only within OCM_TICK_IDLE_DEVICE_US (2 ms) of the
    // last tick that carried traffic; later idle ticks wait on the host (the bell's
    // futex) and then run as plain ticks. 0: always on the host; -1: always on the GPU.
    void set_idle(uint32_t idle_us, uint32_t *bell) {
        idle_us_ = idle_us;
        bell_ = bell;
    }
    void start();
    void stop();
    void abort();          // a peer died: stop ticking, fall back to TCP
    bool up() const { return up_.load() && !failed_.load(); }
    // Queue a record for `dest`. Returns false once the transport has failed.
    bool post(int dest, const Msg &m);
    // Records delivered to this rank (drained by the event loop).
    std::vector<Msg> drain();
    // drain() has records: a spinning event loop looks here on every pass rather
    // than waiting for epoll to report the eventfd.
    bool has_input() const { return in_ready_.load(std::memory_order_acquire); }
    // Readable when drain() has records, a wake-up must be announced, or the
    // transport failed.
    int event_fd() const { return efd_; }
    bool failed() const { return failed_.load(); }
    // A peer asked everybody to perform tick number `tick` (1-based).
    void wake_at(uint64_t tick);
    // True once when this rank starts a burst from idle; `tick` = the tick
    // number the peers must join (broadcast it to them).
    bool take_announce(uint64_t *tick);
    // Records still queued when the transport failed (re-send them over TCP).
    std::vector<TickRecord> take_unsent();
    uint64_t ticks() const { return ticks_.load(); }
    // Latency and host-cost statistics so far (always collected; OCM_TICK_STATS=1
    // also logs them when the transport stops).
    void stats(TickStatsWire *out);
    const char *collective_name() const { return coll_ ? coll_->name() : "none"; }

private:
    void run();
    int rank_, n_;
    CollectiveFactory factory_;
    std::unique_ptr<Collective> coll_;
    std::thread th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<TickRecord> out_;
    std::deque<uint64_t> out_ns_;       // when each queued record was posted (statistics)
    std::vector<Msg> in_;
    std::atomic<bool> stop_{false}, failed_{false}, announce_{false}, up_{false}, in_ready_{false};
    std::atomic<uint64_t> ticks_{0}, wake_upto_{0}, announce_tick_{0};
    TickRing *ring_ = nullptr;  // device-sealed collectives: their outbox (under mu_)
    uint64_t ring_sent_ = 0;    // ring records a completed tick of ours carried
    uint64_t ring_pub_ = 0;     // records appended (host shadow of ring_->published)
    // Post -> delivery latency of this rank's own records,
    // completed-tick periods and start() host time; OCM_TICK_STATS=1 logs them at stop.
    bool stats_ = false, stats_logged_ = false;
    uint64_t post_ns_[kTickRing] = {};
    uint64_t lat_sum_ns_ = 0, lat_n_ = 0, lat_max_ns_ = 0, period_sum_ns_ = 0, period_n_ = 0, last_done_ns_ = 0;
    uint64_t start_sum_ns_ = 0, start_n_ = 0, start_max_ns_ = 0;  // host time inside Collective::start
    uint32_t per_start_ = 1;
    void flush_ring();
    uint64_t unsent() const;
    void ring_bell();                        // bump the doorbell and wake its futex waiters
    uint32_t idle_us_ = 0;
    uint32_t *bell_ = nullptr;
    uint64_t idle_dev_window_ns_ = 2000ull * 1000;  // OCM_TICK_IDLE_DEVICE_US (UINT64_MAX: always)
    uint64_t idle_dev_ticks_ = 0, idle_host_ticks_ = 0;  // idle ticks that waited on the GPU / the host
    std::atomic<bool> lazy_{false};          // the mesh is ticking idle: posts ring the bell
    uint64_t lazy_ticks_ = 0;
    // hop breakdown (TickStatsWire): per own record, post -> its tick queued / -> completion;
    // per delivered batch, completion -> the event loop's drain
    uint64_t wait_sum_ns_ = 0, exec_sum_ns_ = 0, deliver_sum_ns_ = 0, deliver_n_ = 0;
    uint64_t ready_ns_ = 0;                  // when the undrained records were completed (under mu_)
    int efd_ = -1;
    std::vector<int> cpus_;
    // Host-filled collectives: records of issued ticks not yet completed here
    // (and how many each tick took), re-sent by take_unsent if the tick fails.
    std::deque<TickRecord> inflight_;
    std::deque<uint64_t> inflight_ns_;  // their post times
    std::deque<uint32_t> inflight_n_;
    bool timed_out_ = false;  // the watchdog (OCM_TICK_TIMEOUT_MS) ended the transport
};

}  // namespace ocm
