// Tick control transport: daemon<->daemon records carried by collectives
// (ocm/tick.h). Reference parity: the control RPC it can replace, one TCP
// connection per 160-byte record (src/mem.c:62-111 send_recv_msg / send_msg,
// SURVEY K11); the MI355X design carries the records over RCCL on xGMI.
#include "ocm/tick.h"

#include "ocm/affinity.h"

#include <hip/hip_runtime_api.h>
#include <linux/futex.h>
#include <poll.h>
#include <rccl/rccl.h>
#include <fcntl.h>
#include <sys/eventfd.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "ocm/log.h"
#include "ocm/pmsg.h"

namespace ocm {

namespace {

uint64_t mono_now_ns() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

uint64_t slot_rec_xor(const TickSlot &s, uint32_t n) {
    uint64_t x = 0;
    for (uint32_t r = 0; r < n; r++)
        x ^= tick_record_tag(reinterpret_cast<const uint64_t *>(&s.rec[r]), s.first + (uint64_t)r);
    return x;
}

}  // namespace

bool tick_slot_whole(const TickSlot &s, uint64_t tick) {
    if (s.tick != tick || s.count > (uint32_t)kTickMsgs) return false;
    return tick_slot_tag(s.count, s.busy, s.first, s.tick, slot_rec_xor(s, s.count)) == s.tag;
}

void tick_slot_seal_tag(TickSlot *s, uint64_t tick) {
    s->tick = tick;
    s->tag = tick_slot_tag(s->count, s->busy, s->first, tick, slot_rec_xor(*s, std::min<uint32_t>(s->count, kTickMsgs)));
}

namespace {

// Every rank's slot of a gathered tick, read in place while the collective may
// still be writing it: whole copies of the slots sealed for `tick`?
bool gathered_whole(const void *recv, int n, uint64_t tick) {
    const TickSlot *g = static_cast<const TickSlot *>(recv);
    for (int k = 0; k < n; k++) {
        if (__atomic_load_n(&g[k].tick, __ATOMIC_ACQUIRE) != tick) return false;
        TickSlot copy;
        std::memcpy(&copy, &g[k], sizeof(copy));
        if (!tick_slot_whole(copy, tick)) return false;
    }
    return true;
}

// RCCL over xGMI: a ring of depth() tick slots, one ncclAllGather per tick on
// one stream, an event per slot for completion.
//
// Device-sealed (default, OCM_TICK_SEAL=1): the transport appends records to a
// TickRing in pinned host memory; each tick is [seal kernel -> allgather], and
// the seal moves the unsent records into that tick's HBM send slot when the
// tick executes. Records therefore never wait behind queued ticks, and up to
// OCM_TICK_DEPTH (default 2) ticks stay queued while traffic lasts: the GPU
// runs them back to back (an allgather queued behind another costs ~3.5 us,
// a launch-and-wait 12-16 us; profiles/rccl_tick_floor_r02.json). A one-lane
// kernel after each collective stores the tick's number to pinned host memory,
// which the tick thread polls (no runtime query on the fast path).
// 1-daemon remote alloc p50: depth 2 and 3 29.9 us, depth 1 42.9 us, p99 69 /
// 96 / 48 us (profiles/ctrl_probe_r02e_sealed.json).
// Host-filled (OCM_TICK_SEAL=0): the tick thread fills the send slot in pinned
// host memory before queueing the tick (depth 1 by default).
// The gathered slots land in pinned, device-mapped host memory, read in place
// (OCM_TICK_MAPPED=0: HBM plus a D2H copy queued behind the collective).
class RcclCollective : public Collective {
public:
    ~RcclCollective() override {
        for (ncclComm_t c : {comm2_, comm_}) {
            if (!c) continue;
            // A transport that is being stopped (daemon shutdown, a peer gone) aborts:
            // ncclCommAbort never waits on peers that may already have left.
            if (aborted_ || abort_req_.load())
                (void)ncclCommAbort(c);
            else
                (void)ncclCommDestroy(c);
        }
        // Queued ticks read and write the slots: free them only once the stream
        // has drained (an abort ends a collective stuck on a dead peer). If it
        // does not drain within 2 s, leak them rather than free memory a kernel
        // may still touch.
        if (stream_) {
            (void)hipSetDevice(gpu_);
            bool drained = false;
            for (int i = 0; i < 20000 && !drained; i++) {
                const hipError_t q = hipStreamQuery(stream_);
                const hipError_t q2 = stream2_ ? hipStreamQuery(stream2_) : hipSuccess;
                drained = q != hipErrorNotReady && q2 != hipErrorNotReady;
                if (!drained) usleep(100);
            }
            (void)hipGetLastError();
            if (!drained) {
                OCM_WARN("rccl tick stream did not drain; leaving its %zu slots allocated", ring_.size());
                return;
            }
        }
        for (hipGraphExec_t &g : gexec_)
            if (g) (void)hipGraphExecDestroy(g);
        if (tick_ctr_) (void)hipFree(tick_ctr_);
        for (auto &sl : ring_) {
            if (sl.ev) (void)hipEventDestroy(sl.ev);
            if (sl.sealed) (void)hipEventDestroy(sl.sealed);
            if (sl.hsend) (void)hipHostFree(sl.hsend);
            if (sl.hrecv) (void)hipHostFree(sl.hrecv);
            if (sealed_ || !mapped_) (void)hipFree(sl.dsend);
            if (!mapped_) (void)hipFree(sl.drecv);
        }
        if (out_) (void)hipHostFree(out_);
        if (done_) (void)hipHostFree(done_);
        if (bell_seen_) (void)hipFree(bell_seen_);
        if (bell_page_) (void)hipHostUnregister(bell_page_);
        if (consumed_) (void)hipFree(consumed_);
        if (stream2_) (void)hipStreamDestroy(stream2_);
        if (stream_) (void)hipStreamDestroy(stream_);
    }
    int init(int gpu, int rank, int n, const uint8_t *id, size_t bytes, std::string *err) {
        gpu_ = gpu;
        n_ = n;
        bytes_ = bytes;
        auto flag = [](const char *k, bool dflt) {
            const char *v = std::getenv(k);
            return v && *v ? std::strcmp(v, "0") != 0 : dflt;
        };
        mapped_ = flag("OCM_TICK_MAPPED", true);
        sealed_ = flag("OCM_TICK_SEAL", true) && bytes == sizeof(TickSlot);
        // Completion seen in the gathered slots themselves (tick number + tag, read in
        // mapped host memory) instead of a done kernel after each collective.
        // Measured (1 daemon, records to itself, profiles/ctrl_probe_r03_tagged.json): alloc p50
        // 28.3-29.1 us with tagged slots and a 6 us seal wait, against 36-78 us (bimodal) with a done
        // kernel and no wait; the wait is what removes the slow mode (a record posted just after a
        // tick completed had missed the already-running seal of the next one and waited a whole tick).
        done_kernel_ = flag("OCM_TICK_DONE_KERNEL", false) || !sealed_ || !mapped_;
        const char *wv = std::getenv("OCM_TICK_SEAL_WAIT_US");
        wait_us_ = wv && *wv ? (uint32_t)std::max(0, std::atoi(wv)) : 6;
        const char *d = std::getenv("OCM_TICK_DEPTH");
        int depth = std::max(1, std::min(d && *d ? std::atoi(d) : (sealed_ ? 2 : 1), 64));
        // OCM_TICK_STREAMS=2 (sealed ticks): consecutive ticks alternate between two
        // streams and two communicators (the second split from the first), so the next
        // tick's seal waits for records while the previous allgather is still running;
        // the seals stay in order through an event. Depth is then even.
        const char *sv = std::getenv("OCM_TICK_STREAMS");
        nstreams_ = (sealed_ && sv && std::atoi(sv) == 2) ? 2 : 1;
        if (nstreams_ == 2 && depth % 2) depth++;
        // OCM_TICK_GRAPH=K: ticks are queued K at a time as one replay of a captured
        // hipGraph (seal + allgather per tick, the seal numbering the tick from a
        // device counter), two graphs over 2K slots. One tick queued through the
        // runtime and RCCL costs the host 6.6-9.2 us, more than the tick itself
        // runs on the GPU (profiles/tick_timeline_r03.json).
        const char *gv = std::getenv("OCM_TICK_GRAPH");
        graph_k_ = gv && *gv ? std::max(0, std::min(std::atoi(gv), 32)) : kGraphDefault;
        if (graph_k_ <= 1 || !sealed_ || done_kernel_ || !mapped_ || nstreams_ != 1) graph_k_ = 0;
        quantum_ = std::max(1, graph_k_);
        plain_depth_ = depth;
        if (graph_k_) depth = 2 * graph_k_;
        if (hipSetDevice(gpu) != hipSuccess || hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess ||
            (nstreams_ == 2 && hipStreamCreateWithFlags(&stream2_, hipStreamNonBlocking) != hipSuccess)) {
            *err = "rccl: no stream on gpu " + std::to_string(gpu);
            return -1;
        }
        const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable;
        bool ok = true;
        ok = hipHostMalloc(reinterpret_cast<void **>(&done_), 64, fl) == hipSuccess &&
             hipHostGetDevicePointer(reinterpret_cast<void **>(&done_dev_), done_, 0) == hipSuccess;
        if (ok) __atomic_store_n(done_, 0ull, __ATOMIC_RELAXED);
        if (ok && sealed_) {
            // OCM_TICK_OUTBOX_WC=1: the outbox in write-combined host memory (the host only
            // writes it; TickTransport::flush_ring never reads it back), so the seal's read
            // skips the snoop of the CPU's caches. Measured no faster (alloc p50 29.8-38.0 us
            // against 29.0-32.7 coherent, profiles/ctrl_probe_r04_outbox_wc.json): off.
            const unsigned ofl = flag("OCM_TICK_OUTBOX_WC", false)
                                     ? (hipHostMallocMapped | hipHostMallocWriteCombined | hipHostMallocPortable)
                                     : fl;
            ok = hipHostMalloc(reinterpret_cast<void **>(&out_), sizeof(TickRing), ofl) == hipSuccess &&
                 hipHostGetDevicePointer(reinterpret_cast<void **>(&out_dev_), out_, 0) == hipSuccess &&
                 hipMalloc(reinterpret_cast<void **>(&consumed_), sizeof(uint64_t)) == hipSuccess &&
                 hipMemset(consumed_, 0, sizeof(uint64_t)) == hipSuccess;
            if (ok) std::memset(out_, 0, sizeof(TickRing));
        }
        ring_.resize((size_t)depth);
        for (auto &sl : ring_) {
            ok = ok && hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming) == hipSuccess;
            if (nstreams_ == 2) ok = ok && hipEventCreateWithFlags(&sl.sealed, hipEventDisableTiming) == hipSuccess;
            if (sealed_) {
                ok = ok && hipMalloc(&sl.dsend, bytes) == hipSuccess;
            } else if (mapped_) {
                ok = ok && hipHostMalloc(&sl.hsend, bytes, fl) == hipSuccess &&
                     hipHostGetDevicePointer(&sl.dsend, sl.hsend, 0) == hipSuccess;
            } else {
                ok = ok && hipMalloc(&sl.dsend, bytes) == hipSuccess && hipHostMalloc(&sl.hsend, bytes) == hipSuccess;
            }
            if (mapped_) {
                ok = ok && hipHostMalloc(&sl.hrecv, bytes * (size_t)n, fl) == hipSuccess &&
                     hipHostGetDevicePointer(&sl.drecv, sl.hrecv, 0) == hipSuccess;
            } else {
                ok = ok && hipMalloc(&sl.drecv, bytes * (size_t)n) == hipSuccess &&
                     hipHostMalloc(&sl.hrecv, bytes * (size_t)n) == hipSuccess;
            }
            if (!ok) break;
            if (sl.hsend) std::memset(sl.hsend, 0, bytes);
            std::memset(sl.hrecv, 0, bytes * (size_t)n);
        }
        if (!ok) {
            (void)hipGetLastError();
            *err = "rccl: no memory for the tick slots";
            return -1;
        }
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof(uid));
        // Non-blocking init so a rank that never shows up cannot wedge the daemon.
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        ncclResult_t r = ncclCommInitRankConfig(&comm_, n, uid, rank, &cfg);
        while (r == ncclInProgress) {
            if (abort_req_.load()) {
                aborted_ = true;
                *err = "rccl init aborted";
                return -1;
            }
            usleep(100);
            if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess) break;
        }
        if (r != ncclSuccess) {
            *err = std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r);
            return -1;
        }
        if (nstreams_ == 2) {
            // every rank splits the same way (color 0, key = rank): the same membership
            ncclConfig_t cfg2 = NCCL_CONFIG_INITIALIZER;
            cfg2.blocking = 0;
            r = ncclCommSplit(comm_, 0, rank, &comm2_, &cfg2);
            while (r == ncclInProgress) {
                if (abort_req_.load()) {
                    aborted_ = true;
                    *err = "rccl split aborted";
                    return -1;
                }
                usleep(100);
                if (ncclCommGetAsyncError(comm2_, &r) != ncclSuccess) break;
            }
            if (r != ncclSuccess) {
                *err = std::string("ncclCommSplit: ") + ncclGetErrorString(r);
                return -1;
            }
        }
        if (graph_k_ && capture_graphs() != 0) {
            OCM_WARN("rccl tick graphs unavailable (%s): ticks are queued one at a time", err_.c_str());
            err_.clear();
            graph_k_ = 0;
        } else if (graph_k_) {
            OCM_INFO("rank %d: %d ticks per captured graph, two graphs over %d slots", rank, graph_k_, 2 * graph_k_);
        }
        return 0;
    }
    // Two graphs of graph_k_ ticks each: graph g holds slots g*K .. g*K + K - 1.
    int capture_graphs() {
        const int k = graph_k_;
        if (hipMalloc(reinterpret_cast<void **>(&tick_ctr_), sizeof(uint64_t)) != hipSuccess ||
            hipMemsetAsync(tick_ctr_, 0, sizeof(uint64_t), stream_) != hipSuccess ||
            hipStreamSynchronize(stream_) != hipSuccess) {
            (void)hipGetLastError();
            return why("tick counter");
        }
        for (int g = 0; g < 2; g++) {
            if (hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal) != hipSuccess) {
                (void)hipGetLastError();
                return why("begin capture");
            }
            bool ok = true;
            for (int j = 0; j < k && ok; j++) {
                Slot &sl = ring_[(size_t)(g * k + j)];
                ok = tick_seal_launch(out_dev_, consumed_, static_cast<TickSlot *>(sl.dsend), 0, wait_us_, stream_,
                                      tick_ctr_) == hipSuccess &&
                     ncclAllGather(sl.dsend, sl.drecv, bytes_, ncclUint8, comm_, stream_) == ncclSuccess;
            }
            hipGraph_t graph = nullptr;
            const hipError_t ec = hipStreamEndCapture(stream_, &graph);
            if (!ok || ec != hipSuccess || !graph) {
                if (graph) (void)hipGraphDestroy(graph);
                (void)hipGetLastError();
                return why(ok ? "end capture" : "captured tick");
            }
            const hipError_t ei = hipGraphInstantiate(&gexec_[g], graph, nullptr, nullptr, 0);
            (void)hipGraphDestroy(graph);
            if (ei != hipSuccess) {
                gexec_[g] = nullptr;
                (void)hipGetLastError();
                return why(std::string("instantiate: ") + hipGetErrorString(ei));
            }
        }
        return 0;
    }
    void request_abort() { abort_req_ = true; }
    // Idle ticks wait on the device: the seal polls our ring and the host-wide bell.
    bool device_idle_wait() const override { return sealed_ && !graph_k_ && nstreams_ == 1 && bell_dev_; }
    void set_bell(uint32_t *bell) override {
        if (!bell || bell_dev_) return;
        (void)hipSetDevice(gpu_);
        // the bell's page, shared by every daemon of the host, mapped for this GPU
        void *page = reinterpret_cast<void *>(reinterpret_cast<uintptr_t>(bell) & ~(uintptr_t)4095);
        if (hipHostRegister(page, 4096, hipHostRegisterMapped) != hipSuccess ||
            hipHostGetDevicePointer(reinterpret_cast<void **>(&bell_dev_), bell, 0) != hipSuccess ||
            hipMalloc(reinterpret_cast<void **>(&bell_seen_), sizeof(uint32_t)) != hipSuccess ||
            hipMemset(bell_seen_, 0, sizeof(uint32_t)) != hipSuccess) {
            (void)hipGetLastError();
            OCM_WARN("rccl idle ticks: the tick doorbell cannot be mapped for gpu %d; idle ticks wait on the host", gpu_);
            bell_dev_ = nullptr;
            return;
        }
        bell_page_ = page;
    }
    int start_idle(int i, uint32_t wait_us) override {
        if (!device_idle_wait()) return start(i);
        idle_next_ = wait_us;
        const int rc = start(i);
        idle_next_ = 0;
        return rc;
    }
    int depth() const override { return graph_k_ ? 2 * graph_k_ : plain_depth_; }
    int ticks_per_start() const override { return graph_k_ ? graph_k_ : 1; }
    int tick_quantum() const override { return quantum_; }
    TickRing *ring() override { return sealed_ ? out_ : nullptr; }
    void *send_slot(int i) override { return ring_[(size_t)i].hsend; }
    const void *recv_slots(int i) override { return ring_[(size_t)i].hrecv; }
    int start(int i) override {
        if (aborted_) return -1;
        Slot &sl = ring_[(size_t)i];
        (void)hipSetDevice(gpu_);
        if (graph_k_) {
            if (i % graph_k_) return why("graph ticks start on a multiple of K");
            const hipError_t e = hipGraphLaunch(gexec_[(i / graph_k_) & 1], stream_);
            if (e != hipSuccess) return why(std::string("tick graph launch: ") + hipGetErrorString(e));
            for (int j = 0; j < graph_k_; j++) ring_[(size_t)(i + j)].seq = ++started_;
            return 0;
        }
        const uint64_t seq = started_ + 1;
        // two streams: tick i on stream i % 2 (depth is even, so consecutive ticks alternate)
        hipStream_t st = (nstreams_ == 2 && (i & 1)) ? stream2_ : stream_;
        ncclComm_t comm = (nstreams_ == 2 && (i & 1)) ? comm2_ : comm_;
        if (sealed_) {
            if (!out_dev_ || !consumed_ || !sl.dsend || !sl.drecv || !done_dev_) return why("tick slots missing");
            if (nstreams_ == 2 && started_ > 0) {
                // this seal follows the previous tick's seal (the outbox is consumed in order)
                const Slot &prev = ring_[(size_t)((i + (int)ring_.size() - 1) % (int)ring_.size())];
                if (hipStreamWaitEvent(st, prev.sealed, 0) != hipSuccess) return why("seal ordering");
            }
            const hipError_t e =
                idle_next_ ? tick_seal_launch(out_dev_, consumed_, static_cast<TickSlot *>(sl.dsend), seq, idle_next_,
                                              st, nullptr, bell_dev_, bell_seen_)
                           : tick_seal_launch(out_dev_, consumed_, static_cast<TickSlot *>(sl.dsend), seq, wait_us_, st);
            if (e != hipSuccess) return why(std::string("seal launch: ") + hipGetErrorString(e));
            if (nstreams_ == 2 && hipEventRecord(sl.sealed, st) != hipSuccess) return why("seal event");
        } else if (!mapped_ && hipMemcpyAsync(sl.dsend, sl.hsend, bytes_, hipMemcpyHostToDevice, st) != hipSuccess) {
            return -1;
        }
        const ncclResult_t nr = ncclAllGather(sl.dsend, sl.drecv, bytes_, ncclUint8, comm, st);
        if (nr != ncclSuccess) return why(std::string("ncclAllGather: ") + ncclGetErrorString(nr));
        if (!mapped_ && hipMemcpyAsync(sl.hrecv, sl.drecv, bytes_ * (size_t)n_, hipMemcpyDeviceToHost, st) != hipSuccess)
            return -1;
        sl.seq = ++started_;
        if (done_kernel_) {
            const hipError_t de = tick_done_launch(done_dev_, sl.seq, st);
            if (de != hipSuccess) return why(std::string("done launch: ") + hipGetErrorString(de));
        }
        // Completion is read from the gathered slots' tick numbers and tags; the
        // runtime is only the backstop (errors, and a done kernel's absence), for
        // which a stream query serves: no event per tick (host time per start()).
        // Two streams keep per-tick events (a tick on one stream says nothing of the other).
        if (ring_.size() == 1 || (nstreams_ == 1 && !done_kernel_)) return 0;
        return hipEventRecord(sl.ev, st) == hipSuccess ? 0 : -1;
    }
    int test(int i) override {
        // Bounded by abort requests and RCCL async errors: a dead peer never
        // joins the collective, so the event would never fire.
        if (abort_req_.load()) {
            aborted_ = true;
            return why("aborted");
        }
        // The tick's done kernel stored its sequence number: seen without a runtime call.
        if (done_kernel_ ? __atomic_load_n(done_, __ATOMIC_ACQUIRE) >= ring_[(size_t)i].seq
                         : gathered_whole(ring_[(size_t)i].hrecv, n_, ring_[(size_t)i].seq))
            return 1;
        if ((++polls_ & 255) != 0) return 0;
        // Backstop every 256 polls: the runtime's view (errors surface here), and
        // RCCL's async error (a dead peer never joins the collective).
        // One tick in flight: the stream is exactly that tick, and a stream query
        // measured cheaper than an event query (profiles/ctrl_probe_r02c.json).
        // (graph ticks record no events: a drained stream has finished them all)
        const hipError_t q = (ring_.size() == 1 || graph_k_ || (nstreams_ == 1 && !done_kernel_))
                                 ? hipStreamQuery(stream_)  // drained: every queued tick is done
                                 : hipEventQuery(ring_[(size_t)i].ev);
        if (q == hipSuccess) return 1;
        if (q != hipErrorNotReady) return why(std::string("tick completion: ") + hipGetErrorString(q));
        {
            for (ncclComm_t c : {comm_, comm2_}) {
                ncclResult_t async = ncclSuccess;
                if (c && ncclCommGetAsyncError(c, &async) == ncclSuccess && async != ncclSuccess &&
                    async != ncclInProgress)
                    return why(std::string("rccl async error: ") + ncclGetErrorString(async));
            }
        }
        return 0;
    }
    void abort() override { abort_req_ = true; }
    const char *name() const override { return "rccl"; }
    std::string error() const override { return err_; }

private:
    int why(const std::string &e) {
        err_ = e;
        return -1;
    }
    std::string err_;
    struct Slot {
        void *hsend = nullptr, *hrecv = nullptr, *dsend = nullptr, *drecv = nullptr;
        hipEvent_t ev = nullptr;
        hipEvent_t sealed = nullptr;  // two streams: after this tick's seal
        uint64_t seq = 0;  // tick number its done kernel stores
    };
    int gpu_ = 0, n_ = 1;
    size_t bytes_ = 0;
    bool mapped_ = true, sealed_ = true, done_kernel_ = true;
    uint32_t wait_us_ = 0;
    unsigned polls_ = 0;
    ncclComm_t comm_ = nullptr, comm2_ = nullptr;
    hipStream_t stream_ = nullptr, stream2_ = nullptr;
    int nstreams_ = 1;
    std::vector<Slot> ring_;
    TickRing *out_ = nullptr, *out_dev_ = nullptr;  // sealed: the outbox (host view / device view)
    uint64_t *consumed_ = nullptr;                  // sealed: records sealed so far (HBM, this stream only)
    uint64_t *done_ = nullptr, *done_dev_ = nullptr;  // last tick whose done kernel ran (pinned host)
    uint64_t started_ = 0;
    static constexpr int kGraphDefault = 0;
    int graph_k_ = 0, plain_depth_ = 1;    // OCM_TICK_GRAPH: ticks per graph replay (0: none)
    int quantum_ = 1;                      // the configured K, kept if capturing fails
    hipGraphExec_t gexec_[2] = {nullptr, nullptr};
    uint64_t *tick_ctr_ = nullptr;            // graph ticks: the last tick number a seal took (HBM)
    uint32_t *bell_dev_ = nullptr;            // idle ticks: the host-wide doorbell, device view
    uint32_t *bell_seen_ = nullptr;           // the bell value the last idle seal saw (HBM)
    void *bell_page_ = nullptr;               // registered page of the bell
    uint32_t idle_next_ = 0;                  // start(): this tick is idle, its seal waits up to this long
    std::atomic<bool> abort_req_{false};
    bool aborted_ = false;
};

// ---------------------------------------------------------------- sockets

// Ring allgather over abstract unix sockets, done inside start() (depth 1).
// OCM_TICK_SOCKET_SEAL=1 gives it an outbox ring sealed inside start(), the
// CPU stand-in for the RCCL seal kernel: the device-sealed protocol (ring
// accounting, progress from the sender's own gathered slot) then runs
// multi-rank on CPU meshes (tests/test_ctrl_tick.py).
class SocketCollective : public Collective {
public:
    ~SocketCollective() override {
        if (left_ >= 0) close(left_);
        if (right_ >= 0) close(right_);
        if (listen_ >= 0) close(listen_);
    }
    int init(const std::string &ns, int rank, int n, size_t bytes, std::string *err) {
        rank_ = rank;
        n_ = n;
        bytes_ = bytes;
        send_.assign(bytes, 0);
        const char *tf = std::getenv("OCM_TICK_FAULT");
        // fail_after_do_alloc / fail_after_do_free: see test()
        if (tf && bytes == sizeof(TickSlot))
            fault_type_ = std::strcmp(tf, "fail_after_do_alloc") == 0  ? (uint32_t)MSG_DO_ALLOC
                          : std::strcmp(tf, "fail_after_do_free") == 0 ? (uint32_t)MSG_DO_FREE
                                                                        : 0u;
        // stall_after=N: from tick N on this rank stops taking part, without an error
        // (a wedged collective): the peers' watchdogs must end the transport.
        if (tf && std::strncmp(tf, "stall_after=", 12) == 0) stall_after_ = std::atoll(tf + 12);
        const char *to = std::getenv("OCM_TICK_TIMEOUT_MS");
        timeout_ms_ = to && *to ? std::max(1L, std::atol(to)) : 5000;
        const char *sl = std::getenv("OCM_TICK_SOCKET_SEAL");
        if (sl && std::strcmp(sl, "1") == 0 && bytes == sizeof(TickSlot)) {
            outbox_.reset(new TickRing());
            std::memset(outbox_.get(), 0, sizeof(TickRing));
            // OCM_TICK_SOCKET_BATCH=K: start() runs K ticks, like a replay of the RCCL
            // collective's captured graph of K ticks (OCM_TICK_GRAPH), over 2K slots.
            const char *bv = std::getenv("OCM_TICK_SOCKET_BATCH");
            batch_ = bv && *bv ? std::max(1, std::min(std::atoi(bv), 32)) : 1;
            quantum_ = batch_;
            // OCM_TICK_FAULT=no_batch (tests): this rank queues its ticks one at a
            // time, as an RCCL rank whose graph capture failed does
            if (tf && std::strcmp(tf, "no_batch") == 0) batch_ = 1;
        }
        recv_.assign(quantum_ > 1 ? 2 * (size_t)quantum_ : 1, std::vector<char>(bytes * (size_t)n, 0));
        slot_tick_.assign(recv_.size(), 0);
        if (n == 1) return 0;
        listen_ = mbox_listen("ocm_" + ns + "_coll" + std::to_string(rank), 4);
        if (listen_ < 0) {
            *err = "socket collective: listen failed";
            return -1;
        }
        right_ = mbox_connect("ocm_" + ns + "_coll" + std::to_string((rank + 1) % n), 30000);
        if (right_ < 0) {
            *err = "socket collective: cannot reach right neighbour";
            return -1;
        }
        struct pollfd p = {listen_, POLLIN, 0};
        if (poll(&p, 1, 30000) <= 0 || (left_ = mbox_accept(listen_, nullptr)) < 0) {
            *err = "socket collective: left neighbour never connected";
            return -1;
        }
        if (mbox_peer_uid(left_) != (int)getuid()) {  // the ring is same-user daemons only
            *err = "socket collective: left neighbour runs as another user";
            return -1;
        }
        return 0;
    }
    int depth() const override { return (int)recv_.size(); }
    int ticks_per_start() const override { return batch_; }
    int tick_quantum() const override { return quantum_; }
    void *send_slot(int) override { return send_.data(); }
    const void *recv_slots(int i) override { return recv_[(size_t)i % recv_.size()].data(); }
    TickRing *ring() override { return outbox_.get(); }
    int start(int i) override {
        if (i % batch_) return -1;
        for (int j = 0; j < batch_; j++)
            if (tick((size_t)(i + j) % recv_.size()) != 0) return -1;
        return 0;
    }
    int tick(size_t slot_i) {
        if (outbox_) {  // what tick_seal_kernel does, when the tick runs
            TickSlot *slot = reinterpret_cast<TickSlot *>(send_.data());
            const uint64_t pub = __atomic_load_n(&outbox_->published, __ATOMIC_ACQUIRE);
            const uint64_t pending = pub - consumed_;
            const uint32_t n = (uint32_t)std::min<uint64_t>(pending, kTickMsgs);
            for (uint32_t r = 0; r < n; r++) slot->rec[r] = outbox_->rec[(consumed_ + r) & (kTickRing - 1)];
            slot->count = n;
            slot->busy = pending > n ? 1u : 0u;
            slot->first = consumed_;
            consumed_ += n;
            tick_slot_seal_tag(slot, ++ticks_);
            slot_tick_[slot_i] = ticks_;
        }
        if (stall_after_ > 0 && ++started_ >= (uint64_t)stall_after_) {
            while (!aborted_) usleep(1000);  // wedged until the transport is torn down
            return -1;
        }
        char *out = recv_[slot_i].data();
        std::memcpy(out + (size_t)rank_ * bytes_, send_.data(), bytes_);
        // Ring: at step s send block (rank - s) right, receive block (rank - s - 1) from the left.
        for (int s = 0; s < n_ - 1; s++) {
            const int sb = ((rank_ - s) % n_ + n_) % n_;
            const int rb = ((rank_ - s - 1) % n_ + n_) % n_;
            if (xfer(right_, out + (size_t)sb * bytes_, bytes_, true) != 0) return -1;
            if (xfer(left_, out + (size_t)rb * bytes_, bytes_, false) != 0) return -1;
        }
        return 0;
    }
    int test(int i) override {
        if (aborted_) return -1;
        // Sealed emulation: every gathered slot must check out as the RCCL path's
        // done-kernel-less completion requires (same tags, computed on the host).
        const size_t si = (size_t)i % recv_.size();
        if (outbox_ && !gathered_whole(recv_[si].data(), n_, slot_tick_[si])) {
            error_ = "gathered tick slot failed its tag check";
            return -1;
        }
        if (fault_type_ && !fault_fired_) {
            // OCM_TICK_FAULT=fail_after_do_alloc / fail_after_do_free (tests): the tick
            // that carried one of our DO_ALLOC / DO_FREE requests reached every peer,
            // then fails here, so the fallback re-sends a record the owner already has.
            const TickSlot *slot = reinterpret_cast<const TickSlot *>(send_.data());
            for (uint32_t r = 0; r < slot->count && r < (uint32_t)kTickMsgs; r++)
                if (slot->rec[r].msg.type == fault_type_ && slot->rec[r].msg.status == MSG_REQUEST) {
                    fault_fired_ = true;
                    error_ = fault_type_ == MSG_DO_ALLOC ? "injected failure after a DO_ALLOC tick (OCM_TICK_FAULT)"
                                                         : "injected failure after a DO_FREE tick (OCM_TICK_FAULT)";
                    abort();
                    return -1;
                }
        }
        return 1;
    }
    std::string error() const override { return error_; }
    void abort() override {
        aborted_ = true;
        if (left_ >= 0) shutdown(left_, SHUT_RDWR);
        if (right_ >= 0) shutdown(right_, SHUT_RDWR);
    }
    const char *name() const override { return "socket"; }

private:
    int xfer(int fd, char *p, size_t n, bool snd) {
        // Seqpacket records are capped by the socket buffer; move the block in pieces.
        // A neighbour that stops taking part without closing its socket is caught by
        // the same OCM_TICK_TIMEOUT_MS as an RCCL tick that never completes.
        size_t done = 0;
        int idle_ms = 0;
        while (done < n && !aborted_) {
            const size_t piece = std::min<size_t>(n - done, 4096);
            struct pollfd q = {fd, (short)(snd ? POLLOUT : POLLIN), 0};
            int pr = poll(&q, 1, 200);
            if (pr < 0 && errno != EINTR) return -1;
            if (pr <= 0) {
                if ((idle_ms += 200) >= timeout_ms_) {
                    error_ = "no progress within OCM_TICK_TIMEOUT_MS (a peer stopped taking part)";
                    return -1;
                }
                continue;
            }
            idle_ms = 0;
            ssize_t k = snd ? send(fd, p + done, piece, MSG_NOSIGNAL) : recv(fd, p + done, piece, 0);
            if (k <= 0) {
                if (k < 0 && (errno == EAGAIN || errno == EINTR)) continue;
                return -1;
            }
            done += (size_t)k;
        }
        return aborted_ ? -1 : 0;
    }
    int rank_ = 0, n_ = 1, left_ = -1, right_ = -1, listen_ = -1;
    size_t bytes_ = 0;
    std::vector<char> send_;
    std::vector<std::vector<char>> recv_;  // one gathered buffer per slot
    std::vector<uint64_t> slot_tick_;      // sealed emulation: the tick each slot carried
    int batch_ = 1, quantum_ = 1;          // OCM_TICK_SOCKET_BATCH
    std::unique_ptr<TickRing> outbox_;  // OCM_TICK_SOCKET_SEAL
    uint64_t consumed_ = 0;
    std::atomic<bool> aborted_{false};
    uint32_t fault_type_ = 0;  // OCM_TICK_FAULT=fail_after_do_alloc / _do_free: MSG_DO_ALLOC / MSG_DO_FREE
    bool fault_fired_ = false;
    long long stall_after_ = 0;
    uint64_t started_ = 0;
    uint64_t ticks_ = 0;  // sealed emulation: ticks sealed so far
    long timeout_ms_ = 5000;
    std::string error_;
};

}  // namespace

uint32_t *tick_bell_open(const std::string &ns) {
    const std::string name = "/ocm_" + ns + "_tickbell";
    const int fd = shm_open(name.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0600);
    if (fd < 0) return nullptr;
    if (ftruncate(fd, 4096) != 0) {
        close(fd);
        return nullptr;
    }
    void *p = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    return p == MAP_FAILED ? nullptr : static_cast<uint32_t *>(p);
}

void tick_bell_close(uint32_t *bell, const std::string &ns) {
    if (!bell) return;
    munmap(bell, 4096);
    (void)shm_unlink(("/ocm_" + ns + "_tickbell").c_str());
}

int rccl_unique_id(uint8_t out[128], std::string *err) {
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        *err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
        return -1;
    }
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(out, &id, sizeof(id));
    return 0;
}

std::unique_ptr<Collective> make_rccl_collective(int gpu, int rank, int nranks, const uint8_t *id, size_t slot_bytes,
                                                 std::string *err, const std::atomic<bool> *cancel) {
    auto c = std::make_unique<RcclCollective>();
    std::atomic<bool> done{false};
    std::thread watch;
    if (cancel) {
        RcclCollective *raw = c.get();
        watch = std::thread([raw, cancel, &done] {
            while (!done.load()) {
                if (cancel->load()) raw->request_abort();
                usleep(1000);
            }
        });
    }
    int rc = c->init(gpu, rank, nranks, id, slot_bytes, err);
    done = true;
    if (watch.joinable()) watch.join();
    if (rc != 0) return nullptr;
    return c;
}

std::unique_ptr<Collective> make_socket_collective(const std::string &ns, int rank, int nranks, size_t slot_bytes,
                                                   std::string *err, const std::atomic<bool> *cancel) {
    const char *tf = std::getenv("OCM_TICK_FAULT");
    if (tf && std::strcmp(tf, "init_hang") == 0) {
        // Test hook: a communicator that never comes up (a rank that never joins).
        while (cancel && !cancel->load()) usleep(1000);
        *err = "injected: the collective never came up (OCM_TICK_FAULT=init_hang)";
        return nullptr;
    }
    auto c = std::make_unique<SocketCollective>();
    if (c->init(ns, rank, nranks, slot_bytes, err) != 0) return nullptr;
    return c;
}

// ---------------------------------------------------------------- transport

TickTransport::TickTransport(int rank, int nranks, CollectiveFactory factory)
    : rank_(rank), n_(nranks), factory_(std::move(factory)) {
    efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    const char *st = std::getenv("OCM_TICK_STATS");
    stats_ = st && std::strcmp(st, "1") == 0;
}

TickTransport::~TickTransport() {
    stop();
    if (efd_ >= 0) close(efd_);
}

void TickTransport::start() { th_ = std::thread([this] { run(); }); }

void TickTransport::stats(TickStatsWire *out) {
    std::lock_guard<std::mutex> lk(mu_);
    std::memset(out, 0, sizeof(*out));
    out->ticks = ticks_.load();
    out->own_records = lat_n_;
    out->lat_sum_ns = lat_sum_ns_;
    out->lat_max_ns = lat_max_ns_;
    out->periods = period_n_;
    out->period_sum_ns = period_sum_ns_;
    out->starts = start_n_;
    out->start_sum_ns = start_sum_ns_;
    out->start_max_ns = start_max_ns_;
    out->ticks_per_start = per_start_;
    out->wait_sum_ns = wait_sum_ns_;
    out->exec_sum_ns = exec_sum_ns_;
    out->deliver_sum_ns = deliver_sum_ns_;
    out->deliver_n = deliver_n_;
    out->lazy_ticks = lazy_ticks_;
}

// Bump the host-wide doorbell and wake every tick thread sleeping on it (idle ticks).
void TickTransport::ring_bell() {
    if (!bell_) return;
    __atomic_fetch_add(bell_, 1u, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    (void)syscall(SYS_futex, bell_, FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
}

void TickTransport::stop() {
    if (th_.joinable()) {
        stop_ = true;
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (coll_) coll_->abort();
        }
        cv_.notify_all();
        th_.join();
    }
    // logged once the tick thread has ended (it updates these under mu_)
    TickStatsWire st;
    stats(&st);
    if (stats_ && st.own_records && !stats_logged_)
        OCM_INFO("rank %d: tick stats: %llu own records, post -> delivered %.2f us mean (max %.1f); %llu tick "
                 "periods of %.2f us mean; start() %.2f us mean (max %.1f) over %llu ticks",
                 rank_, (unsigned long long)st.own_records, st.lat_sum_ns / 1e3 / (double)st.own_records,
                 st.lat_max_ns / 1e3, (unsigned long long)st.periods,
                 st.periods ? st.period_sum_ns / 1e3 / (double)st.periods : 0.0,
                 st.starts ? st.start_sum_ns / 1e3 / (double)st.starts : 0.0, st.start_max_ns / 1e3,
                 (unsigned long long)st.starts);
    if (stats_ && st.lazy_ticks && !stats_logged_)
        OCM_INFO("rank %d: idle ticks: %llu waited on the GPU, %llu on the host (OCM_TICK_IDLE_DEVICE_US)", rank_,
                 (unsigned long long)idle_dev_ticks_, (unsigned long long)idle_host_ticks_);
    stats_logged_ = true;
}

void TickTransport::abort() {
    failed_ = true;
    stop_ = true;
    std::lock_guard<std::mutex> lk(mu_);
    if (coll_) coll_->abort();
    cv_.notify_all();
}

bool TickTransport::post(int dest, const Msg &m) {
    if (failed_ || !up_) return false;
    {
        std::lock_guard<std::mutex> lk(mu_);
        TickRecord r;
        std::memset(&r, 0, sizeof(r));
        r.dest = dest;
        r.msg = m;
        out_.push_back(r);
        out_ns_.push_back(mono_now_ns());
        flush_ring();
    }
    cv_.notify_all();
    // An idle mesh: every rank's idle tick ends when the bell moves (their seals and
    // tick threads watch it), so this record leaves now instead of at the end of it.
    if (lazy_.load()) ring_bell();
    return true;
}

// Device-sealed collectives: move queued records into the outbox ring while it
// has room (records the seal kernels have not taken yet stay in it). Under mu_.
void TickTransport::flush_ring() {
    if (!ring_ || out_.empty()) return;
    uint64_t pub = ring_pub_;  // never read back: the ring may sit behind a write-combined BAR
    while (!out_.empty() && pub - ring_sent_ < kTickRing) {
        const TickRecord &src = out_.front();
        ring_->rec[pub & (kTickRing - 1)] = src;
        post_ns_[pub & (kTickRing - 1)] = out_ns_.front();  // when it was posted (it may have waited for room)
        // the tag from the private copy: the ring is never read back (write-combined memory)
        ring_->tag[pub & (kTickRing - 1)] = tick_record_tag(reinterpret_cast<const uint64_t *>(&src), pub);
        out_.pop_front();
        out_ns_.pop_front();
        pub++;
    }
    if (pub == ring_pub_) return;
    __builtin_ia32_sfence();                                      // the records before the count
    __atomic_store_n(&ring_->published, pub, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();                                      // and out of the write-combining buffers
    ring_pub_ = pub;
}

uint64_t TickTransport::unsent() const {
    return out_.size() + (ring_ ? ring_pub_ - ring_sent_ : 0);
}

std::vector<Msg> TickTransport::drain() {
    uint64_t v;
    while (read(efd_, &v, sizeof(v)) == (ssize_t)sizeof(v)) {
    }
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<Msg> out;
    out.swap(in_);
    in_ready_.store(false, std::memory_order_relaxed);
    if (!out.empty() && ready_ns_) {
        deliver_sum_ns_ += mono_now_ns() - ready_ns_;
        deliver_n_++;
        ready_ns_ = 0;
    }
    return out;
}

void TickTransport::wake_at(uint64_t tick) {
    uint64_t cur = wake_upto_.load();
    while (tick > cur && !wake_upto_.compare_exchange_weak(cur, tick)) {
    }
    cv_.notify_all();
}

bool TickTransport::take_announce(uint64_t *tick) {
    if (!announce_.exchange(false)) return false;
    *tick = announce_tick_.load();
    return true;
}

std::vector<TickRecord> TickTransport::take_unsent() {
    std::lock_guard<std::mutex> lk(mu_);
    // Ring records past the last completed tick of ours, or (host-filled) the
    // records of ticks issued but not completed here, then the queue. A record of
    // a tick that failed here may still have reached its peer: the fallback may
    // repeat it, and the receiver drops the copy (Daemon::mesh_duplicate).
    std::vector<TickRecord> v;
    if (ring_)
        for (uint64_t j = ring_sent_; j < ring_pub_; j++) v.push_back(ring_->rec[j & (kTickRing - 1)]);
    v.insert(v.end(), inflight_.begin(), inflight_.end());
    v.insert(v.end(), out_.begin(), out_.end());
    inflight_.clear();
    inflight_ns_.clear();
    inflight_n_.clear();
    out_.clear();
    out_ns_.clear();
    ring_sent_ = ring_pub_;
    return v;
}

void TickTransport::run() {
    // Every rank runs the same state machine over identical allgather outputs,
    // so all ranks issue the same ticks: after completing a tick that carried
    // traffic, everybody extends its target by kBusyTicks; an idle rank issues
    // a tick only for its own records (announced to the peers) or a peer's
    // wake-up. Up to depth() ticks are queued at once; tick k's records are
    // read from ring slot (k - 1) % depth.
    constexpr uint64_t kBusyTicks = 64;
    if (!cpus_.empty()) (void)set_thread_cpus(cpus_);
    std::string err;
    std::unique_ptr<Collective> c = factory_(&err, &stop_);
    auto signal = [this] {
        uint64_t one = 1;
        ssize_t w = write(efd_, &one, sizeof(one));
        (void)w;
    };
    if (!c) {
        if (!stop_) OCM_WARN("rank %d: tick transport unavailable: %s", rank_, err.c_str());
        failed_ = true;
        signal();
        return;
    }
    if (idle_us_ && bell_) c->set_bell(bell_);
    {
        std::lock_guard<std::mutex> lk(mu_);
        coll_ = std::move(c);
    }
    Collective *coll = coll_.get();
    // Idle ticks: the seal waits on the GPU (RCCL), or this thread waits on the
    // bell before starting the tick (the socket ring, graph-captured ticks).
    const bool dev_idle = idle_us_ && coll->device_idle_wait();
    if (const char *v = std::getenv("OCM_TICK_IDLE_DEVICE_US"); v && *v) {
        const long long us = std::atoll(v);
        idle_dev_window_ns_ = us < 0 ? UINT64_MAX : (uint64_t)us * 1000ull;
    }
    uint64_t last_traffic_ns = 0;  // completion of the last tick that carried records (0: none yet)
    uint64_t idle_tick = 0;     // number of the idle tick in flight (0: none)
    uint32_t idle_bell = 0;     // the bell when it was queued
    const uint64_t depth = (uint64_t)std::max(1, coll->depth());
    // Ticks are queued `per` at a time (a captured graph of `per` ticks); every
    // rank rounds its target up to the same multiple of `quantum`.
    const uint64_t per = (uint64_t)std::max(1, coll->ticks_per_start());
    const uint64_t quantum = (uint64_t)std::max(1, coll->tick_quantum());
    {
        std::lock_guard<std::mutex> lk(mu_);
        per_start_ = (uint32_t)per;
    }
    {
        std::lock_guard<std::mutex> lk(mu_);
        ring_ = coll->ring();
        flush_ring();
    }
    up_ = true;
    signal();
    uint64_t issued = 0, done = 0, target = 0;
    // Watchdog: a collective that neither completes nor reports an error (a peer
    // that never joins it, a wedged transport) would hold every record queued
    // behind it. After OCM_TICK_TIMEOUT_MS (5 s) the transport fails, and the
    // daemon re-sends over TCP what it had not delivered.
    const uint64_t timeout_ns = [] {
        const char *v = std::getenv("OCM_TICK_TIMEOUT_MS");
        const long ms = v && *v ? std::atol(v) : 5000;
        return (uint64_t)std::max(1L, ms) * 1000000ull;
    }();
    std::vector<uint64_t> issued_at(depth, 0);
    auto mono_ns = [] {
        struct timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
    };
    auto fail = [&] {
        if (!stop_)
            OCM_WARN("rank %d: %s tick transport failed (%s); falling back to TCP", rank_, coll->name(),
                     coll->error().empty() ? "collective error" : coll->error().c_str());
        failed_ = true;
        signal();
    };
    while (!stop_) {
        {
            std::unique_lock<std::mutex> lk(mu_);
            bool idle_now = false, idle_dev = false;
            if (done == issued && issued >= target && idle_us_) {
                // the seal waits on the GPU only shortly after traffic (see set_idle)
                idle_dev = dev_idle && (idle_dev_window_ns_ == UINT64_MAX ||
                                        (last_traffic_ns && mono_ns() - last_traffic_ns < idle_dev_window_ns_));
                // Idle mesh, idle ticks: every rank issues the next tick anyway (each
                // decides from the same gathered ticks), so nobody needs waking over
                // TCP. Its seal (or this thread, below) waits up to idle_us for a
                // record of ours or the host-wide bell.
                lazy_ = true;
                if (unsent() > 0) ring_bell();  // posted before lazy_ was set: tell the peers
                if (!idle_dev) {
                    const uint64_t t_end = mono_ns() + (uint64_t)idle_us_ * 1000ull;
                    const uint32_t b0 = bell_ ? __atomic_load_n(bell_, __ATOMIC_ACQUIRE) : 0u;
                    while (!stop_ && unsent() == 0 && (!bell_ || __atomic_load_n(bell_, __ATOMIC_ACQUIRE) == b0)) {
                        const uint64_t now = mono_ns();
                        if (now >= t_end) break;
                        const uint64_t left = t_end - now;
                        if (bell_) {
                            lk.unlock();
                            struct timespec ts = {(time_t)(left / 1000000000ull), (long)(left % 1000000000ull)};
                            (void)syscall(SYS_futex, bell_, FUTEX_WAIT, b0, &ts, nullptr, 0);
                            lk.lock();
                        } else {
                            cv_.wait_for(lk, std::chrono::nanoseconds(left));
                        }
                    }
                    if (stop_) break;
                }
                target = issued + 1;
                idle_now = true;
                lazy_ticks_++;
                (idle_dev ? idle_dev_ticks_ : idle_host_ticks_)++;
            } else if (done == issued && issued >= target) {
                // Idle: sleep until there is something to send or a peer calls a tick.
                cv_.wait(lk, [&] { return stop_.load() || unsent() > 0 || wake_upto_.load() > target; });
                if (stop_) break;
                if (wake_upto_.load() <= target) {
                    // We start the burst: the peers must join tick issued + 1.
                    announce_tick_ = issued + 1;
                    announce_ = true;
                    target = issued + 1;
                }
            }
            target = std::max(target, wake_upto_.load());
            target = (target + quantum - 1) / quantum * quantum;
            // Queue ticks up to the target, at most `depth` in flight.
            while (issued < target && issued - done + per <= depth) {
                const int i = (int)(issued % depth);
                if (!ring_) {  // host-filled: the slot's records are fixed now
                    TickSlot *slot = static_cast<TickSlot *>(coll->send_slot(i));
                    slot->count = 0;
                    slot->first = 0;
                    while (!out_.empty() && slot->count < (uint32_t)kTickMsgs) {
                        slot->rec[slot->count++] = out_.front();
                        inflight_.push_back(out_.front());  // until the tick completes here
                        inflight_ns_.push_back(out_ns_.front());
                        out_.pop_front();
                        out_ns_.pop_front();
                    }
                    inflight_n_.push_back(slot->count);
                    slot->busy = out_.empty() ? 0 : 1;
                }
                if (announce_.load()) signal();  // let the event loop wake the peers first
                const bool idle_start = idle_now && idle_dev;
                if (idle_start) {
                    idle_tick = issued + 1;
                    idle_bell = bell_ ? __atomic_load_n(bell_, __ATOMIC_ACQUIRE) : 0u;
                }
                idle_now = false;  // only the first tick queued from idle
                lk.unlock();
                const uint64_t t0 = mono_ns();
                const int rc = idle_start ? coll->start_idle(i, idle_us_) : coll->start(i);
                const uint64_t t1 = mono_ns();
                lk.lock();
                if (rc != 0) break;
                start_sum_ns_ += t1 - t0;
                start_n_++;
                start_max_ns_ = std::max(start_max_ns_, t1 - t0);
                for (uint64_t j = 0; j < per; j++) issued_at[(size_t)((issued + j) % depth)] = t1;
                issued += per;
            }
            if (issued < target && issued - done + per <= depth) {  // start() failed
                lk.unlock();
                fail();
                break;
            }
        }
        if (done == issued) continue;
        const int i = (int)(done % depth);
        int t = 0;
        // Spin on the oldest tick without the queue lock (the event loop posts
        // under it); come back to queue more ticks only when there is room.
        for (unsigned spins = 0; !stop_; spins++) {
            t = coll->test(i);
            if (t != 0) break;
            if ((spins & 1023) == 1023 && mono_ns() - issued_at[(size_t)i] > timeout_ns) {
                t = -1;
                timed_out_ = true;
                coll->abort();
                break;
            }
            if (issued - done + per <= depth && (spins & 15) == 15) break;
            // An idle tick in flight, nothing of ours to send and the bell silent: it
            // runs up to idle_us on the GPU, so sleep on the bell (a post anywhere on
            // the host wakes us) instead of spinning a core for it.
            if (idle_tick == done + 1 && bell_ && __atomic_load_n(bell_, __ATOMIC_ACQUIRE) == idle_bell &&
                !in_ready_.load(std::memory_order_relaxed)) {
                bool quiet;
                {
                    std::lock_guard<std::mutex> lk(mu_);
                    quiet = unsent() == 0;
                }
                if (quiet) {
                    // a ring wakes us at once; otherwise look at the tick a few times per idle period
                    struct timespec ts = {0, (long)std::max<uint32_t>(50, idle_us_ / 4) * 1000};
                    (void)syscall(SYS_futex, bell_, FUTEX_WAIT, idle_bell, &ts, nullptr, 0);
                }
            }
        }
        if (t < 0) {
            if (timed_out_ && !stop_)
                OCM_WARN("rank %d: tick %llu did not complete within OCM_TICK_TIMEOUT_MS", rank_,
                         (unsigned long long)(done + 1));
            fail();
            break;
        }
        if (t == 0) continue;
        const TickSlot *got = static_cast<const TickSlot *>(coll->recv_slots(i));
        bool traffic = false;
        size_t delivered = 0;
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (ring_) {
                // Our own slot says how far the seals got through the outbox.
                const TickSlot &mine = got[rank_];
                {
                    const uint64_t t = mono_now_ns();
                    const uint64_t q = issued_at[(size_t)i];
                    for (uint32_t r = 0; r < std::min<uint32_t>(mine.count, kTickMsgs); r++) {
                        const uint64_t p = post_ns_[(mine.first + r) & (kTickRing - 1)];
                        const uint64_t d = t - p;
                        lat_sum_ns_ += d;
                        lat_n_++;
                        lat_max_ns_ = std::max(lat_max_ns_, d);
                        wait_sum_ns_ += q > p ? q - p : 0;  // no tick was queued when it was posted
                        exec_sum_ns_ += t - std::max(p, q);
                    }
                    if (last_done_ns_) {
                        period_sum_ns_ += t - last_done_ns_;
                        period_n_++;
                    }
                    last_done_ns_ = t;
                }
                ring_sent_ = std::max<uint64_t>(ring_sent_, mine.first + std::min<uint32_t>(mine.count, kTickMsgs));
                flush_ring();
            } else if (!inflight_n_.empty()) {
                const uint64_t t = mono_now_ns();
                const uint64_t q = issued_at[(size_t)i];
                for (uint32_t r = 0; r < inflight_n_.front() && !inflight_.empty(); r++) {
                    inflight_.pop_front();
                    const uint64_t p = inflight_ns_.front();
                    const uint64_t d = t - p;  // host-filled: post -> this tick completed here
                    inflight_ns_.pop_front();
                    lat_sum_ns_ += d;
                    lat_n_++;
                    lat_max_ns_ = std::max(lat_max_ns_, d);
                    wait_sum_ns_ += q > p ? q - p : 0;
                    exec_sum_ns_ += t - std::max(p, q);
                }
                inflight_n_.pop_front();
            }
            for (int k = 0; k < n_; k++) {
                const TickSlot &sl = got[k];
                if (sl.count || sl.busy) traffic = true;
                for (uint32_t r = 0; r < sl.count && r < (uint32_t)kTickMsgs; r++)
                    if (sl.rec[r].dest == rank_) {
                        in_.push_back(sl.rec[r].msg);
                        delivered++;
                    }
            }
            if (delivered) {
                if (!ready_ns_) ready_ns_ = mono_now_ns();
                in_ready_.store(true, std::memory_order_release);
            }
        }
        done++;
        ticks_ = done;
        if (idle_tick && done >= idle_tick) idle_tick = 0;
        if (traffic) {
            last_traffic_ns = mono_ns();
            target = std::max(target, done + kBusyTicks);
            lazy_ = false;  // a burst: ticks run back to back, posts need no bell
        }
        if (delivered) signal();
    }
}

}  // namespace ocm
