#include "ocm/tick.h"

#include <hip/hip_runtime_api.h>
#include <poll.h>
#include <rccl/rccl.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>

#include "ocm/log.h"
#include "ocm/pmsg.h"

namespace ocm {

namespace {

// ---------------------------------------------------------------- RCCL

// Each tick is ONE replay of a captured ncclAllGather over persistent slots:
// the send slot and the gathered slots live in pinned, device-mapped host
// memory, so the tick thread writes its records straight into the send slot
// and reads the peers' records straight out of the receive slots (no H2D /
// D2H copies, no per-tick allocation), and the collective is launched as a
// HIP graph (one launch, no RCCL enqueue work per tick). Completion is a
// spin on the stream, bounded by abort requests and RCCL async errors.
// OCM_TICK_GRAPH=0 launches ncclAllGather directly; OCM_TICK_MAPPED=0 keeps
// the slots in HBM with explicit copies (the round-1 path, for A/B).
class RcclCollective : public Collective {
public:
    ~RcclCollective() override {
        if (exec_) (void)hipGraphExecDestroy(exec_);
        if (graph_) (void)hipGraphDestroy(graph_);
        if (comm_) {
            if (aborted_)
                (void)ncclCommAbort(comm_);
            else
                (void)ncclCommDestroy(comm_);
        }
        if (stream_) (void)hipStreamDestroy(stream_);
        if (mapped_) {
            if (hsend_) (void)hipHostFree(hsend_);
            if (hrecv_) (void)hipHostFree(hrecv_);
        } else {
            if (dsend_) (void)hipFree(dsend_);
            if (drecv_) (void)hipFree(drecv_);
            if (hsend_) (void)hipHostFree(hsend_);
            if (hrecv_) (void)hipHostFree(hrecv_);
        }
    }
    int init(int gpu, int rank, int n, const uint8_t *id, std::string *err) {
        gpu_ = gpu;
        n_ = n;
        const char *g = std::getenv("OCM_TICK_GRAPH");
        const char *m = std::getenv("OCM_TICK_MAPPED");
        use_graph_ = !(g && std::strcmp(g, "0") == 0);
        mapped_ = !(m && std::strcmp(m, "0") == 0);
        if (hipSetDevice(gpu) != hipSuccess || hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) {
            *err = "rccl: no stream on gpu " + std::to_string(gpu);
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
        return 0;
    }
    void request_abort() { abort_req_ = true; }
    void *send_slot(size_t bytes) override {
        if (bytes != cap_ && setup(bytes) != 0) return nullptr;
        return hsend_;
    }
    const void *recv_slots() const override { return hrecv_; }
    int allgather(const void *send, void *recv, size_t bytes) override {
        if (aborted_) return -1;
        (void)hipSetDevice(gpu_);
        if (bytes != cap_ && setup(bytes) != 0) return -1;
        if (send != hsend_) std::memcpy(hsend_, send, bytes);
        if (!mapped_ && hipMemcpyAsync(dsend_, hsend_, bytes, hipMemcpyHostToDevice, stream_) != hipSuccess) return -1;
        if (exec_) {
            if (hipGraphLaunch(exec_, stream_) != hipSuccess) return -1;
        } else if (ncclAllGather(dsend_, drecv_, bytes, ncclUint8, comm_, stream_) != ncclSuccess) {
            return -1;
        }
        if (!mapped_ && hipMemcpyAsync(hrecv_, drecv_, bytes * n_, hipMemcpyDeviceToHost, stream_) != hipSuccess)
            return -1;
        // Wait without blocking forever: a dead peer never joins the collective.
        for (unsigned spins = 1;; spins++) {
            hipError_t q = hipStreamQuery(stream_);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) return -1;
            if (abort_req_.load()) {
                aborted_ = true;
                return -1;
            }
            if ((spins & 63) == 0) {
                ncclResult_t async = ncclSuccess;
                if (ncclCommGetAsyncError(comm_, &async) == ncclSuccess && async != ncclSuccess &&
                    async != ncclInProgress)
                    return -1;
            }
        }
        if (recv != hrecv_) std::memcpy(recv, hrecv_, bytes * n_);
        return 0;
    }
    void abort() override { abort_req_ = true; }
    const char *name() const override { return "rccl"; }

private:
    int setup(size_t bytes) {
        if (cap_) return -1;  // the slot size is fixed for the transport's life
        if (mapped_) {
            const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable;
            if (hipHostMalloc(&hsend_, bytes, fl) != hipSuccess || hipHostMalloc(&hrecv_, bytes * n_, fl) != hipSuccess ||
                hipHostGetDevicePointer(&dsend_, hsend_, 0) != hipSuccess ||
                hipHostGetDevicePointer(&drecv_, hrecv_, 0) != hipSuccess) {
                (void)hipGetLastError();
                return -1;
            }
        } else if (hipMalloc(&dsend_, bytes) != hipSuccess || hipMalloc(&drecv_, bytes * n_) != hipSuccess ||
                   hipHostMalloc(&hsend_, bytes) != hipSuccess || hipHostMalloc(&hrecv_, bytes * n_) != hipSuccess) {
            (void)hipGetLastError();
            return -1;
        }
        std::memset(hsend_, 0, bytes);
        std::memset(hrecv_, 0, bytes * n_);
        cap_ = bytes;
        if (use_graph_) {
            // Capture once; every rank captures the same single collective, so replays stay matched.
            hipGraph_t g = nullptr;
            bool ok = hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal) == hipSuccess;
            const bool queued = ok && ncclAllGather(dsend_, drecv_, bytes, ncclUint8, comm_, stream_) == ncclSuccess;
            ok = ok && hipStreamEndCapture(stream_, &g) == hipSuccess && queued;
            ok = ok && hipGraphInstantiate(&exec_, g, nullptr, nullptr, 0) == hipSuccess;
            if (g) graph_ = g;
            if (!ok) {
                (void)hipGetLastError();
                if (exec_) (void)hipGraphExecDestroy(exec_);
                exec_ = nullptr;
                OCM_WARN("rccl tick: graph capture of the allgather failed; launching it directly");
            }
        }
        return 0;
    }
    int gpu_ = 0, n_ = 1;
    ncclComm_t comm_ = nullptr;
    hipStream_t stream_ = nullptr;
    void *dsend_ = nullptr, *drecv_ = nullptr, *hsend_ = nullptr, *hrecv_ = nullptr;
    size_t cap_ = 0;
    bool use_graph_ = true, mapped_ = true;
    hipGraph_t graph_ = nullptr;
    hipGraphExec_t exec_ = nullptr;
    std::atomic<bool> abort_req_{false};
    bool aborted_ = false;
};

// ---------------------------------------------------------------- sockets

class SocketCollective : public Collective {
public:
    ~SocketCollective() override {
        if (left_ >= 0) close(left_);
        if (right_ >= 0) close(right_);
        if (listen_ >= 0) close(listen_);
    }
    int init(const std::string &ns, int rank, int n, std::string *err) {
        rank_ = rank;
        n_ = n;
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
        return 0;
    }
    int allgather(const void *send, void *recv, size_t bytes) override {
        char *out = static_cast<char *>(recv);
        std::memcpy(out + (size_t)rank_ * bytes, send, bytes);
        // Ring: at step s send block (rank - s) right, receive block (rank - s - 1) from the left.
        for (int s = 0; s < n_ - 1; s++) {
            const int sb = ((rank_ - s) % n_ + n_) % n_;
            const int rb = ((rank_ - s - 1) % n_ + n_) % n_;
            if (xfer(right_, out + (size_t)sb * bytes, bytes, true) != 0) return -1;
            if (xfer(left_, out + (size_t)rb * bytes, bytes, false) != 0) return -1;
        }
        return 0;
    }
    void abort() override {
        aborted_ = true;
        if (left_ >= 0) shutdown(left_, SHUT_RDWR);
        if (right_ >= 0) shutdown(right_, SHUT_RDWR);
    }
    const char *name() const override { return "socket"; }

private:
    int xfer(int fd, char *p, size_t n, bool snd) {
        // Seqpacket records are capped by the socket buffer; move the block in pieces.
        size_t done = 0;
        while (done < n && !aborted_) {
            const size_t piece = std::min<size_t>(n - done, 4096);
            struct pollfd q = {fd, (short)(snd ? POLLOUT : POLLIN), 0};
            int pr = poll(&q, 1, 200);
            if (pr < 0 && errno != EINTR) return -1;
            if (pr <= 0) continue;
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
    std::atomic<bool> aborted_{false};
};

}  // namespace

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

std::unique_ptr<Collective> make_rccl_collective(int gpu, int rank, int nranks, const uint8_t *id, std::string *err,
                                                 const std::atomic<bool> *cancel) {
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
    int rc = c->init(gpu, rank, nranks, id, err);
    done = true;
    if (watch.joinable()) watch.join();
    if (rc != 0) return nullptr;
    return c;
}

std::unique_ptr<Collective> make_socket_collective(const std::string &ns, int rank, int nranks, std::string *err,
                                                   const std::atomic<bool> *) {
    auto c = std::make_unique<SocketCollective>();
    if (c->init(ns, rank, nranks, err) != 0) return nullptr;
    return c;
}

// ---------------------------------------------------------------- transport

TickTransport::TickTransport(int rank, int nranks, CollectiveFactory factory)
    : rank_(rank), n_(nranks), factory_(std::move(factory)) {
    efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    recv_.resize((size_t)n_);
}

TickTransport::~TickTransport() {
    stop();
    if (efd_ >= 0) close(efd_);
}

void TickTransport::start() { th_ = std::thread([this] { run(); }); }

void TickTransport::stop() {
    if (!th_.joinable()) return;
    stop_ = true;
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (coll_) coll_->abort();
    }
    cv_.notify_all();
    th_.join();
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
    }
    cv_.notify_all();
    return true;
}

std::vector<Msg> TickTransport::drain() {
    uint64_t v;
    while (read(efd_, &v, sizeof(v)) == (ssize_t)sizeof(v)) {
    }
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<Msg> out;
    out.swap(in_);
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
    *tick = ticks_.load() + 1;
    return true;
}

std::vector<TickRecord> TickTransport::take_unsent() {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<TickRecord> v(out_.begin(), out_.end());
    out_.clear();
    return v;
}

void TickTransport::run() {
    // Every rank runs the same state machine over identical allgather
    // outputs, so all ranks agree on when to tick: after a tick that carried
    // traffic everybody ticks kBusyTicks more times; an idle rank ticks again
    // only for its own records or a peer's wake-up for the current tick count.
    constexpr int kBusyTicks = 64;
    int busy_left = 0;
    TickSlot mine;
    const TickSlot *send = &mine;
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
    {
        std::lock_guard<std::mutex> lk(mu_);
        coll_ = std::move(c);
    }
    up_ = true;
    signal();
    while (!stop_) {
        {
            std::unique_lock<std::mutex> lk(mu_);
            if (busy_left == 0) {
                cv_.wait(lk, [&] {
                    return stop_.load() || !out_.empty() || wake_upto_.load() >= ticks_.load() + 1;
                });
                if (stop_) break;
                if (!out_.empty() && wake_upto_.load() < ticks_.load() + 1) announce_ = true;  // we start the burst
            }
            // Fill the collective's own send slot when it has one (no extra copy).
            TickSlot *slot = static_cast<TickSlot *>(coll_->send_slot(sizeof(TickSlot)));
            if (!slot) slot = &mine;
            slot->count = 0;
            while (!out_.empty() && slot->count < (uint32_t)kTickMsgs) {
                slot->rec[slot->count++] = out_.front();
                out_.pop_front();
            }
            slot->busy = out_.empty() ? 0 : 1;
            send = slot;
        }
        if (announce_.load()) {
            // Let the event loop nudge the peers for this tick before we block in it.
            uint64_t one = 1;
            ssize_t w = write(efd_, &one, sizeof(one));
            (void)w;
        }
        const TickSlot *got = static_cast<const TickSlot *>(coll_->recv_slots());
        if (coll_->allgather(send, got ? const_cast<TickSlot *>(got) : recv_.data(), sizeof(TickSlot)) != 0) {
            if (!stop_) OCM_WARN("rank %d: %s tick transport failed; falling back to TCP", rank_, coll_->name());
            failed_ = true;
            uint64_t one = 1;
            ssize_t w = write(efd_, &one, sizeof(one));
            (void)w;
            break;
        }
        const uint64_t t = ++ticks_;
        bool traffic = false;
        size_t delivered = 0;
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (int k = 0; k < n_; k++) {
                const TickSlot &s = (got ? got : recv_.data())[k];
                if (s.count || s.busy) traffic = true;
                for (uint32_t i = 0; i < s.count && i < (uint32_t)kTickMsgs; i++)
                    if (s.rec[i].dest == rank_) {
                        in_.push_back(s.rec[i].msg);
                        delivered++;
                    }
            }
        }
        busy_left = traffic ? kBusyTicks : (busy_left > 0 ? busy_left - 1 : 0);
        (void)t;
        if (delivered) {
            uint64_t one = 1;
            ssize_t w = write(efd_, &one, sizeof(one));
            (void)w;
        }
    }
}

}  // namespace ocm
