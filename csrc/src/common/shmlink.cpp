// Shared-memory fast path of the app mailbox (see ocm/shmlink.h).
#include "ocm/shmlink.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <new>

namespace ocm {

namespace {
constexpr int kSeals = F_SEAL_SHRINK | F_SEAL_GROW | F_SEAL_SEAL;
constexpr size_t kBytes = (sizeof(ShmLinkLayout) + 4095) & ~size_t(4095);
}  // namespace

int ShmLink::create() {
    close();
    const int fd = memfd_create("ocm_link", MFD_CLOEXEC | MFD_ALLOW_SEALING);
    if (fd < 0) return -1;
    if (ftruncate(fd, (off_t)kBytes) != 0 || fcntl(fd, F_ADD_SEALS, kSeals) != 0) {
        ::close(fd);
        return -1;
    }
    void *p = mmap(nullptr, kBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (p == MAP_FAILED) {
        ::close(fd);
        return -1;
    }
    l_ = new (p) ShmLinkLayout();
    l_->magic = kShmLinkMagic;
    l_->slots = kShmLinkSlots;
    l_->req_taken.store(0, std::memory_order_relaxed);
    l_->rsp_taken.store(0, std::memory_order_relaxed);
    l_->daemon_polling.store(0, std::memory_order_relaxed);
    l_->app_waiting.store(0, std::memory_order_relaxed);
    for (uint32_t i = 0; i < kShmLinkSlots; i++) {
        l_->req[i].seq.store(0, std::memory_order_relaxed);
        l_->rsp[i].seq.store(0, std::memory_order_relaxed);
    }
    sent_ = got_ = peer_taken_ = 0;
    fd_ = fd;
    return 0;
}

int ShmLink::attach(int fd) {
    close();
    struct stat st;
    // Only a memfd sealed against resizing: a file the app could shrink later
    // would turn the daemon's next access into SIGBUS.
    if (fd < 0 || fstat(fd, &st) != 0 || (size_t)st.st_size != kBytes || (fcntl(fd, F_GET_SEALS) & kSeals) != kSeals) {
        if (fd >= 0) ::close(fd);
        return -1;
    }
    void *p = mmap(nullptr, kBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (p == MAP_FAILED) {
        ::close(fd);
        return -1;
    }
    l_ = static_cast<ShmLinkLayout *>(p);
    fd_ = fd;
    sent_ = got_ = peer_taken_ = 0;
    if (l_->magic != kShmLinkMagic || l_->slots != kShmLinkSlots) {
        close();
        return -1;
    }
    return 0;
}

void ShmLink::close() {
    if (l_) munmap(static_cast<void *>(l_), kBytes);
    l_ = nullptr;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
}

// Record n (1-based) lives in slot (n - 1) % slots and is whole once that slot's
// seq reads n. A producer may reuse a slot once the consumer has taken the
// record that was there; it re-reads the consumer's count only when its cached
// one says the ring is full. The peer may write anything anywhere in the
// mapping: all counts are compared with unsigned wrap-around, so a bogus count
// reads as "full" (the daemon then keeps the reply, bounded by kAppBacklogMax).
bool ShmLink::post(ShmLinkSlot *ring, std::atomic<uint64_t> &peer_taken, const Msg &m) {
    if (sent_ - peer_taken_ >= kShmLinkSlots) {
        peer_taken_ = peer_taken.load(std::memory_order_acquire);
        if (sent_ - peer_taken_ >= kShmLinkSlots) return false;
    }
    ShmLinkSlot &sl = ring[sent_ & (kShmLinkSlots - 1)];
    std::memcpy(&sl.msg, &m, sizeof(Msg));
    sl.seq.store(sent_ + 1, std::memory_order_release);
    sent_++;
    return true;
}

bool ShmLink::take(ShmLinkSlot *ring, std::atomic<uint64_t> &taken, Msg *m) {
    ShmLinkSlot &sl = ring[got_ & (kShmLinkSlots - 1)];
    if (sl.seq.load(std::memory_order_acquire) != got_ + 1) return false;
    std::memcpy(m, &sl.msg, sizeof(Msg));
    got_++;
    taken.store(got_, std::memory_order_release);
    return true;
}

bool ShmLink::post_request(const Msg &m) { return post(l_->req, l_->req_taken, m); }
bool ShmLink::take_reply(Msg *m) { return take(l_->rsp, l_->rsp_taken, m); }
bool ShmLink::take_request(Msg *m) { return take(l_->req, l_->req_taken, m); }
bool ShmLink::post_reply(const Msg &m) { return post(l_->rsp, l_->rsp_taken, m); }

bool ShmLink::request_needs_wake() {
    std::atomic_thread_fence(std::memory_order_seq_cst);  // the posted head before the flag's read
    return l_->daemon_polling.load(std::memory_order_relaxed) == 0;
}

bool ShmLink::reply_needs_wake() {
    std::atomic_thread_fence(std::memory_order_seq_cst);
    return l_->app_waiting.load(std::memory_order_relaxed) != 0;
}

void ShmLink::set_daemon_polling(bool on) {
    l_->daemon_polling.store(on ? 1u : 0u, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_seq_cst);  // the flag before the next look at the ring
}

bool ShmLink::requests_pending() {
    return l_->req[got_ & (kShmLinkSlots - 1)].seq.load(std::memory_order_acquire) == got_ + 1;
}

void ShmLink::set_app_waiting(bool on) {
    l_->app_waiting.store(on ? 1u : 0u, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_seq_cst);
}

bool ShmLink::replies_pending() {
    return l_->rsp[got_ & (kShmLinkSlots - 1)].seq.load(std::memory_order_acquire) == got_ + 1;
}

}  // namespace ocm
