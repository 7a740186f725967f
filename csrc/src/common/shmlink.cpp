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
    l_->req_head.store(0, std::memory_order_relaxed);
    l_->req_tail.store(0, std::memory_order_relaxed);
    l_->rsp_head.store(0, std::memory_order_relaxed);
    l_->rsp_tail.store(0, std::memory_order_relaxed);
    l_->daemon_polling.store(0, std::memory_order_relaxed);
    l_->app_waiting.store(0, std::memory_order_relaxed);
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

bool ShmLink::post_request(const Msg &m) {
    const uint64_t h = l_->req_head.load(std::memory_order_relaxed);
    if (h - l_->req_tail.load(std::memory_order_acquire) >= kShmLinkSlots) return false;
    std::memcpy(&l_->req[h & (kShmLinkSlots - 1)], &m, sizeof(Msg));
    l_->req_head.store(h + 1, std::memory_order_release);
    return true;
}

bool ShmLink::take_reply(Msg *m) {
    const uint64_t t = l_->rsp_tail.load(std::memory_order_relaxed);
    if (l_->rsp_head.load(std::memory_order_acquire) == t) return false;
    std::memcpy(m, &l_->rsp[t & (kShmLinkSlots - 1)], sizeof(Msg));
    l_->rsp_tail.store(t + 1, std::memory_order_release);
    return true;
}

bool ShmLink::take_request(Msg *m) {
    // The app owns req_head and may write anything there: bound what we trust.
    const uint64_t t = l_->req_tail.load(std::memory_order_relaxed);
    const uint64_t h = l_->req_head.load(std::memory_order_acquire);
    if (h == t || h - t > kShmLinkSlots) return false;
    std::memcpy(m, &l_->req[t & (kShmLinkSlots - 1)], sizeof(Msg));
    l_->req_tail.store(t + 1, std::memory_order_release);
    return true;
}

bool ShmLink::post_reply(const Msg &m) {
    const uint64_t h = l_->rsp_head.load(std::memory_order_relaxed);
    const uint64_t t = l_->rsp_tail.load(std::memory_order_acquire);
    if (h - t >= kShmLinkSlots) return false;  // full (or a tail the app corrupted): the socket path
    std::memcpy(&l_->rsp[h & (kShmLinkSlots - 1)], &m, sizeof(Msg));
    l_->rsp_head.store(h + 1, std::memory_order_release);
    return true;
}

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
    return l_->req_head.load(std::memory_order_acquire) != l_->req_tail.load(std::memory_order_relaxed);
}

void ShmLink::set_app_waiting(bool on) {
    l_->app_waiting.store(on ? 1u : 0u, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_seq_cst);
}

bool ShmLink::replies_pending() {
    return l_->rsp_head.load(std::memory_order_acquire) != l_->rsp_tail.load(std::memory_order_relaxed);
}

}  // namespace ocm
