#include "ocm/pmsg.h"

#include <dirent.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "ocm/log.h"
#include "ocm/msg.h"

namespace ocm {

std::string pmsg_namespace() {
    const char *ns = std::getenv("OCM_NS");
    std::string s = (ns && *ns) ? ns : "default";
    for (char &c : s)
        if (c == '/' || c == ' ') c = '_';
    return s;
}

std::string daemon_mailbox_name(int rank, const std::string &ns) {
    return "/ocm_" + ns + "_d" + std::to_string(rank);
}

std::string app_mailbox_name(pid_t pid, const std::string &ns) {
    return "/ocm_" + ns + "_p" + std::to_string((long)pid);
}

static long sys_msg_max() {
    FILE *f = fopen("/proc/sys/fs/mqueue/msg_max", "r");
    long v = 10;
    if (f) {
        if (fscanf(f, "%ld", &v) != 1) v = 10;
        fclose(f);
    }
    return v;
}

static void abs_deadline(int timeout_ms, struct timespec *ts) {
    clock_gettime(CLOCK_REALTIME, ts);
    if (timeout_ms <= 0) return;  // already expired: poll semantics
    ts->tv_sec += timeout_ms / 1000;
    ts->tv_nsec += (long)(timeout_ms % 1000) * 1000000L;
    if (ts->tv_nsec >= 1000000000L) {
        ts->tv_sec += 1;
        ts->tv_nsec -= 1000000000L;
    }
}

Mailbox::~Mailbox() { close_self(false); }

int Mailbox::open_self(const std::string &name, size_t msg_size, long depth, bool replace) {
    close_self(false);
    long cap = sys_msg_max();
    if (geteuid() != 0 && depth > cap) depth = cap;
    struct mq_attr attr;
    std::memset(&attr, 0, sizeof(attr));
    attr.mq_maxmsg = depth;
    attr.mq_msgsize = (long)msg_size;
    if (replace) mq_unlink(name.c_str());
    mqd_t q = mq_open(name.c_str(), O_RDONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0660, &attr);
    if (q == (mqd_t)-1) OCM_FAIL(-1, "mq_open(%s): %s", name.c_str(), strerror(errno));
    rx_ = q;
    name_ = name;
    msg_size_ = msg_size;
    return 0;
}

void Mailbox::close_self(bool unlink_queue) {
    for (auto &kv : tx_) mq_close(kv.second);
    tx_.clear();
    if (rx_ != (mqd_t)-1) {
        mq_close(rx_);
        if (unlink_queue) mq_unlink(name_.c_str());
        rx_ = (mqd_t)-1;
    }
}

int Mailbox::recv(void *msg, int timeout_ms) {
    if (rx_ == (mqd_t)-1) OCM_FAIL(-1, "recv on closed mailbox");
    for (;;) {
        ssize_t n;
        if (timeout_ms < 0) {
            n = mq_receive(rx_, static_cast<char *>(msg), msg_size_, nullptr);
        } else {
            struct timespec ts;
            abs_deadline(timeout_ms, &ts);
            n = mq_timedreceive(rx_, static_cast<char *>(msg), msg_size_, nullptr, &ts);
        }
        if (n >= 0) {
            if ((size_t)n != msg_size_) OCM_FAIL(-1, "short mailbox record (%zd bytes)", n);
            return 1;
        }
        if (errno == EINTR) continue;
        if (errno == ETIMEDOUT || errno == EAGAIN) return 0;
        OCM_FAIL(-1, "mq_receive(%s): %s", name_.c_str(), strerror(errno));
    }
}

long Mailbox::pending() const {
    struct mq_attr a;
    if (rx_ == (mqd_t)-1 || mq_getattr(rx_, &a) != 0) return -1;
    return a.mq_curmsgs;
}

int Mailbox::attach(const std::string &peer, bool nonblocking) {
    if (tx_.count(peer)) return 0;
    int flags = O_WRONLY | O_CLOEXEC | (nonblocking ? O_NONBLOCK : 0);
    mqd_t q = mq_open(peer.c_str(), flags);
    if (q == (mqd_t)-1) OCM_FAIL(-1, "attach %s: %s", peer.c_str(), strerror(errno));
    tx_[peer] = q;
    return 0;
}

void Mailbox::detach(const std::string &peer) {
    auto it = tx_.find(peer);
    if (it == tx_.end()) return;
    mq_close(it->second);
    tx_.erase(it);
}

int Mailbox::send(const std::string &peer, const void *msg, int timeout_ms) {
    auto it = tx_.find(peer);
    if (it == tx_.end()) OCM_FAIL(-1, "send to unattached mailbox %s", peer.c_str());
    for (;;) {
        int rc;
        if (timeout_ms < 0) {
            rc = mq_send(it->second, static_cast<const char *>(msg), msg_size_ ? msg_size_ : kMsgBytes, 0);
        } else {
            struct timespec ts;
            abs_deadline(timeout_ms, &ts);
            rc = mq_timedsend(it->second, static_cast<const char *>(msg), msg_size_ ? msg_size_ : kMsgBytes,
                              0, &ts);
        }
        if (rc == 0) return 1;
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == ETIMEDOUT) return 0;
        OCM_FAIL(-1, "mq_send(%s): %s", peer.c_str(), strerror(errno));
    }
}

int Mailbox::peer_fd(const std::string &peer) const {
    auto it = tx_.find(peer);
    return it == tx_.end() ? -1 : static_cast<int>(it->second);
}

int pmsg_cleanup(const std::string &ns) {
    // Only possible when the mqueue filesystem is mounted; daemons otherwise
    // unlink crashed apps' mailboxes themselves (pidfd notification).
    DIR *d = opendir("/dev/mqueue");
    if (!d) return 0;
    const std::string app_prefix = "ocm_" + ns + "_p";
    int removed = 0;
    while (struct dirent *e = readdir(d)) {
        std::string n = e->d_name;
        if (n.compare(0, app_prefix.size(), app_prefix) != 0) continue;
        long pid = std::strtol(n.c_str() + app_prefix.size(), nullptr, 10);
        if (pid > 0 && kill((pid_t)pid, 0) != 0 && errno == ESRCH) {
            if (mq_unlink(("/" + n).c_str()) == 0) removed++;
        }
    }
    closedir(d);
    return removed;
}

}  // namespace ocm

// ---------------- reference-shaped C interface ----------------
namespace {
ocm::Mailbox g_box;
size_t g_size = ocm::kMsgBytes;
std::string peer_name(pid_t pid) {
    const std::string ns = ocm::pmsg_namespace();
    if (pid < 0) return ocm::daemon_mailbox_name(-1 - pid, ns);
    return ocm::app_mailbox_name(pid, ns);
}
}  // namespace

extern "C" {
int pmsg_init(size_t pmsg_size) {
    g_size = pmsg_size;
    return 0;
}
int pmsg_open(pid_t self_pid) { return g_box.open_self(peer_name(self_pid), g_size, 8, self_pid < 0); }
int pmsg_close(void) {
    g_box.close_self(true);
    return 0;
}
int pmsg_attach(pid_t to_pid) { return g_box.attach(peer_name(to_pid), false); }
int pmsg_detach(pid_t to_pid) {
    g_box.detach(peer_name(to_pid));
    return 0;
}
int pmsg_send(pid_t to_pid, void *msg) { return g_box.send(peer_name(to_pid), msg, -1) == 1 ? 0 : -1; }
int pmsg_recv(void *msg, bool block) {
    int rc = g_box.recv(msg, block ? -1 : 0);
    return rc == 1 ? 0 : -1;
}
int pmsg_cleanup_all(void) { return ocm::pmsg_cleanup(ocm::pmsg_namespace()); }
int pmsg_pending(void) { return (int)g_box.pending(); }
}
