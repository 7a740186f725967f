#include "ocm/log.h"

#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <cstdlib>

#include "ocm/msg.h"

namespace ocm {

bool verbose() {
    static const bool v = std::getenv("OCM_VERBOSE") != nullptr;
    return v;
}

void log_line(const char *level, const char *file, const char *func, int line, const char *fmt, ...) {
    char body[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(body, sizeof(body), fmt, ap);
    va_end(ap);
    const char *base = std::strrchr(file, '/');
    base = base ? base + 1 : file;
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    char out[1400];
    const size_t blen = std::strlen(body);
    const char *nl = (blen > 0 && body[blen - 1] == '\n') ? "" : "\n";
    int n = snprintf(out, sizeof(out), "[ocm %s %ld.%06ld pid:%d tid:%ld %s::%s:%d] %s%s", level,
                     (long)ts.tv_sec, ts.tv_nsec / 1000, (int)getpid(), (long)syscall(SYS_gettid),
                     base, func, line, body, nl);
    if (n > 0) {
        ssize_t w = write(2, out, (size_t)(n < (int)sizeof(out) ? n : (int)sizeof(out) - 1));
        (void)w;
    }
}

static thread_local char g_last_error[512];

void set_last_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

const char *last_error() { return g_last_error; }

const char *msg_type_str(uint32_t t) {
    switch (t) {
    case MSG_INVALID: return "MSG_INVALID";
    case MSG_CONNECT: return "MSG_CONNECT";
    case MSG_CONNECT_CONFIRM: return "MSG_CONNECT_CONFIRM";
    case MSG_DISCONNECT: return "MSG_DISCONNECT";
    case MSG_ADD_NODE: return "MSG_ADD_NODE";
    case MSG_REQ_ALLOC: return "MSG_REQ_ALLOC";
    case MSG_DO_ALLOC: return "MSG_DO_ALLOC";
    case MSG_REQ_FREE: return "MSG_REQ_FREE";
    case MSG_DO_FREE: return "MSG_DO_FREE";
    case MSG_RELEASE_APP: return "MSG_RELEASE_APP";
    case MSG_EXTENT: return "MSG_EXTENT";
    case MSG_HELLO: return "MSG_HELLO";
    case MSG_NODE_TABLE: return "MSG_NODE_TABLE";
    case MSG_PLACE_FAIL: return "MSG_PLACE_FAIL";
    case MSG_FREED: return "MSG_FREED";
    case MSG_STATS: return "MSG_STATS";
    case MSG_APP_DEAD: return "MSG_APP_DEAD";
    case MSG_SHUTDOWN: return "MSG_SHUTDOWN";
    case MSG_PING: return "MSG_PING";
    case MSG_TICK_START: return "MSG_TICK_START";
    case MSG_TICK_WAKE: return "MSG_TICK_WAKE";
    case MSG_OWNED: return "MSG_OWNED";
    case MSG_OWNED_DONE: return "MSG_OWNED_DONE";
    case MSG_NODE_LINKS: return "MSG_NODE_LINKS";
    case MSG_SLAB_FD: return "MSG_SLAB_FD";
    case MSG_TICK_STOP: return "MSG_TICK_STOP";
    case MSG_WAKE: return "MSG_WAKE";
    case MSG_TICK_STATS: return "MSG_TICK_STATS";
    default: return "INVALID MSG TYPE";
    }
}

const char *msg_status_str(uint32_t s) {
    switch (s) {
    case MSG_NO_STATUS: return "MSG_NO_STATUS";
    case MSG_REQUEST: return "MSG_REQUEST";
    case MSG_RESPONSE: return "MSG_RESPONSE";
    default: return "INVALID MSG STATUS";
    }
}

}  // namespace ocm
