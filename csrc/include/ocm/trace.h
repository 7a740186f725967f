// Tracing: roctx ranges (visible to rocprofv3 --marker-trace) around every
// control and data-plane operation, per-process counters, and an optional
// JSON-lines op log (OCM_TRACE_FILE=<path>, written at ocm_tini / daemon exit).
// The reference had no tracing at all; its comments only noted
// where timing would go (test/ib_client.c:24, src/extoll.c:148).
#pragma once
#include <cstdint>
#include <string>

namespace ocm {

struct OpCounters {
    uint64_t n_put = 0, n_get = 0, bytes_put = 0, bytes_get = 0;
    uint64_t n_alloc = 0, n_free = 0, n_copy = 0, bytes_copy = 0;
    uint64_t ns_put = 0, ns_get = 0, ns_alloc = 0, ns_free = 0;
    uint64_t n_batch = 0, n_batch_ops = 0, bytes_batch = 0, ns_batch = 0;
    uint64_t n_batch_launches = 0;  // batch kernels launched outside plans (batches, remote->remote copies)
    uint64_t n_slab_fd = 0;         // host-tier slabs imported through an fd from their owner (SCM_RIGHTS)
    uint64_t n_slab_path = 0;       // ... through the /proc/<pid>/fd path fallback
    uint64_t n_link_rpc = 0;        // RPCs posted on the shared-memory link (ocm/shmlink.h)
    uint64_t n_link_wake = 0;       // ... of which had to wake the daemon over the socket
};

bool trace_enabled();  // OCM_TRACE=0 disables the roctx ranges
uint64_t now_ns();
// Record one finished operation into the bounded in-memory log (if enabled).
void trace_op(const char *op, uint64_t bytes, uint64_t t0_ns, uint64_t t1_ns, int rc);
// Write the op log to OCM_TRACE_FILE (append). Returns records written.
int trace_flush(const char *who);

class TraceRange {
public:
    explicit TraceRange(const char *name);
    ~TraceRange();
    TraceRange(const TraceRange &) = delete;
    TraceRange &operator=(const TraceRange &) = delete;

private:
    bool on_;
};

}  // namespace ocm
