#include "ocm/trace.h"

#include <rocprofiler-sdk-roctx/roctx.h>
#include <time.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

namespace ocm {

namespace {
struct Rec {
    const char *op;
    uint64_t bytes, t0, t1;
    int rc;
};
std::mutex g_mu;
std::vector<Rec> g_log;
constexpr size_t kMaxRecs = 1 << 20;

const char *trace_file() {
    static const char *f = std::getenv("OCM_TRACE_FILE");
    return (f && *f) ? f : nullptr;
}
}  // namespace

// roctx ranges cost ~0.4 us per blocking op even with no tool attached
// (profiles/svc_doorbell_r01.json: 4 KiB put 5.57 -> 5.18 us without them), so
// by default they are on only under rocprofv3 (which exports
// ROCPROF_OUTPUT_PATH to the program). OCM_TRACE=1 / =0 forces them on / off.
bool trace_enabled() {
    static const bool on = [] {
        const char *v = std::getenv("OCM_TRACE");
        if (v && *v) return std::strcmp(v, "0") != 0;
        return std::getenv("ROCPROF_OUTPUT_PATH") != nullptr;
    }();
    return on;
}

uint64_t now_ns() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

void trace_op(const char *op, uint64_t bytes, uint64_t t0, uint64_t t1, int rc) {
    if (!trace_file()) return;
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_log.size() < kMaxRecs) g_log.push_back({op, bytes, t0, t1, rc});
}

int trace_flush(const char *who) {
    const char *path = trace_file();
    if (!path) return 0;
    std::lock_guard<std::mutex> lk(g_mu);
    FILE *f = std::fopen(path, "a");
    if (!f) return -1;
    for (const Rec &r : g_log)
        std::fprintf(f, "{\"who\": \"%s\", \"pid\": %d, \"op\": \"%s\", \"bytes\": %llu, \"t0_ns\": %llu, \"us\": %.3f, \"rc\": %d}\n",
                     who, (int)getpid(), r.op, (unsigned long long)r.bytes, (unsigned long long)r.t0,
                     (double)(r.t1 - r.t0) / 1e3, r.rc);
    int n = (int)g_log.size();
    g_log.clear();
    std::fclose(f);
    return n;
}

TraceRange::TraceRange(const char *name) : on_(trace_enabled()) {
    if (on_) roctxRangePushA(name);
}

TraceRange::~TraceRange() {
    if (on_) roctxRangePop();
}

}  // namespace ocm
