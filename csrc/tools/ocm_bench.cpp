// ocm_bench — native benchmark of the OncillaMem runtime, JSON output.
//
// SURVEY §5 (tracing/profiling): the reference timed nothing (test/ocm_test.c:323-425
// has no clock); this tool measures the BASELINE.json metric without Python:
//   * ocm_alloc / ocm_free latency distribution (p50/p99/mean) of a remote pair
//     and of the local malloc-backed kind (config #1);
//   * the reference R/W sweep (ocm_test 4): blocking one-sided get then put of
//     every power-of-two size on a 2*max+1 remote pair, data verified first;
//   * optionally a batch of random 4 KiB gets as one ocm_copy_onesided_batch.
//
//   ocm_bench [--min B] [--max B] [--iters N] [--alloc-samples N]
//             [--kind gpu|rdma] [--place auto|loopback|host|stripe]
//             [--batch N] [--json FILE]
// Attaches to the daemon named by OCM_DAEMON_RANK / OCM_NS like any app.
#include <algorithm>
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "oncillamem.h"

extern "C" long long ocm_x_pattern(void *p, uint64_t words, uint64_t first, uint32_t seed, int check);

namespace {

using clk = std::chrono::steady_clock;

double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

struct Dist {
    double p50 = 0, p99 = 0, mean = 0;
};

Dist dist_us(std::vector<double> v) {
    Dist d;
    if (v.empty()) return d;
    std::sort(v.begin(), v.end());
    d.p50 = v[v.size() / 2] * 1e6;
    d.p99 = v[std::min(v.size() - 1, (size_t)((double)v.size() * 0.99))] * 1e6;
    double s = 0;
    for (double x : v) s += x;
    d.mean = s / (double)v.size() * 1e6;
    return d;
}

struct Opts {
    uint64_t min_b = 4096, max_b = 1ull << 30;
    int iters = 0;  // 0: adaptive
    int alloc_samples = 200;
    enum ocm_kind kind = OCM_REMOTE_GPU;
    std::string place = "auto";
    int batch = 0;
    std::string json;
};

int usage() {
    std::fprintf(stderr,
                 "usage: ocm_bench [--min B] [--max B] [--iters N] [--alloc-samples N] [--kind gpu|rdma]\n"
                 "                 [--place auto|loopback|host|stripe] [--batch N] [--json FILE]\n");
    return 2;
}

uint32_t place_flags(const std::string &p) {
    if (p == "loopback") return OCM_ALLOC_LOOPBACK;
    if (p == "host") return OCM_ALLOC_HOST_TIER;
    if (p == "stripe") return OCM_ALLOC_STRIPE;
    return 0;
}

ocm_alloc_t alloc_pair(const Opts &o, uint64_t local, uint64_t remote) {
    struct ocm_alloc_params ap;
    std::memset(&ap, 0, sizeof(ap));
    ap.local_alloc_bytes = local;
    ap.rem_alloc_bytes = remote;
    ap.kind = o.kind;
    struct ocm_alloc_ex_params ex;
    std::memset(&ex, 0, sizeof(ex));
    ex.remote_rank = -1;
    ex.flags = place_flags(o.place);
    return ex.flags ? ocm_alloc_ex(&ap, &ex) : ocm_alloc(&ap);
}

int iters_for(const Opts &o, uint64_t sz) {
    if (o.iters > 0) return o.iters;
    if (sz <= (4ull << 20)) return 200;
    if (sz <= (64ull << 20)) return 20;
    return 3;
}

}  // namespace

int main(int argc, char **argv) {
    Opts o;
    for (int i = 1; i < argc; i++) {
        std::string k = argv[i];
        auto val = [&]() -> const char * { return i + 1 < argc ? argv[++i] : nullptr; };
        const char *v = nullptr;
        if (k == "--min" && (v = val())) o.min_b = std::strtoull(v, nullptr, 0);
        else if (k == "--max" && (v = val())) o.max_b = std::strtoull(v, nullptr, 0);
        else if (k == "--iters" && (v = val())) o.iters = std::atoi(v);
        else if (k == "--alloc-samples" && (v = val())) o.alloc_samples = std::atoi(v);
        else if (k == "--kind" && (v = val())) o.kind = std::strcmp(v, "rdma") ? OCM_REMOTE_GPU : OCM_REMOTE_RDMA;
        else if (k == "--place" && (v = val())) o.place = v;
        else if (k == "--batch" && (v = val())) o.batch = std::atoi(v);
        else if (k == "--json" && (v = val())) o.json = v;
        else return usage();
    }
    if (o.min_b == 0 || o.min_b > o.max_b) return usage();
    if (ocm_init() < 0) {
        std::fprintf(stderr, "ocm_init: %s\n", ocm_last_error());
        return 1;
    }
    if (o.kind == OCM_REMOTE_GPU && ocm_device() < 0) o.kind = OCM_REMOTE_RDMA;  // CPU-only process

    // ---- alloc / free latency ----
    std::vector<double> ta, tf, tl;
    for (int i = 0; i < o.alloc_samples; i++) {
        auto t0 = clk::now();
        ocm_alloc_t a = alloc_pair(o, 64 << 10, 1 << 20);
        auto t1 = clk::now();
        if (!a) {
            std::fprintf(stderr, "ocm_alloc (remote pair): %s\n", ocm_last_error());
            ocm_tini();
            return 1;
        }
        ocm_free(a);
        auto t2 = clk::now();
        ta.push_back(secs(t0, t1));
        tf.push_back(secs(t1, t2));
        struct ocm_alloc_params lp = {1 << 20, 0, OCM_LOCAL_HOST};
        t0 = clk::now();
        ocm_alloc_t l = ocm_alloc(&lp);
        tl.push_back(secs(t0, clk::now()));
        if (l) ocm_free(l);
    }
    const Dist da = dist_us(ta), df = dist_us(tf), dl = dist_us(tl);

    // ---- the sweep pair (reference: 2 GiB + 1 on each side) ----
    const uint64_t pair_b = 2 * o.max_b + 1;
    ocm_alloc_t a = alloc_pair(o, pair_b, pair_b);
    if (!a) {
        std::fprintf(stderr, "ocm_alloc (%" PRIu64 " B pair): %s\n", pair_b, ocm_last_error());
        ocm_tini();
        return 1;
    }
    struct ocm_remote_info info;
    std::memset(&info, 0, sizeof(info));
    ocm_remote_info(a, &info);
    void *lbuf = nullptr;
    size_t llen = 0;
    ocm_localbuf(a, &lbuf, &llen);

    // verify: pattern -> put -> clobber -> get -> check
    struct ocm_params p;
    std::memset(&p, 0, sizeof(p));
    p.bytes = o.max_b;
    const uint64_t words = o.max_b / 4;
    long long bad = -1;
    p.op_flag = 1;
    if (ocm_x_pattern(lbuf, words, 0, 4242, 0) == 0 && ocm_copy_onesided(a, &p) == 0 &&
        ocm_x_pattern(lbuf, words, 0, 0, 0) == 0) {
        p.op_flag = 0;
        if (ocm_copy_onesided(a, &p) == 0) bad = ocm_x_pattern(lbuf, words, 0, 4242, 1);
    }
    if (bad != 0) {
        std::fprintf(stderr, "verification failed (%lld bad words): %s\n", bad, ocm_last_error());
        ocm_free(a);
        ocm_tini();
        return 1;
    }

    std::string sweep;
    double moved = 0, spent = 0;
    for (uint64_t sz = o.min_b; sz <= o.max_b; sz *= 2) {
        double t[2] = {0, 0};
        for (int op = 0; op < 2; op++) {  // reads first, then writes (reference order)
            p.op_flag = op;
            p.bytes = sz;
            const int n = iters_for(o, sz);
            if (ocm_copy_onesided(a, &p) != 0) {  // warm-up
                std::fprintf(stderr, "one-sided op failed at %" PRIu64 " B: %s\n", sz, ocm_last_error());
                ocm_free(a);
                ocm_tini();
                return 1;
            }
            auto t0 = clk::now();
            for (int i = 0; i < n; i++) ocm_copy_onesided(a, &p);
            t[op] = secs(t0, clk::now()) / n;
            moved += (double)sz;
            spent += t[op];
        }
        char buf[256];
        std::snprintf(buf, sizeof(buf),
                      "%s\"%" PRIu64 "\": {\"get_us\": %.2f, \"put_us\": %.2f, \"get_GiBps\": %.3f, \"put_GiBps\": %.3f}",
                      sweep.empty() ? "" : ", ", sz, t[0] * 1e6, t[1] * 1e6, (double)sz / t[0] / (1ull << 30),
                      (double)sz / t[1] / (1ull << 30));
        sweep += buf;
    }

    // ---- optional batch of random 4 KiB gets ----
    std::string batch = "null";
    if (o.batch > 0) {
        std::vector<struct ocm_params> ops((size_t)o.batch);
        std::mt19937_64 rng(7);
        const uint64_t blocks = pair_b / 4096;
        for (int i = 0; i < o.batch; i++) {
            std::memset(&ops[i], 0, sizeof(ops[i]));
            ops[i].src_offset = (uint64_t)i % blocks * 4096;
            ops[i].dest_offset = (rng() % blocks) * 4096;
            ops[i].bytes = 4096;
            ops[i].op_flag = 0;
        }
        if (ocm_copy_onesided_batch(a, ops.data(), o.batch, 0) != 0) {
            std::fprintf(stderr, "batch failed: %s\n", ocm_last_error());
        } else {
            auto t0 = clk::now();
            const int n = 20;
            for (int i = 0; i < n; i++) ocm_copy_onesided_batch(a, ops.data(), o.batch, 0);
            const double bt = secs(t0, clk::now()) / n;
            char buf[160];
            std::snprintf(buf, sizeof(buf), "{\"ops\": %d, \"us\": %.2f, \"GiBps\": %.2f}", o.batch, bt * 1e6,
                          (double)o.batch * 4096 / bt / (1ull << 30));
            batch = buf;
        }
    }
    ocm_free(a);

    std::string tiers;
    for (uint32_t i = 0; i < info.n_extents; i++)
        tiers += std::string(i ? ", " : "") + (info.tier[i] == OCM_TIER_GPU ? "\"hbm\"" : "\"host\"");
    char head[1024];
    std::snprintf(head, sizeof(head),
                  "{\"tool\": \"ocm_bench\", \"device\": %d, \"rank\": %d, \"nodes\": %d, \"kind\": %d, "
                  "\"place\": \"%s\", \"extents\": %u, \"tiers\": [%s], \"pair_bytes\": %" PRIu64 ", "
                  "\"alloc_us\": {\"p50\": %.2f, \"p99\": %.2f, \"mean\": %.2f}, "
                  "\"free_us\": {\"p50\": %.2f, \"p99\": %.2f, \"mean\": %.2f}, "
                  "\"local_alloc_us\": {\"p50\": %.2f, \"p99\": %.2f, \"mean\": %.2f}, "
                  "\"sweep_GiBps\": %.3f, ",
                  ocm_device(), ocm_rank(), ocm_num_nodes(), (int)o.kind, o.place.c_str(), info.n_extents,
                  tiers.c_str(), pair_b, da.p50, da.p99, da.mean, df.p50, df.p99, df.mean, dl.p50, dl.p99, dl.mean,
                  moved / spent / (1ull << 30));
    std::string out = std::string(head) + "\"batch\": " + batch + ", \"sweep\": {" + sweep + "}}\n";
    std::fputs(out.c_str(), stdout);
    if (!o.json.empty()) {
        FILE *f = std::fopen(o.json.c_str(), "w");
        if (f) {
            std::fputs(out.c_str(), f);
            std::fclose(f);
        }
    }
    ocm_tini();
    return 0;
}
