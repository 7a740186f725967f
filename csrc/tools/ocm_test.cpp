// ocm_test: end-to-end tests through a running ocmd mesh.
//
// Same test numbering and CLI as the reference test/ocm_test.c:18-30,481-530:
//   1 <local MB> <remote MB> <sub>  allocation (sub 1 host, 2 GPU, 3 remote-RDMA, 4 remote-RMA, 5 remote-GPU)
//   2 <local MB> <remote MB>        one-sided read then write of a remote pair
//   3 <local MB> <remote MB>        two-sided ocm_copy matrix (host, GPU, remote)
//   4 <type> <iters>                R/W sweep 64 B .. 1 GiB on a 2 GiB+1 pair (type 0 IB, 1 EXTOLL, 2 GPU)
// Unlike the reference, every transfer is verified against a random fill and
// test 4 is timed (the reference had no timer: SURVEY §4). Extra:
//   5 <MB> <flags>                  striped / placed allocation round trip (ocm_alloc_ex)
// Exit status 0 = pass.
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "oncillamem.h"

namespace {

void fill_random(std::vector<uint8_t> &v, uint64_t seed) {
    std::mt19937_64 g(seed);
    size_t i = 0;
    for (; i + 8 <= v.size(); i += 8) {
        uint64_t x = g();
        std::memcpy(&v[i], &x, 8);
    }
    for (; i < v.size(); i++) v[i] = (uint8_t)g();
}

// Copy between a host vector and an allocation's local half (host or device).
bool to_local(ocm_alloc_t a, const std::vector<uint8_t> &src, size_t off) {
    void *buf;
    size_t len;
    if (ocm_localbuf(a, &buf, &len) || off + src.size() > len) return false;
    hipPointerAttribute_t at;
    bool dev = ocm_device() >= 0 && hipPointerGetAttributes(&at, buf) == hipSuccess && at.type == hipMemoryTypeDevice;
    if (!dev) (void)hipGetLastError();
    if (dev) return hipMemcpy((char *)buf + off, src.data(), src.size(), hipMemcpyHostToDevice) == hipSuccess;
    std::memcpy((char *)buf + off, src.data(), src.size());
    return true;
}

bool from_local(ocm_alloc_t a, std::vector<uint8_t> &dst, size_t off) {
    void *buf;
    size_t len;
    if (ocm_localbuf(a, &buf, &len) || off + dst.size() > len) return false;
    hipPointerAttribute_t at;
    bool dev = ocm_device() >= 0 && hipPointerGetAttributes(&at, buf) == hipSuccess && at.type == hipMemoryTypeDevice;
    if (!dev) (void)hipGetLastError();
    if (dev) return hipMemcpy(dst.data(), (char *)buf + off, dst.size(), hipMemcpyDeviceToHost) == hipSuccess;
    std::memcpy(dst.data(), (char *)buf + off, dst.size());
    return true;
}

enum ocm_kind remote_kind_from_env() {
    const char *k = std::getenv("OCM_TEST_REMOTE_KIND");
    if (k && !std::strcmp(k, "rdma")) return OCM_REMOTE_RDMA;
    if (k && !std::strcmp(k, "rma")) return OCM_REMOTE_RMA;
    return ocm_device() >= 0 ? OCM_REMOTE_GPU : OCM_REMOTE_RDMA;
}

int alloc_test(int sub, uint64_t local_b, uint64_t rem_b) {
    if (ocm_init() < 0) {
        printf("Cannot connect to OCM: %s\n", ocm_last_error());
        return -1;
    }
    struct ocm_alloc_params ap;
    std::memset(&ap, 0, sizeof(ap));
    ap.local_alloc_bytes = local_b;
    switch (sub) {
    case 1: ap.kind = OCM_LOCAL_HOST; break;
    case 2: ap.kind = OCM_LOCAL_GPU; break;
    case 3: ap.kind = OCM_REMOTE_RDMA; ap.rem_alloc_bytes = rem_b; break;
    case 4: ap.kind = OCM_REMOTE_RMA; ap.rem_alloc_bytes = rem_b; break;
    case 5: ap.kind = OCM_REMOTE_GPU; ap.rem_alloc_bytes = rem_b; break;
    default: printf("bad suboption %d\n", sub); return -1;
    }
    for (int i = 0; i < 3; i++) {
        ocm_alloc_t a = ocm_alloc(&ap);
        if (!a) {
            printf("ocm_alloc failed: %s\n", ocm_last_error());
            ocm_tini();
            return -1;
        }
        void *buf;
        size_t len, rlen = 0;
        if (ocm_localbuf(a, &buf, &len) || len != local_b) {
            printf("ocm_localbuf failed\n");
            return -1;
        }
        printf("local buffer size %zu @ %p\n", len, buf);
        const bool want_remote = sub >= 3;
        if (ocm_is_remote(a) != want_remote) {
            printf("ocm_is_remote wrong for kind %d\n", ap.kind);
            return -1;
        }
        if (want_remote) {
            if (ocm_remote_sz(a, &rlen) || rlen != rem_b) {
                printf("ocm_remote_sz wrong (%zu != %" PRIu64 ")\n", rlen, rem_b);
                return -1;
            }
            struct ocm_remote_info info;
            ocm_remote_info(a, &info);
            printf("alloc is remote; size = %zu, extents %u, owner rank %d tier %u\n", rlen, info.n_extents,
                   info.owner_rank[0], info.tier[0]);
        } else if (ocm_remote_sz(a, &rlen) == 0) {
            printf("local alloc reports a remote size\n");
            return -1;
        }
        if (ocm_alloc_kind(a) != ap.kind) {
            printf("ocm_alloc_kind mismatch\n");
            return -1;
        }
        if (ocm_free(a)) {
            printf("ocm_free failed: %s\n", ocm_last_error());
            return -1;
        }
    }
    if (ocm_free(nullptr) == 0) {
        printf("ocm_free(NULL) should fail\n");
        return -1;
    }
    if (ocm_tini() < 0) return -1;
    printf("OCM test completed successfully\n");
    return 0;
}

int copy_onesided_test(uint64_t local_b, uint64_t rem_b) {
    if (ocm_init() < 0) {
        printf("Cannot connect to OCM: %s\n", ocm_last_error());
        return -1;
    }
    struct ocm_alloc_params ap;
    std::memset(&ap, 0, sizeof(ap));
    ap.local_alloc_bytes = local_b + 1;
    ap.rem_alloc_bytes = rem_b + 1;
    ap.kind = remote_kind_from_env();
    ocm_alloc_t a = ocm_alloc(&ap);
    if (!a) {
        printf("ocm_alloc failed: %s\n", ocm_last_error());
        return -1;
    }
    int rc = 0;
    std::vector<uint8_t> pat(local_b), back(local_b, 0);
    fill_random(pat, 1234);
    struct ocm_params p;
    std::memset(&p, 0, sizeof(p));
    p.bytes = local_b;
    // write local -> remote, clobber local, read back, compare
    if (!to_local(a, pat, 0)) rc = -1;
    p.op_flag = 1;
    if (!rc && ocm_copy_onesided(a, &p)) {
        printf("ocm_copy_onesided (write) failed: %s\n", ocm_last_error());
        rc = -1;
    }
    std::vector<uint8_t> zero(local_b, 0);
    if (!rc && !to_local(a, zero, 0)) rc = -1;
    p.op_flag = 0;
    if (!rc && ocm_copy_onesided(a, &p)) {
        printf("ocm_copy_onesided (read) failed: %s\n", ocm_last_error());
        rc = -1;
    }
    if (!rc && (!from_local(a, back, 0) || back != pat)) {
        printf("one-sided round trip mismatch\n");
        rc = -1;
    }
    // offsets: remote[dest_offset] <- local[src_offset]
    if (!rc && local_b >= 8192) {
        p.src_offset = 4096 + 3;
        p.dest_offset = 17;
        p.bytes = local_b - 8192;
        p.op_flag = 1;
        if (ocm_copy_onesided(a, &p)) rc = -1;
        std::vector<uint8_t> z2(local_b, 0);
        to_local(a, z2, 0);
        p.src_offset = 0;
        p.op_flag = 0;
        if (!rc && ocm_copy_onesided(a, &p)) rc = -1;
        std::vector<uint8_t> got(p.bytes);
        if (!rc && (!from_local(a, got, 0) || std::memcmp(got.data(), pat.data() + 4096 + 3, p.bytes) != 0)) {
            printf("offset round trip mismatch\n");
            rc = -1;
        }
    }
    // bounds: must be rejected
    p.src_offset = 0;
    p.dest_offset = rem_b;
    p.bytes = 2;
    if (!rc && ocm_copy_onesided(a, &p) == 0) {
        printf("out-of-bounds one-sided copy was accepted\n");
        rc = -1;
    }
    ocm_free(a);
    ocm_tini();
    if (!rc) printf("OCM test completed successfully\n");
    return rc;
}

int copy_twosided_test(uint64_t local_b, uint64_t rem_b) {
    if (ocm_init() < 0) {
        printf("Cannot connect to OCM: %s\n", ocm_last_error());
        return -1;
    }
    struct ocm_alloc_params ap;
    std::memset(&ap, 0, sizeof(ap));
    ap.local_alloc_bytes = local_b;
    ap.kind = OCM_LOCAL_HOST;
    ocm_alloc_t h1 = ocm_alloc(&ap), h2 = ocm_alloc(&ap), g = nullptr;
    if (ocm_device() >= 0) {
        ap.kind = OCM_LOCAL_GPU;
        g = ocm_alloc(&ap);
    }
    ap.kind = remote_kind_from_env();
    ap.rem_alloc_bytes = rem_b;
    ocm_alloc_t r = ocm_alloc(&ap);
    if (!h1 || !h2 || !r || (ocm_device() >= 0 && !g)) {
        printf("allocation failed: %s\n", ocm_last_error());
        return -1;
    }
    struct ocm_params p;
    std::memset(&p, 0, sizeof(p));
    p.bytes = local_b;
    p.op_flag = 1;
    std::vector<uint8_t> pat(local_b), got(local_b);
    fill_random(pat, 99);
    int rc = 0;
    auto check = [&](ocm_alloc_t a, const char *what) {
        std::fill(got.begin(), got.end(), 0);
        if (!from_local(a, got, 0) || got != pat) {
            printf("ocm_copy %s: data mismatch\n", what);
            rc = -1;
        }
    };
    to_local(h1, pat, 0);
    if (ocm_copy(h2, h1, &p)) rc = -1;  // host -> host
    check(h2, "host->host");
    std::vector<uint8_t> z(local_b, 0);
    if (g) {
        if (ocm_copy(g, h1, &p)) rc = -1;  // host -> GPU
        check(g, "host->GPU");
        to_local(h2, z, 0);
        if (ocm_copy(h2, g, &p)) rc = -1;  // GPU -> host
        check(h2, "GPU->host");
    }
    if (ocm_copy(r, h1, &p)) rc = -1;  // host -> remote (staged, *_2 offsets = 0)
    to_local(h2, z, 0);
    to_local(r, z, 0);
    if (ocm_copy(h2, r, &p)) rc = -1;  // remote -> host
    check(h2, "host->remote->host");
    if (g) {
        to_local(g, z, 0);
        if (ocm_copy(g, r, &p)) rc = -1;  // remote -> GPU
        check(g, "remote->GPU");
        if (ocm_copy(r, g, &p)) rc = -1;  // GPU -> remote
    }
    // op_flag = 0 swaps the roles: read r into h1.
    to_local(h1, z, 0);
    p.op_flag = 0;
    if (ocm_copy(r, h1, &p)) rc = -1;
    check(h1, "read (op_flag=0)");
    // copy_in / copy_out on the remote pair (stubs in the reference).
    std::vector<uint8_t> big(rem_b), bigback(rem_b);
    fill_random(big, 7);
    if (ocm_copy_in(r, big.data()) || ocm_copy_out(bigback.data(), r) || big != bigback) {
        printf("ocm_copy_in/out mismatch\n");
        rc = -1;
    }
    ocm_free(h1);
    ocm_free(h2);
    if (g) ocm_free(g);
    ocm_free(r);
    ocm_tini();
    if (!rc) printf("OCM test completed successfully\n");
    return rc;
}

int read_write_bw_test(int iters, int type, uint64_t max_b) {
    if (ocm_init() < 0) {
        printf("Cannot connect to OCM: %s\n", ocm_last_error());
        return -1;
    }
    struct ocm_alloc_params ap;
    std::memset(&ap, 0, sizeof(ap));
    ap.local_alloc_bytes = 2 * max_b + 1;
    ap.rem_alloc_bytes = 2 * max_b + 1;
    ap.kind = type == 0 ? OCM_REMOTE_RDMA : type == 1 ? OCM_REMOTE_RMA : OCM_REMOTE_GPU;
    if (ap.kind == OCM_REMOTE_GPU && ocm_device() < 0) ap.kind = OCM_REMOTE_RDMA;
    ocm_alloc_t a = ocm_alloc(&ap);
    if (!a) {
        printf("ocm_alloc failed: %s\n", ocm_last_error());
        return -1;
    }
    struct ocm_params p;
    std::memset(&p, 0, sizeof(p));
    for (int op = 0; op < 2; op++) {
        p.op_flag = op;  // reads first, then writes (reference order)
        for (uint64_t sz = 64; sz <= max_b; sz *= 2) {
            p.bytes = sz;
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < iters; i++) {
                if (ocm_copy_onesided(a, &p)) {
                    printf("ocm_copy_onesided (%s) failed at size %" PRIu64 ": %s\n", op ? "write" : "read", sz,
                           ocm_last_error());
                    ocm_free(a);
                    ocm_tini();
                    return -1;
                }
            }
            double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
            printf("%-5s %12" PRIu64 " B  %10.2f us  %9.2f GiB/s\n", op ? "write" : "read", sz, dt * 1e6,
                   (double)sz / dt / (1ull << 30));
        }
    }
    ocm_free(a);
    ocm_tini();
    printf("OCM test completed successfully\n");
    return 0;
}

int striped_test(uint64_t bytes, uint32_t flags) {
    if (ocm_init() < 0) {
        printf("Cannot connect to OCM: %s\n", ocm_last_error());
        return -1;
    }
    struct ocm_alloc_params ap;
    std::memset(&ap, 0, sizeof(ap));
    ap.local_alloc_bytes = bytes;
    ap.rem_alloc_bytes = bytes;
    ap.kind = remote_kind_from_env();
    struct ocm_alloc_ex_params ex;
    std::memset(&ex, 0, sizeof(ex));
    ex.remote_rank = -1;
    ex.flags = flags;
    ex.stripe_unit = 64 * 1024;
    ocm_alloc_t a = ocm_alloc_ex(&ap, &ex);
    if (!a) {
        printf("ocm_alloc_ex failed: %s\n", ocm_last_error());
        return -1;
    }
    struct ocm_remote_info info;
    ocm_remote_info(a, &info);
    printf("extents %u unit %" PRIu64 ":", info.n_extents, info.stripe_unit);
    for (uint32_t i = 0; i < info.n_extents; i++)
        printf(" [rank %d tier %u %" PRIu64 " B]", info.owner_rank[i], info.tier[i], info.extent_bytes[i]);
    printf("\n");
    std::vector<uint8_t> pat(bytes), back(bytes, 0);
    fill_random(pat, 4242);
    int rc = 0;
    if (ocm_copy_in(a, pat.data()) || ocm_copy_out(back.data(), a) || back != pat) {
        printf("striped copy_in/out mismatch\n");
        rc = -1;
    }
    // unaligned one-sided range across stripe boundaries
    struct ocm_params p;
    std::memset(&p, 0, sizeof(p));
    if (!rc && bytes > 300000) {
        p.src_offset = 5;
        p.dest_offset = 65536 - 7;
        p.bytes = 200000;
        p.op_flag = 0;
        std::vector<uint8_t> z(bytes, 0);
        to_local(a, z, 0);
        if (ocm_copy_onesided(a, &p)) rc = -1;
        std::vector<uint8_t> got(bytes);
        if (!rc && (!from_local(a, got, 0) || std::memcmp(got.data() + 5, pat.data() + 65536 - 7, 200000) != 0)) {
            printf("striped unaligned read mismatch\n");
            rc = -1;
        }
    }
    ocm_free(a);
    ocm_tini();
    if (!rc) printf("OCM test completed successfully\n");
    return rc;
}

void usage(const char *p) {
    fprintf(stderr,
            "Usage: %s <test> ...\n"
            "  1 <local MB> <remote MB> <sub>   allocation (1 host, 2 GPU, 3 IB-like, 4 EXTOLL-like, 5 remote GPU)\n"
            "  2 <local MB> <remote MB>         one-sided copy\n"
            "  3 <local MB> <remote MB>         two-sided copy\n"
            "  4 <type 0|1|2> <iters> [max MB]  R/W bandwidth sweep\n"
            "  5 <MB> <flags>                   ocm_alloc_ex (flags: 1 stripe, 2 host tier, 16 loopback)\n",
            p);
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) {
        usage(argv[0]);
        return 2;
    }
    int test = std::atoi(argv[1]);
    auto mb = [](const char *s) { return (uint64_t)(std::strtod(s, nullptr) * (double)(1 << 20)); };
    int rc = -1;
    switch (test) {
    case 1:
        if (argc != 5) break;
        rc = alloc_test(std::atoi(argv[4]), mb(argv[2]), mb(argv[3]));
        break;
    case 2:
        if (argc != 4) break;
        if (mb(argv[2]) > mb(argv[3])) {
            printf("Please use a larger remote buffer size than local size\n");
            return 2;
        }
        rc = copy_onesided_test(mb(argv[2]), mb(argv[3]));
        break;
    case 3:
        if (argc != 4) break;
        rc = copy_twosided_test(mb(argv[2]), mb(argv[3]));
        break;
    case 4:
        if (argc < 4) break;
        rc = read_write_bw_test(std::atoi(argv[3]), std::atoi(argv[2]), argc > 4 ? mb(argv[4]) : (1ull << 30));
        break;
    case 5:
        if (argc != 4) break;
        rc = striped_test(mb(argv[2]), (uint32_t)std::atoi(argv[3]));
        break;
    default: break;
    }
    if (rc == -1 && argc >= 2 && test >= 1 && test <= 5) {
        fprintf(stderr, "FAIL: test %d\n", test);
        return 1;
    }
    if (rc != 0) {
        usage(argv[0]);
        return 2;
    }
    printf("pass: test %d\n", test);
    return 0;
}
