// Raw-backend client (reference test/ib_client.c / test/extoll_rma_client.c):
//   ocm_xgmi_client <endpoint> <test> <MB> [gpu]
//   test 0  one-sided write of 0xdeadbeef, server verifies, read back + verify
//   test 1  string handshake through remote offsets ("buffer size mismatch")
//   test 2  setup / teardown only
//   test 3  R/W sweep 64 B .. buffer size, timed (the reference never timed it)
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ocm/xgmi.h"

static bool is_device(void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

static void put_host(void *dst, const void *src, size_t n) {
    if (is_device(dst))
        (void)hipMemcpy(dst, src, n, hipMemcpyHostToDevice);
    else
        std::memcpy(dst, src, n);
}

static void get_host(void *src, void *dst, size_t n) {
    if (is_device(src))
        (void)hipMemcpy(dst, src, n, hipMemcpyDeviceToHost);
    else
        std::memcpy(dst, src, n);
}

static bool ask(xgmi_t x, const std::string &cmd) {
    char r[400];
    if (xgmi_send_ctrl(x, cmd.c_str()) != 0 || xgmi_recv_ctrl(x, r, sizeof(r), 60000) <= 0) return false;
    if (std::strcmp(r, "OK") != 0) {
        fprintf(stderr, "server: %s -> %s\n", cmd.c_str(), r);
        return false;
    }
    return true;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <endpoint> <test 0-3> <MB> [gpu]\n", argv[0]);
        return 2;
    }
    const int test = std::atoi(argv[2]);
    struct xgmi_params p;
    p.endpoint = argv[1];
    p.buf_len = (size_t)(std::strtod(argv[3], nullptr) * (1 << 20));
    p.gpu = argc > 4 ? std::atoi(argv[4]) : -1;
    p.buf = nullptr;
    xgmi_init();
    xgmi_t x = xgmi_new(&p);
    if (!x || xgmi_connect(x, false) != 0) {
        fprintf(stderr, "connect failed\n");
        return 1;
    }
    size_t len = 0;
    char *buf = static_cast<char *>(xgmi_localbuf(x, &len));
    const size_t rlen = xgmi_remote_len(x);
    const size_t n = std::min(len, rlen);
    int rc = 0;
    if (test == 0) {
        std::vector<uint32_t> v(n / 4, 0xdeadbeefu);
        put_host(buf, v.data(), v.size() * 4);
        if (xgmi_write(x, 0, 0, v.size() * 4) || xgmi_poll(x)) rc = 1;
        if (!rc && !ask(x, "VERIFY 0 " + std::to_string(v.size() * 4) + " deadbeef")) rc = 1;
        std::vector<uint32_t> z(n / 4, 0);
        put_host(buf, z.data(), z.size() * 4);
        if (!rc && (xgmi_read(x, 0, 0, v.size() * 4) || xgmi_poll(x))) rc = 1;
        get_host(buf, z.data(), z.size() * 4);
        for (uint32_t w : z)
            if (w != 0xdeadbeefu) {
                rc = 1;
                break;
            }
        printf("test 0 (write/read 0xdeadbeef, %zu bytes): %s\n", v.size() * 4, rc ? "FAIL" : "pass");
    } else if (test == 1) {
        const std::string msg = "buffer size mismatch";
        const size_t off = n / 2;
        put_host(buf + 64, msg.c_str(), msg.size() + 1);
        if (xgmi_write(x, 64, off, msg.size() + 1) || xgmi_poll(x)) rc = 1;
        if (!rc && !ask(x, "CHECK " + std::to_string(off) + " " + msg)) rc = 1;
        const std::string ans = "acknowledged: " + msg;
        if (!rc && !ask(x, "REPLY 128 " + ans)) rc = 1;
        std::vector<char> got(ans.size() + 1);
        if (!rc && (xgmi_read(x, 4096, 128, got.size()) || xgmi_poll(x))) rc = 1;
        get_host(buf + 4096, got.data(), got.size());
        if (std::strcmp(got.data(), ans.c_str()) != 0) rc = 1;
        printf("test 1 (string handshake): %s\n", rc ? "FAIL" : "pass");
    } else if (test == 2) {
        printf("test 2 (setup/teardown): pass\n");
    } else if (test == 3) {
        for (int op = 0; op < 2; op++) {
            for (size_t sz = 64; sz <= n; sz *= 2) {
                int iters = sz < (1 << 20) ? 50 : 5;
                auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < iters; i++) {
                    if ((op ? xgmi_write(x, 0, 0, sz) : xgmi_read(x, 0, 0, sz)) || xgmi_poll(x)) {
                        rc = 1;
                        break;
                    }
                }
                double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
                printf("%-5s %12zu B %10.2f us %9.2f GiB/s\n", op ? "write" : "read", sz, dt * 1e6,
                       (double)sz / dt / (1ull << 30));
            }
        }
    } else {
        rc = 2;
    }
    xgmi_disconnect(x, false);
    xgmi_free(x);
    return rc;
}
