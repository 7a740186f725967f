// Raw-backend server (reference test/ib_daemon.c / test/extoll_rma_daemon.c):
//   ocm_xgmi_daemon <endpoint> <MB> [gpu]
// Registers a buffer, waits for one client, then serves control requests:
//   VERIFY <off> <len> <word>   check that the client wrote `word` (e.g. 0xdeadbeef)
//   CHECK  <off> <string>       check a string the client wrote at <off>
//   REPLY  <off> <string>       write a string into our buffer for the client to read
//   FILL   <word>               fill our whole buffer with `word`
//   (BYE)                       tear down and exit 0
#include <hip/hip_runtime_api.h>

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

static void read_buf(void *src, void *dst, size_t n) {
    if (is_device(src))
        (void)hipMemcpy(dst, src, n, hipMemcpyDeviceToHost);
    else
        std::memcpy(dst, src, n);
}

static void write_buf(void *dst, const void *src, size_t n) {
    if (is_device(dst))
        (void)hipMemcpy(dst, src, n, hipMemcpyHostToDevice);
    else
        std::memcpy(dst, src, n);
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s <endpoint> <MB> [gpu]\n", argv[0]);
        return 2;
    }
    struct xgmi_params p;
    p.endpoint = argv[1];
    p.buf_len = (size_t)(std::strtod(argv[2], nullptr) * (1 << 20));
    p.gpu = argc > 3 ? std::atoi(argv[3]) : -1;
    p.buf = nullptr;
    xgmi_init();
    xgmi_t x = xgmi_new(&p);
    if (!x) return 1;
    printf("listening on %s (%zu bytes, gpu %d)\n", argv[1], p.buf_len, p.gpu);
    fflush(stdout);
    if (xgmi_connect(x, true) != 0) return 1;
    size_t len = 0;
    char *buf = static_cast<char *>(xgmi_localbuf(x, &len));
    int rc = 0;
    char cmd[400];
    for (;;) {
        int n = xgmi_recv_ctrl(x, cmd, sizeof(cmd), 600000);
        if (n <= 0) break;  // BYE or peer gone
        char verb[16] = {0}, arg[300] = {0};
        unsigned long long off = 0, cnt = 0, word = 0;
        std::string reply = "OK";
        if (sscanf(cmd, "VERIFY %llu %llu %llx", &off, &cnt, &word) == 3) {
            std::vector<uint32_t> v(cnt / 4);
            read_buf(buf + off, v.data(), v.size() * 4);
            size_t bad = 0;
            for (uint32_t w : v) bad += w != (uint32_t)word;
            if (bad) {
                reply = "BAD " + std::to_string(bad);
                rc = 1;
            }
        } else if (sscanf(cmd, "CHECK %llu %299[^\n]", &off, arg) == 2) {
            std::vector<char> got(std::strlen(arg) + 1);
            read_buf(buf + off, got.data(), got.size());
            if (std::strcmp(got.data(), arg) != 0) {
                reply = std::string("BAD got '") + got.data() + "'";
                rc = 1;
            }
        } else if (sscanf(cmd, "REPLY %llu %299[^\n]", &off, arg) == 2) {
            write_buf(buf + off, arg, std::strlen(arg) + 1);
        } else if (sscanf(cmd, "FILL %llx", &word) == 1) {
            std::vector<uint32_t> v(len / 4, (uint32_t)word);
            write_buf(buf, v.data(), v.size() * 4);
        } else if (sscanf(cmd, "%15s", verb) == 1) {
            reply = std::string("UNKNOWN ") + verb;
        }
        xgmi_send_ctrl(x, reply.c_str());
    }
    xgmi_disconnect(x, true);
    xgmi_free(x);
    printf("server done rc=%d\n", rc);
    return rc;
}
