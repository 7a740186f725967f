// Mailbox ping-pong through the reference-shaped pmsg C API (reference
// test/pmsg_daemon.c + test/pmsg_client.c):
//   ocm_pmsg_pingpong server <rank>            echo server on daemon mailbox <rank>
//   ocm_pmsg_pingpong client <rank> <count>    send `count` pings, print p50/p99 RTT
// The client sends MSG_SHUTDOWN at the end so the server exits.
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ocm/msg.h"
#include "ocm/pmsg.h"

using namespace ocm;

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s server <rank> | client <rank> <count>\n", argv[0]);
        return 2;
    }
    const int rank = std::atoi(argv[2]);
    pmsg_init(kMsgBytes);
    Msg m, r;
    if (!std::strcmp(argv[1], "server")) {
        if (pmsg_open(PMSG_DAEMON_PID(rank)) != 0) return 1;
        printf("ready\n");
        fflush(stdout);
        for (;;) {
            if (pmsg_recv(&m, true) != 0) return 1;
            if (m.type == MSG_SHUTDOWN) break;
            m.status = MSG_RESPONSE;
            if (pmsg_send(m.pid, &m) != 0) return 1;  // back on the app's connection
        }
        pmsg_close();
        return 0;
    }
    const int count = argc > 3 ? std::atoi(argv[3]) : 1000;
    if (pmsg_open(getpid()) != 0) return 1;
    for (int i = 0; pmsg_attach(PMSG_DAEMON_PID(rank)) != 0; i++) {
        if (i > 500) return 1;
        usleep(10000);
    }
    std::vector<double> rtt;
    std::memset(&m, 0, sizeof(m));
    m.type = MSG_PING;
    m.pid = getpid();
    for (int i = 0; i < count; i++) {
        m.seq = (uint64_t)i + 1;
        auto t0 = std::chrono::steady_clock::now();
        if (pmsg_send(PMSG_DAEMON_PID(rank), &m) != 0 || pmsg_recv(&r, true) != 0 || r.seq != m.seq ||
            r.status != MSG_RESPONSE) {
            fprintf(stderr, "ping %d failed\n", i);
            return 1;
        }
        rtt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    m.type = MSG_SHUTDOWN;
    pmsg_send(PMSG_DAEMON_PID(rank), &m);
    std::sort(rtt.begin(), rtt.end());
    printf("{\"count\": %d, \"p50_us\": %.2f, \"p99_us\": %.2f}\n", count, rtt[rtt.size() / 2],
           rtt[std::min(rtt.size() - 1, rtt.size() * 99 / 100)]);
    pmsg_close();
    return 0;
}
