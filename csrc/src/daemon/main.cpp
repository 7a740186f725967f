// ocmd entry point: `ocmd <nodefile> [options]` (reference: `oncillamem <nodefile>`,
// src/main.c:187-224). Start one per GPU; rank0 is the master and must be
// reachable within --join-timeout-ms by the others.
#include <pthread.h>
#include <signal.h>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "ocm/daemon.h"
#include "ocm/log.h"

int main(int argc, char **argv) {
    // Block the shutdown signals before anything can start a thread (the HIP
    // runtime does, on first use): threads inherit the mask, so SIGTERM/SIGINT
    // stay pending for the event loop's signalfd and the daemon shuts down in
    // order (directory checkpoint, tick transport, data server). Blocked only
    // later, a runtime thread would take the default action and kill the process.
    sigset_t mask;
    sigemptyset(&mask);
    sigaddset(&mask, SIGINT);
    sigaddset(&mask, SIGTERM);
    pthread_sigmask(SIG_BLOCK, &mask, nullptr);
    // RCCL reads its environment when the tick thread creates the communicator;
    // set here, before any thread exists (setenv is not thread-safe). Captured
    // ticks (OCM_TICK_GRAPH) use plain buffers: no user-buffer registration with
    // the peers while capturing.
    setenv("NCCL_GRAPH_REGISTER", "0", 0);
    ocm::DaemonConfig cfg;
    std::string err;
    const int rc = ocm::parse_daemon_args(argc, argv, &cfg, &err);
    if (rc > 0) {  // --help
        std::printf("%s\n", err.c_str());
        return 0;
    }
    if (rc != 0) {
        std::fprintf(stderr, "%s\n", err.c_str());
        return 2;
    }
    ocm::Daemon d(cfg);
    return d.run();
}
