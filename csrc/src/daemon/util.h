// ocmd internals shared by the daemon's translation units.
#pragma once
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <cstdint>
#include <cstdlib>
#include <fstream>
#include <string>

#include "../../include/oncillamem.h"

namespace ocm {
namespace dm {

// epoll tags: kind in the top byte, fd / pid below

enum Tag : uint64_t { T_MBOX = 1, T_LISTEN, T_CONN, T_PIDFD, T_APPCONN, T_SIGNAL, T_TICK, T_WATCH };
inline uint64_t tag(Tag k, uint64_t id) { return (static_cast<uint64_t>(k) << 56) | (id & 0x00ffffffffffffffull); }
inline Tag tag_kind(uint64_t t) { return static_cast<Tag>(t >> 56); }
inline uint64_t tag_id(uint64_t t) { return t & 0x00ffffffffffffffull; }

inline long now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1000L + ts.tv_nsec / 1000000L;
}

inline int pidfd_open_compat(pid_t pid) { return (int)syscall(SYS_pidfd_open, pid, 0); }

inline bool is_remote_kind(uint32_t kind) {
    return kind == OCM_REMOTE_GPU || kind == OCM_REMOTE_RDMA || kind == OCM_REMOTE_RMA;
}

inline uint64_t parse_bytes(const std::string &s) {
    char *end = nullptr;
    double v = std::strtod(s.c_str(), &end);
    std::string suf = end ? end : "";
    uint64_t mul = 1;
    if (suf == "K" || suf == "KiB" || suf == "k") mul = 1ull << 10;
    else if (suf == "M" || suf == "MiB") mul = 1ull << 20;
    else if (suf == "G" || suf == "GiB") mul = 1ull << 30;
    else if (suf == "T" || suf == "TiB") mul = 1ull << 40;
    return (uint64_t)(v * (double)mul);
}

inline uint64_t mem_available() {
    std::ifstream f("/proc/meminfo");
    std::string k;
    uint64_t v;
    std::string unit;
    while (f >> k >> v >> unit)
        if (k == "MemAvailable:") return v * 1024ull;
    return 0;
}


}  // namespace dm
}  // namespace ocm
