// Registered memory arena of one daemon: HBM slabs + pinned host-tier slabs.
//
// Parity with reference src/alloc.c:150-282 (alloc_ate / dealloc_ate: the owner
// allocates and registers the buffer, then tears it down on free) and the
// registration call sites ibv_reg_mr / rma2_register. Here:
//   * GPU tier: slabs from hipMalloc on the daemon's MI355X, exported once with
//     hipIpcGetMemHandle (64-byte handle carried in the wire Region);
//   * host tier: memfd-backed slabs shared as /proc/<pid>/fd/<n>; importers
//     mmap + hipHostRegister them (pinned, device-mapped) — the spill tier;
//   * requests are sub-allocated from slabs (RangeAllocator), larger requests
//     get a dedicated slab; freed dedicated slabs are released immediately.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "ocm/msg.h"
#include "ocm/range_alloc.h"

namespace ocm {

struct ArenaConfig {
    int gpu = -1;                    // -1: CPU-only daemon, no GPU tier
    uint64_t gpu_capacity = 0;       // max bytes handed out from HBM
    uint64_t host_capacity = 0;      // max bytes handed out from the host tier
    uint64_t slab_bytes = 4ull << 30;  // HBM slab: requests < 2 GiB carve from resident slabs
    uint64_t align = 4096;           // sub-allocation alignment
    bool zero_on_alloc = false;
    int numa_node = -1;              // host-tier pages preferred on this node (the GPU's socket); -1 = any
};

// NUMA node of a GPU's PCIe root (sysfs), -1 when unknown.
int gpu_numa_node(int device);

struct Slab {
    uint32_t id = 0;
    uint32_t tier = TIER_NONE;
    void *base = nullptr;
    uint64_t bytes = 0;
    bool dedicated = false;
    int memfd = -1;                  // host tier
    uint8_t handle[kHandleBytes] = {};
    RangeAllocator ra;
};

class Arena {
public:
    explicit Arena(const ArenaConfig &cfg);
    ~Arena();
    // Allocate `bytes` in `tier`; fills slab id/offset/handle of `out`.
    // Returns 0 or a positive errno.
    int alloc(uint32_t tier, uint64_t bytes, Region *out);
    int free(uint32_t slab_id, uint64_t offset);
    uint64_t used(uint32_t tier) const;
    uint64_t capacity(uint32_t tier) const;
    size_t num_slabs() const;
    const ArenaConfig &config() const { return cfg_; }
    // Raw pointer for daemon-side verification / tests.
    void *resolve(uint32_t slab_id, uint64_t offset) const;
    // Thread-safe bounds check for the network data server: [offset, +len)
    // inside slab `slab_id`; returns its address and tier.
    bool locate(uint32_t slab_id, uint64_t offset, uint64_t len, void **p, uint32_t *tier) const;
    // A dup of host-tier slab `slab_id`'s memfd (the caller closes it), -1 if none.
    int dup_slab_fd(uint32_t slab_id) const;

private:
    Slab *new_slab(uint32_t tier, uint64_t bytes, bool dedicated, int *err);
    void destroy_slab(Slab *s);
    ArenaConfig cfg_;
    uint32_t next_slab_ = 1;
    uint64_t used_gpu_ = 0, used_host_ = 0;
    std::map<uint32_t, std::unique_ptr<Slab>> slabs_;
    mutable std::mutex mu_;  // the event loop mutates, data-server threads locate()
};

}  // namespace ocm
