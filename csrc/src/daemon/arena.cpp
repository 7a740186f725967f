// ocmd memory arenas: 4 GiB HBM slabs (hipMalloc, IPC-exported once) and
// memfd host-tier slabs, sub-allocated with coalescing ranges.
// Reference parity: the server side of alloc_ate / dealloc_ate
// src/alloc.c:150-282 (malloc + ibv_reg_mr / rma2_register of every buffer
// there, src/rdma_server.c:40-236), including the leak it fixes (src/alloc.c:171).
#include "ocm/arena.h"

#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <string>
#include <cstdio>
#include <cstring>

#include "ocm/log.h"

namespace ocm {

static constexpr uint64_t kHugeAlign = 2ull << 20;

int gpu_numa_node(int device) {
    if (device < 0) return -1;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    for (char *c = bus; *c; c++) *c = (char)std::tolower((unsigned char)*c);
    std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
    FILE *f = std::fopen(path.c_str(), "r");
    if (!f) return -1;
    int node = -1;
    if (std::fscanf(f, "%d", &node) != 1) node = -1;
    std::fclose(f);
    return node;
}

Arena::Arena(const ArenaConfig &cfg) : cfg_(cfg) {
    if (cfg_.align == 0 || (cfg_.align & (cfg_.align - 1))) cfg_.align = 4096;
    if (cfg_.slab_bytes < kHugeAlign) cfg_.slab_bytes = kHugeAlign;
}

Arena::~Arena() {
    for (auto &kv : slabs_) destroy_slab(kv.second.get());
    slabs_.clear();
}

uint64_t Arena::used(uint32_t tier) const {
    std::lock_guard<std::mutex> lk(mu_);
    return tier == TIER_GPU ? used_gpu_ : used_host_;
}

size_t Arena::num_slabs() const {
    std::lock_guard<std::mutex> lk(mu_);
    return slabs_.size();
}

bool Arena::locate(uint32_t slab_id, uint64_t offset, uint64_t len, void **p, uint32_t *tier) const {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = slabs_.find(slab_id);
    if (it == slabs_.end() || !it->second->base) return false;
    const Slab &s = *it->second;
    if (offset > s.bytes || len > s.bytes - offset) return false;
    *p = static_cast<char *>(s.base) + offset;
    *tier = s.tier;
    return true;
}

int Arena::dup_slab_fd(uint32_t slab_id) const {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = slabs_.find(slab_id);
    if (it == slabs_.end() || it->second->tier != TIER_HOST || it->second->memfd < 0) return -1;
    return fcntl(it->second->memfd, F_DUPFD_CLOEXEC, 0);
}

uint64_t Arena::capacity(uint32_t tier) const {
    return tier == TIER_GPU ? (cfg_.gpu >= 0 ? cfg_.gpu_capacity : 0) : cfg_.host_capacity;
}

Slab *Arena::new_slab(uint32_t tier, uint64_t bytes, bool dedicated, int *err) {
    auto s = std::make_unique<Slab>();
    s->id = next_slab_++;
    s->tier = tier;
    s->bytes = (bytes + kHugeAlign - 1) & ~(kHugeAlign - 1);
    s->dedicated = dedicated;
    if (tier == TIER_GPU) {
        if (cfg_.gpu < 0) {
            *err = ENODEV;
            return nullptr;
        }
        hipError_t e = hipSetDevice(cfg_.gpu);
        if (e == hipSuccess) e = hipMalloc(&s->base, s->bytes);
        if (e != hipSuccess) {
            OCM_WARN("hipMalloc(%llu) on gpu %d failed: %s", (unsigned long long)s->bytes, cfg_.gpu,
                     hipGetErrorString(e));
            (void)hipGetLastError();
            *err = ENOMEM;
            return nullptr;
        }
        hipIpcMemHandle_t h;
        static_assert(sizeof(h) == kHandleBytes, "hipIpcMemHandle_t must be 64 bytes");
        e = hipIpcGetMemHandle(&h, s->base);
        if (e != hipSuccess) {
            OCM_ERR("hipIpcGetMemHandle failed: %s", hipGetErrorString(e));
            (void)hipFree(s->base);
            *err = EIO;
            return nullptr;
        }
        std::memcpy(s->handle, &h, kHandleBytes);
    } else {
        char name[32];
        snprintf(name, sizeof(name), "ocm_host_slab_%u", s->id);
        s->memfd = memfd_create(name, MFD_CLOEXEC);
        if (s->memfd < 0 || ftruncate(s->memfd, (off_t)s->bytes) != 0) {
            OCM_WARN("host slab memfd(%llu): %s", (unsigned long long)s->bytes, strerror(errno));
            if (s->memfd >= 0) close(s->memfd);
            *err = ENOMEM;
            return nullptr;
        }
        void *p = mmap(nullptr, s->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, s->memfd, 0);
        if (p == MAP_FAILED) {
            close(s->memfd);
            *err = ENOMEM;
            return nullptr;
        }
        s->base = p;
        if (cfg_.numa_node >= 0 && cfg_.numa_node < 64) {
            // Shared policy on the memfd object: whichever process faults the pages in
            // (importers pin them), they land on the GPU's socket, so DMA stays local.
            unsigned long mask = 1ul << cfg_.numa_node;
            if (syscall(SYS_mbind, p, s->bytes, 1 /* MPOL_PREFERRED */, &mask, 64ul, 0u) != 0)
                OCM_WARN("mbind host slab to node %d: %s", cfg_.numa_node, strerror(errno));
        }
        snprintf(reinterpret_cast<char *>(s->handle), kHandleBytes, "/proc/%d/fd/%d", (int)getpid(), s->memfd);
    }
    s->ra.reset(s->bytes);
    Slab *raw = s.get();
    slabs_[raw->id] = std::move(s);
    OCM_LOG("new %s slab %u: %llu bytes%s", tier == TIER_GPU ? "HBM" : "host", raw->id,
            (unsigned long long)raw->bytes, dedicated ? " (dedicated)" : "");
    return raw;
}

void Arena::destroy_slab(Slab *s) {
    if (!s || !s->base) return;
    if (s->tier == TIER_GPU) {
        (void)hipSetDevice(cfg_.gpu);
        (void)hipFree(s->base);
    } else {
        munmap(s->base, s->bytes);
        if (s->memfd >= 0) close(s->memfd);
    }
    s->base = nullptr;
}

int Arena::alloc(uint32_t tier, uint64_t bytes, Region *out) {
    std::lock_guard<std::mutex> lk(mu_);
    if (bytes == 0) return EINVAL;
    if (tier != TIER_GPU && tier != TIER_HOST) return EINVAL;
    const uint64_t cap = capacity(tier), used = tier == TIER_GPU ? used_gpu_ : used_host_;
    if (bytes > cap || used > cap - bytes) return ENOMEM;  // overflow-safe
    // Host slabs: 1 GiB. Importers mmap + hipHostRegister a slab once (pinning
    // costs ~25 ms per 128 MiB), so requests below half a slab carve from one
    // already registered instead of paying that per allocation.
    uint64_t slab_default = tier == TIER_GPU ? cfg_.slab_bytes : std::min<uint64_t>(cfg_.slab_bytes, 1ull << 30);
    // Never map more than the tier may hand out (small capacities in tests / shared GPUs).
    slab_default = std::max(kHugeAlign, std::min(slab_default, (capacity(tier) + kHugeAlign - 1) & ~(kHugeAlign - 1)));
    Slab *slab = nullptr;
    uint64_t off = 0;
    int err = 0;
    if (bytes >= slab_default / 2) {
        slab = new_slab(tier, bytes, true, &err);
        if (!slab) return err;
        slab->ra.alloc(bytes, cfg_.align, &off);
    } else {
        for (auto &kv : slabs_) {
            Slab *s = kv.second.get();
            if (s->tier != tier || s->dedicated) continue;
            if (s->ra.alloc(bytes, cfg_.align, &off)) {
                slab = s;
                break;
            }
        }
        if (!slab) {
            slab = new_slab(tier, slab_default, false, &err);
            if (!slab) return err;
            if (!slab->ra.alloc(bytes, cfg_.align, &off)) return ENOMEM;
        }
    }
    void *p = static_cast<char *>(slab->base) + off;
    if (cfg_.zero_on_alloc) {
        if (tier == TIER_GPU) {
            (void)hipSetDevice(cfg_.gpu);
            (void)hipMemset(p, 0, bytes);
        } else {
            std::memset(p, 0, bytes);
        }
    }
    (tier == TIER_GPU ? used_gpu_ : used_host_) += bytes;
    std::memset(out->handle, 0, sizeof(out->handle));
    std::memcpy(out->handle, slab->handle, kHandleBytes);
    out->slab_id = slab->id;
    out->offset = off;
    out->slab_bytes = slab->bytes;
    out->bytes = bytes;
    out->tier = (uint16_t)tier;
    out->owner_gpu = tier == TIER_GPU ? cfg_.gpu : -1;
    out->flags = (uint16_t)((out->flags & ~REGION_DEDICATED) | (slab->dedicated ? REGION_DEDICATED : 0));
    return 0;
}

int Arena::free(uint32_t slab_id, uint64_t offset) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = slabs_.find(slab_id);
    if (it == slabs_.end()) return ENOENT;
    Slab *s = it->second.get();
    uint64_t before = s->ra.used();
    if (!s->ra.free(offset)) return ENOENT;
    uint64_t freed = before - s->ra.used();
    uint64_t &u = s->tier == TIER_GPU ? used_gpu_ : used_host_;
    u = u >= freed ? u - freed : 0;
    if (s->dedicated) {
        destroy_slab(s);
        slabs_.erase(it);
    }
    return 0;
}

void *Arena::resolve(uint32_t slab_id, uint64_t offset) const {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = slabs_.find(slab_id);
    if (it == slabs_.end() || offset >= it->second->bytes) return nullptr;
    return static_cast<char *>(it->second->base) + offset;
}

}  // namespace ocm
