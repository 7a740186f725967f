// Best-fit range allocator with coalescing (sub-allocation inside a slab).
//
// The reference allocated and registered a whole buffer per request
// (calloc + ibv_reg_mr, src/alloc.c:166-180). Here each daemon registers large
// HBM / host slabs once and hands out aligned ranges of them, so an ocm_alloc
// costs a control round trip, not a hipMalloc + export + import.
#pragma once
#include <cstdint>
#include <cstddef>
#include <map>

namespace ocm {

class RangeAllocator {
public:
    explicit RangeAllocator(uint64_t size = 0) { reset(size); }
    void reset(uint64_t size);
    // Returns true and the offset on success. `align` must be a power of two.
    bool alloc(uint64_t bytes, uint64_t align, uint64_t *off);
    // Frees a range previously returned by alloc (same bytes). Returns false on
    // a double free / unknown range.
    bool free(uint64_t off);
    uint64_t size() const { return size_; }
    uint64_t used() const { return used_; }
    uint64_t largest_free() const;
    size_t num_free_ranges() const { return free_by_off_.size(); }
    size_t num_live() const { return live_.size(); }
    bool empty() const { return live_.empty(); }

private:
    void insert_free(uint64_t off, uint64_t len);
    void erase_free(std::map<uint64_t, uint64_t>::iterator it);
    uint64_t size_ = 0, used_ = 0;
    std::map<uint64_t, uint64_t> free_by_off_;        // off -> len
    std::multimap<uint64_t, uint64_t> free_by_len_;   // len -> off
    std::map<uint64_t, uint64_t> live_;               // off -> len (incl. alignment pad)
};

}  // namespace ocm
