#include "ocm/range_alloc.h"

namespace ocm {

void RangeAllocator::reset(uint64_t size) {
    size_ = size;
    used_ = 0;
    free_by_off_.clear();
    free_by_len_.clear();
    live_.clear();
    if (size) insert_free(0, size);
}

void RangeAllocator::insert_free(uint64_t off, uint64_t len) {
    free_by_off_[off] = len;
    free_by_len_.emplace(len, off);
}

void RangeAllocator::erase_free(std::map<uint64_t, uint64_t>::iterator it) {
    auto range = free_by_len_.equal_range(it->second);
    for (auto j = range.first; j != range.second; ++j) {
        if (j->second == it->first) {
            free_by_len_.erase(j);
            break;
        }
    }
    free_by_off_.erase(it);
}

bool RangeAllocator::alloc(uint64_t bytes, uint64_t align, uint64_t *off) {
    if (bytes == 0 || (align & (align - 1)) != 0) return false;
    // Best fit: smallest free range that can hold bytes after alignment.
    for (auto it = free_by_len_.lower_bound(bytes); it != free_by_len_.end(); ++it) {
        const uint64_t start = it->second, len = it->first;
        const uint64_t aligned = (start + align - 1) & ~(align - 1);
        const uint64_t pad = aligned - start;
        if (pad + bytes > len) continue;
        auto fit = free_by_off_.find(start);
        erase_free(fit);
        if (pad) insert_free(start, pad);  // keep the alignment hole
        const uint64_t tail = len - pad - bytes;
        if (tail) insert_free(aligned + bytes, tail);
        live_[aligned] = bytes;
        used_ += bytes;
        *off = aligned;
        return true;
    }
    return false;
}

bool RangeAllocator::free(uint64_t off) {
    auto lv = live_.find(off);
    if (lv == live_.end()) return false;
    uint64_t start = off, len = lv->second;
    used_ -= len;
    live_.erase(lv);
    // Coalesce with the following free range.
    auto next = free_by_off_.lower_bound(start);
    if (next != free_by_off_.end() && next->first == start + len) {
        len += next->second;
        erase_free(next);
    }
    // Coalesce with the preceding free range.
    auto it = free_by_off_.lower_bound(start);
    if (it != free_by_off_.begin()) {
        auto prev = std::prev(it);
        if (prev->first + prev->second == start) {
            start = prev->first;
            len += prev->second;
            erase_free(prev);
        }
    }
    insert_free(start, len);
    return true;
}

uint64_t RangeAllocator::largest_free() const {
    return free_by_len_.empty() ? 0 : free_by_len_.rbegin()->first;
}

}  // namespace ocm
