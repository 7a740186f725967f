#include "ocm/siphash.h"

#include <cstring>

namespace ocm {

namespace {

inline uint64_t rotl(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }

struct SipState {
    uint64_t v0, v1, v2, v3;
    void round() {
        v0 += v1;
        v1 = rotl(v1, 13);
        v1 ^= v0;
        v0 = rotl(v0, 32);
        v2 += v3;
        v3 = rotl(v3, 16);
        v3 ^= v2;
        v0 += v3;
        v3 = rotl(v3, 21);
        v3 ^= v0;
        v2 += v1;
        v1 = rotl(v1, 17);
        v1 ^= v2;
        v2 = rotl(v2, 32);
    }
    void absorb(uint64_t m) {
        v3 ^= m;
        round();  // c = 2 compression rounds
        round();
        v0 ^= m;
    }
};

inline uint64_t load_le64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}

}  // namespace

uint64_t siphash24(const SipKey &k, const void *data, size_t len) {
    const uint8_t *p = static_cast<const uint8_t *>(data);
    SipState s{k.k0 ^ 0x736f6d6570736575ull, k.k1 ^ 0x646f72616e646f6dull, k.k0 ^ 0x6c7967656e657261ull,
               k.k1 ^ 0x7465646279746573ull};
    const size_t full = len & ~size_t(7);
    for (size_t i = 0; i < full; i += 8) s.absorb(load_le64(p + i));
    uint64_t last = (uint64_t)(len & 0xff) << 56;
    for (size_t i = 0; i < (len & 7); i++) last |= (uint64_t)p[full + i] << (8 * i);
    s.absorb(last);
    s.v2 ^= 0xff;
    for (int i = 0; i < 4; i++) s.round();  // d = 4 finalization rounds
    return s.v0 ^ s.v1 ^ s.v2 ^ s.v3;
}

SipKey sip_derive_key(const std::string &material) {
    // Two independent PRF outputs of the material under fixed, distinct keys.
    const SipKey a{0x6f6e63696c6c6131ull, 0x6d6573682d6b6579ull};
    const SipKey b{0x6f6e63696c6c6132ull, 0x6d6573682d6b6579ull};
    return SipKey{siphash24(a, material.data(), material.size()), siphash24(b, material.data(), material.size())};
}

}  // namespace ocm
