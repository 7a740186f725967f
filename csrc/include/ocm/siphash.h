// SipHash-2-4: a keyed 64-bit PRF (Aumasson & Bernstein, 2012), used as the
// MAC of mesh HELLO records. A 128-bit key derived from the shared mesh key
// signs (ranks, timestamp, nonce). That replaces the reference's unauthenticated
// TCP RPC (src/mem.c:62-111) and round 1's static, replayable hash token.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace ocm {

struct SipKey {
    uint64_t k0 = 0, k1 = 0;
};

uint64_t siphash24(const SipKey &k, const void *data, size_t len);

// Derive a SipHash key from arbitrary key material (namespace + secret).
SipKey sip_derive_key(const std::string &material);

}  // namespace ocm
