// Host check (tests/test_sip_host.py): seed_hash (the build's hoisted per-seed SipRound, used for
// compile-time key lengths) equals prefix_hash (the direct restatement of bf.rs:222-227's
// per-seed part) for random SipHash states, every length byte and seeds 0..255.
#include <cstdio>
#include <random>

#include "../../velarixdb_amd/csrc/sip13.hpp"

int main() {
    std::mt19937_64 rng(20261017);
    long bad = 0, n = 0;
    for (int it = 0; it < 100000; ++it) {
        vbf::Prefix p{};
        p.st = vbf::Sip{rng(), rng(), rng(), rng()};
        p.tail = 0;
        p.r = 0;  // block-aligned prefix: every compile-time key length
        p.total = (uint32_t)(rng() & 0xff);
        const vbf::SeedCtx q = vbf::seed_ctx(p);
        for (uint32_t s = 0; s < 33; ++s, ++n) bad += vbf::prefix_hash(p, s) != vbf::seed_hash(q, s);
        const uint32_t s = (uint32_t)(rng() & 0xff);
        bad += vbf::prefix_hash(p, s) != vbf::seed_hash(q, s);
        ++n;
    }
    std::printf("checked %ld mismatches %ld\n", n, bad);
    return bad != 0;
}
