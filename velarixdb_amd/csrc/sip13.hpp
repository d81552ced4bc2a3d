// sip13.hpp -- SipHash-1-3 (keys 0,0) for gfx950, split into a per-key prefix absorb and a
// per-seed finish so that the k hashes of one key share the `LE64(len) || key` blocks.
//
// What is computed (velarixdb src/filter/bf.rs:222-227, Rust std DefaultHasher):
//   h(key, i) = SipHash-1-3(k0=0, k1=0, [LE64(len(key))] || key || LE64(i))
// The bracketed length block is present for byte keys (`Hash for [u8]`, every production call
// site); callers that pre-encode integer keys pass len_prefix = 0.
//
// On gfx950 a 64-bit add is one v_lshl_add_u64, a rotate by 13/16/17/21 two v_alignbit_b32 (both
// half-rate: ~4.3 cycles per wave-instruction per SIMD against ~2.4-2.9 for v_xor / v_mov,
// tools/isa_rate), and a rotate by 32 a register rename -- plus two v_mov when the swapped value
// next feeds a v_lshl_add_u64, whose operands must sit in aligned register pairs.  One SipRound
// is ~24 VALU instructions, ~80 SIMD cycles per wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vbf {

struct Sip {
    uint64_t v0, v1, v2, v3;
};

// 64-bit rotate by B < 32 as two v_alignbit_b32 (hipcc's own lowering of the C rotate is a
// 64-bit shift + 32-bit shift + or: 22% slower for the whole hash, measured in tools/ubench).
// The SipHash core below is also compiled for the host: the library's own single-key path for
// host-resident (memtable) filters runs the same rounds on the CPU (vbf_api.hip).
template <int B>
__host__ __device__ __forceinline__ uint64_t rotl64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - B);
    const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - B);
    return ((uint64_t)nhi << 32) | nlo;
#else
    return (x << B) | (x >> (64 - B));
#endif
}

// Rotate by 32: swap the halves (free: register renaming).
__host__ __device__ __forceinline__ uint64_t swap32(uint64_t x) { return (x >> 32) | (x << 32); }

__host__ __device__ __forceinline__ void sip_round(Sip& s) {
    s.v0 += s.v1; s.v1 = rotl64<13>(s.v1); s.v1 ^= s.v0; s.v0 = swap32(s.v0);
    s.v2 += s.v3; s.v3 = rotl64<16>(s.v3); s.v3 ^= s.v2;
    s.v0 += s.v3; s.v3 = rotl64<21>(s.v3); s.v3 ^= s.v0;
    s.v2 += s.v1; s.v1 = rotl64<17>(s.v1); s.v1 ^= s.v2; s.v2 = swap32(s.v2);
}

__host__ __device__ __forceinline__ Sip sip_init() {
    return Sip{0x736f6d6570736575ULL, 0x646f72616e646f6dULL, 0x6c7967656e657261ULL,
               0x7465646279746573ULL};
}

// c = 1 compression round per 8-byte block.
__host__ __device__ __forceinline__ void sip_compress(Sip& s, uint64_t m) {
    s.v3 ^= m;
    sip_round(s);
    s.v0 ^= m;
}

// a ^ b ^ c in one v_bitop3_b32 per 32-bit half on gfx950 (truth table 0x96)
__host__ __device__ __forceinline__ uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}
__host__ __device__ __forceinline__ uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
    return ((uint64_t)xor3_32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32) |
           xor3_32((uint32_t)a, (uint32_t)b, (uint32_t)c);
}

// Final block b (length byte << 56 | tail bytes) + d = 3 finalization rounds.  The last round is
// written out to what reaches the output v0 ^ v1 ^ v2 ^ v3: with v0' = swap32(v0) + v3r and
// v3' = rotl21(v3r) ^ v0', v0' cancels (v0' ^ v3' = rotl21(v3r)), so the result is
// rotl21(v3r) ^ rotl17(v1r) ^ v2' ^ swap32(v2') -- one v_bitop3 and one v_xor per half.
__host__ __device__ __forceinline__ uint64_t sip_finish(Sip s, uint64_t b) {
    s.v3 ^= b;
    sip_round(s);
    s.v0 ^= b;
    s.v2 ^= 0xff;
    sip_round(s);
    sip_round(s);
    s.v0 += s.v1;
    const uint64_t v1r = rotl64<13>(s.v1) ^ s.v0;
    s.v2 += s.v3;
    const uint64_t v3r = rotl64<16>(s.v3) ^ s.v2;
    const uint64_t v2n = s.v2 + v1r;
    return xor3_64(rotl64<21>(v3r), rotl64<17>(v1r), v2n) ^ swap32(v2n);
}

// State after absorbing every full block of the seed-independent prefix
// P = [LE64(len)] || key (P bytes).  `tail` holds the last P % 8 bytes (r of them).
struct Prefix {
    Sip st;
    uint64_t tail;
    uint32_t r;      // P % 8
    uint32_t total;  // (P + 8) & 0xff: the length byte of the final block
};

// Hash for seed i: one block (tail bytes || low bytes of LE64(i)), then the final block
// (remaining seed bytes || length byte).  5 SipRounds per seed.
__host__ __device__ __forceinline__ uint64_t prefix_hash(const Prefix& p, uint64_t seed) {
    Sip s = p.st;
    const uint32_t sb = p.r * 8;  // 0..56
    // sb == 0: block = seed, tail = 0.  The double shift keeps every shift count < 64.
    const uint64_t blk = p.tail | (seed << sb);
    const uint64_t hi = (seed >> 1) >> (63 - sb);  // == seed >> (64 - sb), and 0 when sb == 0
    sip_compress(s, blk);
    return sip_finish(s, ((uint64_t)p.total << 56) | hi);
}

// The same hash when the prefix ends on a block boundary (P % 8 == 0: every compile-time key
// length, 8/16/24/32 bytes with or without the length block), with the seed-independent half of
// the first per-seed SipRound done once per key.  The seed block is the seed itself, so that
// round's v0 += v1 / rotl13 / swap and rotl16(v3) do not depend on it: rotl16(v3 ^ seed) =
// rotl16(v3) ^ (seed << 16) for seed < 2^16, and the swapped sum is paired for the next 64-bit
// add once per key instead of once per seed.  Bit-identical to prefix_hash (tests/test_gpu_parity).
struct SeedCtx {
    uint64_t v2, v3, as, b1, r16, r17b;
    uint32_t total;
};
__host__ __device__ __forceinline__ SeedCtx seed_ctx(const Prefix& p) {
    SeedCtx q;
    const uint64_t a = p.st.v0 + p.st.v1;
    q.b1 = rotl64<13>(p.st.v1) ^ a;
    q.as = swap32(a);
    q.v2 = p.st.v2;
    q.v3 = p.st.v3;
    q.r16 = rotl64<16>(p.st.v3);
    q.r17b = rotl64<17>(q.b1);
    q.total = p.total;
    return q;
}
__host__ __device__ __forceinline__ uint64_t seed_hash(const SeedCtx& q, uint32_t seed) {
    const uint64_t c = q.v2 + (q.v3 ^ seed);                             // v2 += v3 ^ m
    const uint64_t d = ((uint64_t)((uint32_t)(q.r16 >> 32) ^ (uint32_t)(c >> 32)) << 32) |
                       xor3_32((uint32_t)q.r16, (uint32_t)c, seed << 16);  // rotl16(v3 ^ m) ^ v2
    const uint64_t e = q.as + d;                                         // v0 += v3
    Sip s;
    s.v3 = rotl64<21>(d) ^ e;
    const uint64_t g = c + q.b1;                                         // v2 += v1
    s.v1 = q.r17b ^ g;
    s.v2 = swap32(g);
    s.v0 = e ^ seed;                                                     // v0 ^= m
    return sip_finish(s, (uint64_t)q.total << 56);
}

// Same, with P % 8 known at compile time (fixed-length keys).
template <uint32_t R>
__device__ __forceinline__ uint64_t prefix_hash_c(const Sip& st, uint64_t tail, uint32_t total,
                                                  uint64_t seed) {
    Sip s = st;
    uint64_t blk, hi;
    if constexpr (R == 0) {
        blk = seed;
        hi = 0;
    } else {
        blk = tail | (seed << (8 * R));
        hi = seed >> (64 - 8 * R);
    }
    sip_compress(s, blk);
    return sip_finish(s, ((uint64_t)total << 56) | hi);
}

// Exact x % m for 0 < m < 2^32 with mu = floor((2^64 - 1) / m) precomputed on the host.
// q = mulhi(x, mu) is floor(x / m) or one less, so one conditional subtract finishes it
// (bit-identical to Rust's `hash % bits.len() as u64`, bf.rs:88).
__device__ __forceinline__ uint32_t fast_mod(uint64_t x, uint64_t m, uint64_t mu) {
    const uint64_t q = __umul64hi(x, mu);
    uint64_t r = x - q * m;
    r = r >= m ? r - m : r;
    return (uint32_t)r;
}

// Same for m <= 2^31: x - q*m < 2m <= 2^32 fits a word, so only the quotient's low word is
// formed (three 32x32 products and the carries into it) and the remainder is taken mod 2^32;
// ~8 VALU ops instead of ~20.  Checked against x % m on 3.4e8 (x, m) pairs incl. the edges.
__device__ __forceinline__ uint32_t fast_mod31(uint64_t x, uint32_t m, uint64_t mu) {
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    const uint32_t ml = (uint32_t)mu, mh = (uint32_t)(mu >> 32);
    const uint64_t t1 = (uint64_t)xl * mh + __umulhi(xl, ml);
    const uint64_t t2 = (uint64_t)xh * ml + (uint32_t)t1;
    const uint32_t ql = xh * mh + (uint32_t)(t1 >> 32) + (uint32_t)(t2 >> 32);
    const uint32_t r = xl - ql * m;
    return min(r, r - m);
}

// x % (2^32 - 1), the reference's saturated size (bf.rs:230-233: every filter of more than 2^32 - 1
// bits, e.g. config 5): 2^32 = 1 (mod m), so x = hi + lo (mod m).  s = hi + lo < 2^33 - 1, and
// u = (s mod 2^32) + (s >> 32) <= m, where u == m means 0.  Four full-rate instructions instead of
// the Barrett step's seven 32x32 products (checked against x % m on the host: edges + 2M random).
__host__ __device__ __forceinline__ uint32_t mod_sat(uint64_t x) {
    const uint64_t s = (x & 0xFFFFFFFFull) + (x >> 32);
    const uint32_t u = (uint32_t)s + (uint32_t)(s >> 32);
    return u == 0xFFFFFFFFu ? 0u : u;
}

// M31: m <= 2^31 known at launch (a template flag of the calling kernel); SAT: m == 2^32 - 1.
template <bool M31, bool SAT = false>
__device__ __forceinline__ uint32_t mod_m(uint64_t x, uint64_t m, uint64_t mu) {
    static_assert(!(M31 && SAT), "m = 2^32 - 1 is above 2^31");
    if constexpr (SAT)
        return mod_sat(x);
    else if constexpr (M31)
        return fast_mod31(x, (uint32_t)m, mu);
    else
        return fast_mod(x, m, mu);
}

}  // namespace vbf
