// keyhash.hpp -- per-key prefix absorption for every key layout the C ABI accepts.
//
// key_prefix<FMT, LP>(kb, j) returns the SipHash state after the seed-independent blocks of key
// j (`LE64(len) || key` when LP), so that h(key, i) = prefix_hash(p, i) costs 5 SipRounds.
//   FMT  > 0 : fixed length FMT bytes (FMT % 8 == 0), 16-byte (or 8-byte) aligned rows
//   FMT == 0 : runtime stride
//   FMT == -1: offsets[n+1], absolute positions into keys
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sip13.hpp"

namespace vbf {

struct DevKeys {
    const uint8_t* keys;
    const uint64_t* offsets;
    uint64_t off_base;
    uint64_t stride;
    uint64_t n;
};

// Aligned 8-byte load of word i of a key whose words start at wstart, or 0 when that word
// starts at or past `end` (a word holding no key byte is never read: no page can fault).
__device__ __forceinline__ uint64_t ld_word(const uint64_t* wbase, uintptr_t wstart, uintptr_t end,
                                            uint64_t i) {
    return (wstart + 8 * i < end) ? wbase[i] : 0ull;
}

// The 8 bytes starting `sh` bits into lo:hi (sh in {0, 8, ..., 56}); shift counts stay < 64.
__device__ __forceinline__ uint64_t funnel(uint64_t lo, uint64_t hi, uint32_t sh) {
    return (lo >> sh) | ((hi << 1) << (63 - sh));
}

// Fixed-length rows (FMT > 0): the row's words, loaded apart from the absorb so a caller can
// issue several rows' loads before hashing any of them.
template <int FMT>
struct FixedWords {
    static_assert(FMT > 0 && FMT % 8 == 0, "fixed fast path needs whole 8-byte words");
    uint64_t w[FMT / 8];
};

template <int FMT>
__device__ __forceinline__ FixedWords<FMT> load_fixed(const DevKeys& a, uint64_t j) {
    constexpr uint32_t NW = FMT / 8;
    FixedWords<FMT> kw;
    const uint8_t* kp = a.keys + j * FMT;
    if constexpr (NW % 2 == 0) {
#pragma unroll
        for (uint32_t c = 0; c < NW; c += 2) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(kp + 8 * c);
            kw.w[c] = v.x;
            kw.w[c + 1] = v.y;
        }
    } else {
#pragma unroll
        for (uint32_t c = 0; c < NW; ++c) kw.w[c] = *reinterpret_cast<const uint64_t*>(kp + 8 * c);
    }
    return kw;
}

template <int FMT, bool LP>
__device__ __forceinline__ Prefix absorb_fixed(const FixedWords<FMT>& kw) {
    Prefix p;
    Sip st = sip_init();
    if constexpr (LP) sip_compress(st, (uint64_t)FMT);
#pragma unroll
    for (uint32_t c = 0; c < FMT / 8; ++c) sip_compress(st, kw.w[c]);
    p.st = st;
    p.tail = 0;
    p.r = 0;
    p.total = (FMT + (LP ? 8 : 0) + 8) & 0xff;
    return p;
}

// A runtime-length key's first five source words (the absorb's first four blocks and the
// shifted-in fifth), loaded apart from the absorb so a caller can issue the next key's loads
// before hashing this one (k_tile_pack's offsets layout: one round of keys ahead).
struct KeyHead {
    const uint64_t* wbase;
    uintptr_t wstart, end;
    uint64_t len;
    uint32_t sh;
    uint64_t w[5];
};

__device__ __forceinline__ KeyHead key_head_load(const uint8_t* keys, uint64_t beg, uint64_t len) {
    KeyHead h;
    const uintptr_t addr = reinterpret_cast<uintptr_t>(keys + beg);
    h.end = addr + len;
    h.wstart = addr & ~(uintptr_t)7;
    h.wbase = reinterpret_cast<const uint64_t*>(h.wstart);
    h.sh = (uint32_t)(addr & 7) * 8;
    h.len = len;
    h.w[0] = len ? ld_word(h.wbase, h.wstart, h.end, 0) : 0ull;
#pragma unroll
    for (int i = 1; i < 5; ++i) h.w[i] = ld_word(h.wbase, h.wstart, h.end, i);
    return h;
}

// The runtime-length absorb from a loaded head.
template <bool LP>
__device__ __forceinline__ Prefix key_prefix_head(const KeyHead& h) {
    Prefix p;
    const uint64_t len = h.len;
    const uint32_t sh = h.sh;
    Sip st = sip_init();
    if constexpr (LP) sip_compress(st, len);
    const uint64_t nfull = len >> 3;
    // Source words c+1..c+4 sit in a[] while words c+5..c+8 are already in flight in b[]:
    // the absorb never waits on a load it just issued (a word past the key reads as 0).
    uint64_t lo = h.w[0];
    uint64_t a[4] = {h.w[1], h.w[2], h.w[3], h.w[4]};
    uint64_t c = 0;
    for (; c + 4 <= nfull; c += 4) {
        uint64_t b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) b[i] = ld_word(h.wbase, h.wstart, h.end, c + 5 + i);
        sip_compress(st, funnel(lo, a[0], sh));
        sip_compress(st, funnel(a[0], a[1], sh));
        sip_compress(st, funnel(a[1], a[2], sh));
        sip_compress(st, funnel(a[2], a[3], sh));
        lo = a[3];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = b[i];
    }
    // 0..3 full blocks left: words c+1.. are a[0..]; the tail's upper word is a[nfull - c]
    const uint32_t left = (uint32_t)(nfull - c);
    uint64_t up = a[0];
    if (left > 0) { sip_compress(st, funnel(lo, a[0], sh)); lo = a[0]; up = a[1]; }
    if (left > 1) { sip_compress(st, funnel(lo, a[1], sh)); lo = a[1]; up = a[2]; }
    if (left > 2) { sip_compress(st, funnel(lo, a[2], sh)); lo = a[2]; up = a[3]; }
    p.st = st;
    p.r = (uint32_t)(len & 7);  // P % 8 == len % 8 (the length block is 8 bytes)
    const uint64_t tmask = p.r ? (~0ull >> (64 - 8 * p.r)) : 0ull;
    p.tail = p.r ? (funnel(lo, up, sh) & tmask) : 0ull;
    p.total = (uint32_t)((len + (LP ? 8 : 0) + 8) & 0xff);
    return p;
}

// Any key given as (byte position in `keys`, length): the runtime-length absorb.
template <bool LP>
__device__ __forceinline__ Prefix key_prefix_at(const uint8_t* keys, uint64_t beg, uint64_t len) {
    return key_prefix_head<LP>(key_head_load(keys, beg, len));
}

template <int FMT, bool LP>
__device__ __forceinline__ Prefix key_prefix(const DevKeys& a, uint64_t j) {
    if constexpr (FMT > 0) {
        return absorb_fixed<FMT, LP>(load_fixed<FMT>(a, j));
    } else if constexpr (FMT < 0) {
        return key_prefix_at<LP>(a.keys, a.offsets[j] - a.off_base, a.offsets[j + 1] - a.offsets[j]);
    } else {
        return key_prefix_at<LP>(a.keys, j * a.stride, a.stride);
    }
}

// Rust `Ord for [u8]`: lexicographic, a proper prefix is smaller.  -1 / 0 / 1.
__device__ __forceinline__ int cmp_bytes(const uint8_t* a, uint64_t la, const uint8_t* b, uint64_t lb) {
    const uint64_t n = la < lb ? la : lb;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t x = a[i], y = b[i];
        if (x != y) return x < y ? -1 : 1;
    }
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// Host-side choice of FMT for a batch: the compile-time fixed layouts need aligned rows.
enum KeyFmt { kFmtOffsets = -1, kFmtStride = 0 };

inline int pick_fmt(const uint8_t* keys, const uint64_t* offsets, uint64_t stride) {
    if (offsets) return kFmtOffsets;
    const uintptr_t k = reinterpret_cast<uintptr_t>(keys);
    if ((stride == 16 || stride == 32) && (k & 15) == 0) return (int)stride;
    if ((stride == 8 || stride == 24) && (k & 7) == 0) return (int)stride;
    return kFmtStride;
}

// Calls f.template operator()<FMT, LP>() for the batch's layout.
template <class F>
inline void with_fmt(int fmt, bool lp, F&& f) {
#define VBF_FMT_CASE(V)                        \
    case V:                                    \
        if (lp)                                \
            f.template operator()<V, true>();  \
        else                                   \
            f.template operator()<V, false>(); \
        break;
    switch (fmt) {
        VBF_FMT_CASE(16)
        VBF_FMT_CASE(32)
        VBF_FMT_CASE(8)
        VBF_FMT_CASE(24)
        VBF_FMT_CASE(-1)
        default:
            if (lp)
                f.template operator()<0, true>();
            else
                f.template operator()<0, false>();
    }
#undef VBF_FMT_CASE
}

}  // namespace vbf
