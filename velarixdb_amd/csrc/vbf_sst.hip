// SST data.db decoder on gfx950: the step before the build on the
// recovery path.  velarixdb rebuilds a lost filter by reading the SST's data.db entry by entry
// into a SkipMap (DataFileNode::load_entries, src/fs/mod.rs:275-332) and then hashing every key
// (key_range/range.rs:117-128).  Here data.db is decoded straight into the build's key layout
// (packed key bytes + u64[n+1] absolute offsets) plus the per-entry value offset, creation time
// and tombstone arrays.
//
// data.db = blocks of whole entries, entry = u32 key_len | key | u32 value offset | i64 created_at
// ms | u8 tombstone (block/block_manager.rs:168-190).  A block never exceeds 4096 bytes
// (set_entry refuses an entry that would overflow it, :121-125), and index.db records every
// block's start offset (table.rs:331-338, index/indexer.rs:151-170).  That index is what makes
// the decode parallel: one wavefront per block.
//
//   k_sst_walk : stage the block in LDS (all of a lane's 16-byte loads in flight at once), walk
//                its entry chain (a dependent chain of u32 reads out of LDS, wave-uniform, scalar
//                control), write the entry starts (u16, 256 slots per block) and the count.  A
//                malformed block (an entry crossing the block end, a block over 64 KiB, offsets
//                out of order) sets the error word instead.  A block of more than 256 entries
//                (never written by the reference: 4096 / 17 = 240) is walked on to its end and
//                counted; its entry starts are not stored (the emit pass re-walks it).
//   exclusive scan of the counts (hipcub) -> entry base E_b of every block; the block's key
//                bytes start at G_b = start_b - 17 * E_b (all bytes before it are entries).
//   k_sst_emit : stage the block again, no walk: lanes write the entry arrays (one lane per
//                entry) and the packed key bytes (one lane per aligned output dword, source
//                entry found by a binary search over the entry starts in LDS).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <hipcub/device/device_reduce.hpp>
#include <hipcub/device/device_scan.hpp>

#include "vbf_kernels.hpp"

namespace vbf {

constexpr int kSstWaves = 4;             // waves per workgroup; one block per wave
constexpr uint32_t kStage = 4096 + 64;   // bytes a wave stages in LDS (writer max block: 4096)
constexpr uint32_t kChunks = (kStage + 16 + 1023) / 1024;  // 16-byte loads per lane to stage
constexpr uint32_t kMaxEnt = 256;        // entries per block (writer max: 4096 / 17 = 240)
constexpr uint32_t kMaxBlock = 65535;    // larger blocks (never written by the reference) fail
constexpr uint32_t kEntryFixed = 17;     // key_len + value offset + created_at + tombstone

enum : uint32_t { kSstErrCross = 1, kSstErrDense = 2, kSstErrBig = 4, kSstErrOrder = 8 };

// A block's bytes: staged in LDS (16-byte aligned image, block byte x at img byte sh + x) or,
// for a block larger than kStage, read in place from global memory.
struct BlockView {
    const uint32_t* lds;
    const uint8_t* glb;
    uint32_t sh;
    __device__ __forceinline__ uint32_t u32(uint32_t x) const {
        if (lds) {
            const uint32_t o = sh + x, w0 = lds[o >> 2], w1 = lds[(o >> 2) + 1];
            return __builtin_amdgcn_alignbyte(w1, w0, o & 3);
        }
        return (uint32_t)glb[x] | ((uint32_t)glb[x + 1] << 8) | ((uint32_t)glb[x + 2] << 16) |
               ((uint32_t)glb[x + 3] << 24);
    }
    __device__ __forceinline__ uint32_t u8(uint32_t x) const {
        if (lds) {
            const uint32_t o = sh + x;
            return (lds[o >> 2] >> ((o & 3) * 8)) & 0xFFu;
        }
        return glb[x];
    }
};

__device__ __forceinline__ void sst_error(const SstArgs& a, uint64_t b, uint32_t bits) {
    atomicOr(a.err, bits);
    atomicMin(a.err + 1, (uint32_t)std::min<uint64_t>(b, 0xFFFFFFFFu));
}

// Block b's byte range; false (error recorded) when the offsets are out of order.
__device__ __forceinline__ bool block_range(const SstArgs& a, uint64_t b, uint64_t& s, uint32_t& blen, uint32_t lane) {
    s = a.blocks[b];
    const uint64_t e = b + 1 < a.nblocks ? a.blocks[b + 1] : a.len;
    if (e <= s || e > a.len || (b == 0 && s != 0)) {
        if (lane == 0) sst_error(a, b, kSstErrOrder);
        return false;
    }
    if (e - s > kMaxBlock) {
        if (lane == 0) sst_error(a, b, kSstErrBig);
        return false;
    }
    blen = (uint32_t)(e - s);
    return true;
}

// Stage [s & ~15, s + blen) into LDS with every 16-byte load of the lane in flight at once.
__device__ __forceinline__ BlockView stage_block(const SstArgs& a, uint64_t s, uint32_t blen, uint32_t* buf,
                                                 uint32_t lane) {
    if (blen > kStage) return BlockView{nullptr, a.data + s, 0};
    const uint64_t a0 = s & ~15ull;
    const uint32_t sh = (uint32_t)(s - a0);
    const uint32_t nc = (sh + blen + 15) / 16;
    uint4 v[kChunks];
#pragma unroll
    for (uint32_t c = 0; c < kChunks; ++c) {  // all full chunks in flight together
        const uint32_t q = lane + 64 * c;
        const uint64_t g = a0 + 16ull * q;
        v[c] = make_uint4(0, 0, 0, 0);
        if (q < nc && g + 16 <= a.len) v[c] = *reinterpret_cast<const uint4*>(a.data + g);
    }
#pragma unroll
    for (uint32_t c = 0; c < kChunks; ++c) {
        const uint32_t q = lane + 64 * c;
        const uint64_t g = a0 + 16ull * q;
        if (q < nc && g + 16 > a.len) {  // the file's last, partial chunk
            uint32_t w[4] = {0, 0, 0, 0};
            for (uint32_t t = 0; t < 16; ++t)
                if (g + t < a.len) w[t >> 2] |= (uint32_t)a.data[g + t] << (8 * (t & 3));
            v[c] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
#pragma unroll
    for (uint32_t c = 0; c < kChunks; ++c) {
        const uint32_t q = lane + 64 * c;
        if (q < nc) *reinterpret_cast<uint4*>(buf + 4 * q) = v[c];
    }
    if (lane == 0) buf[4 * nc] = 0;  // u32() of the last bytes reads one dword past them
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return BlockView{buf, nullptr, sh};
}

// Pass 1: walk each block's entry chain, record the entry starts (u16, kMaxEnt slots per block)
// and the count.  The chain is wave-uniform: its state lives in scalar registers (readfirstlane),
// so a step is one ds_read2 + a handful of SALU ops; entry starts collect in four VGPR slots
// (entry i -> lane i % 64, slot i / 64) and leave with coalesced stores.
template <bool LDS>
__device__ __forceinline__ uint32_t walk_chain(const BlockView& v, uint32_t blen, uint32_t lane, uint32_t (&pr)[4],
                                               uint32_t& bad, uint32_t& lmin, uint32_t& lmax) {
    // Lean loop: no per-step checks.  An entry whose length runs past the block end pushes p
    // beyond blen (a key over 64 KiB cannot fit a block: p jumps to 2^17); the walk is valid iff
    // it ends exactly at blen.  Entry starts go to lane i of slot k by v_writelane.
    uint32_t p = 0, n = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        for (uint32_t i = 0; i < 64 && p < blen; ++i) {
            uint32_t L;
            if constexpr (LDS) {
                const uint32_t o = v.sh + p, w0 = v.lds[o >> 2], w1 = v.lds[(o >> 2) + 1];
                L = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_alignbyte(w1, w0, o & 3));
            } else {
                L = blen - p >= 4 ? __builtin_amdgcn_readfirstlane(v.u32(p)) : 0x10000u;
            }
            // Lane select through m0: two SGPR operands would break gfx9's one-read constant bus.
            // Nothing in this file depends on m0 across the statement (no LDS-DMA, no sendmsg),
            // so the reserved-register clobber LLVM warns about is safe here.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
            asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(pr[k]) : "s"(p), "s"(i) : "m0");
#pragma clang diagnostic pop
            p = L > 0xFFFFu ? 0x20000u : p + L + kEntryFixed;
            lmin = std::min(lmin, L);
            lmax = std::max(lmax, L);
            ++n;
        }
    }
    bad = p != blen ? (p < blen ? kSstErrDense : kSstErrCross) : 0;
    if (bad == kSstErrDense) {  // more than 256 entries: count the rest (starts not recorded)
        for (;;) {
            const uint32_t L = blen - p >= 4 ? __builtin_amdgcn_readfirstlane(v.u32(p)) : 0x10000u;
            p = L > 0xFFFFu ? 0x20000u : p + L + kEntryFixed;
            lmin = std::min(lmin, L);
            lmax = std::max(lmax, L);
            ++n;
            if (p >= blen) break;
        }
        bad = p != blen ? kSstErrCross : 0;
    }
    (void)lane;
    return n;
}

// The same walk with the chain in VECTOR registers (VBF_SST_WALK=1, default).  The scalar walk
// spends ~20 SALU instructions per entry (readfirstlane'd state, m0, loop control), and a CU has
// one scalar unit for all its waves, so the walk was SALU-bound.  Here the (uniform) state stays
// in VGPRs: per entry an LDS read pair, v_alignbyte, a clamp-add and a masked select, and the
// start lands in lane i of slot k by a compare/select.  Four entries per loop check; steps past
// the block end leave p unchanged and record starts >= blen, which the count ignores.  Key length
// range is reduced afterwards from the recorded starts, lane-parallel.  Same outputs and errors.
template <bool LDS>
__device__ __forceinline__ uint32_t walk_chain_v(const BlockView& v, uint32_t blen, uint32_t lane,
                                                 uint32_t (&pr)[4], uint32_t& bad, uint32_t& lmin,
                                                 uint32_t& lmax) {
    // p starts in a VGPR the compiler must treat as divergent (an asm result), or its uniformity
    // analysis would readfirstlane the LDS reads and put the chain back on the scalar unit.
    uint32_t p;
    asm volatile("v_mov_b32 %0, 0" : "=v"(p));
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        pr[k] = 0xFFFFFFFFu;
        if (p >= blen) continue;
        for (uint32_t i = 0; i < 64; i += 4) {
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const bool has4 = p + 4 <= blen;  // a length field lies wholly inside the block
                const uint32_t raw = v.u32(has4 ? p : 0u);  // always a safe read: no branch
                const uint32_t L = has4 ? raw : 0x10000u;
                pr[k] = lane == i + u ? p : pr[k];
                const uint32_t pn = p + std::min(L, 0x10000u) + kEntryFixed;
                p = p < blen ? pn : p;
            }
            if (p >= blen) break;
        }
    }
    // more than 256 entries: walk on to the block end, counting (starts not recorded) and
    // reducing the key-length range on the way
    uint32_t extra = 0, emin = 0xFFFFFFFFu, emax = 0;
    while (p < blen) {
        const bool has4 = p + 4 <= blen;
        const uint32_t raw = v.u32(has4 ? p : 0u);
        const uint32_t L = has4 ? raw : 0x10000u;
        emin = std::min(emin, L);
        emax = std::max(emax, L);
        p += std::min(L, 0x10000u) + kEntryFixed;
        ++extra;
    }
    bad = p != blen ? kSstErrCross : 0;
    uint32_t n = extra;
    lmin = emin;
    lmax = emax;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const bool live = pr[k] < blen;
        n += (uint32_t)__popcll(__ballot(live));
        if (live && pr[k] + 4 <= blen) {  // a malformed tail start is reported, never read past blen
            const uint32_t L = v.u32(pr[k]);
            lmin = std::min(lmin, L);
            lmax = std::max(lmax, L);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lmin = std::min(lmin, (uint32_t)__shfl_xor((int)lmin, o));
        lmax = std::max(lmax, (uint32_t)__shfl_xor((int)lmax, o));
    }
    return n;
}

// Fixed-size entries (every key of the block as long as the first one -- the common case for
// SSTables of fixed-width keys): entry i then starts at i * (L0 + 17).  The guess is checked
// lane-parallel -- the block length is a whole number of such entries and every predicted
// start holds L0 -- and when it holds, the chain walk from 0 would visit exactly these starts
// and end at blen, so the result is identical without the 100+-step dependent chain.  Any
// mismatch (mixed lengths, malformed blocks) falls back to the walk, which reports errors.
template <class View>
__device__ __forceinline__ bool uniform_block(const View& v, uint32_t blen, uint32_t lane, uint32_t (&pr)[4],
                                              uint32_t& n, uint32_t& lmin, uint32_t& lmax) {
    if (blen < 4) return false;
    const uint32_t L0 = v.u32(0);
    if (L0 > 0xFFFFu) return false;
    const uint32_t E = L0 + kEntryFixed;
    if (blen % E != 0) return false;
    const uint32_t cnt = blen / E;
    bool ok = true;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t i = lane + 64 * k;
        pr[k] = i < cnt ? i * E : 0xFFFFFFFFu;
        if (i < cnt) ok &= v.u32(i * E) == L0;
    }
    for (uint32_t i = lane + 64 * 4; i < cnt; i += 64) ok &= v.u32(i * E) == L0;  // dense blocks
    if (__ballot(!ok)) return false;
    n = cnt;
    lmin = lmax = L0;
    return true;
}

__global__ __launch_bounds__(64 * kSstWaves) void k_sst_walk(SstArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[kSstWaves][kStage / 4 + 8];
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t b = (uint64_t)blockIdx.x * kSstWaves + wave;
    if (b >= a.nblocks) return;  // no workgroup barriers: waves are independent
    uint64_t s;
    uint32_t blen;
    if (!block_range(a, b, s, blen, lane)) return;
    BlockView v;
    if (a.ablate == 12 || a.ablate == 13) v = BlockView{stage[wave], nullptr, 0};  // timing: no staging
    else v = stage_block(a, s, blen, stage[wave], lane);
    uint32_t pr[4] = {0, 0, 0, 0}, bad = 0, lmin = 0xFFFFFFFFu, lmax = 0;
    uint32_t n = 0;
    if (a.ablate == 11) {  // timing experiment: staging only, no walk
        n = (stage[wave][lane] == 0x12345678u) ? 1 : 0;
    } else if (a.ablate == 13 || a.ablate == 14) {  // dependent LDS chain of 124 steps
        uint32_t o = 0;
        for (uint32_t i = 0; i < 124; ++i) {
            const uint32_t w = stage[wave][(o >> 2) & 1023];
            o = __builtin_amdgcn_readfirstlane(o + 33 + (w & 0x80000000u ? 1 : 0));
        }
        pr[0] = o;
        n = 124;
    } else if (a.ablate == 12) {  // walk a synthetic chain of 124 entries
        for (uint32_t i = 0; i < 124; ++i) {
            const uint32_t o = i * 33 + (stage[wave][i & 15] & 1);
            pr[i & 3] += __builtin_amdgcn_readfirstlane(o);
        }
        n = 124;
    } else {
        static_assert(kMaxEnt == 256, "four 64-lane slots of entry starts");
        if (a.walk_v && uniform_block(v, blen, lane, pr, n, lmin, lmax)) {
            // every entry has the first entry's key length: starts known without the chain
        } else if (a.walk_v)
            n = v.lds ? walk_chain_v<true>(v, blen, lane, pr, bad, lmin, lmax)
                      : walk_chain_v<false>(v, blen, lane, pr, bad, lmin, lmax);
        else
            n = v.lds ? walk_chain<true>(v, blen, lane, pr, bad, lmin, lmax)
                      : walk_chain<false>(v, blen, lane, pr, bad, lmin, lmax);
    }
    if (bad) {
        if (lane == 0) sst_error(a, b, bad);
        return;
    }
    // Blocks whose keys all have one length need no starts: entry i is at i * (L + 17), which
    // is how the emit pass finds them (lmin == lmax), so the 512-byte start list is not written.
    uint16_t* out = a.pos + b * kMaxEnt;
    if (lmin != lmax && n <= kMaxEnt) {
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            if (lane + 64 * k < n) out[lane + 64 * k] = (uint16_t)pr[k];
    }
    if (lane == 0) {
        a.counts[b] = n;
        a.lmin[b] = lmin;  // key-length range (reduced after the pass): uniform lengths let the
        a.lmax[b] = lmax;  // build use the fixed-stride key path
    }
}

// Pass 2: no walk -- stage the block again, read its entry starts, write the outputs.
__global__ __launch_bounds__(64 * kSstWaves) void k_sst_emit(SstArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[kSstWaves][kStage / 4 + 8];
    __shared__ uint16_t pos[kSstWaves][kMaxEnt];
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t b = (uint64_t)blockIdx.x * kSstWaves + wave;
    if (b >= a.nblocks) return;
    const uint64_t s = a.blocks[b];
    const uint32_t blen = (uint32_t)((b + 1 < a.nblocks ? a.blocks[b + 1] : a.len) - s);  // validated by pass 1
    const uint32_t n = a.counts[b];
    const uint32_t L0 = a.lmin[b];
    const bool uni = a.lmax[b] == L0;  // one key length: entry i starts at i * (L0 + 17)
    uint16_t* ps = pos[wave];
    if (!uni) {
        const uint16_t* pin = a.pos + b * kMaxEnt;
        for (uint32_t i = lane; i < n && i < kMaxEnt; i += 64) ps[i] = pin[i];
    }
    const BlockView v = stage_block(a, s, blen, stage[wave], lane);  // its barrier covers ps too
    auto start = [&](uint32_t i) { return uni ? i * (L0 + kEntryFixed) : (uint32_t)ps[i]; };
    const uint64_t E = a.ebase[b];
    const uint64_t G = s - (uint64_t)kEntryFixed * E;  // key bytes before this block
    const uint64_t K = blen - (uint64_t)kEntryFixed * n;  // this block's key bytes
    if (!uni && n > kMaxEnt) {
        // a block of more than 256 entries of mixed key lengths (hand-written files only): its
        // starts were not stored, so re-walk the chain 64 entries at a time, lane u taking entry
        // base + u, and copy the key bytes per entry
        uint32_t p = 0;
        for (uint32_t base = 0; base < n; base += 64) {
            uint32_t mine = 0;
            for (uint32_t u = 0; u < 64 && base + u < n; ++u) {
                mine = lane == u ? p : mine;
                p += v.u32(p) + kEntryFixed;
            }
            const uint32_t i = base + lane;
            if (i >= n) continue;
            const uint32_t q = mine, L = v.u32(q);
            const uint64_t dst = G + q - (uint64_t)kEntryFixed * i;
            if (a.offsets) a.offsets[E + i] = dst;
            if (a.val_off) a.val_off[E + i] = v.u32(q + 4 + L);
            if (a.created) a.created[E + i] = (uint64_t)v.u32(q + 8 + L) | ((uint64_t)v.u32(q + 12 + L) << 32);
            if (a.tomb) a.tomb[E + i] = v.u8(q + 16 + L) == 1;
            if (a.keys)
                for (uint32_t t = 0; t < L; ++t) a.keys[dst + t] = (uint8_t)v.u8(q + 4 + t);
        }
        if (a.offsets && b + 1 == a.nblocks && lane == 0) a.offsets[E + n] = G + K;
        return;
    }
    for (uint32_t i = lane; i < n; i += 64) {
        const uint32_t q = start(i);
        const uint32_t L = v.u32(q);
        if (a.offsets) a.offsets[E + i] = G + q - kEntryFixed * i;
        if (a.val_off) a.val_off[E + i] = v.u32(q + 4 + L);
        if (a.created) a.created[E + i] = (uint64_t)v.u32(q + 8 + L) | ((uint64_t)v.u32(q + 12 + L) << 32);
        if (a.tomb) a.tomb[E + i] = v.u8(q + 16 + L) == 1;
    }
    if (a.offsets && b + 1 == a.nblocks && lane == 0) a.offsets[E + n] = G + K;
    if (!a.keys || K == 0) return;
    // Fixed-size entries whose key length is a multiple of 4 (the walk's fast-path layout, with
    // G then dword aligned): output dword x is word x % (L0/4) of key x / (L0/4) -- no search.
    if (uni && (L0 & 3) == 0 && (G & 3) == 0) {
        const uint32_t wpk = L0 >> 2, nw = (uint32_t)(K >> 2);
        uint32_t* kout = reinterpret_cast<uint32_t*>(a.keys + G);
        for (uint32_t x = lane; x < nw; x += 64) {
            const uint32_t i = x / wpk;
            kout[x] = v.u32(4 * x + 4 + kEntryFixed * i);
        }
        return;
    }
    // packed key bytes [G, G + K), one lane per aligned output dword: output byte d lies in the
    // last entry i with cum(i) = pos(i) - 17 i <= d, at block byte d + 4 + 17 i
    auto cum = [&](uint32_t i) { return start(i) - kEntryFixed * i; };
    const uint64_t w_lo = G >> 2, w_hi = (G + K + 3) >> 2;
    uint32_t hint = 0;  // lanes move forward through the block: start the search at the last hit
    for (uint64_t w = w_lo + lane; w < w_hi; w += 64) {
        const uint64_t g0 = w << 2;
        const uint32_t d0 = g0 < G ? 0 : (uint32_t)(g0 - G);
        uint32_t lo = hint, hi = n - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (cum(mid) <= d0) lo = mid;
            else hi = mid - 1;
        }
        uint32_t i = lo;
        hint = lo;
        const bool full = g0 >= G && g0 + 4 <= G + K;
        const uint32_t next = i + 1 < n ? cum(i + 1) : (uint32_t)K;
        if (full && d0 + 4 <= next) {
            reinterpret_cast<uint32_t*>(a.keys)[w] = v.u32(d0 + 4 + kEntryFixed * i);
            continue;
        }
        uint32_t val = 0;
        for (uint32_t t = 0; t < 4; ++t) {
            const uint64_t g = g0 + t;
            if (g < G || g >= G + K) continue;
            const uint32_t d = (uint32_t)(g - G);
            while (i + 1 < n && cum(i + 1) <= d) ++i;
            const uint32_t byte = v.u8(d + 4 + kEntryFixed * i);
            if (full) val |= byte << (8 * t);
            else a.keys[g] = (uint8_t)byte;
        }
        if (full) reinterpret_cast<uint32_t*>(a.keys)[w] = val;
    }
}

hipError_t sst_count(const SstArgs& a, hipStream_t s) {
    if (a.nblocks == 0) return hipSuccess;
    const uint64_t grid = (a.nblocks + kSstWaves - 1) / kSstWaves;
    hipLaunchKernelGGL(k_sst_walk, dim3((uint32_t)grid), dim3(64 * kSstWaves), 0, s, a);
    return hipGetLastError();
}

hipError_t sst_emit(const SstArgs& a, hipStream_t s) {
    if (a.nblocks == 0) return hipSuccess;
    const uint64_t grid = (a.nblocks + kSstWaves - 1) / kSstWaves;
    hipLaunchKernelGGL(k_sst_emit, dim3((uint32_t)grid), dim3(64 * kSstWaves), 0, s, a);
    return hipGetLastError();
}

uint64_t sst_pos_bytes(uint64_t nblocks) { return nblocks * kMaxEnt * 2; }

hipError_t sst_len_range(const uint32_t* lmin, const uint32_t* lmax, uint64_t nblocks, uint32_t* out2, void* tmp,
                         size_t* tmp_bytes, hipStream_t s) {
    size_t need = 0, b1 = 0;
    hipError_t e = hipcub::DeviceReduce::Min(nullptr, need, lmin, out2, (int)nblocks, s);
    if (e != hipSuccess) return e;
    e = hipcub::DeviceReduce::Max(nullptr, b1, lmax, out2 + 1, (int)nblocks, s);
    if (e != hipSuccess) return e;
    need = std::max(need, b1);
    if (!tmp) {
        *tmp_bytes = need;
        return hipSuccess;
    }
    e = hipcub::DeviceReduce::Min(tmp, need, lmin, out2, (int)nblocks, s);
    if (e != hipSuccess) return e;
    return hipcub::DeviceReduce::Max(tmp, need, lmax, out2 + 1, (int)nblocks, s);
}

hipError_t sst_scan(const uint32_t* counts, uint64_t* ebase, uint64_t nblocks, void* tmp, size_t* tmp_bytes,
                    hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveScan(tmp, *tmp_bytes, counts, ebase, hipcub::Sum(), (uint64_t)0,
                                             (int)nblocks, s);
}

// Synthetic data.db of fixed-length keys (bench / tests): entry j = the config generator's key j
// (vbf_gen_fixed_dev), value offset (u32)j, created_at 1720785462000 + j, tombstone j % 97 == 0,
// blocked exactly as Table::write_to_file does (equal entries -> floor(4096 / (L+17)) per block).
__device__ __forceinline__ uint64_t sm64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_gen_sst_fixed(uint64_t seed, uint64_t base, uint64_t n, uint32_t len,
                                                       uint32_t per_block, uint8_t* data, uint32_t* blocks) {
    const uint64_t jj = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (jj >= n) return;
    const uint64_t j = base + jj, es = len + kEntryFixed;
    uint8_t* o = data + jj * es;
    auto put = [&](uint32_t at, uint64_t v, int nb) {
        for (int i = 0; i < nb; ++i) o[at + i] = (uint8_t)(v >> (8 * i));
    };
    put(0, len, 4);
    for (uint32_t c = 0; c * 8 < len; ++c) {
        const uint64_t w = c == 0 ? sm64(seed ^ j) : c == 1 ? j : sm64(seed ^ j ^ (c * 0x9E3779B97F4A7C15ull));
        for (uint32_t b = 0; b < 8 && c * 8 + b < len; ++b) o[4 + c * 8 + b] = (uint8_t)(w >> (8 * b));
    }
    put(4 + len, (uint32_t)j, 4);
    put(8 + len, 1720785462000ull + j, 8);
    o[16 + len] = (j % 97) == 0;
    if (jj % per_block == 0) blocks[jj / per_block] = (uint32_t)(jj * es);
}

hipError_t gen_sst_fixed(uint64_t seed, uint64_t base, uint64_t n, uint32_t len, uint8_t* data, uint32_t* blocks,
                         hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t per_block = 4096 / (len + kEntryFixed);
    hipLaunchKernelGGL(k_gen_sst_fixed, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, seed, base, n, len,
                       per_block, data, blocks);
    return hipGetLastError();
}

}  // namespace vbf
