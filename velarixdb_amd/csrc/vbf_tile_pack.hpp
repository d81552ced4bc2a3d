// vbf_tile_pack.hpp -- K1 of the partitioned Bloom build (k_tile_pack) and the plan it runs on,
// shared by vbf_partition.hip (the compiled-k kernels and the launch) and vbf_partition_rk.hip
// (the runtime-k classes, compiled in a translation unit of their own so the library builds in
// parallel).  Every kernel instantiation lives in exactly one translation unit.
#pragma once
#include "vbf_partition.hpp"

namespace vbf {

struct PartPlan {
    uint32_t k;
    uint32_t R;           // hashing rounds per lane (ceil(KT / 1024))
    uint32_t KT;          // keys per tile
    uint32_t C;           // indices per tile (KT * k)
    uint32_t CP;          // capacity: C rounded up to a multiple of 8 (whole groups)
    uint32_t nseg, nseg_pad, G;
    uint32_t tile_words;  // u32 words per tile in the workspace: 5 per group, rounded up to 4
    uint32_t lds1;        // K1 dynamic LDS bytes
    uint32_t stagger_lo, stagger_hi, stagger_sleeps;
    uint32_t ablate;      // ablation builds only (VBF_ABLATE, vbf_kernels.hpp): 1 skip place+copy
    uint32_t k3v;         // k_seg_or tile-loop variant (VBF_K3, see k_seg_or); 0 = by run length
    uint32_t len_order;   // offsets layout: deal keys to lanes by length (VBF_LEN_ORDER, default 1)
    uint32_t stage_keys;  // the lo16 image holds perm + (begin, length) per key (VBF_STAGE_KEYS)
    uint32_t fresh;       // K3: the words hold no filter yet -- write the segment without reading it
    uint32_t nsegS;       // row stride of ends[tile][seg] (nseg rounded up to 8: 16-byte rows)
    uint32_t ntS;         // row stride of endsT[seg][tile] (tiles rounded up to 8)
    uint32_t c16;         // K1's segment counters are u16 pairs (half the LDS: larger tiles)
    uint32_t cnt_words;   // K1's counter words (a multiple of 4: the image stays 16-byte aligned)
    uint32_t k1v;         // K1's workgroup shape (k1_shape; VBF_K1)
    uint32_t ends_t;      // K1 writes the run ends transposed, endsT[seg][tile] (VBF_ENDS_T)
    uint32_t kc;          // K1 runtime-k class: k <= kc seeds per key in a kc-slot stash (0: none)
    uint32_t lp;          // the batch hashes the length prefix (selects the class kernels' LP)
    uint32_t gd_words;    // group pack: LDS words of its per-segment u16 table (0 for the build)
    uint32_t CPg;         // group pack: entries per tile in HBM, every run padded to whole groups
    uint32_t nfull;       // K3: segments [0, nfull) one workgroup each; the rest split in P parts
    uint32_t P;
    uint64_t m, mu, nwords;
    uint64_t perm_off;    // POS = 2 with the length order: u16 elements from posv to perm[tile][KT]
};

// Variable-length keys (offsets layout): a wave runs the prefix-absorb loop as long as its
// longest key, and with Zipf lengths almost every wave holds one long key.  So the tile's keys
// are dealt to lanes in order of length -- a counting sort on min(len / 8, 31) into perm[] in
// LDS -- and a wave's lanes absorb similar numbers of blocks.  The build is an OR over keys, so
// the order changes speed only.  hist[kLenBuckets] must be zero on entry; ends with a barrier.
constexpr int kLenBuckets = 32;

// With sbeg/slen (not null) the second pass also stages each key's (begin - base, length) at its
// sorted slot, so the hashing rounds read them from LDS instead of a dependent offsets load.
template <int BS = kPBlock>
__device__ __forceinline__ void length_order(const DevKeys& dk, uint64_t key0, uint32_t nk, uint16_t* perm,
                                             uint32_t* hist, uint32_t* sbeg = nullptr, uint32_t* slen = nullptr,
                                             uint64_t base = 0) {
    const uint32_t tid = threadIdx.x;
    auto bucket = [&](uint32_t l) {
        const uint64_t len = dk.offsets[key0 + l + 1] - dk.offsets[key0 + l];
        return (uint32_t)std::min<uint64_t>(len >> 3, kLenBuckets - 1);
    };
    for (uint32_t l = tid; l < nk; l += BS) atomicAdd(&hist[bucket(l)], 1u);
    __syncthreads();
    if (tid < 64) {
        const uint32_t v = tid < kLenBuckets ? hist[tid] : 0u;
        uint32_t incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (tid >= (uint32_t)o) incl += y;
        }
        if (tid < kLenBuckets) hist[tid] = incl - v;
    }
    __syncthreads();
    for (uint32_t l = tid; l < nk; l += BS) {
        const uint64_t b = dk.offsets[key0 + l], len = dk.offsets[key0 + l + 1] - b;
        const uint32_t pos = atomicAdd(&hist[(uint32_t)std::min<uint64_t>(len >> 3, kLenBuckets - 1)], 1u);
        perm[pos] = (uint16_t)l;
        if (sbeg) {
            sbeg[pos] = (uint32_t)(b - base);
            slen[pos] = (uint32_t)len;
        }
    }
    __syncthreads();
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;

// The tile image is read back only by k_seg_or after this launch (2.5 GB at config 2: far beyond
// the L2 and the Infinity Cache), so its copy-out is a streaming store (VBF_IMAGE_NT, default on):
// it does not evict from the L2 the key bytes and offsets the other workgroups of the XCD are still
// reading (config 3's keys are read in length order, every line several times).
#ifndef VBF_IMAGE_NT
#define VBF_IMAGE_NT 1
#endif
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void image_store(uint32_t* dst, u32x4 v) {
    if constexpr (VBF_IMAGE_NT)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
    else
        *reinterpret_cast<u32x4*>(dst) = v;
}
__device__ __forceinline__ void lds_add(lds_u32* p) {
    (void)__hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_add_rtn(lds_u32* p) {
    return __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_add(lds_u32* p, uint32_t v) {
    (void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_add_rtn(lds_u32* p, uint32_t v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Segment counters of K1.  C16 = false: one u32 per segment.  C16 = true: two u16 per word
// (segment s in half s & 1 of word s >> 1; no half ever carries into the other: every count and
// start is < CP <= 65535), which halves the counters' LDS -- at k = 10 (954 segments) the tile
// then holds its three full stash rounds (3 072 keys instead of 3 020), at k = 19 (1 812
// segments) likewise (1 536 instead of 1 472).  The half of segment s is bit 20 of the index:
// shift = (idx >> 16) & 16.
// SB: segment = 2^SB positions (the build: 2^20 filter bits; the multi-SST group pack: 2^17 bytes
// of interleaved filters, vbf_multi_part.hip).
template <bool C16, int SB = kSegBits>
__device__ __forceinline__ void seg_count(lds_u32* cnt0, uint32_t idx) {
    if constexpr (C16) lds_add(&cnt0[idx >> (SB + 1)], 1u << ((idx >> (SB - 4)) & 16u));
    else lds_add(&cnt0[idx >> SB]);
}
template <bool C16, int SB = kSegBits>
__device__ __forceinline__ uint32_t seg_rank(lds_u32* cnt0, uint32_t idx) {
    if constexpr (C16) {
        const uint32_t sh = (idx >> (SB - 4)) & 16u;
        return (lds_add_rtn(&cnt0[idx >> (SB + 1)], 1u << sh) >> sh) & 0xFFFFu;
    } else {
        return lds_add_rtn(&cnt0[idx >> SB]);
    }
}
template <bool C16>
__device__ __forceinline__ uint32_t seg_get(const uint32_t* cnt, uint32_t s) {
    if constexpr (C16) return (cnt[s >> 1] >> ((s & 1u) * 16)) & 0xFFFFu;
    else return cnt[s];
}

// The packed tile image: entry e lives in group e >> 3, 20 bytes = 5 words: words 0..3 hold the
// group's eight u16 low halves (entry e at u16 (e >> 3) * 10 + (e & 7)), word 4 its eight 4-bit
// nibbles (entry e at bits 4 * (e & 7)).
constexpr uint32_t kGroupWords = 5;
__host__ __device__ constexpr uint32_t group_words(uint32_t entries) { return (entries + 7) / 8 * kGroupWords; }

// K > 0: k known at compile time (the stash and seed loops unroll, no indexed register moves);
// K == 0, KC > 0: a runtime-k class -- any k <= KC (pl.k) in the compiled kernel's KC-slot stash
// (the seed loop unrolls to KC with a wave-uniform `i < k` guard, the unused slots hold sentinels),
// on the 512-thread shape: k outside {4, 9, 10, 19} (p = 1e-3 gives k = 14, 1e-5 k = 23,
// cfg/config.rs:102-106) keeps its stash in registers;
// K == 0, KC == 0: any k <= kStash at run time, the stash in scratch memory (VBF_KCLASS=0).  V = 0: __launch_bounds__(1024, 8): two workgroups per CU
// (the hashing of one overlaps the other's sort), i.e. at most 64 VGPRs; the offsets-layout
// kernels would otherwise take 80-90 and drop to one workgroup per CU.  V = 1: 512 threads, two
// workgroups per CU at 4 waves per SIMD, 128 VGPRs (k1_shape).
//
// POS = 1 (the multi-SST group pack, vbf_multi_part.hip, SB < kSegBits; and the round-4 probe pack):
// segments of 2^SB positions, every run padded to whole groups in the image, and every entry's
// place in the tile image is also written to posv[tile][stash slot][lane] (u16), so the group output
// pass finds a key's k results without re-reading the image.
// POS = 2 (the round-6 probe pack, vbf_probe_pu.hip): the build's own unpadded image, and beside it
// the places the entries WOULD have with every run padded to whole groups -- those index the
// per-entry result bits the segment pass writes (each run owns whole result bytes, so no two
// workgroups write one byte) -- in posv, and the run ends as u32 pairs (unpadded end | padded
// end << 16) in endsT.  No padding reserve shrinks the tile (POS = 1 reserves 7 entries per segment
// of LDS: at m = 2^32 - 1 that is the whole image).
// SAT: m == 2^32 - 1 (the reference's saturated size), remainders by mod_sat (sip13.hpp).
template <int FMT, bool LP, int K, bool M31, bool C16 = false, int V = 0, int KC = 0, int SB = kSegBits,
          int POS = 0, bool SAT = false>
__global__ __launch_bounds__(V == 1 ? 512 : kPBlock, V == 1 ? 4 : 8) void k_tile_pack(DevKeys dk, PartPlan pl,
                                                                                      uint32_t* tiles, uint16_t* ends,
                                                                                      uint16_t* posv) {
    constexpr int BS = V == 1 ? 512 : kPBlock;  // k1_shape(K, FMT > 0, V).bs
    static_assert(V == 0 || K > 0 || KC > 0, "the 512-thread shape is for compiled k and k classes");
    static_assert(KC == 0 || (K == 0 && V == 1 && !C16), "k classes run on the 512-thread shape");
    static_assert(POS != 2 || (K > 0 || KC > 0), "the probe pack keeps its stash in registers");
    constexpr int KK = K > 0 ? K : KC;  // seed slots per key in the stash (0: the scratch stash)
    extern __shared__ __attribute__((aligned(16))) uint32_t smem_all[];
    // The per-segment counters first, at LDS address 0 (the kernel has no static LDS, so the
    // dynamic allocation starts there; launch_build_partitioned checks it): the count and rank
    // atomics address them through an LDS-space pointer to 0, so a counter's address is the
    // segment number times 4 with no base to add -- one VALU instruction fewer per bit index in
    // each of the two passes.  Then the tile image, 16-byte aligned.
    uint32_t* cnt = smem_all;                           // nseg_pad (C16: nseg_pad / 2) words
    lds_u32* const cnt0 = reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(0));  // == cnt
    const uint32_t cnt_words = pl.cnt_words;
    uint32_t* wsum = cnt + cnt_words;                   // 16
    uint32_t* lhist = wsum + 16;                        // kLenBuckets (offsets layout)
    uint32_t* gd = lhist + kLenBuckets;                 // POS: gd_words (a multiple of 4)
    uint32_t* smem = gd + pl.gd_words;                  // the image: (cnt_words + 48) * 4 % 16 == 0
    uint16_t* lo = reinterpret_cast<uint16_t*>(smem);  // before placement: perm (offsets layout)
    const uint32_t tid = threadIdx.x;
    // Stagger (VBF_STAGGER, speed only, off by default since round 5): the second workgroup
    // dispatched to each CU may start a few s_sleeps later, so the two co-resident workgroups
    // alternate hashing (VALU) and sorting (LDS) from the first tile on.
    if (blockIdx.x >= pl.stagger_lo && blockIdx.x < pl.stagger_hi) {
        for (uint32_t i = 0; i < pl.stagger_sleeps; ++i) __builtin_amdgcn_s_sleep(127);
    }
    for (uint32_t s = tid; s < cnt_words; s += BS) cnt[s] = 0;
    if (FMT < 0 && tid < kLenBuckets) lhist[tid] = 0;
    __syncthreads();

    // SPL lanes per key (k1_shape): lane tid takes key slot r * (BS / SPL) + tid / SPL and
    // seeds [KL * (tid % SPL), KL * (tid % SPL) + KL) of it
    constexpr int SPL = KK > 0 ? k1_shape(KK, FMT > 0, V).spl : 1;
    constexpr int KL = KK > 0 ? k1_shape(KK, FMT > 0, V).kl : 1;
    constexpr uint32_t kKeysPerRound = BS / SPL;
    constexpr int RMK = KK > 0 ? k1_shape(KK, FMT > 0, V).rounds : 1;
    uint32_t stash[KK > 0 ? RMK * KL : kStash];
    // the tile: with ends_t, XCD-aware (blocks are dealt round-robin over the 8 XCDs; each XCD
    // takes a contiguous range of tiles, so the endsT columns its workgroups write at one time are
    // neighbours and fill whole L2 lines); otherwise the block number
    uint32_t tile = blockIdx.x;
    if (pl.ends_t) {
        const uint32_t nwg = gridDim.x, q = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
        tile = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + blockIdx.x / 8;
    }
    const uint64_t key0 = (uint64_t)tile * pl.KT;
    const uint64_t key_end = std::min<uint64_t>(dk.n, key0 + pl.KT);
    const uint32_t nk = (uint32_t)(key_end - key0);
    // perm lives in the (not yet used) tile image; every read of it precedes the barrier below
    const bool perm = FMT < 0 && pl.len_order;
    // Staged keys (offsets layout, compiled k, plan says the image holds perm + 2 words per key,
    // and the tile's bytes span < 4 GiB): (begin, length) at smem[sw0 ..) and smem[sw0 + nk ..).
    const uint32_t sw0 = (nk + 1) / 2;
    bool staged = false;
    uint64_t sbase = 0;
    if constexpr (FMT < 0) {
        if (perm) {
            if (KK > 0 && pl.stage_keys) {
                sbase = dk.offsets[key0];
                staged = dk.offsets[key_end] - sbase < (1ull << 32);
            }
            if (staged)
                length_order<BS>(dk, key0, nk, lo, lhist, smem + sw0, smem + sw0 + nk, sbase);
            else
                length_order<BS>(dk, key0, nk, lo, lhist);
        }
    }
    auto key_of = [&](uint32_t slot) -> uint64_t { return key0 + (perm ? (uint32_t)lo[slot] : slot); };
    uint32_t ns;  // wave-uniform: every lane stores R*k entries (sentinels past the end)
    if constexpr (KK > 0) {
        constexpr int RM = RMK;
        // One instance per round with r a compile-time constant: the stash index r*K+i stays
        // static even where the round body holds a runtime loop (the offsets layout's absorb),
        // which keeps LLVM from unrolling a plain `for` -- the stash then went to scratch
        // memory (128 B per lane of scratch stores and loads per key, variable-length builds).
        // Runtime-length layouts on the 512-thread shape (128 VGPRs): the first five source words
        // of a lane's next-round key are loaded before this round's absorb, so they arrive while
        // this round hashes (config 3: the absorb waited on its first loads).
        constexpr bool PF = FMT <= 0 && V == 1;
        auto key_span = [&](uint32_t slot, uint64_t& beg, uint64_t& len) {
            if constexpr (FMT < 0) {
                if (staged) {
                    beg = sbase - dk.off_base + smem[sw0 + slot];
                    len = smem[sw0 + nk + slot];
                } else {
                    const uint64_t j = key_of(slot);
                    beg = dk.offsets[j] - dk.off_base;
                    len = dk.offsets[j + 1] - dk.offsets[j];
                }
            } else {
                beg = key_of(slot) * dk.stride;
                len = dk.stride;
            }
        };
        auto head_of = [&](uint32_t rr) -> KeyHead {
            const uint32_t slot = rr * kKeysPerRound + tid / SPL;
            uint64_t beg = 0, len = 0;  // no key: a zero-length head reads nothing
            if (rr < pl.R && slot < nk) key_span(slot, beg, len);
            return key_head_load(dk.keys, beg, len);
        };
        KeyHead head_cur{};
        if constexpr (PF) head_cur = head_of(0);
        auto round = [&](auto rc) {
            constexpr int r = decltype(rc)::value;
            const uint32_t slot = (uint32_t)r * kKeysPerRound + tid / SPL;
            const uint32_t seed0 = (uint32_t)KL * (tid % SPL);
            const bool valid = (uint32_t)r < pl.R && slot < nk;
            // ablation builds only (VBF_ABLATE = 8 / 9, timing experiments): no key loads, no SipHash
            const bool nohash = VBF_ABLATION_BUILD && (pl.ablate == 8 || pl.ablate == 9);
            Prefix p{};
            if (nohash) {
            } else if constexpr (PF) {
                const KeyHead h = head_cur;
                if constexpr (r + 1 < RM) head_cur = head_of(r + 1);
                if (valid) p = key_prefix_head<LP>(h);
            } else if (valid) {
                if constexpr (FMT < 0) {
                    uint64_t beg, len;
                    key_span(slot, beg, len);
                    p = key_prefix_at<LP>(dk.keys, beg, len);
                } else {
                    p = key_prefix<FMT, LP>(dk, key_of(slot));
                }
            }
            // compile-time key lengths end the prefix on a block boundary: the seed loop shares
            // half of its first SipRound (seed_hash, sip13.hpp)
            SeedCtx q{};
            if constexpr (FMT > 0) q = seed_ctx(p);
            // one instance per seed slot with i a compile-time constant (a fold, like the rounds):
            // a `#pragma unroll` loop was left rolled for the 32-slot class with runtime-length keys
            // and the Barrett remainder, which put the stash in scratch memory (272 B per lane)
            auto seed = [&](auto ic) {
                constexpr int i = decltype(ic)::value;
                uint32_t idx = kSentinel;
                // class kernels: seeds past the runtime k (wave-uniform) leave sentinels
                if (valid && (SPL == 1 || seed0 + i < (uint32_t)K) && (KC == 0 || (uint32_t)i < pl.k)) {
                    const uint64_t h =
                        nohash ? (key0 + slot) * 0x9E3779B97F4A7C15ull ^ (uint64_t)(seed0 + i + 1) * 0xC2B2AE3D27D4EB4Full
                        : FMT > 0 ? seed_hash(q, seed0 + i) : prefix_hash(p, seed0 + i);
                    idx = mod_m<M31, SAT>(h, pl.m, pl.mu);
                    seg_count<C16, SB>(cnt0, idx);
                }
                stash[r * KL + i] = idx;
            };
            [&]<int... Is>(std::integer_sequence<int, Is...>) {
                (seed(std::integral_constant<int, Is>{}), ...);
            }(std::make_integer_sequence<int, KL>{});
        };
        [&]<int... Rs>(std::integer_sequence<int, Rs...>) {
            (round(std::integral_constant<int, Rs>{}), ...);
        }(std::make_integer_sequence<int, RM>{});
        ns = RM * KL;
    } else {
        ns = 0;
        for (uint32_t r = 0; r < pl.R; ++r) {
            const uint32_t slot = r * BS + tid;
            const bool valid = slot < nk;
            Prefix p{};
            if (valid) p = key_prefix<FMT, LP>(dk, key_of(slot));
            for (uint32_t i = 0; i < pl.k; ++i) {
                uint32_t idx = kSentinel;
                if (valid) {
                    idx = mod_m<M31, SAT>(prefix_hash(p, i), pl.m, pl.mu);
                    seg_count<C16, SB>(cnt0, idx);
                }
                stash[ns++] = idx;
            }
        }
    }
    __syncthreads();
    if constexpr (POS == 2 && FMT < 0) {
        // the probe answers keys in key order: the length order's slot -> key map goes out beside
        // the positions (perm[tile][slot]) before the placement overwrites it
        if (perm) {
            uint16_t* pm = posv + pl.perm_off + (uint64_t)tile * pl.KT;
            for (uint32_t l = tid; l < nk; l += BS) pm[l] = lo[l];
        }
    }
    // run starts; the 512-thread shape scans up to 8 counters per thread where m > 2^31
    // (up to 4 096 segments)
    constexpr int SPER = (V == 1 && !M31) ? 8 : 4;
    auto gd_get = [&](uint32_t sg) -> uint32_t { return (gd[sg >> 1] >> ((sg & 1u) * 16)) & 0xFFFFu; };
    if constexpr (POS == 1) {
        // every run padded to whole groups in HBM: gd = groups per segment (u16 pairs), scanned
        // after the counters into each run's first group, then turned into the run's shift
        // dlt(s) = 8 * gstart(s) - start(s) (< 7 * nseg) for the positions written to posv
        static_assert(!C16, "the group pack keeps plain counters");
        for (uint32_t w = tid; w < (pl.nseg + 1) / 2; w += BS) {
            const uint32_t s0 = 2 * w, s1 = s0 + 1;
            gd[w] = ((cnt[s0] + 7) >> 3) | (s1 < pl.nseg ? ((cnt[s1] + 7) >> 3) << 16 : 0u);
        }
        __syncthreads();
        block_exclusive_scan<false, SPER>(cnt, pl.nseg, wsum);
        __syncthreads();
        block_exclusive_scan16<false, SPER>(gd, pl.nseg, wsum);
        __syncthreads();
        for (uint32_t w = tid; w < (pl.nseg + 1) / 2; w += BS) {
            const uint32_t s0 = 2 * w, s1 = s0 + 1, g = gd[w];
            const uint32_t d0 = 8 * (g & 0xFFFFu) - cnt[s0];
            const uint32_t d1 = s1 < pl.nseg ? 8 * (g >> 16) - cnt[s1] : 0u;
            gd[w] = d0 | (d1 << 16);
        }
    } else if constexpr (POS == 2) {
        // one u32 per segment: count in the low half, its whole result bytes (count rounded up to 8)
        // in the high half -- one scan makes both the run's start and its padded start, and no half
        // carries (C + 7 * nseg <= 65535, probe_pu_enabled); each rank atomic adds 1 to both
        static_assert(!C16, "the probe pack keeps one counter word per segment");
        for (uint32_t sg = tid; sg < pl.nseg; sg += BS) cnt[sg] |= ((cnt[sg] + 7) & ~7u) << 16;
        __syncthreads();
        block_exclusive_scan<false, SPER>(cnt, pl.nseg, wsum);
    } else if constexpr (C16) {
        block_exclusive_scan16<false, SPER>(cnt, pl.nseg, wsum);
    } else {
        block_exclusive_scan<false, SPER>(cnt, pl.nseg, wsum);
    }
    // the groups' nibble words start clear (ORed into below); the image held perm / staged keys
    // until the hashing rounds ended
    for (uint32_t g = tid; g < (POS == 1 ? pl.CPg : pl.CP) / 8; g += BS) smem[g * kGroupWords + 4] = 0;
    __syncthreads();
    if (pl.ablate == 1 || pl.ablate == 2 || (VBF_ABLATION_BUILD && pl.ablate == 9)) {  // timing experiment: keep the stash live, skip the sort
        uint32_t acc = 0;
        for (uint32_t t = 0; t < ns; ++t) acc ^= stash[t];
        if (acc == 0x12345678u) ends[blockIdx.x] = (uint16_t)acc;
        return;
    }
    // rank + place, 8 returning LDS atomics in flight before their results are used
    // the bound is a compile-time constant for K > 0 (ns == RM * K); K == 0 stops at ns
    constexpr uint32_t kNsMax = KK > 0 ? (uint32_t)(RMK * KL) : (uint32_t)kStash;
#pragma unroll
    for (uint32_t t = 0; t < kNsMax; t += 8) {
        if (t >= ns) break;
        uint32_t pos[8], val[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            val[q] = (t + q < ns) ? stash[t + q] : kSentinel;
            if constexpr (POS == 2)  // place | padded place << 16
                pos[q] = val[q] != kSentinel ? lds_add_rtn(&cnt0[val[q] >> SB], 0x10001u) : 0u;
            else
                pos[q] = val[q] != kSentinel ? seg_rank<C16, SB>(cnt0, val[q]) : 0u;
        }
        if constexpr (POS == 1) {  // the group pack places every run at its padded place (whole groups)
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (val[q] != kSentinel) pos[q] += gd_get(val[q] >> SB);
        }
        // the image addresses as 32-bit LDS byte addresses from LDS address 0 (a generic pointer's
        // index took a 64-bit v_mad_u64_u32 per entry); p < 2^16, so a 24-bit multiply
        const uint32_t img0 = (cnt_words + 16 + kLenBuckets + pl.gd_words) * 4u;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (val[q] != kSentinel) {
                const uint32_t p = POS == 2 ? pos[q] & 0xFFFFu : pos[q];
                const uint32_t gb = img0 + __umul24(p >> 3, kGroupWords * 4), e7 = p & 7;
                *reinterpret_cast<lds_u16*>((uintptr_t)(gb + e7 * 2)) = (uint16_t)val[q];
                (void)__hip_atomic_fetch_or(reinterpret_cast<lds_u32*>((uintptr_t)(gb + 16)),
                                            ((val[q] >> 16) & ((1u << (SB - 16)) - 1u)) << (e7 * 4), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        if constexpr (POS != 0) {  // coalesced: for a pair of stash slots the lanes write consecutive u32
            static_assert(KK > 0, "the group pack runs compiled k");
            uint32_t* pv = reinterpret_cast<uint32_t*>(posv);
            // POS 1: the place itself (the image is padded); POS 2: the padded place
            auto pp = [&](int q) -> uint32_t { return val[q] == kSentinel ? 0u : POS == 2 ? pos[q] >> 16 : pos[q]; };
#pragma unroll
            for (int q = 0; q < 8; q += 2)
                if (val[q] != kSentinel || val[q + 1] != kSentinel)
                    pv[((uint64_t)tile * ((kNsMax + 1) / 2) + (t + q) / 2) * BS + tid] = pp(q) | (pp(q + 1) << 16);
        }
    }
    __syncthreads();
    // cnt[s] = start(s) + count(s) = the end of segment s's run.  The last group's low halves past
    // the tile's end are whatever LDS held: every reader masks entries by the run bounds.
    const uint32_t total = seg_get<C16>(cnt, pl.nseg - 1) & (POS == 2 ? 0xFFFFu : 0xFFFFFFFFu);
    uint32_t* out = tiles + (uint64_t)tile * pl.tile_words;
    if constexpr (POS == 2) {
        // the unpadded image, as the build writes it; endsT[s][tile] = end(s) | padded end(s) << 16
        // (cnt[s] = end | (padded start + count) << 16; the padded start is a multiple of 8)
        static_assert(SPL == 1, "posv holds one key's seeds per lane");
        const uint32_t words = group_words(total);
        for (uint32_t w = tid * 4; w < words; w += BS * 4) {
            if (w + 4 <= words)
                image_store(out + w, *reinterpret_cast<const u32x4*>(smem + w));
            else
                for (uint32_t x = w; x < words; ++x) out[x] = smem[x];
        }
        uint32_t* e32 = reinterpret_cast<uint32_t*>(ends);
        for (uint32_t sg = tid; sg < pl.nseg; sg += BS) {
            const uint32_t c = cnt[sg];
            e32[(uint64_t)sg * pl.ntS + tile] = (c & 0xFFFFu) | ((((c >> 16) + 7) & ~7u) << 16);
        }
        return;
    }
    if constexpr (POS == 1) {
        // the padded image is already in LDS: copy its whole groups; run ends in padded entries
        // (multiples of 8): end(s) + dlt(s), rounded up to the group
        const uint32_t pwords = group_words((total + gd_get(pl.nseg - 1) + 7) & ~7u);
        for (uint32_t w = tid * 4; w < pwords; w += BS * 4) {
            if (w + 4 <= pwords)
                *reinterpret_cast<uint4*>(out + w) = *reinterpret_cast<const uint4*>(smem + w);
            else
                for (uint32_t x = w; x < pwords; ++x) out[x] = smem[x];
        }
        for (uint32_t sg = tid; sg < pl.nseg; sg += BS)
            ends[(uint64_t)sg * pl.ntS + tile] = (uint16_t)((cnt[sg] + gd_get(sg) + 7) & ~7u);
        return;
    }
    const uint32_t words = group_words(total);
    for (uint32_t w = tid * 4; w < words; w += BS * 4) {
        if (w + 4 <= words)
            image_store(out + w, *reinterpret_cast<const u32x4*>(smem + w));
        else
            for (uint32_t x = w; x < words; ++x) out[x] = smem[x];
    }
    if (pl.ends_t) {  // straight into endsT[seg][tile] (no transpose pass)
        for (uint32_t s = tid; s < pl.nseg; s += BS) ends[(uint64_t)s * pl.ntS + tile] = (uint16_t)seg_get<C16>(cnt, s);
    } else {
        uint16_t* eo = ends + (uint64_t)tile * pl.nsegS;
        for (uint32_t s = tid; s < pl.nseg; s += BS) eo[s] = (uint16_t)seg_get<C16>(cnt, s);
    }
}

// The multi-SST group pack (vbf_partition.hip, used by vbf_multi_part.hip): k_tile_pack over
// 2^17-position segments of an interleaved group (k = 10 or 19, keys hashed with the length prefix,
// m <= 2^28 positions), writing the tile images, endsT[seg][tile] (row stride pl.ntS, set by the
// caller) and every entry's padded place in posv: u16 pairs, posv32[tile][slot / 2][lane] (slot =
// round * k + seed; (group_pack_slots(k) + 1) / 2 pairs of 512 lanes per tile).
// The same over 2^20-bit segments of one filter (sb = kSegBits) serves the single-filter
// partitioned probe (vbf_probe_part.hip).
bool group_pack_supported(uint64_t m, uint32_t k, int sb = kByteSegBits);
PartPlan make_group_plan(uint32_t m, uint32_t k, bool fixed, int sb = kByteSegBits);
uint32_t group_pack_slots(uint32_t k);
// m == 2^32 - 1 with the length prefix and compiled k (4, 9, 10, 19) on the 1 024-thread shape: the
// SAT kernels (vbf_partition_sat.hip).  hipErrorNotSupported when none fits (the caller then runs
// the general m > 2^31 kernel).
hipError_t launch_tile_pack_sat(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles,
                                uint16_t* ends, hipStream_t s);
// The compiled-k K1 of the build (vbf_tile_pack_main.hpp): launch_tile_pack_main dispatches the
// key layout to launch_tile_pack_main_a (16/32-byte rows), _b (8/24) or _c (offsets, runtime
// stride), each in a translation unit of its own.
hipError_t launch_tile_pack_main(int fmt, bool lp, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                 uint32_t* tiles, uint16_t* ends, hipStream_t s);
hipError_t launch_tile_pack_main_a(int fmt, bool lp, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                   uint32_t* tiles, uint16_t* ends, hipStream_t s);
hipError_t launch_tile_pack_main_b(int fmt, bool lp, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                   uint32_t* tiles, uint16_t* ends, hipStream_t s);
hipError_t launch_tile_pack_main_c(int fmt, bool lp, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                   uint32_t* tiles, uint16_t* ends, hipStream_t s);
hipError_t launch_group_pack(const KeyBatch& kb, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                             uint32_t* tiles, uint16_t* endsT, uint16_t* posv, int sb, hipStream_t s);
// The round-6 probe on the build's image (vbf_probe_pu.hip): the build's plan with keys in key order
// (posv maps a key's seeds to their places), K1 with POS = 2.
PartPlan make_probe_pu_plan(uint32_t m, uint32_t k, bool fixed, bool lp);
bool probe_pu_enabled(uint32_t m, uint32_t k, bool lp, bool fixed);
uint64_t probe_pu_workspace_bytes(uint64_t n, uint32_t m, uint32_t k, bool lp);
hipError_t launch_probe_pu(const KeyBatch& kb, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
                           unsigned long long* count, void* ws, uint64_t ws_bytes, hipStream_t s);

}  // namespace vbf
