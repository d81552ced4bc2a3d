// vbf_probe_pack.hpp -- Q1 of the partitioned probe (k_probe_pack), shared by vbf_probe_part.hip (the
// compiled k and the scratch-stash kernel) and vbf_probe_part_rk_{a,b,c,d}.hip (the runtime-k
// classes, translation units of their own so the library builds in parallel).
#pragma once
#include "vbf_tile_pack.hpp"

namespace vbf {

constexpr uint32_t kOffMask = (1u << kSegBits) - 1;
static_assert(kSegBits == 20, "probe entries hold a 12-bit key id above the 20-bit offset");

// SB: segment = 2^SB filter positions (bits of one filter: 20; bytes of an interleaved group of
// filters, vbf_multi_part.hip: 17).  An entry is (tile-local key id << SB) | offset in segment.
// SAT: m == 2^32 - 1, remainders by mod_sat (sip13.hpp).
// Per segment one LDS word holds the run's count (-> start -> end) in its low half and its padded
// start in the high half: both stay below 2^16 (C + 7 * nseg <= cap <= 65535, probe_partition_
// supported), so one scan of the words scans both and no half carries into the other -- half the
// counters' LDS of two u32 arrays, which at m = 2^32 - 1 (4 096 segments) buys 33 % larger tiles.
// KC > 0 (K == 0): a runtime-k class -- any k <= KC (pl.k) in a KC-slot register stash, seeds past k
// leaving sentinels (the build's class kernels, vbf_tile_pack_rk.hpp); K == 0 == KC: the stash in
// scratch memory (k > 32 never reaches here: probe_partition_supported).
template <int FMT, bool LP, int K, bool M31, int SB, bool SAT = false, int KC = 0>
__global__ __launch_bounds__(kPBlock, 8) void k_probe_pack(DevKeys dk, ProbePlan pl, uint32_t* tiles, uint16_t* ends) {
    static_assert(KC == 0 || K == 0, "a class kernel takes its k at run time");
    constexpr int KK = K > 0 ? K : KC;  // seed slots per key in the stash (0: the scratch stash)
    constexpr uint32_t kOff = (1u << SB) - 1;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t* ent = smem;               // C entries
    uint32_t* cnt = ent + pl.C;         // nseg_pad: count | padded count << 16 -> starts -> end | padded start
    uint32_t* wsum = cnt + pl.nseg_pad; // 16
    const uint32_t tid = threadIdx.x;
    for (uint32_t s = tid; s < pl.nseg; s += kPBlock) cnt[s] = 0;
    __syncthreads();
    uint32_t stash[KK > 0 ? rounds_max(KK) * KK : kStash];
    const uint64_t key0 = (uint64_t)blockIdx.x * pl.KT;
    const uint64_t key_end = std::min<uint64_t>(dk.n, key0 + pl.KT);
    uint32_t ns;
    if constexpr (KK > 0) {
        constexpr int RM = rounds_max(KK);
        // compile-time r per round (see k_tile_pack): keeps the stash out of scratch memory
        auto round = [&](auto rc) {
            constexpr int r = decltype(rc)::value;
            const uint64_t j = key0 + (uint64_t)r * kPBlock + tid;
            const bool valid = (uint32_t)r < pl.R && j < key_end;
            Prefix p{};
            if (valid) p = key_prefix<FMT, LP>(dk, j);
            SeedCtx q{};
            if constexpr (FMT > 0) q = seed_ctx(p);  // block-aligned prefix: seed_hash (sip13.hpp)
            // the seed slots as a fold with a compile-time slot number, as in k_tile_pack
            auto seed = [&](auto ic) {
                constexpr int i = decltype(ic)::value;
                uint32_t idx = kSentinel;
                if (valid && (KC == 0 || (uint32_t)i < pl.k)) {  // class: seeds past k stay sentinels
                    idx = mod_m<M31, SAT>(FMT > 0 ? seed_hash(q, i) : prefix_hash(p, i), pl.m, pl.mu);
                    atomicAdd(&cnt[idx >> SB], 1u);
                }
                stash[r * KK + i] = idx;
            };
            [&]<int... Is>(std::integer_sequence<int, Is...>) {
                (seed(std::integral_constant<int, Is>{}), ...);
            }(std::make_integer_sequence<int, KK>{});
        };
        [&]<int... Rs>(std::integer_sequence<int, Rs...>) {
            (round(std::integral_constant<int, Rs>{}), ...);
        }(std::make_integer_sequence<int, RM>{});
        ns = RM * KK;
    } else {
        ns = 0;
        for (uint32_t r = 0; r < pl.R; ++r) {
            const uint64_t j = key0 + (uint64_t)r * kPBlock + tid;
            const bool valid = j < key_end;
            Prefix p{};
            if (valid) p = key_prefix<FMT, LP>(dk, j);
            for (uint32_t i = 0; i < pl.k; ++i) {
                uint32_t idx = kSentinel;
                if (valid) {
                    idx = mod_m<M31>(prefix_hash(p, i), pl.m, pl.mu);
                    atomicAdd(&cnt[idx >> SB], 1u);
                }
                stash[ns++] = idx;
            }
        }
    }
    __syncthreads();
    for (uint32_t s = tid; s < pl.nseg; s += kPBlock) cnt[s] |= ((cnt[s] + 7) & ~7u) << 16;
    __syncthreads();
    block_exclusive_scan(cnt, pl.nseg, wsum);
    __syncthreads();
    const uint32_t per = KK > 0 ? (uint32_t)KK : pl.k;  // stash slots per key (round r = slot / per)
    // the bound is a compile-time constant for KK > 0 (ns == RM * KK); the scratch stash stops at ns
    constexpr uint32_t kNsMax = KK > 0 ? (uint32_t)(rounds_max(KK) * KK) : (uint32_t)kStash;
#pragma unroll
    for (uint32_t t = 0; t < kNsMax; t += 8) {
        if (t >= ns) break;
        uint32_t pos[8], val[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            val[q] = (t + q < ns) ? stash[t + q] : kSentinel;
            pos[q] = val[q] != kSentinel ? atomicAdd(&cnt[val[q] >> SB], 1u) & 0xFFFFu : 0u;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (val[q] != kSentinel) {
                const uint32_t local = ((t + q) / per) * kPBlock + tid;  // round r = slot / k
                ent[pos[q]] = (local << SB) | (val[q] & kOff);
            }
    }
    __syncthreads();
    // runs -> global, padded to multiples of 8; 8-lane groups, one run at a time
    const uint32_t grp = tid >> 3, q = tid & 7;
    uint32_t* out = tiles + (uint64_t)blockIdx.x * pl.cap;
    uint16_t* eo = ends + (uint64_t)blockIdx.x * pl.nseg;
    for (uint32_t s = grp; s < pl.nseg; s += kPBlock / 8) {
        const uint32_t st = s ? cnt[s - 1] & 0xFFFFu : 0, en = cnt[s] & 0xFFFFu, c = en - st, pc = (c + 7) & ~7u;
        const uint32_t d = cnt[s] >> 16;
        for (uint32_t x = q; x < pc; x += 8) out[d + x] = ent[std::min(st + x, en - 1)];
        if (q == 0) eo[s] = (uint16_t)(d + pc);
    }
}

// The runtime-k class probe packs on 2^20-bit segments: vbf_probe_part_rk_a.hip (classes 5, 8, 12)
// and _b (16, 21, 24, 32) for keys hashed with the length prefix, _c / _d the same without it (the
// pre-encoded integer keys of bf.rs:275-424); hipErrorNotSupported for other shapes.
hipError_t launch_probe_pack_class_a(int fmt, uint32_t kc, const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles,
                                     uint32_t* tiles, uint16_t* ends, hipStream_t s);
hipError_t launch_probe_pack_class_b(int fmt, uint32_t kc, const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles,
                                     uint32_t* tiles, uint16_t* ends, hipStream_t s);
hipError_t launch_probe_pack_class_c(int fmt, uint32_t kc, const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles,
                                     uint32_t* tiles, uint16_t* ends, hipStream_t s);
hipError_t launch_probe_pack_class_d(int fmt, uint32_t kc, const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles,
                                     uint32_t* tiles, uint16_t* ends, hipStream_t s);

// The same classes over 2^17-position segments (the multi-SST probe's interleaved filters,
// vbf_multi_part.hip: m <= 2^28 positions), keys with the length prefix: _a17 (5, 8, 12), _b17 (16,
// 21, 24, 32) -- round 6: the multi-SST pack at k outside {10, 19} no longer keeps a scratch stash.
hipError_t launch_probe_pack_class_a17(int fmt, uint32_t kc, const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles,
                                       uint32_t* tiles, uint16_t* ends, hipStream_t s);
hipError_t launch_probe_pack_class_b17(int fmt, uint32_t kc, const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles,
                                       uint32_t* tiles, uint16_t* ends, hipStream_t s);

// One class kernel: m <= 2^31 takes the one-word remainder, above it the general one (2^17-position
// segments: always m <= 2^28).
template <int FMT, bool LP, int KC, int SB = kSegBits>
hipError_t launch_probe_pack_one_class(const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles, uint32_t* tiles,
                                       uint16_t* ends, hipStream_t s) {
    auto fn = SB != kSegBits || pl.m <= (1ull << 31) ? k_probe_pack<FMT, LP, 0, true, SB, false, KC>
                                                     : k_probe_pack<FMT, LP, 0, false, SB, false, KC>;
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)pl.lds1);
    if (err == hipSuccess) hipLaunchKernelGGL(fn, dim3(ntiles), dim3(kPBlock), pl.lds1, s, dk, pl, tiles, ends);
    return err;
}

template <bool LPC, int SB, int... KCs>
hipError_t launch_probe_pack_classes(int fmt, uint32_t kc, const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles,
                                     uint32_t* tiles, uint16_t* ends, hipStream_t s) {
    hipError_t err = hipErrorNotSupported;
    with_fmt(fmt, LPC, [&]<int FMT, bool LP>() {
        if constexpr (LP == LPC)
            ((kc == (uint32_t)KCs
                  ? (void)(err = launch_probe_pack_one_class<FMT, LP, KCs, SB>(dk, pl, ntiles, tiles, ends, s))
                  : (void)0),
             ...);
    });
    return err;
}

}  // namespace vbf
