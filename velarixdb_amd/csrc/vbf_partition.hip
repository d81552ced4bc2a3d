// vbf_partition.hip -- the partitioned Bloom build: no global atomics on the hot path.
//
// Random `atomicOr`s into a 125 MB bit array run at the memory-side atomic rate (~27 G/s on
// MI355X, measured: profiles/r01), 1e9 of them per 100M-key build.  Instead:
//
//   K1 k_tile_sort : one 1024-thread workgroup per tile of R*1024 keys.  Each lane hashes its
//                    keys (k SipHash-1-3 per key, shared prefix), keeps the k bit indices in
//                    registers (stash), counts them per 2^20-bit segment in LDS, scans the
//                    counts, scatters the indices into an LDS copy of the tile sorted by
//                    segment, and writes that copy out with coalesced stores, plus the tile's
//                    per-segment end offsets (u16).
//   K2 k_transpose : ends[tile][seg] -> endsT[seg][tile] so each segment reads one row.
//   K3 k_seg_or    : one workgroup per 2^20-bit segment (128 KiB of LDS): gathers that
//                    segment's run from every tile, ORs the bits into LDS with ds_or, then
//                    writes the segment's 32768 words with coalesced stores (or merges them
//                    with word-wise atomics when several workgroups share a segment).
//
// Results are bit-identical to the per-key atomic kernel (OR is order-independent); the
// build still ORs into the existing words (bf.rs:89 never clears bits).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "keyhash.hpp"
#include "sip13.hpp"
#include "vbf_kernels.hpp"

namespace vbf {

constexpr int kPBlock = 1024;      // threads per K1 / K3 workgroup
constexpr int kStash = 32;         // max bit indices a lane keeps in registers (k <= kStash)
constexpr int kSegBits = 20;       // segment = 2^20 bits = 128 KiB of LDS
constexpr uint32_t kSegWords = 1u << (kSegBits - 5);
constexpr uint32_t kSentinel = 0xFFFFFFFFu;  // never a bit index: idx < m <= 2^32 - 1

struct PartPlan {
    uint32_t k, KS, R, KT, C, nseg, G;
    uint64_t m, mu, nwords;
};

// Exclusive scan of v[0..n) in LDS (n <= 4 * kPBlock); returns nothing, v holds the prefix.
__device__ __forceinline__ void block_exclusive_scan(uint32_t* v, uint32_t n, uint32_t* wsum) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t loc[4];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t s = tid * 4 + q;
        loc[q] = s < n ? v[s] : 0;
        sum += loc[q];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= (uint32_t)o) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    if (wave == 0) {
        uint32_t w = lane < kPBlock / 64 ? wsum[lane] : 0;
        uint32_t wi = w;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const uint32_t y = __shfl_up(wi, o);
            if (lane >= (uint32_t)o) wi += y;
        }
        if (lane < kPBlock / 64) wsum[lane] = wi - w;  // exclusive wave offsets
    }
    __syncthreads();
    uint32_t run = wsum[wave] + incl - sum;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t s = tid * 4 + q;
        if (s < n) v[s] = run;
        run += loc[q];
    }
}

// KS = stash slots per lane: 32 -> one 1024-thread workgroup per CU (big tiles, long runs);
// 16 -> two per CU (8 waves/SIMD for the hashing, shorter runs).
template <int FMT, bool LP, int KS>
__global__ __launch_bounds__(kPBlock, KS == 16 ? 8 : 4) void k_tile_sort(DevKeys dk, PartPlan pl,
                                                                         uint32_t* tiles, uint16_t* ends) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t* sorted = smem;            // C entries
    uint32_t* cnt = smem + pl.C;        // nseg entries (+ pad)
    uint32_t* wsum = cnt + ((pl.nseg + 3) & ~3u);
    const uint32_t tid = threadIdx.x;
    for (uint32_t s = tid; s < pl.nseg; s += kPBlock) cnt[s] = 0;
    __syncthreads();

    uint32_t stash[KS];
    uint32_t ns = 0;  // wave-uniform: every lane stores R*k entries (sentinels past the end)
    const uint64_t key0 = (uint64_t)blockIdx.x * pl.KT;
    for (uint32_t r = 0; r < pl.R; ++r) {
        const uint64_t j = key0 + (uint64_t)r * kPBlock + tid;
        const bool valid = j < dk.n;
        Prefix p{};
        if (valid) p = key_prefix<FMT, LP>(dk, j);
        for (uint32_t i = 0; i < pl.k; ++i) {
            uint32_t idx = kSentinel;
            if (valid) {
                idx = fast_mod(prefix_hash(p, i), pl.m, pl.mu);
                atomicAdd(&cnt[idx >> kSegBits], 1u);
            }
            stash[ns++] = idx;
        }
    }
    __syncthreads();
    block_exclusive_scan(cnt, pl.nseg, wsum);
    __syncthreads();
    // rank + place, 8 returning LDS atomics in flight before their results are used
    for (uint32_t t = 0; t < ns; t += 8) {
        uint32_t pos[8], val[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            val[q] = (t + q < ns) ? stash[t + q] : kSentinel;
            pos[q] = val[q] != kSentinel ? atomicAdd(&cnt[val[q] >> kSegBits], 1u) : 0u;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (val[q] != kSentinel) sorted[pos[q]] = val[q];
    }
    __syncthreads();
    // cnt[s] now holds the end of segment s's run within the sorted tile
    const uint32_t total = cnt[pl.nseg - 1];
    uint32_t* out = tiles + (uint64_t)blockIdx.x * pl.C;
    const uint32_t total4 = total & ~3u;
    for (uint32_t e = tid * 4; e < total4; e += kPBlock * 4)
        *reinterpret_cast<uint4*>(out + e) = *reinterpret_cast<const uint4*>(sorted + e);
    for (uint32_t e = total4 + tid; e < total; e += kPBlock) out[e] = sorted[e];
    uint16_t* eo = ends + (uint64_t)blockIdx.x * pl.nseg;
    for (uint32_t s = tid; s < pl.nseg; s += kPBlock) eo[s] = (uint16_t)cnt[s];
}

// Same tile contract, no LDS copy of the tile: each index is stored straight to its sorted slot
// in the tile's global region (the block's 120 KiB of scattered 4-byte stores land in L2 within
// a few microseconds and leave as whole lines).  LDS holds only the counters, so two
// 1024-thread workgroups fit per CU (8 waves/SIMD for the hashing).
template <int FMT, bool LP>
__global__ __launch_bounds__(kPBlock) void k_tile_sort_direct(DevKeys dk, PartPlan pl, uint32_t* tiles,
                                                                 uint16_t* ends) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t* cnt = smem;  // nseg entries (+ pad)
    uint32_t* wsum = cnt + ((pl.nseg + 3) & ~3u);
    const uint32_t tid = threadIdx.x;
    for (uint32_t s = tid; s < pl.nseg; s += kPBlock) cnt[s] = 0;
    __syncthreads();

    uint32_t stash[kStash];
    uint32_t ns = 0;
    const uint64_t key0 = (uint64_t)blockIdx.x * pl.KT;
    for (uint32_t r = 0; r < pl.R; ++r) {
        const uint64_t j = key0 + (uint64_t)r * kPBlock + tid;
        const bool valid = j < dk.n;
        Prefix p{};
        if (valid) p = key_prefix<FMT, LP>(dk, j);
        for (uint32_t i = 0; i < pl.k; ++i) {
            uint32_t idx = kSentinel;
            if (valid) {
                idx = fast_mod(prefix_hash(p, i), pl.m, pl.mu);
                atomicAdd(&cnt[idx >> kSegBits], 1u);
            }
            stash[ns++] = idx;
        }
    }
    __syncthreads();
    block_exclusive_scan(cnt, pl.nseg, wsum);
    __syncthreads();
    uint32_t* out = tiles + (uint64_t)blockIdx.x * pl.C;
    for (uint32_t t = 0; t < ns; t += 8) {
        uint32_t pos[8], val[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            val[q] = (t + q < ns) ? stash[t + q] : kSentinel;
            pos[q] = val[q] != kSentinel ? atomicAdd(&cnt[val[q] >> kSegBits], 1u) : 0u;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (val[q] != kSentinel) out[pos[q]] = val[q];
    }
    __syncthreads();
    uint16_t* eo = ends + (uint64_t)blockIdx.x * pl.nseg;
    for (uint32_t s = tid; s < pl.nseg; s += kPBlock) eo[s] = (uint16_t)cnt[s];
}

// ends[rows][cols] -> endsT[cols][rows], 64x64 tiles through LDS.
__global__ __launch_bounds__(256) void k_transpose_u16(const uint16_t* in, uint16_t* out, uint32_t rows,
                                                       uint32_t cols) {
    __shared__ uint16_t t[64][65];
    const uint32_t c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
    const uint32_t tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (uint32_t y = ty; y < 64; y += 4) {
        const uint32_t r = r0 + y, c = c0 + tx;
        if (r < rows && c < cols) t[y][tx] = in[(uint64_t)r * cols + c];
    }
    __syncthreads();
    for (uint32_t y = ty; y < 64; y += 4) {
        const uint32_t c = c0 + y, r = r0 + tx;
        if (r < rows && c < cols) out[(uint64_t)c * rows + r] = t[tx][y];
    }
}

// Runs are read by 8-lane groups: lane q of a group loads words [4q, 4q+4) and [32+4q, 32+4q+4)
// of its run with 16-byte loads (4-byte aligned: gfx950 global loads need only dword alignment),
// so one wave instruction covers 8 runs x 128 contiguous bytes.  All 16 loads of the 64 runs a
// wave owns are issued before the first ds_or; the few runs longer than 64 words finish in a
// tail loop.  Words past a run's end belong to the next run of the same tile (or to the
// workspace's tail pad) and are masked off.
__global__ __launch_bounds__(kPBlock) void k_seg_or(const uint32_t* tiles, const uint16_t* endsT,
                                                    uint32_t ntiles, PartPlan pl, bool atomic_merge,
                                                    uint32_t* words) {
    __shared__ __attribute__((aligned(16))) uint32_t bitmap[kSegWords];
    const uint32_t seg = blockIdx.x / pl.G, part = blockIdx.x % pl.G;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t wbase = (uint64_t)seg * kSegWords;
    const uint32_t wn = (uint32_t)std::min<uint64_t>(kSegWords, pl.nwords - wbase);
    const bool own = (pl.G == 1) && !atomic_merge;  // sole writer: start from the existing words
    for (uint32_t w = tid * 4; w < kSegWords; w += kPBlock * 4) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (own) {
            if (w + 4 <= wn)
                v = *reinterpret_cast<const uint4*>(words + wbase + w);
            else if (w < wn) {
                v.x = words[wbase + w];
                if (w + 1 < wn) v.y = words[wbase + w + 1];
                if (w + 2 < wn) v.z = words[wbase + w + 2];
            }
        }
        *reinterpret_cast<uint4*>(bitmap + w) = v;
    }
    __syncthreads();

    const uint32_t t_lo = (uint32_t)((uint64_t)part * ntiles / pl.G);
    const uint32_t t_hi = (uint32_t)((uint64_t)(part + 1) * ntiles / pl.G);
    const uint16_t* row_end = endsT + (uint64_t)seg * ntiles;
    const uint16_t* row_beg = seg ? endsT + (uint64_t)(seg - 1) * ntiles : nullptr;
    const uint32_t grp = lane >> 3, q4 = (lane & 7) * 4;
    for (uint32_t tg = t_lo + wave * 64; tg < t_hi; tg += kPBlock) {
        // element offsets fit u32: one chunk holds < 2^30 + C indices (kPartChunkIdx)
        uint32_t off[8], len[8];
        uint4 d0[8], d1[8];
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const uint32_t t = tg + g * 8 + grp;  // the 8 lanes of a group read the same u16
            uint32_t st = 0, en = 0;
            if (t < t_hi) {
                st = row_beg ? row_beg[t] : 0;
                en = row_end[t];
            }
            off[g] = t * pl.C + st + q4;
            len[g] = en - st;
        }
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            if (q4 < len[g]) __builtin_memcpy(&d0[g], tiles + off[g], 16);
            if (q4 + 32 < len[g]) __builtin_memcpy(&d1[g], tiles + off[g] + 32, 16);
        }
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const uint32_t a[4] = {d0[g].x, d0[g].y, d0[g].z, d0[g].w};
            const uint32_t b[4] = {d1[g].x, d1[g].y, d1[g].z, d1[g].w};
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (q4 + c < len[g]) atomicOr(&bitmap[(a[c] >> 5) & (kSegWords - 1)], 1u << (a[c] & 31));
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (q4 + 32 + c < len[g]) atomicOr(&bitmap[(b[c] >> 5) & (kSegWords - 1)], 1u << (b[c] & 31));
        }
        // tail: runs longer than 64 words (rare at the default plan; common for tiny m)
#pragma unroll 1
        for (int g = 0; g < 8; ++g) {
            for (uint32_t e = q4 + 64; e < len[g]; e += 32) {
                uint4 v;
                __builtin_memcpy(&v, tiles + off[g] - q4 + e, 16);
                const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (e + c < len[g]) atomicOr(&bitmap[(x[c] >> 5) & (kSegWords - 1)], 1u << (x[c] & 31));
            }
        }
    }
    __syncthreads();
    if (own) {
        for (uint32_t w = tid * 4; w < wn; w += kPBlock * 4) {
            if (w + 4 <= wn)
                *reinterpret_cast<uint4*>(words + wbase + w) = *reinterpret_cast<const uint4*>(bitmap + w);
            else
                for (uint32_t x = w; x < wn; ++x) words[wbase + x] = bitmap[x];
        }
    } else {
        for (uint32_t w = tid; w < wn; w += kPBlock) {
            const uint32_t v = bitmap[w];
            if (v) atomicOr(words + wbase + w, v);
        }
    }
}

static int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}

static uint32_t stash_slots(uint32_t k) {
    static const int env = env_int("VBF_TILE_KS", 0);
    if (env == 16 && k <= 16) return 16;
    return 32;
}

// K1 variant: 0 = LDS-sorted tile copy, 1 = direct scattered stores (VBF_TILE_DIRECT)
static int tile_direct() {
    static const int env = env_int("VBF_TILE_DIRECT", 0);
    return env;
}

static PartPlan make_plan(uint32_t m, uint32_t k) {
    PartPlan pl{};
    pl.k = k;
    pl.KS = stash_slots(k);
    pl.R = pl.KS / k;
    pl.KT = pl.R * kPBlock;
    pl.C = pl.KT * k;
    pl.m = m;
    pl.mu = ~0ull / m;
    pl.nwords = ((uint64_t)m + 31) / 32;
    pl.nseg = (uint32_t)(((uint64_t)m + (1u << kSegBits) - 1) >> kSegBits);
    return pl;
}

bool partition_supported(uint32_t m, uint32_t k) { return m > 0 && k >= 1 && k <= (uint32_t)kStash; }

// Bytes of workspace one launch_build_partitioned call needs for n keys.
uint64_t partition_workspace_bytes(uint64_t n, uint32_t m, uint32_t k) {
    if (!partition_supported(m, k)) return 0;
    const PartPlan pl = make_plan(m, k);
    uint64_t chunk_keys = std::min<uint64_t>(n, kPartChunkIdx / k);
    const uint64_t ntiles = (chunk_keys + pl.KT - 1) / pl.KT;
    return ntiles * ((uint64_t)pl.C * 4 + (uint64_t)pl.nseg * 4) + 512;
}

hipError_t launch_build_partitioned(const KeyBatch& kb, uint32_t m, uint32_t k, uint32_t* words,
                                    void* ws, uint64_t ws_bytes, bool atomic_merge, hipStream_t s) {
    if (kb.n == 0 || k == 0) return hipSuccess;
    if (!partition_supported(m, k)) return hipErrorInvalidValue;
    PartPlan pl = make_plan(m, k);
    const uint64_t chunk_keys = std::min<uint64_t>(kb.n, (kPartChunkIdx / k) / pl.KT * pl.KT);
    const uint64_t max_tiles = (chunk_keys + pl.KT - 1) / pl.KT;
    if (ws_bytes < partition_workspace_bytes(kb.n, m, k)) return hipErrorInvalidValue;
    uint32_t* tiles = reinterpret_cast<uint32_t*>(ws);
    uint16_t* ends = reinterpret_cast<uint16_t*>(tiles + max_tiles * pl.C);
    uint16_t* endsT = ends + max_tiles * pl.nseg;

    const bool direct = tile_direct() && pl.KS == 32;
    const size_t lds1 = ((size_t)(direct ? 0 : pl.C) + ((pl.nseg + 3) & ~3u) + 64) * 4;
    for (uint64_t lo = 0; lo < kb.n; lo += chunk_keys) {
        const uint64_t cn = std::min<uint64_t>(chunk_keys, kb.n - lo);
        DevKeys dk{kb.keys, kb.offsets, kb.off_base, kb.stride, cn};
        if (kb.offsets)
            dk.offsets = kb.offsets + lo;
        else
            dk.keys = kb.keys + lo * kb.stride;
        const uint32_t ntiles = (uint32_t)((cn + pl.KT - 1) / pl.KT);
        hipError_t err = hipSuccess;
        phase_begin(kPhaseTileSort, s);
        with_fmt(pick_fmt(dk.keys, dk.offsets, dk.stride), kb.len_prefix, [&]<int FMT, bool LP>() {
            auto fn = direct ? k_tile_sort_direct<FMT, LP>
                             : pl.KS == 16 ? k_tile_sort<FMT, LP, 16> : k_tile_sort<FMT, LP, 32>;
            err = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1);
            if (err == hipSuccess)
                hipLaunchKernelGGL(fn, dim3(ntiles), dim3(kPBlock), lds1, s, dk, pl, tiles, ends);
        });
        if (err != hipSuccess) return err;
        phase_end(kPhaseTileSort, s);
        phase_begin(kPhaseTranspose, s);
        hipLaunchKernelGGL(k_transpose_u16, dim3((pl.nseg + 63) / 64, (ntiles + 63) / 64), dim3(256), 0, s,
                           ends, endsT, ntiles, pl.nseg);
        // several workgroups per segment when there are few segments (small m)
        pl.G = std::max<uint32_t>(1, std::min<uint32_t>(ntiles, (512 + pl.nseg - 1) / pl.nseg));
        const bool merge = atomic_merge || pl.G > 1;
        phase_end(kPhaseTranspose, s);
        phase_begin(kPhaseSegOr, s);
        hipLaunchKernelGGL(k_seg_or, dim3(pl.nseg * pl.G), dim3(kPBlock), 0, s, tiles, endsT, ntiles, pl,
                           merge, words);
        phase_end(kPhaseSegOr, s);
        err = hipGetLastError();
        if (err != hipSuccess) return err;
    }
    return hipSuccess;
}

}  // namespace vbf
