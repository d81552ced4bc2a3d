// vbf_partition.hip -- the partitioned Bloom build: no global atomics on the hot path.
//
// Random `atomicOr`s into a 125 MB bit array run at the memory-side atomic rate (27 G/s on
// MI355X whatever the array size, tools/ubench), 1e9 of them per 100M-key build.  Instead:
//
//   K1 k_tile_pack : one 1024-thread workgroup per tile of KT keys, two workgroups per CU.  Each
//                    lane hashes its keys (k SipHash-1-3 per key over a shared prefix) and keeps
//                    the k bit indices in registers; the workgroup counts them per 2^20-bit
//                    segment in LDS, scans the counts, and places every index into an LDS copy
//                    of the tile sorted by segment.  The copy is PACKED: an index inside its
//                    segment is 20 bits, stored as a u16 low half plus a 4-bit nibble (2.5 B per
//                    index instead of 4), in 8-entry GROUPS of 20 bytes -- the 8 low halves, then
//                    the group's 8 nibbles in one word -- so that a run's low halves and nibbles
//                    share cache lines (k_seg_or's time follows the L2 requests it makes, one
//                    per 128-byte line a run touches: group layout 1.7 lines per run at k = 10
//                    against 2.6 with the nibbles in a separate area, tools/rdgroup).  The tile
//                    and its per-segment run ends (u16) are written out with coalesced stores.
//   K2 k_transpose : ends[tile][seg] -> endsT[seg][tile] so each segment reads one row.
//   K3 k_seg_or    : one workgroup per segment (128 KiB of LDS): lanes read that segment's run
//                    from every tile one 20-byte group each, all issued before the first ds_or,
//                    then the segment's 32768 words are written with coalesced stores (or
//                    merged with word atomics when several workgroups share it).
//
// Results are bit-identical to the per-key atomic kernel (OR is order-independent); the build
// ORs into the existing words (bf.rs:89 never clears bits).
#include "vbf_partition.hpp"
#include "vbf_tile_pack.hpp"
#include "vbf_tile_pack_rk.hpp"

namespace vbf {


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

void launch_transpose_u16(const uint16_t* in, uint16_t* out, uint32_t rows, uint32_t cols, hipStream_t s) {
    hipLaunchKernelGGL(k_transpose_u16, dim3((cols + 63) / 64, (rows + 63) / 64), dim3(256), 0, s, in, out, rows, cols);
}

// in[rows][in_stride] -> out[cols][out_stride] with both strides multiples of 8 and 16-byte aligned
// buffers: a 64 x 64 tile moves as 16-byte vectors (512 per tile, two per thread each way) instead
// of 2-byte elements -- one eighth of the memory instructions (the build's k = 19 ends array is
// 250 MB).  The vectors may cover stride padding past rows / cols: in stays inside in_stride,
// out inside out_stride, and the padding is never read.  LDS rows of 66 u16 (33 dwords) keep the
// column reads of the write phase on different banks.
__global__ __launch_bounds__(256) void k_transpose_u16_v(const uint16_t* in, uint16_t* out, uint32_t rows,
                                                         uint32_t cols, uint32_t in_stride, uint32_t out_stride) {
    __shared__ uint32_t t[64 * 33];
    const uint32_t c0 = blockIdx.x * 64, r0 = blockIdx.y * 64, tid = threadIdx.x;
#pragma unroll
    for (uint32_t q = tid; q < 512; q += 256) {
        const uint32_t r = q >> 3, cv = (q & 7) * 8;
        if (r0 + r < rows && c0 + cv < cols) {
            const uint4 v = *reinterpret_cast<const uint4*>(in + (uint64_t)(r0 + r) * in_stride + c0 + cv);
            uint32_t* d = t + r * 33 + cv / 2;
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
    }
    __syncthreads();
    const uint16_t* t16 = reinterpret_cast<const uint16_t*>(t);
#pragma unroll
    for (uint32_t q = tid; q < 512; q += 256) {
        const uint32_t c = q >> 3, rv = (q & 7) * 8;
        if (c0 + c < cols && r0 + rv < rows) {
            uint32_t w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                w[i] = (uint32_t)t16[(rv + 2 * i) * 66 + c] | ((uint32_t)t16[(rv + 2 * i + 1) * 66 + c] << 16);
            *reinterpret_cast<uint4*>(out + (uint64_t)(c0 + c) * out_stride + r0 + rv) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

// Any strides (the fallback of launch_transpose_u16_strided): 64 x 64 tiles of u16 elements.
__global__ __launch_bounds__(256) void k_transpose_u16_s(const uint16_t* in, uint16_t* out, uint32_t rows,
                                                         uint32_t cols, uint32_t in_stride, uint32_t out_stride) {
    __shared__ uint16_t t[64][65];
    const uint32_t c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
    const uint32_t tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (uint32_t y = ty; y < 64; y += 4) {
        const uint32_t r = r0 + y, c = c0 + tx;
        if (r < rows && c < cols) t[y][tx] = in[(uint64_t)r * in_stride + c];
    }
    __syncthreads();
    for (uint32_t y = ty; y < 64; y += 4) {
        const uint32_t c = c0 + y, r = r0 + tx;
        if (r < rows && c < cols) out[(uint64_t)c * out_stride + r] = t[tx][y];
    }
}

hipError_t launch_transpose_u16_strided(const uint16_t* in, uint16_t* out, uint32_t rows, uint32_t cols,
                                        uint32_t in_stride, uint32_t out_stride, hipStream_t s) {
    if (rows == 0 || cols == 0) return hipSuccess;
    if (in_stride < cols || out_stride < rows) return hipErrorInvalidValue;
    const bool vec = in_stride % 8 == 0 && out_stride % 8 == 0 && (reinterpret_cast<uintptr_t>(in) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    const dim3 grid((cols + 63) / 64, (rows + 63) / 64);
    if (vec)
        hipLaunchKernelGGL(k_transpose_u16_v, grid, dim3(256), 0, s, in, out, rows, cols, in_stride, out_stride);
    else
        hipLaunchKernelGGL(k_transpose_u16_s, grid, dim3(256), 0, s, in, out, rows, cols, in_stride, out_stride);
    return hipGetLastError();
}

// OR entries [a, b) of one group (8 u16 low halves in l, their 8 nibbles in nib) into the segment
// bitmap.
__device__ __forceinline__ void or_group(uint32_t* bitmap, uint4 l, uint32_t nib, uint32_t a, uint32_t b,
                                         uint32_t abl = 0) {
    if (abl == 3) {  // timing experiment: consume the loads without touching LDS
        if ((l.x ^ l.y ^ l.z ^ l.w ^ nib) == 0x12345678u && b == 9) bitmap[0] = a;
        return;
    }
    const uint32_t w[4] = {l.x, l.y, l.z, l.w};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        if ((uint32_t)c >= a && (uint32_t)c < b) {
            const uint32_t idx = ((w[c >> 1] >> ((c & 1) * 16)) & 0xFFFFu) | (((nib >> (4 * c)) & 15u) << 16);
            atomicOr(&bitmap[idx >> 5], 1u << (idx & 31));
        }
    }
}

// Loads group g of a packed tile: 16 bytes of low halves and the nibble word after them (the group
// is 4-byte aligned; bytes past the tile's last entry are masked by the caller).
__device__ __forceinline__ void load_group(const uint32_t* tile, uint32_t g, uint4& l, uint32_t& nib) {
    __builtin_memcpy(&l, tile + g * kGroupWords, 16);
    nib = tile[g * kGroupWords + 4];
}

// Entries of group gi inside the run [st, en): [a, b) packed as a | b << 4 (0: none).
__device__ __forceinline__ uint32_t group_range(uint32_t gi, uint32_t st, uint32_t en) {
    if (gi * 8 >= en || gi * 8 + 8 <= st) return 0u;
    const uint32_t a = gi * 8 < st ? st - gi * 8 : 0u, b = std::min<uint32_t>(8, en - gi * 8);
    return a | (b << 4);
}

// K3 tile-loop variants (speed only; identical results).  By default the plan picks V7 with NG = 5
// for runs of >= kShortRun entries on average (C / nseg) and NG = 4 below; VBF_K3 forces one:
//   1: two-stage -- run bounds of batch b+1 (8 u16 loads per lane) in flight with batch b's data
//   3: three-stage -- bounds of b+2, data of b+1 and the ORs of b overlap; run bounds loaded
//      coalesced (one u16 pair per lane for the wave's tiles) and handed to the 8-lane groups with
//      ds_bpermute; lane q of a group reads the run's q-th group (and q+8, ... past 8 groups);
//      data loads unconditional (idle lanes re-read their run's first group) so vmcnt waits stay
//      exact; NG runs per 8-lane group per batch (VBF_K3 3: 1024 threads NG=4; 4: 1024, NG=5;
//      5: 768, NG=6; 6: 768, NG=8; 8: 1024, NG=6; NG=8 at 1024 spills); VBF_K3 13: 4-lane groups,
//      NG=4 (16 runs per load instruction, no idle lanes on short runs, no prefix search).
//   6: flattened -- a wave's runs' groups dealt to lanes back to back, no lane idles on a short
//      run (VBF_K3 10: NG=4, 11: NG=5, 12: NG=6).  At k = 19 (m = 1.9e9, ~16-entry runs) it is
//      the one that keeps K3 from idling most of its lanes.
//   7: the flattened reader with each group's run found from per-wave run marks in LDS and a DPP
//      max-scan instead of the binary search (round 6; VBF_K3 14: NG=4, 15: NG=5, 16: NG=6).
//   Measured and dropped (tools/env_ab.sh): coalesced bounds in the two-stage loop (-3 %);
//   raw buffer loads with out-of-range offsets for idle lanes (no duplicate requests): the same
//   as the duplicates (the texture addresser coalesces them).
template <int V, int BS = kPBlock, int NG = 8, int LPR = 8>
__global__ __launch_bounds__(BS) void k_seg_or(const uint32_t* tiles, const uint16_t* endsT,
                                                    uint32_t ntiles, PartPlan pl, bool atomic_merge,
                                                    uint32_t* words) {
    __shared__ __attribute__((aligned(16))) uint32_t bitmap[kSegWords];
    // V = 7 (the flattened reader with the run marks, below): per wave, a byte per group slot of the
    // batch and the batch's 64 run bounds
    constexpr bool MK = V == 7;
    __shared__ __attribute__((aligned(16))) uint32_t marks[BS / 64][MK ? NG * 16 : 1];
    __shared__ __attribute__((aligned(16))) uint2 rinfo[BS / 64][MK ? 64 : 1];
    // XCD-aware order (blocks are dealt round-robin over the 8 XCDs; speed only, never
    // correctness): consecutive segments run on one XCD at the same time, and since a tile
    // stores its segments' runs back to back, they share the L2 lines those short runs sit in.
    // Blocks [0, nfull): whole segments.  The rest: the last segments split into P parts (tile
    // ranges) each, merged with word atomics -- the tail of the launch, dispatched last over all
    // XCDs, so the last round of segments does not run on a few CUs while the others idle (k = 19:
    // 1 812 segments = 7 rounds of 256 CUs + 20; launch_build_partitioned).
    uint32_t seg, part, parts;
    if (blockIdx.x < pl.nfull) {
        const uint32_t nwg = pl.nfull, q = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
        seg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + blockIdx.x / 8;
        part = 0;
        parts = 1;
    } else {
        const uint32_t r = blockIdx.x - pl.nfull;
        seg = pl.nfull + r / pl.P;
        part = r % pl.P;
        parts = pl.P;
    }
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t wbase = (uint64_t)seg * kSegWords;
    const uint32_t wn = (uint32_t)std::min<uint64_t>(kSegWords, pl.nwords - wbase);
    const bool own = parts == 1 && !atomic_merge;  // sole writer: start from the existing words
    for (uint32_t w = tid * 4; w < kSegWords; w += BS * 4) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (own && !pl.fresh && pl.ablate < 6) {
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

    const uint32_t t_lo = (uint32_t)((uint64_t)part * ntiles / parts);
    const uint32_t t_hi = (uint32_t)((uint64_t)(part + 1) * ntiles / parts);
    const uint16_t* row_end = endsT + (uint64_t)seg * pl.ntS;
    const uint16_t* row_beg = seg ? endsT + (uint64_t)(seg - 1) * pl.ntS : nullptr;
    // V 0 / 3: LPR-lane groups, one run each (RPW runs per wave per load instruction)
    static_assert(LPR == 4 || LPR == 8, "lanes per run");
    constexpr uint32_t RPW = 64 / LPR;
    static_assert(V != 3 || RPW * NG <= 64, "one coalesced bounds load per batch covers 64 tiles");
    static_assert(V != 0 || LPR == 8, "the two-stage loop deals 8-lane groups");
    const uint32_t grp = lane / LPR, q8 = lane % LPR;
    // a wave serves RPW * NG tiles per batch (NG runs per lane group)
    const uint32_t step = (BS / 64) * RPW * NG;
    uint32_t tg = t_lo + wave * RPW * NG;
    const uint32_t abl = VBF_ABLATION_BUILD ? pl.ablate : 0u;
    // groups LPR.. of a run that spans more than LPR (rare at the default plans; common for tiny m)
    auto tail = [&](uint32_t t, uint32_t st, uint32_t en) {
        const uint32_t* tile = tiles + (uint64_t)t * pl.tile_words;
#pragma unroll 1
        for (uint32_t gi = (st >> 3) + q8 + LPR; gi * 8 < en; gi += LPR) {
            uint4 lt;
            uint32_t nt;
            load_group(tile, gi, lt, nt);
            const uint32_t ab = group_range(gi, st, en);
            or_group(bitmap, lt, nt, ab & 15u, ab >> 4);
        }
    };
    auto spans_more = [](uint32_t st, uint32_t en) { return en > st && ((en + 7) >> 3) - (st >> 3) > LPR; };
    // packed bounds (begin | end << 16) of tile tg + lane, one coalesced u16 pair per lane
    auto lb = [&](uint32_t t0) -> uint32_t {
        const uint32_t t = t0 + lane;
        uint32_t v = 0;
        if (t < t_hi) v = (row_beg ? (uint32_t)row_beg[t] : 0u) | ((uint32_t)row_end[t] << 16);
        return v;
    };

    if (pl.ablate >= 5) {
        // 5-7: timing experiments, fixed costs only
    } else if constexpr (V == 6 || V == 7) {
        // Flattened groups for SHORT runs (large k or m: C / nseg entries per run): the groups of
        // a wave's 64 runs (one per tile, bounds in lane order) are dealt to lanes back to back,
        // so no lane idles on a short run.  A lane finds its run by a 6-step binary search over
        // the wave's exclusive group prefix (ds_bpermute).  Pipelined like V3: the bounds of batch
        // b+2, the group loads of batch b+1 and the ORs of batch b in flight together.  Groups
        // beyond NG * 64 per batch are loaded and ORed at consume time.
        const uint32_t wstep = (BS / 64) * 64;
        struct FB {
            uint32_t v, excl, total;
            uint4 l[NG];
            uint32_t nib[NG], ab[NG];
        };
        auto prep = [&](uint32_t v, FB& b) {
            const uint32_t st = v & 0xFFFFu, en = v >> 16;
            const uint32_t ch = en > st ? ((en + 7) >> 3) - (st >> 3) : 0u;
            uint32_t incl = ch;
            if constexpr (MK) {  // DPP: no LDS instruction
                incl = wave_incl_scan_dpp(ch);
                b.total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            } else {
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(incl, o);
                    if (lane >= (uint32_t)o) incl += y;
                }
                b.total = (uint32_t)__shfl((int)incl, 63);
            }
            b.v = v;
            b.excl = incl - ch;
        };
        // group c of the batch at t0 -> (tile, group index, live entries a | b << 4; 0 past the end)
        auto locate = [&](const FB& b, uint32_t t0, uint32_t c, const uint32_t*& tile, uint32_t& gi) -> uint32_t {
            uint32_t r = 0;
#pragma unroll
            for (int sft = 32; sft; sft >>= 1)
                if ((uint32_t)__shfl((int)b.excl, (int)r + sft) <= c) r += sft;
            const uint32_t rv = (uint32_t)__shfl((int)b.v, (int)r), rex = (uint32_t)__shfl((int)b.excl, (int)r);
            const uint32_t rst = rv & 0xFFFFu, ren = rv >> 16;
            tile = tiles + (uint64_t)std::min(t0 + r, t_hi - 1) * pl.tile_words;
            gi = (rst >> 3) + (c - rex);
            return c < b.total ? group_range(gi, rst, ren) : 0u;
        };
        auto issue = [&](uint32_t t0, FB& b) {
            if constexpr (MK) {
                // Round 6 (V = 7): the binary search costs 8 ds_bpermute per group -- more LDS
                // instructions than the group's ORs.  Instead the run marks (vbf_partition.hpp) and the
                // run's bounds from rinfo: ~2 LDS instructions per group (tools/rdg6,
                // profiles/r06/rdg6.log: -14 / -17 / -21 % at k = 10 / 19 / config 5).  Slots past
                // 64 * NG keep the search (consume).
                rinfo[wave][lane] = make_uint2(b.v, b.excl);
                run_marks_set<NG>(marks[wave], (b.v >> 16) > (b.v & 0xFFFFu), b.excl, lane);
                uint32_t carry = 0;
#pragma unroll
                for (int q = 0; q < NG; ++q) {
                    const uint32_t c = (uint32_t)q * 64 + lane;
                    const uint32_t r1 = run_marks_find(marks[wave], c, carry);
                    b.ab[q] = 0;
                    if (c < b.total) {  // r1 >= 1: some run starts at or before c
                        const uint2 ri = rinfo[wave][r1 - 1];
                        const uint32_t rst = ri.x & 0xFFFFu, ren = ri.x >> 16;
                        const uint32_t gi = (rst >> 3) + (c - ri.y);
                        b.ab[q] = group_range(gi, rst, ren);
                        load_group(tiles + (uint64_t)std::min(t0 + r1 - 1, t_hi - 1) * pl.tile_words, gi, b.l[q],
                                   b.nib[q]);
                    }
                }
            } else {
#pragma unroll
                for (int q = 0; q < NG; ++q) {
                    const uint32_t* tile;
                    uint32_t gi;
                    b.ab[q] = locate(b, t0, (uint32_t)q * 64 + lane, tile, gi);
                    if (b.ab[q]) load_group(tile, gi, b.l[q], b.nib[q]);
                }
            }
        };
        auto consume = [&](uint32_t t0, const FB& b) {
#pragma unroll
            for (int q = 0; q < NG; ++q)
                if (b.ab[q]) or_group(bitmap, b.l[q], b.nib[q], b.ab[q] & 15u, b.ab[q] >> 4, abl);
#pragma unroll 1
            for (uint32_t c0 = 64 * NG; c0 < b.total; c0 += 64) {
                const uint32_t* tile;
                uint32_t gi;
                const uint32_t ab = locate(b, t0, c0 + lane, tile, gi);
                if (ab) {
                    uint4 lt;
                    uint32_t nt;
                    load_group(tile, gi, lt, nt);
                    or_group(bitmap, lt, nt, ab & 15u, ab >> 4, abl);
                }
            }
        };
        uint32_t t0 = t_lo + wave * 64;
        FB A, B;
        uint32_t v1 = lb(t0 + wstep);
        prep(lb(t0), A);
        if (t0 < t_hi) issue(t0, A);
        while (t0 < t_hi) {
            prep(v1, B);
            uint32_t v2 = lb(t0 + 2 * wstep);
            const bool more = t0 + wstep < t_hi;
            if (more) issue(t0 + wstep, B);
            consume(t0, A);
            t0 += wstep;
            if (!more) break;
            prep(v2, A);
            v1 = lb(t0 + 2 * wstep);
            const bool more2 = t0 + wstep < t_hi;
            if (more2) issue(t0 + wstep, A);
            consume(t0, B);
            t0 += wstep;
            if (!more2) break;
        }
    } else if constexpr (V == 3) {
        struct Batch {
            uint32_t be[NG];
            uint4 l[NG];
            uint32_t nib[NG];
        };
        auto spread = [&](uint32_t v, Batch& b) {
#pragma unroll
            for (int g = 0; g < NG; ++g) b.be[g] = (uint32_t)__shfl((int)v, g * RPW + grp);
        };
        auto issue = [&](uint32_t t0, Batch& b) {
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                const uint32_t st = b.be[g] & 0xFFFFu, en = b.be[g] >> 16;
                const uint32_t t = std::min(t0 + g * RPW + grp, t_hi - 1);
                // idle lanes re-read the run's first group (same lines, always in bounds)
                const uint32_t gi = ((st >> 3) + q8) * 8 < en ? (st >> 3) + q8 : st >> 3;
                if (VBF_ABLATION_BUILD && pl.ablate == 4) {  // timing experiment: no tile loads
                    b.l[g] = make_uint4(t * 2654435761u + g, lane * 40503u, t ^ lane, gi * 977u);
                    b.nib[g] = t + lane;
                } else {
                    load_group(tiles + (uint64_t)t * pl.tile_words, gi, b.l[g], b.nib[g]);
                }
            }
        };
        auto consume = [&](uint32_t t0, const Batch& b) {
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                const uint32_t st = b.be[g] & 0xFFFFu, en = b.be[g] >> 16;
                const uint32_t ab = group_range((st >> 3) + q8, st, en);
                if (ab) or_group(bitmap, b.l[g], b.nib[g], ab & 15u, ab >> 4, abl);
            }
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                const uint32_t st = b.be[g] & 0xFFFFu, en = b.be[g] >> 16;
                if (spans_more(st, en)) tail(t0 + g * RPW + grp, st, en);
            }
        };
        Batch A, B;
        uint32_t v0 = lb(tg), v1 = lb(tg + step);
        spread(v0, A);
        if (tg < t_hi) issue(tg, A);
        // invariant at the top: A = batch tg (data in flight), v1 = bounds of tg + step
        while (tg < t_hi) {
            spread(v1, B);
            uint32_t v2 = lb(tg + 2 * step);
            const bool more = tg + step < t_hi;
            if (more) issue(tg + step, B);
            consume(tg, A);
            tg += step;
            if (!more) break;
            v1 = v2;
            spread(v1, A);
            v2 = lb(tg + 2 * step);
            const bool more2 = tg + step < t_hi;
            if (more2) issue(tg + step, A);
            consume(tg, B);
            tg += step;
            if (!more2) break;
            v1 = v2;
        }
    } else {
        // Two-stage pipeline over the wave's 64-tile batches: the run bounds of batch b+1 and the
        // data of batch b are in flight together, so each batch costs one memory latency, not two.
        auto bounds = [&](uint32_t t0, uint32_t (&st)[8], uint32_t (&en)[8]) {
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const uint32_t t = t0 + g * 8 + grp;  // the 8 lanes of a group read the same u16
                uint32_t b = 0, e = 0;
                if (t < t_hi) {
                    b = row_beg ? row_beg[t] : 0;
                    e = row_end[t];
                }
                st[g] = b;
                en[g] = e;
            }
        };
        uint32_t st[8], en[8];
        bounds(tg, st, en);
        while (tg < t_hi) {
            uint32_t nib[8], ab[8];
            uint4 l[8];
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const uint32_t gi = (st[g] >> 3) + q8;
                ab[g] = group_range(gi, st[g], en[g]);
                if (ab[g]) {
                    const uint32_t* tile = tiles + (uint64_t)(tg + g * 8 + grp) * pl.tile_words;
                    load_group(tile, gi, l[g], nib[g]);
                }
            }
            const uint32_t tn = tg + step;
            uint32_t st2[8], en2[8];
            bounds(tn, st2, en2);
#pragma unroll
            for (int g = 0; g < 8; ++g)
                if (ab[g]) or_group(bitmap, l[g], nib[g], ab[g] & 15u, ab[g] >> 4, abl);
#pragma unroll
            for (int g = 0; g < 8; ++g)
                if (spans_more(st[g], en[g])) tail(tg + g * 8 + grp, st[g], en[g]);
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                st[g] = st2[g];
                en[g] = en2[g];
            }
            tg = tn;
        }
    }
    __syncthreads();
    if (pl.ablate == 7) return;
    if (own) {
        for (uint32_t w = tid * 4; w < wn; w += BS * 4) {
            if (w + 4 <= wn)
                *reinterpret_cast<uint4*>(words + wbase + w) = *reinterpret_cast<const uint4*>(bitmap + w);
            else
                for (uint32_t x = w; x < wn; ++x) words[wbase + x] = bitmap[x];
        }
    } else {
        for (uint32_t w = tid; w < wn; w += BS) {
            const uint32_t v = bitmap[w];
            if (v) atomicOr(words + wbase + w, v);
        }
    }
}

// Tile size: the largest KT (<= kStash/k rounds of 1024 keys) whose packed LDS image fits two
// workgroups per CU; one per CU only when two cannot hold a single round of keys.
// fixed: the batch has a compile-time key length (pick_fmt > 0), which allows more stash rounds
// for some k (build_rounds_max).
// lp: the batch hashes the length prefix (Hash for [u8]; only such batches take the runtime-k
// class kernels).  group_sb != 0: the position-table pack of the probes (vbf_multi_part.hip:
// segments of 2^17 bytes of 8 interleaved filters; vbf_probe_part.hip: 2^20 filter bits) -- the
// 512-thread shape, keys in key order, runs padded to whole groups.
static PartPlan make_plan(uint32_t m, uint32_t k, bool fixed = true, bool lp = true, int group_sb = 0, bool pu = false) {
    PartPlan pl{};
    const bool group = group_sb != 0;
    const int sb = group ? group_sb : kSegBits;
    pl.k = k;
    pl.m = m;
    pl.mu = ~0ull / m;
    pl.nwords = ((uint64_t)m + 31) / 32;
    pl.nseg = (uint32_t)(((uint64_t)m + (1u << sb) - 1) >> sb);
    pl.nseg_pad = (pl.nseg + 3) & ~3u;
    // runtime k (the K = 0 kernel) keeps kStash / k rounds; compiled K values their own
    const bool ck = k == 4 || k == 9 || k == 10 || k == 19;
    // any other k <= 32 (with the length prefix) takes a runtime-k class kernel on the 512-thread
    // shape, its stash in registers (VBF_KCLASS = 0: the generic scratch-stash kernel, A/B)
    static const int kcls = [] { const char* e = getenv("VBF_KCLASS"); return e ? atoi(e) : 1; }();
    pl.kc = (!ck && kcls != 0) ? tile_pack_class(k) : 0u;
    pl.lp = lp ? 1u : 0u;
    // K1 shape (k1_shape): the 512-thread one-lane-per-key workgroups where they exist (compiled
    // k = 10 / 19, a scan of <= 4 * 512 segments), by default (profiles/r03/matrix1.log, one box:
    // k = 19 tile_sort 6.76 -> 6.24 ms; k = 10 even with packed counters, and with plain ones
    // 3.36 -> 3.28 ms, matrix7.log).  Runtime-length layouts take it with plain counters only.
    // VBF_K1 = 0 / 1 forces V = 0 / V = 1 where it exists.
    static const int k1env = [] { const char* e = getenv("VBF_K1"); return e ? atoi(e) : -1; }();
    pl.k1v = (uint32_t)((k1env >= 0 ? k1env == 1 : true) && (k == 10 || k == 19) && pl.nseg <= 4 * 512);
    if (pl.kc) pl.k1v = 1;
    if (group) {
        pl.kc = 0;
        pl.k1v = 1;
    }
    // packed u16 counters where they buy tile (VBF_C16 = 0 / 1 forces them off / on: A/B)
    static const int c16env = [] { const char* e = getenv("VBF_C16"); return e ? atoi(e) : -1; }();
    // measured: with the split image (runs padded, CP = C + nseg) they bought k = 10 its full
    // third stash round (3 020 -> 3 072 keys, +1 %, profiles/r03/ab_c16.log); the group image
    // needs no run padding and holds 3 072 keys with plain counters, which then skip the packing's
    // VALU (the 512-thread k = 19 K1: 6.18 -> 6.05 ms, matrix3.log; k = 10 even).  Only the
    // 1 024-thread k = 19 shape (two lanes per key: m > 2^31) keeps them, for its 1 536-key tile.
    // k = 4 above 2 048 segments (m = 2^32 - 1, config 5): 16 KiB of plain counters would cap the
    // tile at 6 532 keys, packed ones leave room for the 7 168 of seven stash rounds
    pl.c16 = (uint32_t)(!group && (k == 19 || k == 4 || k == 10) &&
                        (c16env >= 0 ? c16env != 0 : ((k == 19 && !pl.k1v) || (k == 4 && pl.nseg > 2048))));
    if (!fixed && pl.c16) pl.k1v = 0;
    // VBF_K1_4=1 (A/B, speed only): k = 4 at m = 2^32 - 1 with a fixed layout and packed counters on
    // the 512-thread shape -- only the SAT kernels have it (vbf_partition_sat.hip), so VBF_SAT must
    // be on as well
    static const int k14env = [] { const char* e = getenv("VBF_K1_4"); return e ? atoi(e) : 0; }();
    static const int satenv = [] { const char* e = getenv("VBF_SAT"); return e ? atoi(e) : 1; }();
    if (k14env == 1 && satenv != 0 && k == 4 && fixed && lp && m == 0xFFFFFFFFu && !group && pl.c16) pl.k1v = 1;
    // the round-6 probe pack (K1 with POS = 2, vbf_probe_pu.hip): one u32 counter per segment (the
    // run's place and padded place in its two halves)
    if (pu) {  // k = 4 at m = 2^32 - 1: the 1 024-thread shape; k = 10 / 19 keep the build's 512-thread one
        pl.c16 = 0;
        if (k == 4 && m == 0xFFFFFFFFu) {
            pl.k1v = 0;
        } else if ((k == 4 || k == 9) && kcls != 0) {  // below it the pack has no compiled k = 4 / 9: a class
            pl.kc = tile_pack_class(k);
            pl.k1v = 1;
        }
    }
    const K1Shape sh = k1_shape((int)(pl.kc ? pl.kc : k), fixed, (int)pl.k1v);
    const uint32_t rmax = (uint32_t)(ck || pl.kc ? sh.rounds : rounds_max((int)k));
    const uint32_t kpr = (uint32_t)sh.bs / (uint32_t)(ck ? sh.spl : 1);  // keys per round
    // K1 writes endsT[seg][tile] itself, no transpose pass (k = 19: -0.15 ms per 100M keys, k = 10
    // -0.025 ms; VBF_ENDS_T = 0 keeps the transpose)
    static const int etenv = [] { const char* e = getenv("VBF_ENDS_T"); return e ? atoi(e) : 1; }();
    pl.ends_t = (uint32_t)(etenv != 0);
    const uint32_t cnt_words = pl.c16 ? ((pl.nseg + 7) & ~7u) / 2 : pl.nseg_pad;
    pl.cnt_words = cnt_words;
    pl.gd_words = group ? (((pl.nseg + 1) / 2 + 3) & ~3u) : 0u;  // the group pack's u16 run table
    for (uint32_t per_cu : {2u, 1u}) {
        const uint32_t budget = kLdsPerCu / per_cu;
        const int64_t avail = (int64_t)budget - 4 * (16 + kLenBuckets) - 4 * (int64_t)cnt_words - 4 * (int64_t)pl.gd_words;
        // LDS = 2.5 * CP with CP <= C + 7 (the group pack: runs padded to whole groups in LDS,
        // up to 7 more entries per segment)
        const int64_t cmax = avail * 2 / 5 - 8 - (group ? 7 * (int64_t)pl.nseg : 0);
        const int64_t kt = std::min<int64_t>((int64_t)rmax * kpr, cmax / k);
        if (kt >= kpr || per_cu == 1) {
            pl.KT = (uint32_t)std::max<int64_t>(kt, 1);
            break;
        }
    }
    pl.R = (pl.KT + kpr - 1) / kpr;
    pl.C = pl.KT * k;
    pl.CP = (pl.C + 7) & ~7u;
    // the group pack pads every run to whole groups in HBM (<= 7 entries per segment)
    pl.CPg = group ? (pl.C + 7 * pl.nseg + 7) & ~7u : pl.CP;
    pl.tile_words = (group_words(pl.CPg) + 3) & ~3u;  // tiles start 16-byte aligned
    // VBF_TILE_PAD (speed only; default 4 words): extra words per tile in the workspace, which
    // move the tile stride off large powers of two -- k_seg_or reads the runs of consecutive tiles
    // at the same offset in each, and k = 10's 76 800-byte stride is a multiple of 1 KiB (seg_or
    // 0.848 -> 0.829 ms with 16 bytes of pad, k = 19 even; profiles/r03/matrix6.log)
    static const int tpad = [] { const char* e = getenv("VBF_TILE_PAD"); return e ? atoi(e) : 4; }();
    pl.tile_words += (uint32_t)std::max(0, tpad) & ~3u;
    pl.nsegS = (pl.nseg + 7) & ~7u;
    pl.lds1 = (group_words(group ? pl.CPg : pl.CP) + cnt_words + 16 + kLenBuckets + pl.gd_words) * 4;
    // VBF_TILE_LDS_MIN (experiments, speed only): request at least this much LDS per k_tile_pack
    // workgroup, e.g. > 80 KiB to hold one workgroup per CU
    static const int lds_min = [] { const char* e = getenv("VBF_TILE_LDS_MIN"); return e ? atoi(e) : 0; }();
    if (lds_min > 0) pl.lds1 = std::max<uint32_t>(pl.lds1, std::min<uint32_t>((uint32_t)lds_min, kLdsPerCu));
    // VBF_STAGGER = n (A/B): the second resident workgroup per CU starts n x s_sleep 127 (8128
    // cycles, ~3.7 us) later.  Off by default since round 5: with the current kernels 0 measured
    // best at k = 10 and 19 (monotonic over 0..14, two passes; configs 3 / 5 within noise,
    // profiles/r05/stagger_r5.txt, stagger_cfg_r5.txt) -- the workgroups fall out of step by
    // themselves after the first tile.
    static const int env = [] { const char* e = getenv("VBF_STAGGER"); return e ? atoi(e) : -1; }();
    const uint32_t sleeps = env >= 0 ? (uint32_t)env : 0;
    pl.stagger_lo = 256;
    pl.stagger_hi = 512;
    pl.stagger_sleeps = sleeps;
    static const int abl = [] {
        const char* e = VBF_ABLATION_BUILD ? getenv("VBF_ABLATE") : nullptr;  // vbf_kernels.hpp
        return e ? atoi(e) : 0;
    }();
    pl.ablate = (uint32_t)abl;
    static const int k3v = [] { const char* e = getenv("VBF_K3"); return e ? atoi(e) : 0; }();
    pl.k3v = (uint32_t)k3v;
    static const int lord = [] { const char* e = getenv("VBF_LEN_ORDER"); return e ? atoi(e) : 1; }();
    pl.len_order = (uint32_t)(lord != 0 && !group);  // the group pack's positions are in key order
    static const int stg = [] { const char* e = getenv("VBF_STAGE_KEYS"); return e ? atoi(e) : 1; }();
    // words: perm (KT u16) + begin + length (KT u32 each) inside the image's words
    pl.stage_keys = (uint32_t)(stg != 0 && (uint64_t)(pl.KT + 1) / 2 + 2ull * pl.KT <= group_words(pl.CP));
    return pl;
}

bool partition_supported(uint32_t m, uint32_t k) {
    if (m == 0 || k < 1 || k > (uint32_t)kStash) return false;
    for (bool fixed : {true, false})
        for (bool lp : {true, false}) {
            const PartPlan pl = make_plan(m, k, fixed, lp);
            if (pl.lds1 > kLdsPerCu || pl.CP > 65535) return false;
        }
    return true;
}

// Bit indices per build chunk: kBuildChunkIdx, or 2^VBF_BUILD_CHUNK_LOG2 (speed only: each chunk's
// k_seg_or re-reads and re-writes the whole filter, fewer chunks need a larger workspace)
static uint64_t build_chunk_idx() {
    static const uint64_t v = [] {
        const char* e = getenv("VBF_BUILD_CHUNK_LOG2");
        return e ? 1ull << std::max(20, std::min(33, atoi(e))) : kBuildChunkIdx;
    }();
    return v;
}

uint64_t build_chunk_default() { return build_chunk_idx(); }

static uint64_t chunk_keys_for(const PartPlan& pl, uint64_t n, uint64_t chunk_idx = 0) {
    const uint64_t tiles_per_chunk = std::max<uint64_t>(1, (chunk_idx ? chunk_idx : build_chunk_idx()) / pl.C);
    return std::min<uint64_t>(n, tiles_per_chunk * pl.KT);
}

// Bytes of workspace one launch_build_partitioned call needs for n keys.
uint64_t partition_workspace_bytes(uint64_t n, uint32_t m, uint32_t k, uint64_t chunk_idx) {
    if (!partition_supported(m, k)) return 0;
    uint64_t need = 0;
    for (bool fixed : {true, false})  // the largest of the layouts' plans
        for (bool lp : {true, false}) {
            const PartPlan pl = make_plan(m, k, fixed, lp);
            const uint64_t ntiles = (chunk_keys_for(pl, n, chunk_idx) + pl.KT - 1) / pl.KT;
            // tiles, then ends[ntiles][nsegS] and endsT[nsegS][ntiles rounded up to 8] (16-byte aligned)
            need = std::max<uint64_t>(need,
                                      ntiles * (uint64_t)pl.tile_words * 4 + (ntiles + 8) * (uint64_t)pl.nsegS * 4 + 512);
        }
    return need;
}

bool partition_fresh_ok(uint64_t n, uint32_t m, uint32_t k, uint64_t chunk_idx) {
    if (!partition_supported(m, k) || n == 0) return false;
    for (bool fixed : {true, false})
        for (bool lp : {true, false}) {
            const PartPlan pl = make_plan(m, k, fixed, lp);
            const uint64_t ck = chunk_keys_for(pl, n, chunk_idx);
            const uint64_t ntiles = (ck + pl.KT - 1) / pl.KT;
            const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)ntiles, (512 + pl.nseg - 1) / pl.nseg));
            if (ck < n || G > 1) return false;
        }
    return true;
}

// ---- the position-table pack of the probes: K1 with 2^sb-position segments ----
bool group_pack_supported(uint64_t m, uint32_t k, int sb) {
    if (m == 0 || m > (2048ull << sb) || m > (1ull << 31) || (k != 10 && k != 19)) return false;  // <= 2 048 segments
    for (bool fixed : {true, false}) {
        const PartPlan pl = make_plan((uint32_t)m, k, fixed, true, sb);
        if (pl.lds1 > kLdsPerCu / 2 || pl.CPg > 65535 || pl.nseg > 4 * 512) return false;
        // the worst-case run padding (7 entries per segment) must leave the tile most of the LDS:
        // at k = 19, m = 1.9e9 (1 812 segments) it would take half of it, the tile would drop to
        // 823 keys and the segment pass would read 2.7x the runs (measured slower than the round-3
        // probe: 15.4 vs 14.2 ms per 100M positives, profiles/r04/bench_k19.log)
        if (7ull * pl.nseg * 20 > 9ull * pl.C) return false;
    }
    return true;
}

PartPlan make_group_plan(uint32_t m, uint32_t k, bool fixed, int sb) { return make_plan(m, k, fixed, true, sb); }

PartPlan make_probe_pu_plan(uint32_t m, uint32_t k, bool fixed, bool lp) {
    PartPlan pl = make_plan(m, k, fixed, lp, 0, true);
    pl.stage_keys = 0;  // the tile image holds the length order's perm only (written out before placement)
    return pl;
}

uint32_t group_pack_slots(uint32_t k) {
    const K1Shape sh = k1_shape((int)k, true, 1);
    return (uint32_t)(sh.rounds * sh.kl);
}

hipError_t launch_group_pack(const KeyBatch& kb, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                             uint32_t* tiles, uint16_t* endsT, uint16_t* posv, int sb, hipStream_t s) {
    hipError_t err = hipErrorInvalidValue;
    if (!kb.len_prefix || (pl.k != 10 && pl.k != 19) || pl.k1v != 1 || !pl.ends_t) return err;
    if (sb != kByteSegBits && sb != kSegBits) return err;
    with_fmt(pick_fmt(dk.keys, dk.offsets, dk.stride), true, [&]<int FMT, bool LP>() {
        if constexpr (LP) {
            auto fn = sb == kByteSegBits
                          ? (pl.k == 10 ? k_tile_pack<FMT, true, 10, true, false, 1, 0, kByteSegBits, true>
                                        : k_tile_pack<FMT, true, 19, true, false, 1, 0, kByteSegBits, true>)
                          : (pl.k == 10 ? k_tile_pack<FMT, true, 10, true, false, 1, 0, kSegBits, true>
                                        : k_tile_pack<FMT, true, 19, true, false, 1, 0, kSegBits, true>);
            hipFuncAttributes fa{};
            err = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(fn));
            if (err == hipSuccess && fa.sharedSizeBytes != 0) err = hipErrorInvalidKernelFile;
            if (err == hipSuccess)
                err = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.lds1);
            if (err == hipSuccess) {
                hipLaunchKernelGGL(fn, dim3(ntiles), dim3(512), pl.lds1, s, dk, pl, tiles, endsT, posv);
                err = hipGetLastError();
            }
        }
    });
    return err;
}

hipError_t launch_tile_pack_main(int fmt, bool lp, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                 uint32_t* tiles, uint16_t* ends, hipStream_t s) {
    switch (fmt) {
        case 16: case 32: return launch_tile_pack_main_a(fmt, lp, dk, pl, ntiles, tiles, ends, s);
        case 8: case 24: return launch_tile_pack_main_b(fmt, lp, dk, pl, ntiles, tiles, ends, s);
        default: return launch_tile_pack_main_c(fmt, lp, dk, pl, ntiles, tiles, ends, s);
    }
}

hipError_t launch_build_partitioned(const KeyBatch& kb, uint32_t m, uint32_t k, uint32_t* words,
                                    void* ws, uint64_t ws_bytes, bool atomic_merge, hipStream_t s, bool fresh,
                                    uint64_t chunk_idx) {
    if (kb.n == 0 || k == 0) return hipSuccess;
    if (!partition_supported(m, k)) return hipErrorInvalidValue;
    // every chunk keeps the batch's alignment (chunks are whole tiles of keys), so one layout
    PartPlan pl = make_plan(m, k, pick_fmt(kb.keys, kb.offsets, kb.stride) > 0, kb.len_prefix);
    const uint64_t chunk_keys = chunk_keys_for(pl, kb.n, chunk_idx);
    const uint64_t max_tiles = (chunk_keys + pl.KT - 1) / pl.KT;
    if (ws_bytes < partition_workspace_bytes(kb.n, m, k, chunk_idx)) return hipErrorInvalidValue;
    uint32_t* tiles = reinterpret_cast<uint32_t*>(ws);
    uint16_t* ends = reinterpret_cast<uint16_t*>(
        (reinterpret_cast<uintptr_t>(tiles + max_tiles * pl.tile_words) + 15) & ~(uintptr_t)15);
    uint16_t* endsT = ends + max_tiles * pl.nsegS;  // nsegS % 8 == 0: stays 16-byte aligned

    for (uint64_t lo = 0; lo < kb.n; lo += chunk_keys) {
        const uint64_t cn = std::min<uint64_t>(chunk_keys, kb.n - lo);
        DevKeys dk{kb.keys, kb.offsets, kb.off_base, kb.stride, cn};
        if (kb.offsets)
            dk.offsets = kb.offsets + lo;
        else
            dk.keys = kb.keys + lo * kb.stride;
        const uint32_t ntiles = (uint32_t)((cn + pl.KT - 1) / pl.KT);
        pl.ntS = (ntiles + 7) & ~7u;
        hipError_t err = hipSuccess;
        phase_begin(kPhaseTileSort, s);
        if (pl.kc) {  // a runtime-k class kernel (translation units of their own)
            const int fmt = pick_fmt(dk.keys, dk.offsets, dk.stride);
            uint16_t* e = pl.ends_t ? endsT : ends;
            err = pl.kc <= 12 ? (pl.lp ? launch_tile_pack_class_a(fmt, dk, pl, ntiles, tiles, e, s)
                                       : launch_tile_pack_class_c(fmt, dk, pl, ntiles, tiles, e, s))
                              : (pl.lp ? launch_tile_pack_class_b(fmt, dk, pl, ntiles, tiles, e, s)
                                       : launch_tile_pack_class_d(fmt, dk, pl, ntiles, tiles, e, s));
        } else if (kb.len_prefix && m == 0xFFFFFFFFu &&
                   (err = launch_tile_pack_sat(pick_fmt(dk.keys, dk.offsets, dk.stride), dk, pl, ntiles, tiles,
                                               pl.ends_t ? endsT : ends, s)) != hipErrorNotSupported) {
            // m = 2^32 - 1 (the reference's saturated size): end-around-carry remainders (SAT kernels)
        } else {
            err = launch_tile_pack_main(pick_fmt(dk.keys, dk.offsets, dk.stride), kb.len_prefix, dk, pl, ntiles, tiles,
                                        pl.ends_t ? endsT : ends, s);
        }
        if (err != hipSuccess) return err;
        phase_end(kPhaseTileSort, s);
        if (!pl.ends_t) {
            phase_begin(kPhaseTranspose, s);
            err = launch_transpose_u16_strided(ends, endsT, ntiles, pl.nseg, pl.nsegS, pl.ntS, s);
            if (err != hipSuccess) return err;
            phase_end(kPhaseTranspose, s);
        }
        // several workgroups per segment when there are few segments (small m)
        pl.G = std::max<uint32_t>(1, std::min<uint32_t>(ntiles, (512 + pl.nseg - 1) / pl.nseg));
        const bool merge = atomic_merge || pl.G > 1;
        // only the first chunk, and only where each segment has one sole writer, skips the read
        pl.fresh = (fresh && lo == 0 && !merge) ? 1u : 0u;
        if (fresh && lo == 0 && merge) return hipErrorInvalidValue;  // the caller zeroes first
        // K3 runs one workgroup per CU (128 KiB of LDS); when the segments leave a last round of
        // few workgroups (nseg % CUs small), those segments are split over several workgroups each
        pl.nfull = pl.G > 1 ? 0u : pl.nseg;
        pl.P = pl.G;
        if (pl.G == 1 && tail_split_enabled()) {
            const uint32_t ncu = device_cu_count(), rem = ncu ? pl.nseg % ncu : 0u;
            if (pl.nseg > ncu && rem > 0 && ncu / rem >= 2) {
                pl.P = std::min<uint32_t>(std::min<uint32_t>(ncu / rem, 16u), ntiles);
                pl.nfull = pl.nseg - rem;
            }
        }
        if (pl.fresh && pl.nfull < pl.nseg) {  // the split segments' words: zero, then ORed into
            const uint64_t w0 = (uint64_t)pl.nfull * kSegWords;
            err = hipMemsetAsync(words + w0, 0, (pl.nwords - w0) * 4, s);
            if (err != hipSuccess) return err;
        }
        phase_begin(kPhaseSegOr, s);
        // the flattened variant, NG = 4 for short runs (large k or m), 5 otherwise (group layout,
        // profiles/r03/matrix1.log: k = 10 seg_or 1.011 (V3) -> 0.861 ms, k = 19 NG 4 2.26 vs NG 5
        // 2.34 ms), with the run marks since round 6 (V7); VBF_K3 overrides (10 / 11: round 5's)
        const uint32_t k3v = pl.k3v ? pl.k3v : (pl.C / std::max(pl.nseg, 1u) < kShortRun ? 14u : 15u);
        auto k3 = k3v == 14 ? k_seg_or<7, kPBlock, 4>
                : k3v == 15 ? k_seg_or<7, kPBlock, 5>
                : k3v == 16 ? k_seg_or<7, kPBlock, 6>
                : k3v == 13 ? k_seg_or<3, kPBlock, 4, 4>
                : k3v == 10 ? k_seg_or<6, kPBlock, 4>
                : k3v == 11 ? k_seg_or<6, kPBlock, 5>
                : k3v == 12 ? k_seg_or<6, kPBlock, 6>
                : k3v == 8 ? k_seg_or<3, kPBlock, 6>
                : k3v == 3 ? k_seg_or<3, kPBlock, 4>
                : k3v == 5 ? k_seg_or<3, 768, 6>
                : k3v == 6 ? k_seg_or<3, 768, 8>
                : k3v == 1 ? k_seg_or<0>
                           : k_seg_or<3, kPBlock, 5>;
        const int bs = (k3v == 5 || k3v == 6) ? 768 : kPBlock;
        // VBF_K3_PASSES = q (experiments, speed only): the segment pass in q launches over consecutive
        // tile windows -- each launch boundary re-aligns the workgroups that share tile lines in an
        // XCD's L2 (they drift apart within one launch); every window after the first reads the
        // segment's words back (the previous window's result) and writes them again
        static const uint32_t k3passes = [] {
            const char* e = getenv("VBF_K3_PASSES");
            return (uint32_t)std::max(1, e ? atoi(e) : 1);
        }();
        const uint32_t passes = std::max<uint32_t>(1, std::min<uint32_t>(k3passes, ntiles / std::max<uint32_t>(pl.P, 16)));
        for (uint32_t ps = 0; ps < passes; ++ps) {
            const uint32_t a = (uint32_t)((uint64_t)ntiles * ps / passes), b = (uint32_t)((uint64_t)ntiles * (ps + 1) / passes);
            PartPlan pp = pl;
            if (ps > 0) pp.fresh = 0;
            hipLaunchKernelGGL(k3, dim3(pl.nfull + (pl.nseg - pl.nfull) * pl.P), dim3(bs), 0, s,
                               tiles + (uint64_t)a * pl.tile_words, endsT + a, b - a, pp, merge, words);
        }
        phase_end(kPhaseSegOr, s);
        err = hipGetLastError();
        if (err != hipSuccess) return err;
    }
    return hipSuccess;
}
}  // namespace vbf
