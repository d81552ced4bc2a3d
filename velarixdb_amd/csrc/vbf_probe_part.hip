// vbf_probe_part.hip -- the partitioned probe (contains() for large batches): the build's
// tile/segment scheme (vbf_partition.hip) applied to lookups.
#include "vbf_probe_pack.hpp"
#include "vbf_tile_pack_rk.hpp"

namespace vbf {

// =================================================================================================
// Partitioned probe (contains() for large batches, bf.rs:95-105).  The same idea as the build:
// random filter loads (~55 G/s chip-wide) become LDS bit tests.
//   Q1 k_probe_pack : per tile of keys, hash all k indices, sort the entries (tile-local key id
//                     << 20 | offset in segment) by 2^20-bit segment in LDS, write each run padded
//                     to a multiple of 8 entries (repeating its last entry) + the padded run ends.
//   (K2 transpose of the run ends, shared with the build)
//   Q3 k_probe_seg  : one workgroup per segment loads the segment's 128 KiB of filter words into
//                     LDS once and tests every tile's run against it, 8 entries -> 1 result byte.
//   Q4 k_probe_out  : per tile, AND each key's k results (a clear bit anywhere -> false) and write
//                     the answer byte (or count the hits).
// Without early exit every key costs k hashes, but no probe leaves the chip's LDS.
// =================================================================================================
// Q3 variants (VBF_Q3, speed only; identical answers):
//   0: one pass per 8-lane group and tile, 8 tiles per wave-step
//   1: the k_seg_or<3> scheme -- a wave serves 8 * NG tiles per batch, run bounds loaded
//      coalesced and spread with ds_bpermute, bounds of b+2 / entries of b+1 / bit tests of b in
//      flight together, unconditional entry loads (idle lanes re-read their run's start)
// Blocks [0, nfull): whole segments, XCD-aware.  The rest: segments [nfull, nseg) split into P
// tile ranges each (every segment when segments are few; otherwise the last, short round of
// segment workgroups, spread over the idle CUs).  Results are per entry, so parts need no merge:
// a split costs only the segment's filter words loaded once more per part.
template <int V, int NG = 4>
__global__ __launch_bounds__(kPBlock) void k_probe_seg(const uint32_t* tiles, const uint16_t* endsT, uint32_t ntiles,
                                                       ProbePlan pl, uint32_t nfull, uint32_t P, const uint32_t* words,
                                                       uint8_t* res) {
    __shared__ __attribute__((aligned(16))) uint32_t bitmap[kSegWords];
    uint32_t seg, part, parts;
    if (blockIdx.x < nfull) {
        const uint32_t qq = nfull / 8, r8 = nfull % 8, xcd = blockIdx.x % 8;
        seg = (xcd < r8 ? xcd * (qq + 1) : r8 * (qq + 1) + (xcd - r8) * qq) + blockIdx.x / 8;
        part = 0;
        parts = 1;
    } else {
        const uint32_t r = blockIdx.x - nfull;
        seg = nfull + r / P;
        part = r % P;
        parts = P;
    }
    const uint32_t t_lo = (uint32_t)((uint64_t)part * ntiles / parts);
    const uint32_t t_hi = (uint32_t)((uint64_t)(part + 1) * ntiles / parts);
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t wbase = (uint64_t)seg * kSegWords;
    const uint32_t wn = (uint32_t)std::min<uint64_t>(kSegWords, pl.nwords - wbase);
    for (uint32_t w = tid * 4; w < kSegWords; w += kPBlock * 4) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (w + 4 <= wn) {
            v = *reinterpret_cast<const uint4*>(words + wbase + w);
        } else if (w < wn) {
            v.x = words[wbase + w];
            if (w + 1 < wn) v.y = words[wbase + w + 1];
            if (w + 2 < wn) v.z = words[wbase + w + 2];
        }
        *reinterpret_cast<uint4*>(bitmap + w) = v;
    }
    __syncthreads();
    const uint16_t* row_end = endsT + (uint64_t)seg * ntiles;
    const uint16_t* row_beg = seg ? endsT + (uint64_t)(seg - 1) * ntiles : nullptr;
    const uint32_t grp = lane >> 3, q8 = (lane & 7) * 8;
    // 8 entries -> 1 result byte (bit c = entry c's filter bit)
    auto test8 = [&](const uint4& a, const uint4& b) -> uint32_t {
        const uint32_t e[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t r = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint32_t off = e[c] & kOffMask;
            r |= ((bitmap[off >> 5] >> (off & 31)) & 1u) << c;
        }
        return r;
    };
    if constexpr (V == 1) {
        const uint32_t step = (kPBlock / 64) * 8 * NG;
        uint32_t tg = t_lo + wave * 8 * NG;
        auto lb = [&](uint32_t t0) -> uint32_t {
            const uint32_t t = t0 + lane;
            uint32_t v = 0;
            if (t < t_hi) v = (row_beg ? (uint32_t)row_beg[t] : 0u) | ((uint32_t)row_end[t] << 16);
            return v;
        };
        struct Batch {
            uint32_t be[NG];
            uint4 a[NG], b[NG];
        };
        auto spread = [&](uint32_t v, Batch& bt) {
#pragma unroll
            for (int g = 0; g < NG; ++g) bt.be[g] = (uint32_t)__shfl((int)v, g * 8 + grp);
        };
        auto issue = [&](uint32_t t0, Batch& bt) {
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                const uint32_t st = bt.be[g] & 0xFFFFu, len = (bt.be[g] >> 16) - st;
                const uint32_t t = std::min(t0 + g * 8 + grp, t_hi - 1);
                const uint32_t x = q8 < len ? st + q8 : st;
                const uint32_t* run = tiles + (uint64_t)t * pl.cap + x;
                bt.a[g] = *reinterpret_cast<const uint4*>(run);
                bt.b[g] = *reinterpret_cast<const uint4*>(run + 4);
            }
        };
        auto consume = [&](uint32_t t0, const Batch& bt) {
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                const uint32_t st = bt.be[g] & 0xFFFFu, len = (bt.be[g] >> 16) - st;
                const uint64_t t = t0 + g * 8 + grp;
                if (q8 < len) {
                    const uint32_t r = test8(bt.a[g], bt.b[g]);
                    if (r != 0xFFu) res[(t * pl.cap + st + q8) >> 3] = (uint8_t)r;  // bytes start all ones
                }
            }
#pragma unroll
            for (int g = 0; g < NG; ++g) {  // runs longer than 64 entries
                const uint32_t st = bt.be[g] & 0xFFFFu, len = (bt.be[g] >> 16) - st;
                const uint64_t t = t0 + g * 8 + grp;
#pragma unroll 1
                for (uint32_t x = st + q8 + 64; x < st + len; x += 64) {
                    const uint32_t* run = tiles + t * pl.cap + x;
                    const uint32_t r =
                        test8(*reinterpret_cast<const uint4*>(run), *reinterpret_cast<const uint4*>(run + 4));
                    if (r != 0xFFu) res[(t * pl.cap + x) >> 3] = (uint8_t)r;
                }
            }
        };
        Batch A, B;
        uint32_t v0 = lb(tg), v1 = lb(tg + step);
        spread(v0, A);
        if (tg < t_hi) issue(tg, A);
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
        // 8-lane group per tile, 8 tiles per wave-step: each lane tests 8 entries -> 1 byte
        for (uint32_t t = t_lo + wave * 8 + grp; t < t_hi; t += (kPBlock / 64) * 8) {
            const uint32_t beg = row_beg ? row_beg[t] : 0, end = row_end[t];
            const uint32_t* run = tiles + (uint64_t)t * pl.cap;
            for (uint32_t x = beg + q8; x < end; x += 64) {
                const uint4 a = *reinterpret_cast<const uint4*>(run + x);
                const uint4 b = *reinterpret_cast<const uint4*>(run + x + 4);
                const uint32_t r = test8(a, b);
                if (r != 0xFFu) res[((uint64_t)t * pl.cap + x) >> 3] = (uint8_t)r;
            }
        }
    }
}

// OUT: 0 answer bytes, 1 hit count.
template <int OUT>
__global__ __launch_bounds__(kPBlock) void k_probe_out(const uint32_t* tiles, const uint16_t* ends, const uint8_t* res,
                                                       ProbePlan pl, uint64_t n, uint8_t* out, uint32_t* partial) {
    __shared__ uint32_t ok[4096 / 32];
    __shared__ uint32_t wsum[kPBlock / 64];
    const uint32_t tid = threadIdx.x;
    const uint64_t key0 = (uint64_t)blockIdx.x * pl.KT;
    const uint32_t nk = (uint32_t)std::min<uint64_t>(pl.KT, n - key0);
    for (uint32_t w = tid; w < (nk + 31) / 32; w += kPBlock) ok[w] = 0xFFFFFFFFu;
    __syncthreads();
    const uint32_t total = ends[(uint64_t)blockIdx.x * pl.nseg + pl.nseg - 1];
    const uint32_t* tl = tiles + (uint64_t)blockIdx.x * pl.cap;
    // 32 result bits per lane (cap is a multiple of 32, so each tile's bytes are dword aligned);
    // only the clear bits -- entries whose filter bit is 0 -- cost a tile read and an LDS AND
    const uint32_t* rs = reinterpret_cast<const uint32_t*>(res + ((uint64_t)blockIdx.x * pl.cap >> 3));
    for (uint32_t w = tid; w * 32 < total; w += kPBlock) {
        const uint32_t valid = std::min<uint32_t>(32, total - w * 32);
        uint32_t z = ~rs[w];
        if (valid < 32) z &= (1u << valid) - 1u;
        while (z) {
            const uint32_t c = __builtin_ctz(z);
            z &= z - 1;
            const uint32_t local = tl[w * 32 + c] >> kSegBits;
            atomicAnd(&ok[local >> 5], ~(1u << (local & 31)));
        }
    }
    __syncthreads();
    if constexpr (OUT == 0) {
        for (uint32_t l = tid; l < nk; l += kPBlock) out[key0 + l] = (ok[l >> 5] >> (l & 31)) & 1u;
    } else {  // hits of the tile -> partial[tile] (summed by one finishing workgroup)
        uint32_t c = 0;
        for (uint32_t w = tid; w < (nk + 31) / 32; w += kPBlock) {
            const uint32_t valid = (w + 1) * 32 <= nk ? 0xFFFFFFFFu : ((1u << (nk & 31)) - 1u);
            c += __popc(ok[w] & valid);
        }
        for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
        if ((tid & 63) == 0) wsum[tid >> 6] = c;
        __syncthreads();
        if (tid == 0) {
            uint32_t t = 0;
            for (int w = 0; w < kPBlock / 64; ++w) t += wsum[w];
            partial[blockIdx.x] = t;
        }
    }
}

// ---- Round 4: the partitioned probe on the build's image (k = 10 / 19 with the length prefix,
// m <= 2^31; VBF_PROBE_GP = 0 keeps the pipeline above) ----
// PP1 launch_group_pack(sb = 20): k_tile_pack writing the 2.5-byte 8-entry group image with every
// run padded to whole groups, the padded run ends transposed, and every entry's padded place in
// posv (u16 pairs per stash slot pair and lane).
// PP3 k_probe_seg2: k_seg_or's flattened reader over a segment's runs (whole groups): a group's 8
// filter bits -> one result byte at res[tile][group] (no run shares a group, so one plain store).
// PP4 k_probe_out2: the tile's result bits staged in LDS, each key's k bits found through posv and
// ANDed: the answer byte, or the tile's hit count.
template <int NG = 4>
__global__ __launch_bounds__(kPBlock) void k_probe_seg2(const uint32_t* tiles, const uint16_t* endsT, uint32_t ntiles,
                                                        PartPlan pl, uint32_t G, const uint32_t* words, uint8_t* res) {
    __shared__ __attribute__((aligned(16))) uint32_t bitmap[kSegWords];
    __shared__ __attribute__((aligned(16))) uint32_t marks[kPBlock / 64][NG * 16];
    __shared__ __attribute__((aligned(16))) uint2 rinfo[kPBlock / 64][64];
    const uint32_t nwg = gridDim.x, qq = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
    const uint32_t wg = (xcd < r8 ? xcd * (qq + 1) : r8 * (qq + 1) + (xcd - r8) * qq) + blockIdx.x / 8;
    const uint32_t seg = wg / G, part = wg % G;
    const uint32_t t_lo = (uint32_t)((uint64_t)part * ntiles / G), t_hi = (uint32_t)((uint64_t)(part + 1) * ntiles / G);
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t wbase = (uint64_t)seg * kSegWords;
    const uint32_t wn = (uint32_t)std::min<uint64_t>(kSegWords, pl.nwords - wbase);
    for (uint32_t w = tid * 4; w < kSegWords; w += kPBlock * 4) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (w + 4 <= wn) {
            v = *reinterpret_cast<const uint4*>(words + wbase + w);
        } else if (w < wn) {
            v.x = words[wbase + w];
            if (w + 1 < wn) v.y = words[wbase + w + 1];
            if (w + 2 < wn) v.z = words[wbase + w + 2];
        }
        *reinterpret_cast<uint4*>(bitmap + w) = v;
    }
    __syncthreads();
    const uint16_t* row_end = endsT + (uint64_t)seg * pl.ntS;
    const uint16_t* row_beg = seg ? endsT + (uint64_t)(seg - 1) * pl.ntS : nullptr;
    const uint32_t rstride = pl.CPg / 8;  // result bytes per tile
    auto lb = [&](uint32_t t0) -> uint32_t {
        const uint32_t t = t0 + lane;
        uint32_t v = 0;
        if (t < t_hi) v = (row_beg ? (uint32_t)row_beg[t] : 0u) | ((uint32_t)row_end[t] << 16);
        return v;
    };
    auto answer = [&](uint32_t t, uint32_t gi, uint4 l, uint32_t nib) {
        const uint32_t w[4] = {l.x, l.y, l.z, l.w};
        uint32_t r = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint32_t off = ((w[c >> 1] >> ((c & 1) * 16)) & 0xFFFFu) | (((nib >> (4 * c)) & 15u) << 16);
            r |= ((bitmap[off >> 5] >> (off & 31)) & 1u) << c;
        }
        if (r != 0xFFu) res[(uint64_t)t * rstride + gi] = (uint8_t)r;  // bytes start all ones
    };
    const uint32_t wstep = (kPBlock / 64) * 64;
    struct FB {
        uint32_t v, excl, total;
        uint4 l[NG];
        uint32_t nib[NG], ok[NG], t[NG], gi[NG];
    };
    auto prep = [&](uint32_t v, FB& b) {  // padded runs: whole groups
        const uint32_t ch = ((v >> 16) - (v & 0xFFFFu)) >> 3;
        const uint32_t incl = wave_incl_scan_dpp(ch);
        b.v = v;
        b.excl = incl - ch;
        b.total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    };
    auto locate = [&](const FB& b, uint32_t t0, uint32_t c, uint32_t& t, uint32_t& gi) -> uint32_t {
        uint32_t r = 0;
#pragma unroll
        for (int sft = 32; sft; sft >>= 1)
            if ((uint32_t)__shfl((int)b.excl, (int)r + sft) <= c) r += sft;
        const uint32_t rv = (uint32_t)__shfl((int)b.v, (int)r), rex = (uint32_t)__shfl((int)b.excl, (int)r);
        t = std::min(t0 + r, t_hi - 1);
        gi = ((rv & 0xFFFFu) >> 3) + (c - rex);
        return c < b.total ? 1u : 0u;
    };
    auto issue = [&](uint32_t t0, FB& b) {  // round 6: the run marks (vbf_partition.hpp)
        rinfo[wave][lane] = make_uint2(b.v, b.excl);
        run_marks_set<NG>(marks[wave], (b.v >> 16) > (b.v & 0xFFFFu), b.excl, lane);
        uint32_t carry = 0;
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            const uint32_t c = (uint32_t)q * 64 + lane;
            const uint32_t r1 = run_marks_find(marks[wave], c, carry);
            b.ok[q] = c < b.total ? 1u : 0u;
            if (b.ok[q]) {
                const uint2 ri = rinfo[wave][r1 - 1];
                b.t[q] = std::min(t0 + r1 - 1, t_hi - 1);
                b.gi[q] = ((ri.x & 0xFFFFu) >> 3) + (c - ri.y);
                const uint32_t* tile = tiles + (uint64_t)b.t[q] * pl.tile_words;
                __builtin_memcpy(&b.l[q], tile + b.gi[q] * 5, 16);
                b.nib[q] = tile[b.gi[q] * 5 + 4];
            }
        }
    };
    auto consume = [&](uint32_t t0, const FB& b) {
#pragma unroll
        for (int q = 0; q < NG; ++q)
            if (b.ok[q]) answer(b.t[q], b.gi[q], b.l[q], b.nib[q]);
#pragma unroll 1
        for (uint32_t c0 = 64 * NG; c0 < b.total; c0 += 64) {
            uint32_t t, gi;
            if (locate(b, t0, c0 + lane, t, gi)) {
                const uint32_t* tile = tiles + (uint64_t)t * pl.tile_words;
                uint4 l;
                __builtin_memcpy(&l, tile + gi * 5, 16);
                answer(t, gi, l, tile[gi * 5 + 4]);
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
}

// PP4 (OUT 0: answer bytes, 1: hits of the tile -> partial[tile]).  K compile-time: a lane issues the
// position loads of its KPT keys together.
template <int K, int KPT, int OUT>
__global__ __launch_bounds__(kPBlock) void k_probe_out2(const uint8_t* res, const uint32_t* posv, PartPlan pl,
                                                        uint32_t pairs, uint64_t n, uint8_t* out, uint32_t* partial) {
    __shared__ uint32_t rl32[65536 / 8 / 4];  // the tile's result bits (<= CPg / 8 bytes)
    __shared__ uint32_t wsum[kPBlock / 64];
    const uint8_t* rl = reinterpret_cast<const uint8_t*>(rl32);
    const uint32_t tid = threadIdx.x, tile = blockIdx.x;
    const uint64_t key0 = (uint64_t)tile * pl.KT;
    const uint32_t nk = (uint32_t)std::min<uint64_t>(pl.KT, n - key0);
    const uint32_t rbytes = pl.CPg / 8;
    const uint8_t* src = res + (uint64_t)tile * rbytes;
    uint32_t all = 0xFFu;
    for (uint32_t b = tid; b < rbytes; b += kPBlock) {
        const uint8_t v = src[b];
        reinterpret_cast<uint8_t*>(rl32)[b] = v;
        all &= v;
    }
    // no failing entry in the tile (the segment pass stored none of its result bytes): every key
    // passes without reading the position table
    if (__syncthreads_and(all == 0xFFu)) {
        if constexpr (OUT == 0) {
            for (uint32_t l = tid; l < nk; l += kPBlock) out[key0 + l] = 1;
        } else if (tid == 0) {
            partial[blockIdx.x] = nk;
        }
        return;
    }
    const uint32_t* pt = posv + (uint64_t)tile * pairs * 512;
    constexpr int NW = K / 2 + 1;
    uint32_t wv[KPT][NW];
#pragma unroll
    for (int x = 0; x < KPT; ++x) {
        const uint32_t l = tid + x * kPBlock;
        const uint32_t r = l >> 9, ln = l & 511u;
        const uint32_t wb = (r * K) >> 1;
#pragma unroll
        for (int j = 0; j < NW; ++j) wv[x][j] = (l < nk && wb + j < pairs) ? pt[(wb + j) * 512 + ln] : 0u;
    }
    auto bit_at = [&](int x, int i, uint32_t odd) -> uint32_t {
        const uint32_t q = odd + (uint32_t)i;
        const uint32_t p = (wv[x][q >> 1] >> ((q & 1u) * 16)) & 0xFFFFu;
        return (rl[p >> 3] >> (p & 7)) & 1u;
    };
    uint32_t hits = 0;
#pragma unroll
    for (int x = 0; x < KPT; ++x) {
        const uint32_t l = tid + x * kPBlock;
        if (l >= nk) break;
        uint32_t ok = 1;
        const uint32_t odd = ((l >> 9) * K) & 1u;
        if (odd) {
#pragma unroll
            for (int i = 0; i < K; ++i) ok &= bit_at(x, i, 1u);
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) ok &= bit_at(x, i, 0u);
        }
        if constexpr (OUT == 0) out[key0 + l] = (uint8_t)ok;
        else hits += ok;
    }
    if constexpr (OUT == 1) {
        for (int o = 32; o > 0; o >>= 1) hits += __shfl_down(hits, o);
        if ((tid & 63) == 0) wsum[tid >> 6] = hits;
        __syncthreads();
        if (tid == 0) {
            uint32_t t = 0;
            for (int w = 0; w < kPBlock / 64; ++w) t += wsum[w];
            partial[blockIdx.x] = t;
        }
    }
}

static bool pp_enabled(uint32_t m, uint32_t k, bool lp) {
    const char* e = getenv("VBF_PROBE_GP");  // read per call (A/B)
    return (e ? atoi(e) : 1) != 0 && lp && group_pack_supported(m, k, kSegBits);
}

static uint64_t pp_chunk_keys(const PartPlan& pl, uint64_t n) {
    const uint64_t tiles_per_chunk = std::max<uint64_t>(1, kPartChunkIdx / pl.C);
    return std::min<uint64_t>(n, tiles_per_chunk * pl.KT);
}

// tiles, endsT[nseg][ntS], res[tiles][CPg / 8], posv (u16 pairs), partial counts
static uint64_t pp_workspace_bytes(uint64_t n, uint32_t m, uint32_t k) {
    uint64_t need = 0;
    for (bool fixed : {true, false}) {
        const PartPlan pl = make_group_plan(m, k, fixed, kSegBits);
        const uint64_t nt = (pp_chunk_keys(pl, n) + pl.KT - 1) / pl.KT, ntS = (nt + 7) & ~7ull;
        need = std::max<uint64_t>(need, nt * (uint64_t)pl.tile_words * 4 + ntS * pl.nseg * 2 + nt * (pl.CPg / 8) +
                                            nt * (uint64_t)((group_pack_slots(k) + 1) / 2) * 512 * 4 + nt * 4 +
                                            5 * 256);
    }
    return need;
}

static hipError_t launch_probe_pp(const KeyBatch& kb, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
                                  unsigned long long* count, void* ws, hipStream_t s) {
    auto align256 = [](uint64_t x) { return (x + 255) & ~255ull; };
    PartPlan pl = make_group_plan(m, k, pick_fmt(kb.keys, kb.offsets, kb.stride) > 0, kSegBits);
    const uint32_t pairs = (group_pack_slots(k) + 1) / 2;
    const uint64_t chunk_keys = pp_chunk_keys(pl, kb.n);
    const uint64_t max_tiles = (chunk_keys + pl.KT - 1) / pl.KT, max_ntS = (max_tiles + 7) & ~7ull;
    char* base = static_cast<char*>(ws);
    const uint64_t o_ends = align256(max_tiles * pl.tile_words * 4);
    const uint64_t o_res = align256(o_ends + max_ntS * pl.nseg * 2);
    const uint64_t o_pos = align256(o_res + max_tiles * (pl.CPg / 8));
    const uint64_t o_part = align256(o_pos + max_tiles * pairs * 512 * 4);
    uint32_t* tiles = reinterpret_cast<uint32_t*>(base);
    uint16_t* endsT = reinterpret_cast<uint16_t*>(base + o_ends);
    uint8_t* res = reinterpret_cast<uint8_t*>(base + o_res);
    uint32_t* posv = reinterpret_cast<uint32_t*>(base + o_pos);
    uint32_t* partial = reinterpret_cast<uint32_t*>(base + o_part);
    const bool k10 = k == 10;
    if (pl.KT > 1024u * (k10 ? 3u : 2u) || pl.CPg / 8 > 65536 / 8) return hipErrorInvalidValue;
    for (uint64_t lo = 0; lo < kb.n; lo += chunk_keys) {
        const uint64_t cn = std::min<uint64_t>(chunk_keys, kb.n - lo);
        DevKeys dk{kb.keys, kb.offsets, kb.off_base, kb.stride, cn};
        if (kb.offsets)
            dk.offsets = kb.offsets + lo;
        else
            dk.keys = kb.keys + lo * kb.stride;
        const uint32_t ntiles = (uint32_t)((cn + pl.KT - 1) / pl.KT);
        pl.ntS = (ntiles + 7) & ~7u;
        phase_begin(kPhaseProbePack, s);
        hipError_t err = launch_group_pack(kb, dk, pl, ntiles, tiles, endsT, reinterpret_cast<uint16_t*>(posv), kSegBits, s);
        if (err != hipSuccess) return err;
        phase_end(kPhaseProbePack, s);
        phase_begin(kPhaseProbeSeg, s);
        // every result bit starts "pass": the segment pass stores only bytes holding a failing entry
        // (a positive probe stores none; the scattered byte stores cost the segment pass most)
        err = hipMemsetAsync(res, 0xFF, (uint64_t)ntiles * (pl.CPg / 8), s);
        if (err != hipSuccess) return err;
        const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>(ntiles, (512 + pl.nseg - 1) / pl.nseg));
        hipLaunchKernelGGL(k_probe_seg2<4>, dim3(pl.nseg * G), dim3(kPBlock), 0, s, tiles, endsT, ntiles, pl, G, words,
                           res);
        phase_end(kPhaseProbeSeg, s);
        phase_begin(kPhaseProbeOut, s);
        if (count) {
            auto fn = k10 ? k_probe_out2<10, 3, 1> : k_probe_out2<19, 2, 1>;
            hipLaunchKernelGGL(fn, dim3(ntiles), dim3(kPBlock), 0, s, res, posv, pl, pairs, cn, nullptr, partial);
            err = launch_count_finish(partial, ntiles, count, s);
            if (err != hipSuccess) return err;
        } else {
            auto fn = k10 ? k_probe_out2<10, 3, 0> : k_probe_out2<19, 2, 0>;
            hipLaunchKernelGGL(fn, dim3(ntiles), dim3(kPBlock), 0, s, res, posv, pl, pairs, cn, out + lo, nullptr);
        }
        phase_end(kPhaseProbeOut, s);
        err = hipGetLastError();
        if (err != hipSuccess) return err;
    }
    return hipSuccess;
}

// The runtime-k class a probe pack of k takes (0: a compiled k, k > 32 or VBF_KCLASS=0): over 2^20-bit
// segments for k outside {4, 10, 19}; over 2^17-position multi-SST segments (keys with the length
// prefix) for k outside {4, 10, 19} too (round 6).
uint32_t probe_class(uint32_t k, int sb) {
    static const int kcls = [] { const char* e = getenv("VBF_KCLASS"); return e ? atoi(e) : 1; }();
    if (kcls == 0 || k == 4 || k == 10 || k == 19 || (sb != kSegBits && sb != kByteSegBits)) return 0;
    return tile_pack_class(k);
}

ProbePlan make_probe_plan(uint32_t m, uint32_t k, int sb) {
    ProbePlan pl{};
    pl.k = k;
    pl.m = m;
    pl.mu = ~0ull / m;
    pl.nwords = ((uint64_t)m + 31) / 32;
    pl.nseg = (uint32_t)(((uint64_t)m + (1u << sb) - 1) >> sb);
    pl.nseg_pad = (pl.nseg + 3) & ~3u;
    // k outside {4, 10, 19} on 2^20-bit segments: the runtime-k class kernel's rounds (its stash holds
    // rounds_max(class) rounds of class slots; the scratch-stash kernel runs any round count)
    const uint32_t kc = probe_class(k, sb);
    const uint32_t rmax = (uint32_t)rounds_max((int)(kc ? kc : k));
    const int64_t avail = (int64_t)(kLdsPerCu / 2) - 64 - 4 * (int64_t)pl.nseg_pad;
    const int64_t kt = std::min<int64_t>(std::min<int64_t>((int64_t)rmax * kPBlock, avail / 4 / k), 4096);
    pl.KT = (uint32_t)std::max<int64_t>(kt, 1);
    pl.R = (pl.KT + kPBlock - 1) / kPBlock;
    pl.C = pl.KT * k;
    pl.cap = (pl.C + 7 * pl.nseg + 31) & ~31u;  // multiple of 32: k_probe_out reads result dwords
    pl.lds1 = (pl.C + pl.nseg_pad + 16) * 4;
    return pl;
}

bool probe_partition_supported(uint32_t m, uint32_t k) {
    if (m == 0 || k < 1 || k > (uint32_t)kStash) return false;
    const ProbePlan pl = make_probe_plan(m, k, kSegBits);
    return pl.KT >= 64 && pl.lds1 <= kLdsPerCu / 2 && pl.cap <= 65535;
}

static uint64_t probe_chunk_keys(const ProbePlan& pl, uint64_t n) {
    const uint64_t tiles_per_chunk = std::max<uint64_t>(1, kPartChunkIdx / pl.C);
    return std::min<uint64_t>(n, tiles_per_chunk * pl.KT);
}

uint64_t probe_workspace_bytes(uint64_t n, uint32_t m, uint32_t k) {
    if (!probe_partition_supported(m, k)) return 0;
    const ProbePlan pl = make_probe_plan(m, k, kSegBits);
    const uint64_t ntiles = (probe_chunk_keys(pl, n) + pl.KT - 1) / pl.KT;
    uint64_t need = ntiles * ((uint64_t)pl.cap * 4 + pl.cap / 8 + (uint64_t)pl.nseg * 4 + 4) + 1024;
    if (group_pack_supported(m, k, kSegBits)) need = std::max<uint64_t>(need, pp_workspace_bytes(n, m, k));
    if (probe_pu_enabled(m, k, true, true)) need = std::max<uint64_t>(need, probe_pu_workspace_bytes(n, m, k, true));
    return need;
}

uint64_t probe_count_partials(uint64_t n, uint32_t m, uint32_t k) {
    const ProbePlan pl = make_probe_plan(m, k, kSegBits);
    return (probe_chunk_keys(pl, n) + pl.KT - 1) / pl.KT;
}

template <int FMT, bool LP, int SB>
hipError_t launch_probe_pack_fmt(const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles, uint32_t* tiles,
                                 uint16_t* ends, hipStream_t s) {
    const uint32_t k = pl.k;
    auto pick = [&]<bool S>() {
        return k == 10 ? k_probe_pack<FMT, LP, 10, S, SB>
             : k == 4  ? k_probe_pack<FMT, LP, 4, S, SB>
             : k == 19 ? k_probe_pack<FMT, LP, 19, S, SB>  // the reference's default p = 1e-4
                       : k_probe_pack<FMT, LP, 0, false, SB>;
    };
    if constexpr (SB == kByteSegBits && LP) {
        // the multi-SST probe's interleaved filters (2^17-position segments): the class kernels
        // too (round 6; make_probe_plan sizes the tile by the class)
        const uint32_t kc = probe_class(k, SB);
        if (kc)
            return kc <= 12 ? launch_probe_pack_class_a17(FMT, kc, dk, pl, ntiles, tiles, ends, s)
                            : launch_probe_pack_class_b17(FMT, kc, dk, pl, ntiles, tiles, ends, s);
    }
    if constexpr (SB == kSegBits) {
        // k outside the compiled set: the runtime-k class kernels (register stash) -- unless
        // VBF_KCLASS=0 keeps the scratch-stash kernel (A/B)
        const uint32_t kc = probe_class(k, SB);
        if (kc) {
            if constexpr (LP)
                return kc <= 12 ? launch_probe_pack_class_a(FMT, kc, dk, pl, ntiles, tiles, ends, s)
                                : launch_probe_pack_class_b(FMT, kc, dk, pl, ntiles, tiles, ends, s);
            else
                return kc <= 12 ? launch_probe_pack_class_c(FMT, kc, dk, pl, ntiles, tiles, ends, s)
                                : launch_probe_pack_class_d(FMT, kc, dk, pl, ntiles, tiles, ends, s);
        }
    }
    auto fn = pl.m <= (1ull << 31) ? pick.template operator()<true>() : pick.template operator()<false>();
    if constexpr (LP && SB == kSegBits) {  // m = 2^32 - 1 (the reference's saturated size): SAT kernels
        if (pl.m == 0xFFFFFFFFull && (k == 4 || k == 10 || k == 19))
            fn = k == 4 ? k_probe_pack<FMT, LP, 4, false, SB, true>
               : k == 10 ? k_probe_pack<FMT, LP, 10, false, SB, true> : k_probe_pack<FMT, LP, 19, false, SB, true>;
    }
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)pl.lds1);
    if (err == hipSuccess) hipLaunchKernelGGL(fn, dim3(ntiles), dim3(kPBlock), pl.lds1, s, dk, pl, tiles, ends);
    return err;
}

hipError_t launch_probe_pack(const KeyBatch& kb, const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles,
                             uint32_t* tiles, uint16_t* ends, int sb, hipStream_t s) {
    hipError_t err = hipErrorInvalidValue;
    with_fmt(pick_fmt(dk.keys, dk.offsets, dk.stride), kb.len_prefix, [&]<int FMT, bool LP>() {
        if (sb == kSegBits)
            err = launch_probe_pack_fmt<FMT, LP, kSegBits>(dk, pl, ntiles, tiles, ends, s);
        else if (sb == kByteSegBits)
            err = launch_probe_pack_fmt<FMT, LP, kByteSegBits>(dk, pl, ntiles, tiles, ends, s);
    });
    return err;
}

hipError_t launch_probe_partitioned(const KeyBatch& kb, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
                                    unsigned long long* count, void* ws, uint64_t ws_bytes, hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    if (!probe_partition_supported(m, k)) return hipErrorInvalidValue;
    const ProbePlan pl = make_probe_plan(m, k, kSegBits);
    const uint64_t chunk_keys = probe_chunk_keys(pl, kb.n);
    const uint64_t max_tiles = (chunk_keys + pl.KT - 1) / pl.KT;
    if (ws_bytes < probe_workspace_bytes(kb.n, m, k)) return hipErrorInvalidValue;
    if (probe_pu_enabled(m, k, kb.len_prefix, pick_fmt(kb.keys, kb.offsets, kb.stride) > 0))  // round 6: the build's image (vbf_probe_pu.hip)
        return launch_probe_pu(kb, m, k, words, out, count, ws, ws_bytes, s);
    if (pp_enabled(m, k, kb.len_prefix)) return launch_probe_pp(kb, m, k, words, out, count, ws, s);
    auto align16 = [](uint64_t x) { return (x + 15) & ~15ull; };
    char* base = static_cast<char*>(ws);
    uint32_t* tiles = reinterpret_cast<uint32_t*>(base);
    const uint64_t o_res = align16(max_tiles * pl.cap * 4);
    const uint64_t o_ends = align16(o_res + max_tiles * pl.cap / 8);
    const uint64_t o_endsT = align16(o_ends + max_tiles * pl.nseg * 2);
    const uint64_t o_part = align16(o_endsT + max_tiles * pl.nseg * 2);
    uint32_t* partial = reinterpret_cast<uint32_t*>(base + o_part);
    uint8_t* res = reinterpret_cast<uint8_t*>(base + o_res);
    uint16_t* ends = reinterpret_cast<uint16_t*>(base + o_ends);
    uint16_t* endsT = reinterpret_cast<uint16_t*>(base + o_endsT);
    for (uint64_t lo = 0; lo < kb.n; lo += chunk_keys) {
        const uint64_t cn = std::min<uint64_t>(chunk_keys, kb.n - lo);
        DevKeys dk{kb.keys, kb.offsets, kb.off_base, kb.stride, cn};
        if (kb.offsets)
            dk.offsets = kb.offsets + lo;
        else
            dk.keys = kb.keys + lo * kb.stride;
        const uint32_t ntiles = (uint32_t)((cn + pl.KT - 1) / pl.KT);
        hipError_t err = hipSuccess;
        phase_begin(kPhaseProbePack, s);
        with_fmt(pick_fmt(dk.keys, dk.offsets, dk.stride), kb.len_prefix, [&]<int FMT, bool LP>() {
            err = launch_probe_pack_fmt<FMT, LP, kSegBits>(dk, pl, ntiles, tiles, ends, s);
        });
        if (err != hipSuccess) return err;
        launch_transpose_u16(ends, endsT, ntiles, pl.nseg, s);
        phase_end(kPhaseProbePack, s);
        phase_begin(kPhaseProbeSeg, s);
        err = hipMemsetAsync(res, 0xFF, (uint64_t)ntiles * (pl.cap / 8), s);  // bytes start all ones
        if (err != hipSuccess) return err;
        const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>(ntiles, (512 + pl.nseg - 1) / pl.nseg));
        uint32_t nfull = G > 1 ? 0u : pl.nseg, P = G;
        if (G == 1 && probe_split_enabled()) {
            // the last round's rem segments in P parts: P minimising ceil(rem * P / CUs) / P, the
            // rounds of part-workgroups the tail then takes (k = 19, m = 1.9e9: 1 812 = 7 x 256 +
            // 20 -> P = 12; k = 10, m = 1e9: 954 = 3 x 256 + 186 -> P = 11)
            const uint32_t ncu = device_cu_count(), rem = ncu ? pl.nseg % ncu : 0u;
            if (pl.nseg > ncu && rem > 0) {
                double best = 1.0;
                for (uint32_t p = 2; p <= 16 && p <= ntiles; ++p) {
                    const double t = (double)((rem * p + ncu - 1) / ncu) / p;
                    if (t < best - 1e-9) { best = t; P = p; }
                }
                if (P > 1) nfull = pl.nseg - rem;
            }
        }
        static const int q3v = [] { const char* e = getenv("VBF_Q3"); return e ? atoi(e) : 1; }();
        hipLaunchKernelGGL(q3v == 1 ? k_probe_seg<1> : k_probe_seg<0>, dim3(nfull + (pl.nseg - nfull) * P),
                           dim3(kPBlock), 0, s, tiles, endsT, ntiles, pl, nfull, P, words, res);
        phase_end(kPhaseProbeSeg, s);
        phase_begin(kPhaseProbeOut, s);
        if (count) {
            hipLaunchKernelGGL(k_probe_out<1>, dim3(ntiles), dim3(kPBlock), 0, s, tiles, ends, res, pl, cn, nullptr,
                               partial);
            err = launch_count_finish(partial, ntiles, count, s);
            if (err != hipSuccess) return err;
        } else {
            hipLaunchKernelGGL(k_probe_out<0>, dim3(ntiles), dim3(kPBlock), 0, s, tiles, ends, res, pl, cn, out + lo,
                               nullptr);
        }
        phase_end(kPhaseProbeOut, s);
        err = hipGetLastError();
        if (err != hipSuccess) return err;
    }
    return hipSuccess;
}

}  // namespace vbf
