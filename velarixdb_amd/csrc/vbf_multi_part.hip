// vbf_multi_part.hip -- batched read-path probe for groups of SSTs whose filters share (m, k)
// (KeyRange::filter_sstables_by_key_range, src/key_range/range.rs:91-147).
//
// calculate_hash(key, i) does not depend on the filter (bf.rs:222-227), and the bit a filter
// tests for it is hash % m (bf.rs:99): filters with the same m test the SAME position for a key.
// So up to 8 such filters are interleaved into one byte per position (bit g = filter g's bit) and
// each of a key's k positions is looked up once for the whole group.  Filters with one (m, k) are
// the common case: every memtable-born SST is sized from the write buffer (mem.rs:188-191), and
// equally sized compaction outputs get equal m (sized.rs:192).
//
// The lookups themselves go through the partitioned probe (vbf_probe_part.hip) with byte
// positions: Q1 hashes a tile of keys and sorts its (key id, position) entries by 2^17-position
// segment; MQ3 stages a segment's 128 KiB of interleaved bytes in LDS and answers each entry with
// its byte; MQ4 ANDs each key's k bytes and writes, per member SST, range test && bit.  No entry
// is answered from HBM: random loads (~55 G/s chip-wide) become LDS reads.
#include "vbf_tile_pack.hpp"

namespace vbf {

// bytes[i] bit g = bit i of filter g (positions i < m; the pad up to a multiple of 32 is 0).
__global__ __launch_bounds__(256) void k_interleave(MultiGroup g, uint64_t nwords, uint32_t* bytes) {
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (w >= nwords) return;
    uint32_t src[kMaxGroup];
#pragma unroll
    for (uint32_t q = 0; q < kMaxGroup; ++q) src[q] = q < g.G ? g.words[q][w] : 0u;
    uint32_t out[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) {  // output dword d = positions 4d .. 4d+3
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            uint32_t byte = 0;
#pragma unroll
            for (uint32_t q = 0; q < kMaxGroup; ++q) byte |= ((src[q] >> (4 * d + b)) & 1u) << q;
            v |= byte << (8 * b);
        }
        out[d] = v;
    }
    uint4* o = reinterpret_cast<uint4*>(bytes + w * 8);
    o[0] = make_uint4(out[0], out[1], out[2], out[3]);
    o[1] = make_uint4(out[4], out[5], out[6], out[7]);
}

constexpr uint32_t kByteSeg = 1u << kByteSegBits;  // positions (bytes) per segment: 128 KiB of LDS
constexpr uint32_t kByteOff = kByteSeg - 1;

// MQ3: one workgroup per segment; the k_probe_seg<1> pipeline (bounds of batch b+2, entries of
// b+1 and the lookups of b in flight together), answering each entry with its group byte.
template <int NG = 4>
__global__ __launch_bounds__(kPBlock) void k_group_seg(const uint32_t* tiles, const uint16_t* endsT, uint32_t ntiles,
                                                       ProbePlan pl, uint32_t G, const uint32_t* bytes, uint64_t nbytes,
                                                       uint8_t* res) {
    __shared__ __attribute__((aligned(16))) uint32_t seg_bytes[kByteSeg / 4];
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(seg_bytes);
    const uint32_t nwg = gridDim.x, qq = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
    const uint32_t wg = (xcd < r8 ? xcd * (qq + 1) : r8 * (qq + 1) + (xcd - r8) * qq) + blockIdx.x / 8;
    const uint32_t seg = wg / G, part = wg % G;
    const uint32_t t_lo = (uint32_t)((uint64_t)part * ntiles / G), t_hi = (uint32_t)((uint64_t)(part + 1) * ntiles / G);
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t b0 = (uint64_t)seg * kByteSeg;  // nbytes is a multiple of 16
    const uint32_t bn = (uint32_t)std::min<uint64_t>(kByteSeg, nbytes - b0);
    for (uint32_t w = tid * 4; w < kByteSeg / 4; w += kPBlock * 4) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (w * 4 < bn) v = *reinterpret_cast<const uint4*>(bytes + b0 / 4 + w);
        *reinterpret_cast<uint4*>(seg_bytes + w) = v;
    }
    __syncthreads();
    const uint16_t* row_end = endsT + (uint64_t)seg * ntiles;
    const uint16_t* row_beg = seg ? endsT + (uint64_t)(seg - 1) * ntiles : nullptr;
    const uint32_t grp = lane >> 3, q8 = (lane & 7) * 8;
    auto look8 = [&](const uint4& a, const uint4& b) -> uint2 {
        const uint32_t e[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t r[2] = {0, 0};
#pragma unroll
        for (int c = 0; c < 8; ++c) r[c >> 2] |= (uint32_t)sb[e[c] & kByteOff] << (8 * (c & 3));
        return make_uint2(r[0], r[1]);
    };
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
            const uint32_t x = q8 < len ? st + q8 : st;  // idle lanes re-read the run's start
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
            if (q8 < len) *reinterpret_cast<uint2*>(res + t * pl.cap + st + q8) = look8(bt.a[g], bt.b[g]);
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) {  // runs longer than 64 entries
            const uint32_t st = bt.be[g] & 0xFFFFu, len = (bt.be[g] >> 16) - st;
            const uint64_t t = t0 + g * 8 + grp;
#pragma unroll 1
            for (uint32_t x = st + q8 + 64; x < st + len; x += 64) {
                const uint32_t* run = tiles + t * pl.cap + x;
                *reinterpret_cast<uint2*>(res + t * pl.cap + x) =
                    look8(*reinterpret_cast<const uint4*>(run), *reinterpret_cast<const uint4*>(run + 4));
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
}

// MQ4: per tile, AND each key's k group bytes (bf.rs:97-103 for every member at once), then for
// every member SST: out = key in [smallest, biggest] (range.rs:113) && its bit.
__global__ __launch_bounds__(kPBlock) void k_group_out(const uint32_t* tiles, const uint16_t* ends, const uint8_t* res,
                                                       ProbePlan pl, DevKeys dk, MultiGroup g, const uint8_t* bounds,
                                                       uint8_t* out, uint32_t out_stride) {
    __shared__ uint32_t msk[4096 / 4];  // one byte per key of the tile (KT <= 4096)
    const uint32_t tid = threadIdx.x;
    const uint64_t key0 = (uint64_t)blockIdx.x * pl.KT;
    const uint32_t nk = (uint32_t)std::min<uint64_t>(pl.KT, dk.n - key0);
    for (uint32_t w = tid; w < (nk + 3) / 4; w += kPBlock) msk[w] = 0xFFFFFFFFu;
    __syncthreads();
    const uint32_t total = ends[(uint64_t)blockIdx.x * pl.nseg + pl.nseg - 1];
    const uint32_t* tl = tiles + (uint64_t)blockIdx.x * pl.cap;
    const uint32_t* rs = reinterpret_cast<const uint32_t*>(res + (uint64_t)blockIdx.x * pl.cap);
    const uint32_t full = g.G >= 8 ? 0xFFu : ((1u << g.G) - 1u);
    // 4 entries per lane: one dword of result bytes and one 16-byte load of their entries (most
    // entries of a multi-member group have some member's bit clear, so the entries are read
    // unconditionally); cap % 32 == 0 keeps both aligned
    for (uint32_t w = tid; w * 4 < total; w += kPBlock) {
        const uint32_t r = rs[w];
        const uint4 ev = *reinterpret_cast<const uint4*>(tl + w * 4);
        const uint32_t ee[4] = {ev.x, ev.y, ev.z, ev.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t b = (r >> (8 * c)) & full;
            if (w * 4 + c < total && b != full) {  // some member's bit is clear: drop those members
                const uint32_t local = ee[c] >> kByteSegBits;
                atomicAnd(&msk[local >> 2], ~(((~b) & full) << ((local & 3) * 8)));
            }
        }
    }
    __syncthreads();
    // members in consecutive columns from an 8-aligned one and 8-byte rows: one 8-byte store per key
    bool packed = g.G == 8 && (out_stride & 7u) == 0 && (g.col[0] & 7u) == 0 && !bounds &&
                  (reinterpret_cast<uintptr_t>(out) & 7u) == 0;
    for (uint32_t q = 1; q < g.G && packed; ++q) packed = g.col[q] == g.col[0] + q;
    for (uint32_t l = tid; l < nk; l += kPBlock) {
        const uint64_t j = key0 + l;
        const uint32_t mk = (msk[l >> 2] >> ((l & 3) * 8)) & 0xFFu;
        uint8_t* row = out + j * out_stride;
        if (packed) {
            // byte q = bit q of mk: spread the 8 bits to the low bit of 8 bytes
            uint64_t v = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) v |= (uint64_t)((mk >> q) & 1u) << (8 * q);
            *reinterpret_cast<uint64_t*>(row + g.col[0]) = v;
        } else if (bounds) {
            const uint8_t* kp;
            uint64_t kl;
            if (dk.offsets) {
                kp = dk.keys + (dk.offsets[j] - dk.off_base);
                kl = dk.offsets[j + 1] - dk.offsets[j];
            } else {
                kp = dk.keys + j * dk.stride;
                kl = dk.stride;
            }
            for (uint32_t q = 0; q < g.G; ++q) {
                bool hit = (mk >> q) & 1u;
                if (hit)
                    hit = cmp_bytes(kp, kl, bounds + g.lo_beg[q], g.lo_end[q] - g.lo_beg[q]) >= 0 &&
                          cmp_bytes(kp, kl, bounds + g.hi_beg[q], g.hi_end[q] - g.hi_beg[q]) <= 0;
                row[g.col[q]] = hit ? 1 : 0;
            }
        } else {
            for (uint32_t q = 0; q < g.G; ++q) row[g.col[q]] = (mk >> q) & 1u;
        }
    }
}

// ---- Round 4: the group pipeline on the build's image (k = 10 / 19 with the length prefix) ----
// GP1 launch_group_pack (k_tile_pack with 2^17-position segments): the tile image in the build's
// 2.5-byte 8-entry groups instead of 4-byte (key id, position) entries, each run padded to whole
// groups in HBM (the LDS image stays unpadded; the copy-out repacks), the padded run ends written
// transposed, and each entry's padded place in its tile in posv[tile][slot][lane].
// GP3 k_group_seg2: k_seg_or's flattened reader over a segment's runs, each entry answered with its
// interleaved byte at the entry's place, res[tile][e]: whole groups, one 8-byte store each (runs
// never share a group; the piecewise path for a partial group is kept for unpadded images).
// GP4 k_group_out2: per tile, the result bytes staged in LDS; a key's k results are found through
// posv (coalesced u16 reads) instead of re-reading and decoding every entry, then ANDed.
template <int NG = 4>
__global__ __launch_bounds__(kPBlock) void k_group_seg2(const uint32_t* tiles, const uint16_t* endsT, uint32_t ntiles,
                                                        PartPlan pl, uint32_t G, const uint32_t* bytes, uint64_t nbytes,
                                                        uint8_t* res) {
    __shared__ __attribute__((aligned(16))) uint32_t seg_bytes[kByteSeg / 4];
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(seg_bytes);
    const uint32_t nwg = gridDim.x, qq = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
    const uint32_t wg = (xcd < r8 ? xcd * (qq + 1) : r8 * (qq + 1) + (xcd - r8) * qq) + blockIdx.x / 8;
    const uint32_t seg = wg / G, part = wg % G;
    const uint32_t t_lo = (uint32_t)((uint64_t)part * ntiles / G), t_hi = (uint32_t)((uint64_t)(part + 1) * ntiles / G);
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t b0 = (uint64_t)seg * kByteSeg;  // nbytes is a multiple of 16
    const uint32_t bn = (uint32_t)std::min<uint64_t>(kByteSeg, nbytes - b0);
    for (uint32_t w = tid * 4; w < kByteSeg / 4; w += kPBlock * 4) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (w * 4 < bn) v = *reinterpret_cast<const uint4*>(bytes + b0 / 4 + w);
        *reinterpret_cast<uint4*>(seg_bytes + w) = v;
    }
    __syncthreads();
    const uint16_t* row_end = endsT + (uint64_t)seg * pl.ntS;
    const uint16_t* row_beg = seg ? endsT + (uint64_t)(seg - 1) * pl.ntS : nullptr;
    auto lb = [&](uint32_t t0) -> uint32_t {
        const uint32_t t = t0 + lane;
        uint32_t v = 0;
        if (t < t_hi) v = (row_beg ? (uint32_t)row_beg[t] : 0u) | ((uint32_t)row_end[t] << 16);
        return v;
    };
    // entries [a, b) of group gi of tile t: their bytes, stored at res[t][gi * 8 + c]
    auto answer = [&](uint32_t t, uint32_t gi, uint4 l, uint32_t nib, uint32_t a, uint32_t b) {
        const uint32_t w[4] = {l.x, l.y, l.z, l.w};
        uint32_t r[2] = {0, 0};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint32_t off = ((w[c >> 1] >> ((c & 1) * 16)) & 0xFFFFu) | (((nib >> (4 * c)) & 1u) << 16);
            r[c >> 2] |= (uint32_t)sb[off] << (8 * (c & 3));
        }
        uint8_t* dst = res + (uint64_t)t * pl.CPg + gi * 8;
        if (a == 0 && b == 8) {
            *reinterpret_cast<uint2*>(dst) = make_uint2(r[0], r[1]);
        } else {  // a group shared with a neighbouring run: only [a, b), in aligned pieces
            // greedy aligned pieces (4, 2 or 1 bytes): at most four stores for any [a, b) of 8
            const uint64_t v = (uint64_t)r[0] | ((uint64_t)r[1] << 32);
            uint32_t c = a;
#pragma unroll
            for (int step = 0; step < 4; ++step) {
                if (c >= b) break;
                if ((c & 3) == 0 && c + 4 <= b) {
                    *reinterpret_cast<uint32_t*>(dst + c) = (uint32_t)(v >> (8 * c));
                    c += 4;
                } else if ((c & 1) == 0 && c + 2 <= b) {
                    *reinterpret_cast<uint16_t*>(dst + c) = (uint16_t)(v >> (8 * c));
                    c += 2;
                } else {
                    dst[c] = (uint8_t)(v >> (8 * c));
                    c += 1;
                }
            }
        }
    };
    const uint32_t wstep = (kPBlock / 64) * 64;
    struct FB {
        uint32_t v, excl, total;
        uint4 l[NG];
        uint32_t nib[NG], ab[NG], t[NG], gi[NG];
    };
    auto prep = [&](uint32_t v, FB& b) {
        const uint32_t st = v & 0xFFFFu, en = v >> 16;
        const uint32_t ch = en > st ? ((en + 7) >> 3) - (st >> 3) : 0u;
        uint32_t incl = ch;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= (uint32_t)o) incl += y;
        }
        b.v = v;
        b.excl = incl - ch;
        b.total = (uint32_t)__shfl((int)incl, 63);
    };
    // (the run marks of k_seg_or, vbf_partition.hpp, measured 1.3 % slower in this pass, whose
    // result-byte stores bound it: profiles/r06/ab_marks_multi.log)
    auto locate = [&](const FB& b, uint32_t t0, uint32_t c, uint32_t& t, uint32_t& gi) -> uint32_t {
        uint32_t r = 0;
#pragma unroll
        for (int sft = 32; sft; sft >>= 1)
            if ((uint32_t)__shfl((int)b.excl, (int)r + sft) <= c) r += sft;
        const uint32_t rv = (uint32_t)__shfl((int)b.v, (int)r), rex = (uint32_t)__shfl((int)b.excl, (int)r);
        const uint32_t rst = rv & 0xFFFFu, ren = rv >> 16;
        t = std::min(t0 + r, t_hi - 1);
        gi = (rst >> 3) + (c - rex);
        if (c >= b.total || gi * 8 >= ren || gi * 8 + 8 <= rst) return 0u;
        const uint32_t a = gi * 8 < rst ? rst - gi * 8 : 0u, e = std::min<uint32_t>(8, ren - gi * 8);
        return a | (e << 4);
    };
    auto issue = [&](uint32_t t0, FB& b) {
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            b.ab[q] = locate(b, t0, (uint32_t)q * 64 + lane, b.t[q], b.gi[q]);
            if (b.ab[q]) {
                const uint32_t* tile = tiles + (uint64_t)b.t[q] * pl.tile_words;
                __builtin_memcpy(&b.l[q], tile + b.gi[q] * 5, 16);
                b.nib[q] = tile[b.gi[q] * 5 + 4];
            }
        }
    };
    auto consume = [&](uint32_t t0, const FB& b) {
#pragma unroll
        for (int q = 0; q < NG; ++q)
            if (b.ab[q]) answer(b.t[q], b.gi[q], b.l[q], b.nib[q], b.ab[q] & 15u, b.ab[q] >> 4);
#pragma unroll 1
        for (uint32_t c0 = 64 * NG; c0 < b.total; c0 += 64) {
            uint32_t t, gi;
            const uint32_t ab = locate(b, t0, c0 + lane, t, gi);
            if (ab) {
                const uint32_t* tile = tiles + (uint64_t)t * pl.tile_words;
                uint4 l;
                __builtin_memcpy(&l, tile + gi * 5, 16);
                answer(t, gi, l, tile[gi * 5 + 4], ab & 15u, ab >> 4);
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

// GP4: dynamic LDS = the tile's result bytes (pl.CPg, a multiple of 8).  K compile-time: a lane
// issues the K position loads of each of its KPT keys together (one memory latency, not K * KPT).
template <int K, int KPT>
__global__ __launch_bounds__(kPBlock) void k_group_out2(const uint8_t* res, const uint32_t* posv, const uint16_t* endsT,
                                                        PartPlan pl, uint32_t pairs, DevKeys dk, MultiGroup g,
                                                        const uint8_t* bounds, uint8_t* out, uint32_t out_stride) {
    extern __shared__ __attribute__((aligned(16))) uint32_t rl32[];
    const uint8_t* rl = reinterpret_cast<const uint8_t*>(rl32);
    const uint32_t tid = threadIdx.x, tile = blockIdx.x;
    const uint64_t key0 = (uint64_t)tile * pl.KT;
    const uint32_t nk = (uint32_t)std::min<uint64_t>(pl.KT, dk.n - key0);
    const uint32_t total = endsT[(uint64_t)(pl.nseg - 1) * pl.ntS + tile];
    const uint2* src = reinterpret_cast<const uint2*>(res + (uint64_t)tile * pl.CPg);
    for (uint32_t w = tid; w * 8 < total; w += kPBlock) reinterpret_cast<uint2*>(rl32)[w] = src[w];
    __syncthreads();
    const uint32_t full = g.G >= 8 ? 0xFFu : ((1u << g.G) - 1u);
    const uint32_t* pt = posv + (uint64_t)tile * pairs * 512;
    bool packed = g.G == 8 && (out_stride & 7u) == 0 && (g.col[0] & 7u) == 0 && !bounds &&
                  (reinterpret_cast<uintptr_t>(out) & 7u) == 0;
    for (uint32_t q = 1; q < g.G && packed; ++q) packed = g.col[q] == g.col[0] + q;
    // key l: stash round r = l / 512, lane l % 512; its slots r*K .. r*K+K-1 sit in the u16 pairs
    // (r*K)/2 ..; for odd K a round starts on the pair's high half when r is odd (wave-uniform:
    // a wave's 64 keys share r)
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
    auto pos_of = [&](int x, int i, uint32_t odd) -> uint32_t {
        const uint32_t q = odd + (uint32_t)i;
        return (wv[x][q >> 1] >> ((q & 1u) * 16)) & 0xFFFFu;
    };
#pragma unroll
    for (int x = 0; x < KPT; ++x) {
        const uint32_t l = tid + x * kPBlock;
        if (l >= nk) break;
        uint32_t mk = full;
        const uint32_t odd = ((l >> 9) * K) & 1u;
        if (odd) {
#pragma unroll
            for (int i = 0; i < K; ++i) mk &= rl[pos_of(x, i, 1u)];
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) mk &= rl[pos_of(x, i, 0u)];
        }
        const uint64_t j = key0 + l;
        uint8_t* row = out + j * out_stride;
        if (packed) {
            uint64_t v = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) v |= (uint64_t)((mk >> q) & 1u) << (8 * q);
            *reinterpret_cast<uint64_t*>(row + g.col[0]) = v;
        } else if (bounds) {
            const uint8_t* kp;
            uint64_t kl;
            if (dk.offsets) {
                kp = dk.keys + (dk.offsets[j] - dk.off_base);
                kl = dk.offsets[j + 1] - dk.offsets[j];
            } else {
                kp = dk.keys + j * dk.stride;
                kl = dk.stride;
            }
            for (uint32_t q = 0; q < g.G; ++q) {
                bool hit = (mk >> q) & 1u;
                if (hit)
                    hit = cmp_bytes(kp, kl, bounds + g.lo_beg[q], g.lo_end[q] - g.lo_beg[q]) >= 0 &&
                          cmp_bytes(kp, kl, bounds + g.hi_beg[q], g.hi_end[q] - g.hi_beg[q]) <= 0;
                row[g.col[q]] = hit ? 1 : 0;
            }
        } else {
            for (uint32_t q = 0; q < g.G; ++q) row[g.col[q]] = (mk >> q) & 1u;
        }
    }
}

static uint64_t group_nbytes(uint64_t m) { return ((m + 31) / 32) * 32; }

bool multi_group_supported(uint64_t m, uint32_t k) {
    if (m == 0 || m > 0xFFFFFFFFull || k < 1 || k > (uint32_t)kStash) return false;
    const ProbePlan pl = make_probe_plan((uint32_t)m, k, kByteSegBits);
    return pl.KT >= 64 && pl.KT <= 4096 && pl.lds1 <= kLdsPerCu / 2 && pl.cap <= 65535;
}

static uint64_t group_chunk_keys(const ProbePlan& pl, uint64_t n) {
    const uint64_t tiles_per_chunk = std::max<uint64_t>(1, kPartChunkIdx / pl.C);
    return std::min<uint64_t>(n, tiles_per_chunk * pl.KT);
}

// The round-4 pipeline (GP1-GP4) where it exists; VBF_MULTI_GP = 0 keeps the round-3 one (A/B).
static bool gp_enabled(uint64_t m, uint32_t k, bool lp) {
    const char* e = getenv("VBF_MULTI_GP");  // read per call, like VBF_MULTI
    return (e ? atoi(e) : 1) != 0 && lp && group_pack_supported(m, k);
}

static uint64_t gp_chunk_keys(const PartPlan& pl, uint64_t n) {
    const uint64_t tiles_per_chunk = std::max<uint64_t>(1, kPartChunkIdx / pl.C);
    return std::min<uint64_t>(n, tiles_per_chunk * pl.KT);
}

// GP workspace after the interleaved bytes: tiles, endsT[nseg][ntS], res[tiles][CP], posv.
static uint64_t gp_workspace_bytes(uint64_t n, uint64_t m, uint32_t k) {
    uint64_t need = 0;
    for (bool fixed : {true, false}) {
        const PartPlan pl = make_group_plan((uint32_t)m, k, fixed);
        const uint64_t nt = (gp_chunk_keys(pl, n) + pl.KT - 1) / pl.KT, ntS = (nt + 7) & ~7ull;
        need = std::max<uint64_t>(need, nt * (uint64_t)pl.tile_words * 4 + ntS * pl.nseg * 2 + nt * pl.CPg +
                                            nt * (uint64_t)((group_pack_slots(k) + 1) / 2) * 512 * 4 + 4 * 256);
    }
    return need;
}

uint64_t multi_group_workspace_bytes(uint64_t n, uint64_t m, uint32_t k) {
    if (!multi_group_supported(m, k)) return 0;
    const ProbePlan pl = make_probe_plan((uint32_t)m, k, kByteSegBits);
    const uint64_t nt = (group_chunk_keys(pl, n) + pl.KT - 1) / pl.KT;
    uint64_t need = group_nbytes(m) + 256 + nt * ((uint64_t)pl.cap * 5 + (uint64_t)pl.nseg * 4) + 1024;
    if (group_pack_supported(m, k)) need = std::max<uint64_t>(need, group_nbytes(m) + 256 + gp_workspace_bytes(n, m, k));
    return need;
}

static hipError_t launch_multi_probe_gp(const KeyBatch& kb, const MultiGroup& g, const uint8_t* bounds, uint8_t* out,
                                        uint32_t out_stride, char* base, hipStream_t s) {
    auto align256 = [](uint64_t x) { return (x + 255) & ~255ull; };
    PartPlan pl = make_group_plan((uint32_t)g.m, g.k, pick_fmt(kb.keys, kb.offsets, kb.stride) > 0);
    const uint32_t slots = group_pack_slots(g.k);
    const uint64_t chunk_keys = gp_chunk_keys(pl, kb.n);
    const uint64_t max_tiles = (chunk_keys + pl.KT - 1) / pl.KT, max_ntS = (max_tiles + 7) & ~7ull;
    const uint64_t nbytes = group_nbytes(g.m);
    uint32_t* bytes = reinterpret_cast<uint32_t*>(base);
    const uint64_t o_tiles = align256(nbytes);
    const uint64_t o_ends = align256(o_tiles + max_tiles * pl.tile_words * 4);
    const uint64_t o_res = align256(o_ends + max_ntS * pl.nseg * 2);
    const uint64_t o_pos = align256(o_res + max_tiles * pl.CPg);
    uint32_t* tiles = reinterpret_cast<uint32_t*>(base + o_tiles);
    uint16_t* endsT = reinterpret_cast<uint16_t*>(base + o_ends);
    uint8_t* res = reinterpret_cast<uint8_t*>(base + o_res);
    uint16_t* posv = reinterpret_cast<uint16_t*>(base + o_pos);
    const uint32_t pairs = (slots + 1) / 2;
    const uint64_t nwords = (g.m + 31) / 32;
    hipLaunchKernelGGL(k_interleave, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, s, g, nwords, bytes);
    // k_group_out2's dynamic LDS: the tile's result bytes (up to 64 KiB); keys per lane: KT / 1024
    auto out2 = g.k == 10 ? k_group_out2<10, 3> : k_group_out2<19, 2>;
    if (pl.KT > 1024u * (g.k == 10 ? 3u : 2u)) return hipErrorInvalidValue;
    hipError_t e0 = hipFuncSetAttribute(reinterpret_cast<const void*>(out2),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    if (e0 != hipSuccess) return e0;
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
        hipError_t err = launch_group_pack(kb, dk, pl, ntiles, tiles, endsT, posv, kByteSegBits, s);
        if (err != hipSuccess) return err;
        phase_end(kPhaseProbePack, s);
        phase_begin(kPhaseProbeSeg, s);
        const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>(ntiles, (512 + pl.nseg - 1) / pl.nseg));
        hipLaunchKernelGGL(k_group_seg2<4>, dim3(pl.nseg * G), dim3(kPBlock), 0, s, tiles, endsT, ntiles, pl, G, bytes,
                           nbytes, res);
        phase_end(kPhaseProbeSeg, s);
        phase_begin(kPhaseProbeOut, s);
        hipLaunchKernelGGL(out2, dim3(ntiles), dim3(kPBlock), (pl.CPg + 15) & ~15u, s, res,
                           reinterpret_cast<const uint32_t*>(posv), endsT, pl, pairs, dk, g, bounds,
                           out + lo * out_stride, out_stride);
        phase_end(kPhaseProbeOut, s);
        err = hipGetLastError();
        if (err != hipSuccess) return err;
    }
    return hipSuccess;
}

hipError_t launch_multi_probe_group(const KeyBatch& kb, const MultiGroup& g, const uint8_t* bounds, uint8_t* out,
                                    uint32_t out_stride, void* ws, uint64_t ws_bytes, hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    if (!multi_group_supported(g.m, g.k) || g.G < 1 || g.G > kMaxGroup) return hipErrorInvalidValue;
    if (ws_bytes < multi_group_workspace_bytes(kb.n, g.m, g.k)) return hipErrorInvalidValue;
    if (gp_enabled(g.m, g.k, kb.len_prefix))
        return launch_multi_probe_gp(kb, g, bounds, out, out_stride, static_cast<char*>(ws), s);
    const ProbePlan pl = make_probe_plan((uint32_t)g.m, g.k, kByteSegBits);
    const uint64_t chunk_keys = group_chunk_keys(pl, kb.n);
    const uint64_t max_tiles = (chunk_keys + pl.KT - 1) / pl.KT;
    auto align256 = [](uint64_t x) { return (x + 255) & ~255ull; };
    char* base = static_cast<char*>(ws);
    const uint64_t nbytes = group_nbytes(g.m);
    uint32_t* bytes = reinterpret_cast<uint32_t*>(base);
    const uint64_t o_tiles = align256(nbytes);
    uint32_t* tiles = reinterpret_cast<uint32_t*>(base + o_tiles);
    const uint64_t o_res = align256(o_tiles + max_tiles * pl.cap * 4);
    const uint64_t o_ends = align256(o_res + max_tiles * pl.cap);
    const uint64_t o_endsT = align256(o_ends + max_tiles * pl.nseg * 2);
    uint8_t* res = reinterpret_cast<uint8_t*>(base + o_res);
    uint16_t* ends = reinterpret_cast<uint16_t*>(base + o_ends);
    uint16_t* endsT = reinterpret_cast<uint16_t*>(base + o_endsT);

    const uint64_t nwords = (g.m + 31) / 32;
    hipLaunchKernelGGL(k_interleave, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, s, g, nwords, bytes);
    for (uint64_t lo = 0; lo < kb.n; lo += chunk_keys) {
        const uint64_t cn = std::min<uint64_t>(chunk_keys, kb.n - lo);
        DevKeys dk{kb.keys, kb.offsets, kb.off_base, kb.stride, cn};
        if (kb.offsets)
            dk.offsets = kb.offsets + lo;
        else
            dk.keys = kb.keys + lo * kb.stride;
        const uint32_t ntiles = (uint32_t)((cn + pl.KT - 1) / pl.KT);
        phase_begin(kPhaseProbePack, s);
        hipError_t err = launch_probe_pack(kb, dk, pl, ntiles, tiles, ends, kByteSegBits, s);
        if (err != hipSuccess) return err;
        launch_transpose_u16(ends, endsT, ntiles, pl.nseg, s);
        phase_end(kPhaseProbePack, s);
        phase_begin(kPhaseProbeSeg, s);
        const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>(ntiles, (512 + pl.nseg - 1) / pl.nseg));
        hipLaunchKernelGGL(k_group_seg<4>, dim3(pl.nseg * G), dim3(kPBlock), 0, s, tiles, endsT, ntiles, pl, G, bytes,
                           nbytes, res);
        phase_end(kPhaseProbeSeg, s);
        phase_begin(kPhaseProbeOut, s);
        hipLaunchKernelGGL(k_group_out, dim3(ntiles), dim3(kPBlock), 0, s, tiles, ends, res, pl, dk, g, bounds,
                           out + lo * out_stride, out_stride);
        phase_end(kPhaseProbeOut, s);
        err = hipGetLastError();
        if (err != hipSuccess) return err;
    }
    return hipSuccess;
}

}  // namespace vbf
