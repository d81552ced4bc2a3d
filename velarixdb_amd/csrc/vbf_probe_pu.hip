// vbf_probe_pu.hip -- the round-6 partitioned probe: contains() over large batches
// (bf.rs:95-105) on the BUILD's own tile image.
//
// The round-3 probe (vbf_probe_part.hip) sorts 4-byte entries (key id << 20 | offset) and so fits
// 4 092-key tiles at m = 2^32 - 1 (config 5): 4-entry runs, twice the build's.  The round-4 probe
// writes the 2.5-byte group image but pads every run to whole groups in LDS, which at 4 096
// segments would take the whole image.  Here:
//   U1 k_tile_pack<POS = 2> : the build's K1 -- same tile, same unpadded 2.5-byte group image --
//                             plus, per entry, its place in a PADDED numbering (every run rounded up
//                             to whole bytes of result bits) in posv, and the run ends as u32
//                             (end | padded end << 16) in endsT.
//   U3 k_probe_seg3         : k_seg_or's flattened reader over a segment's runs: 8 filter bits per
//                             group, realigned to the run's own result bytes with the next group's
//                             bits (a lane shuffle), one byte store per result byte.  A run owns
//                             whole result bytes, so no two workgroups write one byte.
//   U4 k_probe_out3         : per tile, the result bytes staged in LDS, each key's k bits found
//                             through posv and ANDed: the answer byte, or the tile's hit count.
// The same hashing as the build, the build's run count for the segment pass, and no key id stored.
#include "vbf_tile_pack.hpp"
#include "vbf_tile_pack_rk.hpp"

namespace vbf {

// U1 for the runtime-k classes (k outside {4, 9, 10, 19}, m <= 2^31, every key layout):
// vbf_probe_pu_rk_a.hip (classes 5, 8, 12) and _b (16, 21, 24, 32), compiled in parallel.
hipError_t launch_pu_pack_class_a(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles,
                                  uint32_t* endsT, uint32_t* posv, hipStream_t s);
hipError_t launch_pu_pack_class_b(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles,
                                  uint32_t* endsT, uint32_t* posv, hipStream_t s);
static hipError_t launch_pu_pack_class(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                       uint32_t* tiles, uint32_t* endsT, uint32_t* posv, hipStream_t s) {
    return pl.kc <= 12 ? launch_pu_pack_class_a(fmt, dk, pl, ntiles, tiles, endsT, posv, s)
                       : launch_pu_pack_class_b(fmt, dk, pl, ntiles, tiles, endsT, posv, s);
}

// U3.  Blocks: G consecutive tile ranges per segment, XCD-aware (neighbouring segments on one XCD
// share the L2 lines their short runs sit in, as in k_seg_or).
// MK: a group's run from per-wave run marks and a DPP max-scan (as k_seg_or V7, vbf_partition.hip)
// instead of the binary search's ds_bpermutes.
template <int NG = 4, bool MK = true>
__global__ __launch_bounds__(kPBlock) void k_probe_seg3(const uint32_t* tiles, const uint32_t* endsT, uint32_t ntiles,
                                                        PartPlan pl, uint32_t G, const uint32_t* words, uint8_t* res,
                                                        uint32_t rstride) {
    __shared__ __attribute__((aligned(16))) uint32_t bitmap[kSegWords];
    __shared__ __attribute__((aligned(16))) uint32_t marks[kPBlock / 64][MK ? NG * 16 : 1];
    __shared__ __attribute__((aligned(16))) uint4 rinfo[kPBlock / 64][MK ? 64 : 1];
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
    const uint32_t* row_end = endsT + (uint64_t)seg * pl.ntS;
    const uint32_t* row_beg = seg ? endsT + (uint64_t)(seg - 1) * pl.ntS : nullptr;
    // a group's 8 filter bits (bit c = entry c of the group; entries outside the run are masked later)
    auto test8 = [&](uint4 l, uint32_t nib) -> uint32_t {
        const uint32_t w[4] = {l.x, l.y, l.z, l.w};
        uint32_t r = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint32_t off = ((w[c >> 1] >> ((c & 1) * 16)) & 0xFFFFu) | (((nib >> (4 * c)) & 15u) << 16);
            r |= ((bitmap[off >> 5] >> (off & 31)) & 1u) << c;
        }
        return r;
    };
    auto load_test = [&](uint32_t t, uint32_t gi) -> uint32_t {
        const uint32_t* tile = tiles + (uint64_t)t * pl.tile_words;
        uint4 l;
        __builtin_memcpy(&l, tile + gi * kGroupWords, 16);
        return test8(l, tile[gi * kGroupWords + 4]);
    };
    // bounds of tile t0 + lane: b = the previous segment's (end | padded end << 16) = this run's
    // (begin | padded begin << 16), e = this segment's
    struct FB {
        uint32_t b, e, excl, total;
        uint4 l[NG];
        uint32_t nib[NG];
        uint32_t t[NG], j[NG], ok[NG], rb[NG], re[NG];
    };
    auto prep = [&](uint32_t t0, FB& f) {
        const uint32_t t = t0 + lane;
        uint32_t b = 0, e = 0;
        if (t < t_hi) {
            b = row_beg ? row_beg[t] : 0u;
            e = row_end[t];
        }
        const uint32_t st = b & 0xFFFFu, en = e & 0xFFFFu;
        const uint32_t ch = en > st ? ((en + 7) >> 3) - (st >> 3) : 0u;
        uint32_t incl = ch;
        if constexpr (MK) {
            incl = wave_incl_scan_dpp(ch);
            f.total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        } else {
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= (uint32_t)o) incl += y;
            }
            f.total = (uint32_t)__shfl((int)incl, 63);
        }
        f.b = b;
        f.e = e;
        f.excl = incl - ch;
    };
    // group c of the batch -> run r (binary search over the exclusive prefix), tile, group index and
    // the group's number j within its run
    auto locate = [&](const FB& f, uint32_t t0, uint32_t c, uint32_t& t, uint32_t& gi, uint32_t& j, uint32_t& rb,
                      uint32_t& re) -> uint32_t {
        uint32_t r = 0;
#pragma unroll
        for (int sft = 32; sft; sft >>= 1)
            if ((uint32_t)__shfl((int)f.excl, (int)r + sft) <= c) r += sft;
        rb = (uint32_t)__shfl((int)f.b, (int)r);
        re = (uint32_t)__shfl((int)f.e, (int)r);
        const uint32_t rex = (uint32_t)__shfl((int)f.excl, (int)r);
        t = std::min(t0 + r, t_hi - 1);
        j = c - rex;
        gi = ((rb & 0xFFFFu) >> 3) + j;
        return c < f.total ? 1u : 0u;
    };
    // result byte j of run [st, en) with padded begin pb: entries st + 8j .. st + 8j + 7 = the high
    // bits of group j from slot sh = st & 7 on and the low bits of group j + 1.  The result bytes
    // start all ones (the launcher fills them), so only a byte with a clear bit -- an entry whose
    // filter bit is 0 -- is stored: a positive sweep stores nothing, and the scattered byte stores
    // were what the segment pass waited on (one per run: 21.9 ms per 1B keys at config 5 against
    // the build's 7.9 ms for the same runs)
    auto emit = [&](uint32_t t, uint32_t j, uint32_t rb, uint32_t re, uint32_t bits, uint32_t nbits) {
        const uint32_t st = rb & 0xFFFFu, len = (re & 0xFFFFu) - st, sh = st & 7u;
        if (8 * j >= len) return;
        uint32_t v = ((bits >> sh) | (nbits << (8 - sh))) & 0xFFu;
        if (len - 8 * j < 8) v = (v | (0xFFu << (len - 8 * j))) & 0xFFu;  // bits past the run: pass
        if (v != 0xFFu) res[(uint64_t)t * rstride + ((rb >> 16) >> 3) + j] = (uint8_t)v;
    };
    // lane 63 of the last slot of a step: its run's next group belongs to the next step -- load it
    auto next_own = [&](uint32_t t, uint32_t gi, uint32_t j, uint32_t rb, uint32_t re) -> uint32_t {
        const uint32_t st = rb & 0xFFFFu, len = (re & 0xFFFFu) - st;
        return ((st & 7u) && 8 * j + 8 - (st & 7u) < len) ? load_test(t, gi + 1) : 0u;
    };
    const uint32_t wstep = (kPBlock / 64) * 64;
    auto issue = [&](uint32_t t0, FB& f) {
        if constexpr (MK) {
            // the run marks (vbf_partition.hpp) and the runs' bounds in rinfo (slots past 64 * NG:
            // the search, in consume)
            rinfo[wave][lane] = make_uint4(f.b, f.e, f.excl, 0u);
            run_marks_set<NG>(marks[wave], (f.e & 0xFFFFu) > (f.b & 0xFFFFu), f.excl, lane);
            uint32_t carry = 0;
#pragma unroll
            for (int q = 0; q < NG; ++q) {
                const uint32_t c = (uint32_t)q * 64 + lane;
                const uint32_t r1 = run_marks_find(marks[wave], c, carry);
                f.ok[q] = c < f.total ? 1u : 0u;
                if (f.ok[q]) {
                    const uint4 ri = rinfo[wave][r1 - 1];
                    f.rb[q] = ri.x;
                    f.re[q] = ri.y;
                    f.t[q] = std::min(t0 + r1 - 1, t_hi - 1);
                    f.j[q] = c - ri.z;
                    const uint32_t gi = ((ri.x & 0xFFFFu) >> 3) + f.j[q];
                    const uint32_t* tile = tiles + (uint64_t)f.t[q] * pl.tile_words;
                    __builtin_memcpy(&f.l[q], tile + gi * kGroupWords, 16);
                    f.nib[q] = tile[gi * kGroupWords + 4];
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < NG; ++q) {
                uint32_t gi;
                f.ok[q] = locate(f, t0, (uint32_t)q * 64 + lane, f.t[q], gi, f.j[q], f.rb[q], f.re[q]);
                if (f.ok[q]) {
                    const uint32_t* tile = tiles + (uint64_t)f.t[q] * pl.tile_words;
                    __builtin_memcpy(&f.l[q], tile + gi * kGroupWords, 16);
                    f.nib[q] = tile[gi * kGroupWords + 4];
                }
            }
        }
    };
    auto consume = [&](uint32_t t0, const FB& f) {
        uint32_t bits[NG];
#pragma unroll
        for (int q = 0; q < NG; ++q) bits[q] = f.ok[q] ? test8(f.l[q], f.nib[q]) : 0u;
        // slot (q, lane)'s next group is (q, lane + 1), or (q + 1, 0) for lane 63
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            uint32_t nb = (uint32_t)__shfl_down((int)bits[q], 1);
            const uint32_t n0 = (uint32_t)__shfl((int)bits[q + 1 < NG ? q + 1 : q], 0);
            if (lane == 63) nb = q + 1 < NG ? n0 : (f.ok[q] ? next_own(f.t[q], ((f.rb[q] & 0xFFFFu) >> 3) + f.j[q], f.j[q], f.rb[q], f.re[q]) : 0u);
            if (f.ok[q]) emit(f.t[q], f.j[q], f.rb[q], f.re[q], bits[q], nb);
        }
#pragma unroll 1
        for (uint32_t c0 = 64 * NG; c0 < f.total; c0 += 64) {
            uint32_t t, gi, j, rb, re;
            const uint32_t ok = locate(f, t0, c0 + lane, t, gi, j, rb, re);
            const uint32_t bits1 = ok ? load_test(t, gi) : 0u;
            uint32_t nb = (uint32_t)__shfl_down((int)bits1, 1);
            if (lane == 63 && ok) nb = next_own(t, gi, j, rb, re);
            if (ok) emit(t, j, rb, re, bits1, nb);
        }
    };
    uint32_t t0 = t_lo + wave * 64;
    FB A, B;
    prep(t0, A);
    if (t0 < t_hi) issue(t0, A);
    while (t0 < t_hi) {
        prep(t0 + wstep, B);
        const bool more = t0 + wstep < t_hi;
        if (more) issue(t0 + wstep, B);
        consume(t0, A);
        t0 += wstep;
        if (!more) break;
        prep(t0 + wstep, A);
        const bool more2 = t0 + wstep < t_hi;
        if (more2) issue(t0 + wstep, A);
        consume(t0, B);
        t0 += wstep;
        if (!more2) break;
    }
}

// U4 (OUT 0: answer bytes, 1: hits of the tile -> partial[tile]).  posv: u16 pairs per pair of stash
// slots, [tile][slot / 2][lane of BS]; key l of the tile = round l / BS on lane l % BS, its seeds in
// slots round * K + i.  K compile-time: a lane issues the position loads of its KPT keys together.
// RK: K is a runtime-k class (the stash slots per key); the key's k = pl.k <= K seeds are ANDed.
// PERM: the pack dealt the keys to lanes in length order (offsets layout): slot l is key perm[l].
template <int K, int BS, int KPT, int OUT, bool RK = false, bool PERM = false>
__global__ __launch_bounds__(kPBlock) void k_probe_out3(const uint8_t* res, const uint32_t* posv, PartPlan pl,
                                                        uint32_t pairs, uint32_t rbytes, uint64_t n, uint8_t* out,
                                                        uint32_t* partial) {
    __shared__ uint32_t rl32[65536 / 8 / 4];  // the tile's result bits (rbytes <= 8 KiB)
    __shared__ uint32_t wsum[kPBlock / 64];
    const uint8_t* rl = reinterpret_cast<const uint8_t*>(rl32);
    const uint32_t tid = threadIdx.x, tile = blockIdx.x;
    const uint64_t key0 = (uint64_t)tile * pl.KT;
    const uint32_t nk = (uint32_t)std::min<uint64_t>(pl.KT, n - key0);
    // rbytes is a multiple of 4 and res 256-byte aligned (pu_layout): dword copies
    const uint32_t* src = reinterpret_cast<const uint32_t*>(res + (uint64_t)tile * rbytes);
    uint32_t all = 0xFFFFFFFFu;
    for (uint32_t w = tid; w < rbytes / 4; w += kPBlock) {
        const uint32_t v = src[w];
        rl32[w] = v;
        all &= v;
    }
    // no entry of the tile failed (the segment pass stored none of its result bytes): every key
    // passes, and the position table need not be read -- a positive sweep's common case
    if (__syncthreads_and(all == 0xFFFFFFFFu)) {
        if constexpr (OUT == 0) {
            for (uint32_t l = tid; l < nk; l += kPBlock) out[key0 + l] = 1;
        } else if (tid == 0) {
            partial[blockIdx.x] = nk;
        }
        return;
    }
    const uint32_t* pt = posv + (uint64_t)tile * pairs * BS;
    constexpr int NW = K / 2 + 1;
    uint32_t wv[KPT][NW];
#pragma unroll
    for (int x = 0; x < KPT; ++x) {
        const uint32_t l = tid + x * kPBlock;
        const uint32_t r = l / BS, ln = l % BS;
        const uint32_t wb = (r * K) >> 1;
#pragma unroll
        for (int j = 0; j < NW; ++j) wv[x][j] = (l < nk && wb + j < pairs) ? pt[(wb + j) * BS + ln] : 0u;
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
        const uint32_t odd = ((l / BS) * K) & 1u;
        if (odd) {
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (!RK || (uint32_t)i < pl.k) ok &= bit_at(x, i, 1u);
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (!RK || (uint32_t)i < pl.k) ok &= bit_at(x, i, 0u);
        }
        if constexpr (OUT == 0) {
            if constexpr (PERM)
                out[key0 + reinterpret_cast<const uint16_t*>(posv)[pl.perm_off + (uint64_t)tile * pl.KT + l]] = (uint8_t)ok;
            else
                out[key0 + l] = (uint8_t)ok;
        } else {
            hits += ok;
        }
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

// ---- host side ----

// The shapes U1 has kernels for, every key layout (16 / 32 / 8 / 24-byte rows, any stride, offsets:
// the length order's slot -> key map goes beside the positions) hashed with the length prefix
// (every Vec<u8> key):
//   k = 4 at m = 2^32 - 1 (config 5: SAT remainders, the 1 024-thread shape, seven stash rounds);
//   k = 10 and 19 (p = 1e-4, velarixdb's default) at m <= 2^31: the build's 512-thread
//   one-lane-per-key shape with its full tile -- where the round-4 pipeline (vbf_probe_part.hip)
//   reserves 7 entries of LDS per segment for run padding;
//   any other k <= 32 at m <= 2^31 (k = 4 and 9 too): the runtime-k class packs (_rk_a / _rk_b).
// Other batches take the round-3 / round-4 pipelines; VBF_PROBE_PU = 0 keeps them for these too (A/B).
static bool pu_shape(const PartPlan& pl, bool lp) {
    if (!lp || pl.c16 || !pl.ends_t) return false;
    if (pl.kc) return pl.m <= (1ull << 31) && pl.k1v == 1;  // a runtime-k class (round 6, late)
    if (pl.k == 4) return pl.m == 0xFFFFFFFFull && pl.k1v == 0;
    return (pl.k == 10 || pl.k == 19) && pl.m <= (1ull << 31) && pl.k1v == 1;
}

bool probe_pu_enabled(uint32_t m, uint32_t k, bool lp, bool fixed) {
    const char* e = getenv("VBF_PROBE_PU");  // read per call (A/B)
    static const int sat = [] { const char* v = getenv("VBF_SAT"); return v ? atoi(v) : 1; }();
    if ((e && atoi(e) == 0) || !lp || m == 0) return false;
    // every k but 10 / 19 below 2^32 - 1 runs a runtime-k class pack (k = 4 and 9 included)
    const bool cls = k != 10 && k != 19 && tile_pack_class(k) != 0;
    (void)fixed;
    if (!((k == 4 && m == 0xFFFFFFFFu && sat) || ((k == 10 || k == 19 || cls) && m <= (1u << 31)))) return false;
    const PartPlan pl = make_probe_pu_plan(m, k, fixed, lp);
    // padded ends must fit u16 (C + 7 per segment)
    return pu_shape(pl, lp) && pl.C + 7ull * pl.nseg <= 65535 && pl.CP <= 65535;
}

// bit indices per probe chunk (VBF_PROBE_CHUNK_LOG2, 22-32, read per call): every chunk's segment
// pass reloads the whole filter; the workspace holds one chunk (~5.4 B per bit index)
static uint64_t pu_chunk_idx() {
    const char* e = getenv("VBF_PROBE_CHUNK_LOG2");
    return 1ull << (e ? std::max(22, std::min(32, atoi(e))) : 31);
}

struct PuLayout {
    uint64_t chunk_keys, max_tiles, o_ends, o_res, o_pos, o_perm, o_part, bytes;
    uint32_t rstride, pairs;
};

static PuLayout pu_layout(const PartPlan& pl, bool fixed, uint64_t n) {
    auto align256 = [](uint64_t x) { return (x + 255) & ~255ull; };
    PuLayout L{};
    const uint64_t tiles_per_chunk = std::max<uint64_t>(1, pu_chunk_idx() / pl.C);
    L.chunk_keys = std::min<uint64_t>(n, tiles_per_chunk * pl.KT);
    L.max_tiles = (L.chunk_keys + pl.KT - 1) / pl.KT;
    const uint64_t ntS = (L.max_tiles + 7) & ~7ull;
    // stash slots per lane of the kernel (SPL = 1): its compile-time rounds x seeds
    const K1Shape sh = k1_shape((int)(pl.kc ? pl.kc : pl.k), fixed, (int)pl.k1v);
    L.pairs = (uint32_t)(sh.rounds * sh.kl + 1) / 2;
    // result bytes per tile: every run rounded up to whole bytes, <= (C + 7 * nseg) / 8, 4-aligned
    L.rstride = (uint32_t)(((pl.C + 7ull * pl.nseg + 7) / 8 + 3) & ~3ull);
    L.o_ends = align256(L.max_tiles * pl.tile_words * 4);
    L.o_res = align256(L.o_ends + ntS * pl.nseg * 4);
    L.o_pos = align256(L.o_res + L.max_tiles * L.rstride);
    L.o_perm = align256(L.o_pos + L.max_tiles * (uint64_t)L.pairs * (uint32_t)sh.bs * 4);  // u16 [tile][KT]
    L.o_part = align256(L.o_perm + (fixed ? 0 : L.max_tiles * (uint64_t)pl.KT * 2));
    L.bytes = L.o_part + L.max_tiles * 4 + 256;
    return L;
}

uint64_t probe_pu_workspace_bytes(uint64_t n, uint32_t m, uint32_t k, bool lp) {
    uint64_t need = 0;
    for (bool fixed : {true, false})
        need = std::max(need, pu_layout(make_probe_pu_plan(m, k, fixed, lp), fixed, n).bytes);
    return need;
}

template <int FMT>
static hipError_t launch_pu_pack(const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles,
                                 uint32_t* endsT, uint32_t* posv, hipStream_t s) {
    auto fn = pl.k == 4    ? k_tile_pack<FMT, true, 4, false, false, 0, 0, kSegBits, 2, true>
              : pl.k == 10 ? k_tile_pack<FMT, true, 10, true, false, 1, 0, kSegBits, 2, false>
                           : k_tile_pack<FMT, true, 19, true, false, 1, 0, kSegBits, 2, false>;
    // the segment counters sit at LDS address 0: no static LDS may precede them
    hipFuncAttributes fa{};
    hipError_t err = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(fn));
    if (err == hipSuccess && fa.sharedSizeBytes != 0) err = hipErrorInvalidKernelFile;
    if (err == hipSuccess)
        err = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)pl.lds1);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(fn, dim3(ntiles), dim3(pl.k1v ? 512 : kPBlock), pl.lds1, s, dk, pl, tiles,
                       reinterpret_cast<uint16_t*>(endsT), reinterpret_cast<uint16_t*>(posv));
    return hipGetLastError();
}

hipError_t launch_probe_pu(const KeyBatch& kb, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
                           unsigned long long* count, void* ws, uint64_t ws_bytes, hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    const int fmt = pick_fmt(kb.keys, kb.offsets, kb.stride);
    PartPlan pl = make_probe_pu_plan(m, k, fmt > 0, kb.len_prefix);
    if (!probe_pu_enabled(m, k, kb.len_prefix, fmt > 0) || !pu_shape(pl, kb.len_prefix)) return hipErrorInvalidValue;
    const PuLayout L = pu_layout(pl, fmt > 0, kb.n);
    if (ws_bytes < L.bytes || L.rstride > 65536 / 8) return hipErrorInvalidValue;
    char* base = static_cast<char*>(ws);
    uint32_t* tiles = reinterpret_cast<uint32_t*>(base);
    uint32_t* endsT = reinterpret_cast<uint32_t*>(base + L.o_ends);
    uint8_t* res = reinterpret_cast<uint8_t*>(base + L.o_res);
    uint32_t* posv = reinterpret_cast<uint32_t*>(base + L.o_pos);
    pl.perm_off = (L.o_perm - L.o_pos) / 2;  // the length order's slot -> key map (offsets layout)
    const bool permuted = fmt < 0 && pl.len_order;
    uint32_t* partial = reinterpret_cast<uint32_t*>(base + L.o_part);
    for (uint64_t lo = 0; lo < kb.n; lo += L.chunk_keys) {
        const uint64_t cn = std::min<uint64_t>(L.chunk_keys, kb.n - lo);
        DevKeys dk{kb.keys, kb.offsets, kb.off_base, kb.stride, cn};
        if (kb.offsets)
            dk.offsets = kb.offsets + lo;
        else
            dk.keys = kb.keys + lo * kb.stride;
        const uint32_t ntiles = (uint32_t)((cn + pl.KT - 1) / pl.KT);
        pl.ntS = (ntiles + 7) & ~7u;
        hipError_t err = hipErrorInvalidValue;
        phase_begin(kPhaseProbePack, s);
        if (pl.kc) err = launch_pu_pack_class(fmt, dk, pl, ntiles, tiles, endsT, posv, s);
        else switch (fmt) {
            case 16: err = launch_pu_pack<16>(dk, pl, ntiles, tiles, endsT, posv, s); break;
            case 32: err = launch_pu_pack<32>(dk, pl, ntiles, tiles, endsT, posv, s); break;
            case 8: err = launch_pu_pack<8>(dk, pl, ntiles, tiles, endsT, posv, s); break;
            case 24: err = launch_pu_pack<24>(dk, pl, ntiles, tiles, endsT, posv, s); break;
            case -1: err = launch_pu_pack<-1>(dk, pl, ntiles, tiles, endsT, posv, s); break;
            default: err = launch_pu_pack<0>(dk, pl, ntiles, tiles, endsT, posv, s); break;
        }
        if (err != hipSuccess) return err;
        phase_end(kPhaseProbePack, s);
        phase_begin(kPhaseProbeSeg, s);
        // every result bit starts "pass"; the segment pass stores only bytes with a failing entry
        err = hipMemsetAsync(res, 0xFF, (uint64_t)ntiles * L.rstride, s);
        if (err != hipSuccess) return err;
        const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>(ntiles, (512 + pl.nseg - 1) / pl.nseg));
        hipLaunchKernelGGL(k_probe_seg3<4>, dim3(pl.nseg * G), dim3(kPBlock), 0, s, tiles, endsT, ntiles, pl, G, words,
                           res, L.rstride);
        phase_end(kPhaseProbeSeg, s);
        phase_begin(kPhaseProbeOut, s);
        // KPT = ceil(KT / 1024) keys per thread (k = 4: 7 for the 6 532-key tile, posv rows of 1 024
        // lanes; k = 10: 3 for 3 072, k = 19: 2 for 1 536, rows of 512)
        // classes: K = the class's slots per key, k at run time; KPT from the class's rounds of 512
        auto pick = [&]<int OUT, bool PM>() {
            switch (pl.kc) {
                case 5: return k_probe_out3<5, 512, 3, OUT, true, PM>;
                case 8: return k_probe_out3<8, 512, 3, OUT, true, PM>;
                case 12: return k_probe_out3<12, 512, 3, OUT, true, PM>;
                case 16: return k_probe_out3<16, 512, 2, OUT, true, PM>;
                case 21: return k_probe_out3<21, 512, 2, OUT, true, PM>;
                case 24: return k_probe_out3<24, 512, 1, OUT, true, PM>;
                case 32: return k_probe_out3<32, 512, 1, OUT, true, PM>;
                default: break;
            }
            return pl.k == 4    ? k_probe_out3<4, kPBlock, 7, OUT, false, PM>
                   : pl.k == 10 ? k_probe_out3<10, 512, 3, OUT, false, PM>
                                : k_probe_out3<19, 512, 2, OUT, false, PM>;
        };
        const uint32_t kpt_max = pl.kc ? (pl.kc <= 12 ? 3u : pl.kc <= 21 ? 2u : 1u)
                                       : pl.k == 4 ? 7u : pl.k == 10 ? 3u : 2u;
        if ((pl.KT + kPBlock - 1) / kPBlock > kpt_max) return hipErrorInvalidValue;
        if (count) {
            auto fn = pick.template operator()<1, false>();
            hipLaunchKernelGGL(fn, dim3(ntiles), dim3(kPBlock), 0, s, res, posv, pl, L.pairs,
                               L.rstride, cn, nullptr, partial);
            err = launch_count_finish(partial, ntiles, count, s);
            if (err != hipSuccess) return err;
        } else {
            auto fn = permuted ? pick.template operator()<0, true>() : pick.template operator()<0, false>();
            hipLaunchKernelGGL(fn, dim3(ntiles), dim3(kPBlock), 0, s, res, posv, pl, L.pairs,
                               L.rstride, cn, out + lo, nullptr);
        }
        phase_end(kPhaseProbeOut, s);
        err = hipGetLastError();
        if (err != hipSuccess) return err;
    }
    return hipSuccess;
}

}  // namespace vbf
