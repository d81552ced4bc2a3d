// Compaction merge on gfx950: the step before the build on the
// compaction path.
//
// velarixdb merges a bucket by folding its tables pairwise -- merged = tables[0]; merged =
// merge_sstables(merged, t) for every further table (compactors/sized.rs:170-200) -- and each
// pairwise merge passes every surviving entry through tombstone_check (:286-320), whose
// `tombstones` map persists across merges and buckets.  The output feeds
// BloomFilter::new(p, n) + build_filter_from_entries (:192-193).
//
// The fold's outcome for one key depends only on that key's entries (at most one per table,
// tables being SkipMaps) and on the map's value for that key, so the GPU version is:
//   1. k_merge_level x ceil(log2 B): stable merge-path merges of the sorted runs (entry ids,
//      ties keep the earlier table first) -> every entry in key order;
//   2. k_fold: one lane per distinct key replays the fold over the B-1 pairwise merges for that
//      key (skipping the merges that cannot change it) with the map value looked up in the
//      sorted input map; it emits the surviving entry id and the key's final map value;
//   3. select (hipcub) -> merged ids in key order, map updates.
// Bit-exact with the literal fold (oracle/oracle.c ora_compact_merge).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <hipcub/device/device_scan.hpp>
#include <hipcub/device/device_select.hpp>

#include "vbf_kernels.hpp"

namespace vbf {

constexpr uint32_t kNone = 0xFFFFFFFFu;

// Rust `Ord for [u8]` on two keys of the arena: 8 bytes at a time as big-endian words (global
// memory takes unaligned 8-byte loads), then the tail byte by byte.
__device__ __forceinline__ uint64_t ld_be64(const uint8_t* p) {
    uint64_t w;
    __builtin_memcpy(&w, p, 8);
    return __builtin_bswap64(w);
}

__device__ __forceinline__ int cmp_keys(const uint8_t* ka, uint64_t la, const uint8_t* kb, uint64_t lb) {
    const uint64_t n = la < lb ? la : lb;
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        const uint64_t x = ld_be64(ka + i), y = ld_be64(kb + i);
        if (x != y) return x < y ? -1 : 1;
    }
    for (; i < n; ++i) {
        const uint32_t x = ka[i], y = kb[i];
        if (x != y) return x < y ? -1 : 1;
    }
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

__device__ __forceinline__ int cmp_ids(const CompactArgs& a, uint32_t x, uint32_t y) {
    const uint64_t bx = a.offsets[x], by = a.offsets[y];
    return cmp_keys(a.keys + bx, a.offsets[x + 1] - bx, a.keys + by, a.offsets[y + 1] - by);
}

// Big-endian 8-byte prefix of a key (zero-padded): prefixes order keys except on ties.
__device__ __forceinline__ uint64_t key_prefix8(const uint8_t* k, uint64_t len) {
    if (len >= 8) return ld_be64(k);
    uint64_t w = 0;
    for (uint64_t i = 0; i < len; ++i) w |= (uint64_t)k[i] << (56 - 8 * i);
    return w;
}

__global__ __launch_bounds__(256) void k_prefixes(CompactArgs a, uint32_t* ids, uint64_t* pfx) {
    const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= a.run_off_host_total) return;
    const uint64_t b = a.offsets[e];
    ids[e] = (uint32_t)e;
    pfx[e] = key_prefix8(a.keys + b, a.offsets[e + 1] - b);
}

// (prefix, id) order: prefixes first, the full keys only on a prefix tie.
__device__ __forceinline__ int cmp_pid(const CompactArgs& a, uint64_t px, uint32_t x, uint64_t py, uint32_t y) {
    if (px != py) return px < py ? -1 : 1;
    return cmp_ids(a, x, y);
}

// Merge levels, two-level merge path.  Pairs (2p, 2p+1) of segments [bnd[s], bnd[s+1]) are cut
// into tiles of kTile outputs; k_merge_split finds every tile's start on its merge path (one
// binary search per tile, over the carried prefixes), k_merge_tile stages the tile's two input
// ranges (ids + prefixes) in LDS and merges them there, 8 outputs per lane.  Stable: on equal
// keys the left (earlier-table) side first.
constexpr uint32_t kTile = 2048;
constexpr uint32_t kTileIpt = kTile / 256;

struct LevelGeom {
    const uint64_t* bnd;       // nseg + 1 segment boundaries
    const uint64_t* tile_base; // npairs + 1: first tile of each pair
    uint32_t nseg, npairs;
    uint64_t ntiles;
};

__device__ __forceinline__ void tile_pair(const LevelGeom& g, uint64_t t, uint32_t& p, uint64_t& a0, uint64_t& a1,
                                          uint64_t& b1) {
    uint32_t lo = 0, hi = g.npairs - 1;  // last pair whose first tile <= t
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) / 2;
        if (g.tile_base[mid] <= t) lo = mid;
        else hi = mid - 1;
    }
    p = lo;
    a0 = g.bnd[2 * p];
    a1 = g.bnd[std::min(2 * p + 1, g.nseg)];
    b1 = g.bnd[std::min(2 * p + 2, g.nseg)];
}

// split[t] = number of A items among the first d outputs of tile t's pair (d = tile start).
__global__ __launch_bounds__(256) void k_merge_split(CompactArgs a, LevelGeom g, const uint32_t* in,
                                                     const uint64_t* pin, uint64_t* split) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= g.ntiles) return;
    uint32_t p;
    uint64_t a0, a1, b1;
    tile_pair(g, t, p, a0, a1, b1);
    const uint64_t na = a1 - a0, nb = b1 - a1, d = (t - g.tile_base[p]) * kTile;
    uint64_t l = d > nb ? d - nb : 0, h = d < na ? d : na;
    while (l < h) {
        const uint64_t mid = (l + h) / 2;
        const uint64_t y = a1 + d - 1 - mid;
        if (cmp_pid(a, pin[a0 + mid], in[a0 + mid], pin[y], in[y]) <= 0) l = mid + 1;
        else h = mid;
    }
    split[t] = l;
}

__global__ __launch_bounds__(256) void k_merge_tile(CompactArgs a, LevelGeom g, const uint32_t* in,
                                                    const uint64_t* pin, const uint64_t* split, uint32_t* out,
                                                    uint64_t* pout) {
    __shared__ uint64_t sp[kTile];
    __shared__ uint32_t si[kTile];
    const uint64_t t = blockIdx.x;
    uint32_t p;
    uint64_t a0, a1, b1;
    tile_pair(g, t, p, a0, a1, b1);
    const uint64_t na = a1 - a0, nb = b1 - a1, n = na + nb;
    const uint64_t d0 = (t - g.tile_base[p]) * kTile, d1 = std::min<uint64_t>(d0 + kTile, n);
    const uint64_t i0 = split[t], j0 = d0 - i0;
    const uint64_t i1 = (t + 1 < g.tile_base[p + 1]) ? split[t + 1] : na, j1 = d1 - i1;
    const uint32_t la = (uint32_t)(i1 - i0), lb = (uint32_t)(j1 - j0);  // la + lb = d1 - d0
    for (uint32_t x = threadIdx.x; x < la + lb; x += 256) {
        const uint64_t src = x < la ? a0 + i0 + x : a1 + j0 + (x - la);
        si[x] = in[src];
        sp[x] = pin[src];
    }
    __syncthreads();
    // this lane's outputs [dt, dt + kTileIpt) of the tile: its own merge path in LDS
    const uint32_t dt = threadIdx.x * kTileIpt, tot = la + lb;
    if (dt >= tot) return;
    uint32_t l = dt > lb ? dt - lb : 0, h = dt < la ? dt : la;
    while (l < h) {
        const uint32_t mid = (l + h) / 2;
        const uint32_t y = la + dt - 1 - mid;
        if (cmp_pid(a, sp[mid], si[mid], sp[y], si[y]) <= 0) l = mid + 1;
        else h = mid;
    }
    uint32_t i = l, j = dt - l;
    const uint32_t stop = std::min(dt + kTileIpt, tot);
    const uint64_t ob = a0 + d0;
    for (uint32_t o = dt; o < stop; ++o) {
        bool take_a;
        if (j >= lb) take_a = true;
        else if (i >= la) take_a = false;
        else take_a = cmp_pid(a, sp[i], si[i], sp[la + j], si[la + j]) <= 0;
        const uint32_t x = take_a ? i++ : la + j++;
        out[ob + o] = si[x];
        pout[ob + o] = sp[x];
    }
}

__device__ __forceinline__ uint32_t run_of(const CompactArgs& a, uint32_t id) {
    uint32_t lo = 0, hi = a.nruns - 1;  // last r with run_off[r] <= id
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) / 2;
        if (a.run_off[mid] <= id) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// One lane per position; lanes at the first entry of a key replay that key's fold.
__global__ __launch_bounds__(256) void k_fold(CompactArgs a, const uint32_t* order, const uint64_t* opfx,
                                              uint64_t total, uint8_t* keep, uint32_t* sel, uint8_t* upd,
                                              int64_t* upd_time) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= total) return;
    keep[p] = 0;
    upd[p] = 0;
    const uint32_t first = order[p];
    const uint64_t fp = opfx[p];
    if (p > 0 && cmp_pid(a, opfx[p - 1], order[p - 1], fp, first) == 0) return;  // not the key's first entry
    uint64_t q = p + 1;
    while (q < total && cmp_pid(a, fp, first, opfx[q], order[q]) == 0) ++q;  // group [p, q): one per table
    const uint8_t* kp = a.keys + a.offsets[first];
    const uint64_t kl = a.offsets[first + 1] - a.offsets[first];

    // the map's value for this key (sorted unique map keys)
    bool has = false;
    int64_t t = 0;
    if (a.map_n) {
        uint64_t l = 0, h = a.map_n;
        while (l < h) {
            const uint64_t mid = (l + h) / 2;
            const int c = cmp_keys(a.map_keys + a.map_off[mid], a.map_off[mid + 1] - a.map_off[mid], kp, kl);
            if (c < 0) l = mid + 1;
            else h = mid;
        }
        if (l < a.map_n &&
            cmp_keys(a.map_keys + a.map_off[l], a.map_off[l + 1] - a.map_off[l], kp, kl) == 0) {
            has = true;
            t = a.map_time[l];
        }
    }
    bool changed = false;
    auto expired = [&](uint32_t e, uint64_t ttl) { return a.now_ms > (uint64_t)a.created[e] + ttl; };
    // tombstone_check (sized.rs:291-320)
    auto check = [&](uint32_t e) -> bool {
        const int64_t c = a.created[e];
        const bool tb = a.tomb[e] != 0;
        if (has) {
            if (c > t) {
                if (tb) {
                    t = c;
                    changed = true;
                    return !expired(e, a.tomb_ttl_ms);
                }
                return a.use_ttl ? !expired(e, a.entry_ttl_ms) : true;
            }
            return false;
        }
        if (tb) {
            has = true;
            t = c;
            changed = true;
            return !expired(e, a.tomb_ttl_ms);
        }
        return a.use_ttl ? !expired(e, a.entry_ttl_ms) : true;
    };
    // the fold: merged = tables[0]; for j in 1..B: merged = merge(merged, tables[j])
    uint64_t gi = p;
    uint32_t cur = kNone;
    if (run_of(a, first) == 0) {
        cur = first;
        ++gi;
    }
    bool stable = false;  // cur is a live non-tombstone that already passed a check
    uint32_t j = 1;
    while (j < a.nruns) {
        const uint32_t next = gi < q ? run_of(a, order[gi]) : a.nruns;
        if (cur == kNone || stable) {
            // merges without an entry of this key in tables[j] cannot change it
            if (next >= a.nruns) break;
            j = next;
        }
        uint32_t b = kNone;
        if (gi < q && next == j) b = order[gi++];
        const uint32_t pick = cur == kNone ? b : b == kNone ? cur : (a.created[cur] > a.created[b] ? cur : b);
        cur = check(pick) ? pick : kNone;
        stable = cur != kNone && !a.tomb[cur];
        ++j;
    }
    if (cur != kNone) {
        keep[p] = 1;
        sel[p] = cur;
    }
    if (changed) {
        upd[p] = 1;
        upd_time[p] = t;
    }
}

// Every run must be strictly increasing (a SkipMap): err[0] = 1 + the first bad position.
__global__ __launch_bounds__(256) void k_check_sorted(CompactArgs a, uint32_t* err) {
    const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (e + 1 >= a.run_off_host_total) return;
    // e and e+1 in the same run?
    uint32_t lo = 0, hi = a.nruns - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) / 2;
        if (a.run_off[mid] <= e + 1) lo = mid;
        else hi = mid - 1;
    }
    if (a.run_off[lo] == e + 1) return;  // e + 1 starts a run
    if (cmp_ids(a, (uint32_t)e, (uint32_t)(e + 1)) >= 0) atomicMin(err, (uint32_t)std::min<uint64_t>(e + 1, 0xFFFFFFFEu));
}

__global__ __launch_bounds__(256) void k_iota(uint32_t* out, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = (uint32_t)i;
}

hipError_t launch_iota_u32(uint32_t* out, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_iota, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, out, n);
    return hipGetLastError();
}

hipError_t compact_check_sorted(const CompactArgs& a, uint32_t* err, hipStream_t s) {
    if (a.run_off_host_total < 2) return hipSuccess;
    hipLaunchKernelGGL(k_check_sorted, dim3((uint32_t)((a.run_off_host_total + 255) / 256)), dim3(256), 0, s, a, err);
    return hipGetLastError();
}

hipError_t compact_merge_levels(const CompactArgs& a, const uint64_t* d_bnd_all, const uint64_t* d_tiles_all,
                                const uint32_t* nseg_per_level, const uint64_t* ntiles_per_level, uint32_t nlevels,
                                uint32_t* ping, uint32_t* pong, uint64_t* pping, uint64_t* ppong, uint64_t* split,
                                uint32_t** result, uint64_t** presult, hipStream_t s) {
    const uint64_t total = a.run_off_host_total;
    hipLaunchKernelGGL(k_prefixes, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, a, ping, pping);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    uint32_t* in = ping;
    uint32_t* out = pong;
    uint64_t* pin = pping;
    uint64_t* pout = ppong;
    const uint64_t* bnd = d_bnd_all;
    const uint64_t* tb = d_tiles_all;
    for (uint32_t l = 0; l < nlevels; ++l) {
        const uint32_t nseg = nseg_per_level[l], npairs = (nseg + 1) / 2;
        const LevelGeom g{bnd, tb, nseg, npairs, ntiles_per_level[l]};
        hipLaunchKernelGGL(k_merge_split, dim3((uint32_t)((g.ntiles + 255) / 256)), dim3(256), 0, s, a, g, in, pin,
                           split);
        hipLaunchKernelGGL(k_merge_tile, dim3((uint32_t)g.ntiles), dim3(256), 0, s, a, g, in, pin, split, out, pout);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        bnd += nseg + 1;
        tb += npairs + 1;
        std::swap(in, out);
        std::swap(pin, pout);
    }
    *result = in;
    *presult = pin;
    return hipSuccess;
}

uint32_t compact_tile() { return kTile; }

hipError_t compact_fold(const CompactArgs& a, const uint32_t* order, const uint64_t* opfx, uint64_t total,
                        uint8_t* keep, uint32_t* sel, uint8_t* upd, int64_t* upd_time, hipStream_t s) {
    hipLaunchKernelGGL(k_fold, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, a, order, opfx, total, keep,
                       sel, upd, upd_time);
    return hipGetLastError();
}

template <class T>
static hipError_t select_flagged(void* tmp, size_t* bytes, const T* in, const uint8_t* flags, T* out,
                                 uint64_t* nsel, uint64_t n, hipStream_t s) {
    return hipcub::DeviceSelect::Flagged(tmp, *bytes, in, flags, out, nsel, (int)n, s);
}

hipError_t select_u32(void* tmp, size_t* bytes, const uint32_t* in, const uint8_t* flags, uint32_t* out,
                      uint64_t* nsel, uint64_t n, hipStream_t s) {
    return select_flagged(tmp, bytes, in, flags, out, nsel, n, s);
}
hipError_t select_i64(void* tmp, size_t* bytes, const int64_t* in, const uint8_t* flags, int64_t* out,
                      uint64_t* nsel, uint64_t n, hipStream_t s) {
    return select_flagged(tmp, bytes, in, flags, out, nsel, n, s);
}

// ---- gather: ids -> packed keys + offsets (+ per-entry arrays), the build's input layout ----
__global__ __launch_bounds__(256) void k_gather_lens(const uint64_t* offsets, const uint32_t* ids, uint64_t n,
                                                     uint64_t* lens) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) lens[i] = offsets[ids[i] + 1] - offsets[ids[i]];
    else if (i == n) lens[i] = 0;
}

__global__ __launch_bounds__(256) void k_gather(GatherArgs g) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= g.n) return;
    const uint32_t id = g.ids[i];
    const uint64_t b = g.offsets[id], len = g.offsets[id + 1] - b, o = g.out_off[i];
    for (uint64_t x = 0; x < len; ++x) g.out_keys[o + x] = g.keys[b + x];
    if (g.out_created) g.out_created[i] = g.created[id];
    if (g.out_tomb) g.out_tomb[i] = g.tomb[id];
    if (g.out_val) g.out_val[i] = g.val[id];
}

hipError_t gather_lens(const uint64_t* offsets, const uint32_t* ids, uint64_t n, uint64_t* lens, hipStream_t s) {
    hipLaunchKernelGGL(k_gather_lens, dim3((uint32_t)((n + 1 + 255) / 256)), dim3(256), 0, s, offsets, ids, n, lens);
    return hipGetLastError();
}

hipError_t scan_u64(void* tmp, size_t* bytes, const uint64_t* in, uint64_t* out, uint64_t n, hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, *bytes, in, out, (int)n, s);
}

hipError_t gather(const GatherArgs& g, hipStream_t s) {
    if (g.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather, dim3((uint32_t)((g.n + 255) / 256)), dim3(256), 0, s, g);
    return hipGetLastError();
}

}  // namespace vbf
