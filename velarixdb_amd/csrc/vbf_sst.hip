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
//   k_sst_blocks<EMIT=false>: stage the block in LDS (coalesced dword loads), walk its entry
//                             chain (a dependent chain of u32 reads, but out of LDS), write the
//                             entry count.  A malformed block (an entry crossing the block end,
//                             more than kMaxEnt entries, a block over kStage bytes) sets the
//                             error word instead.
//   exclusive scan of the counts (hipcub) -> entry base E_b of every block; the block's key
//                             bytes start at G_b = start_b - 17 * E_b (all bytes before it are
//                             entries).
//   k_sst_blocks<EMIT=true> : stage + walk again, then lanes write the entry arrays (one lane per
//                             entry) and the packed key bytes (one lane per aligned output dword,
//                             source found by a binary search over the entry starts in LDS).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <hipcub/device/device_scan.hpp>

#include "vbf_kernels.hpp"

namespace vbf {

constexpr int kSstWaves = 4;            // waves per workgroup; one block per wave
constexpr uint32_t kStage = 8192;       // bytes of a block a wave stages (writer max: 4096)
constexpr uint32_t kMaxEnt = 512;       // entries per block (writer max: 4096 / 17 = 240)
constexpr uint32_t kEntryFixed = 17;    // key_len + value offset + created_at + tombstone

enum : uint32_t { kSstErrCross = 1, kSstErrDense = 2, kSstErrBig = 4, kSstErrOrder = 8 };

// u32 at byte offset `o` of an LDS byte image held as dwords (unaligned: two reads + alignbyte).
__device__ __forceinline__ uint32_t lds_u32(const uint32_t* buf, uint32_t o) {
    const uint32_t w0 = buf[o >> 2], w1 = buf[(o >> 2) + 1];
    return __builtin_amdgcn_alignbyte(w1, w0, o & 3);
}
__device__ __forceinline__ uint32_t lds_u8(const uint32_t* buf, uint32_t o) {
    return (buf[o >> 2] >> ((o & 3) * 8)) & 0xFFu;
}

template <bool EMIT>
__global__ __launch_bounds__(64 * kSstWaves) void k_sst_blocks(SstArgs a) {
    __shared__ uint32_t stage[kSstWaves][kStage / 4 + 2];
    __shared__ uint16_t pos[kSstWaves][kMaxEnt];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t b = (uint64_t)blockIdx.x * kSstWaves + wave;
    uint32_t* buf = stage[wave];
    uint16_t* ps = pos[wave];
    if (b >= a.nblocks) return;  // no workgroup barriers below: each wave is independent

    const uint64_t s = a.blocks[b];
    const uint64_t e = b + 1 < a.nblocks ? a.blocks[b + 1] : a.len;
    if (e <= s || e > a.len || (b == 0 && s != 0)) {
        if (lane == 0) {
            atomicOr(a.err, kSstErrOrder);
            atomicMin(a.err + 1, (uint32_t)std::min<uint64_t>(b, 0xFFFFFFFFu));
        }
        return;
    }
    const uint32_t blen = (uint32_t)std::min<uint64_t>(e - s, kStage + 1);
    if (blen > kStage) {
        if (lane == 0) {
            atomicOr(a.err, kSstErrBig);
            atomicMin(a.err + 1, (uint32_t)std::min<uint64_t>(b, 0xFFFFFFFFu));
        }
        return;
    }
    // stage [s & ~3, e) as dwords; byte x of the block is at buf byte sh + x
    const uint64_t a0 = s & ~3ull;
    const uint32_t sh = (uint32_t)(s - a0);
    const uint32_t nw = (sh + blen + 3) / 4;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.data + a0);
    for (uint32_t w = lane; w < nw; w += 64) {
        const uint64_t g = a0 + 4ull * w;
        uint32_t v;
        if (g + 4 <= a.len) {
            v = src[w];
        } else {
            v = 0;
            for (uint32_t t = 0; t < 4; ++t)
                if (g + t < a.len) v |= (uint32_t)a.data[g + t] << (8 * t);
        }
        buf[w] = v;
    }
    if (lane == 0) buf[nw] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // walk the entry chain (every lane in step: same LDS addresses, broadcast reads)
    uint32_t p = 0, n = 0, bad = 0;
    while (p < blen) {
        if (blen - p < 4) {
            bad = kSstErrCross;
            break;
        }
        const uint32_t L = lds_u32(buf, sh + p);
        if ((uint64_t)blen - p - 4 < (uint64_t)L + 13) {
            bad = kSstErrCross;
            break;
        }
        if (n == kMaxEnt) {
            bad = kSstErrDense;
            break;
        }
        if (EMIT && lane == 0) ps[n] = (uint16_t)p;
        p += L + kEntryFixed;
        ++n;
    }
    if (bad) {
        if (lane == 0) {
            atomicOr(a.err, bad);
            atomicMin(a.err + 1, (uint32_t)std::min<uint64_t>(b, 0xFFFFFFFFu));
        }
        return;
    }
    if constexpr (!EMIT) {
        if (lane == 0) a.counts[b] = n;
        return;
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint64_t E = a.ebase[b];
        const uint64_t G = s - (uint64_t)kEntryFixed * E;  // key bytes before this block
        // per-entry arrays
        for (uint32_t i = lane; i < n; i += 64) {
            const uint32_t q = ps[i];
            const uint32_t L = lds_u32(buf, sh + q);
            if (a.offsets) a.offsets[E + i] = G + q - kEntryFixed * i;
            if (a.val_off) a.val_off[E + i] = lds_u32(buf, sh + q + 4 + L);
            if (a.created) {
                const uint64_t lo = lds_u32(buf, sh + q + 8 + L), hi = lds_u32(buf, sh + q + 12 + L);
                a.created[E + i] = lo | (hi << 32);
            }
            if (a.tomb) a.tomb[E + i] = lds_u8(buf, sh + q + 16 + L) == 1;
        }
        const uint64_t K = blen - (uint64_t)kEntryFixed * n;  // this block's key bytes
        if (a.offsets && b + 1 == a.nblocks && lane == 0) a.offsets[E + n] = G + K;
        if (!a.keys || K == 0) return;
        // packed key bytes [G, G + K): lane per aligned output dword.  Output byte d of the
        // block lies in entry i = the last entry with cum(i) = pos(i) - 17 i <= d, at block byte
        // d + 4 + 17 i.
        auto cum = [&](uint32_t i) { return (uint32_t)ps[i] - kEntryFixed * i; };
        const uint64_t w_lo = G >> 2, w_hi = (G + K + 3) >> 2;
        for (uint64_t w = w_lo + lane; w < w_hi; w += 64) {
            const uint64_t g0 = w << 2;
            const uint32_t d0 = g0 < G ? 0 : (uint32_t)(g0 - G);  // first byte of the dword in range
            uint32_t lo = 0, hi = n - 1;                          // last i with cum(i) <= d0
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (cum(mid) <= d0) lo = mid;
                else hi = mid - 1;
            }
            uint32_t i = lo;
            const bool full = g0 >= G && g0 + 4 <= G + K;
            const uint32_t next = i + 1 < n ? cum(i + 1) : (uint32_t)K;
            if (full && d0 + 4 <= next) {  // whole dword inside one key
                reinterpret_cast<uint32_t*>(a.keys)[w] = lds_u32(buf, sh + d0 + 4 + kEntryFixed * i);
                continue;
            }
            uint32_t v = 0;
            for (uint32_t t = 0; t < 4; ++t) {
                const uint64_t g = g0 + t;
                if (g < G || g >= G + K) continue;
                const uint32_t d = (uint32_t)(g - G);
                while (i + 1 < n && cum(i + 1) <= d) ++i;
                const uint32_t byte = lds_u8(buf, sh + d + 4 + kEntryFixed * i);
                if (full) v |= byte << (8 * t);
                else a.keys[g] = (uint8_t)byte;
            }
            if (full) reinterpret_cast<uint32_t*>(a.keys)[w] = v;
        }
    }
}

hipError_t sst_count(const SstArgs& a, hipStream_t s) {
    if (a.nblocks == 0) return hipSuccess;
    const uint64_t grid = (a.nblocks + kSstWaves - 1) / kSstWaves;
    hipLaunchKernelGGL(k_sst_blocks<false>, dim3((uint32_t)grid), dim3(64 * kSstWaves), 0, s, a);
    return hipGetLastError();
}

hipError_t sst_emit(const SstArgs& a, hipStream_t s) {
    if (a.nblocks == 0) return hipSuccess;
    const uint64_t grid = (a.nblocks + kSstWaves - 1) / kSstWaves;
    hipLaunchKernelGGL(k_sst_blocks<true>, dim3((uint32_t)grid), dim3(64 * kSstWaves), 0, s, a);
    return hipGetLastError();
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
