// vbf_partition.hpp -- constants and LDS helpers shared by the partitioned build
// (vbf_partition.hip) and the partitioned probe (vbf_probe_part.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <utility>

#include "keyhash.hpp"
#include "sip13.hpp"
#include "vbf_kernels.hpp"

#ifndef VBF_SEG_BITS
#define VBF_SEG_BITS 20
#endif

namespace vbf {

constexpr int kPBlock = 1024;                // threads per K1 / K3 workgroup
constexpr int kStash = 32;                   // max bit indices a lane keeps in registers
constexpr int kSegBits = VBF_SEG_BITS;       // segment = 2^20 bits = 128 KiB of LDS (default)
constexpr uint32_t kSegWords = 1u << (kSegBits - 5);
constexpr uint32_t kNibMask = (1u << (kSegBits - 16)) - 1;  // in-segment offset bits above 16
static_assert(kSegBits > 16 && kSegBits <= 20, "offset = u16 + up to 4 nibble bits");
constexpr uint32_t kSentinel = 0xFFFFFFFFu;  // never a bit index: idx < m <= 2^32 - 1
constexpr uint32_t kLdsPerCu = 163840;
constexpr uint32_t kShortRun = 24;  // mean entries per (tile, segment) run below which K3 flattens

// Rounds of 1024 keys a lane can stash: kStash / k indices, but k = 4 keeps 24 so the fully
// unrolled K = 4 kernel stays within 64 VGPRs (two workgroups per CU) without spilling.
__host__ __device__ constexpr int rounds_max(int k) { return k == 4 ? 6 : kStash / k; }
// Lanes per key of the build kernels: K = 19 (velarixdb's default p = 1e-4) with a compile-time
// key length splits a key's seeds over two lanes (0..9 and 10..18).  One lane per key stashes 19
// indices per round and fits one round (1 024 keys) in the 64 VGPRs two workgroups per CU allow,
// while the tile's LDS image holds ~1 500 keys: ~11-entry runs for k_seg_or.  Two lanes per key
// stash 10 each, three rounds of 512 keys, and fill the image (the seed-independent prefix is
// absorbed twice: +3 % hashing).  Runtime-length layouts keep more live state and would spill:
// they stay at one lane per key.
__host__ __device__ constexpr int build_spl(int k, bool fixed) { return (k == 19 && fixed) ? 2 : 1; }
// Seeds per lane and stash rounds of the build kernels.
__host__ __device__ constexpr int build_kl(int k, bool fixed) {
    return (k + build_spl(k, fixed) - 1) / build_spl(k, fixed);
}
// The build's fixed-layout K = 4 kernels stash 7 rounds (28 indices; 56-62 VGPRs, no scratch):
// 7 168-key tiles where the LDS holds them (m = 2^32 - 1: with packed counters), 17 % fewer
// k_seg_or runs.  Runtime-length layouts keep 6 (7 spills 12-20 bytes of scratch there).
__host__ __device__ constexpr int build_rounds_max(int k, bool fixed) {
    return build_spl(k, fixed) != 1 ? kStash / build_kl(k, fixed) : (k == 4 && fixed) ? 7 : rounds_max(k);
}

// K1 workgroup shapes (k_tile_pack template parameter V).  V = 0: 1024 threads with the lanes per
// key, seeds per lane and rounds above, at most 64 VGPRs (two workgroups per CU = 8 waves per SIMD).
// V = 1 (compiled k = 10 / 19, <= 2048 segments; runtime-length layouts with plain counters): 512
// threads, one lane per key,
// up to 128 VGPRs -- two workgroups per CU are then 4 waves per SIMD, and the stash holds
// kStashWide indices: k = 19 takes three rounds of 512 keys on one lane each (no idle 20th seed
// slot, the prefix absorbed once), the same 1 536-key tile as V = 0.
constexpr int kStashWide = 64;
struct K1Shape {
    int bs, spl, kl, rounds;
};
__host__ __device__ constexpr K1Shape k1_shape(int k, bool fixed, int v) {
    // k = 4 on this shape (m = 2^32 - 1, VBF_K1_4): fourteen rounds, a 7 168-key tile
    if (v == 1) return K1Shape{512, 1, k, k == 4 ? 14 : kStashWide / k < 6 ? kStashWide / k : 6};
    return K1Shape{kPBlock, build_spl(k, fixed), build_kl(k, fixed), build_rounds_max(k, fixed)};
}

// Inclusive sum over the lanes of a wave with DPP row shifts and row broadcasts (gfx9 wave64): no
// ds_bpermute and so no lane-address registers (hipcc hoists and keeps those alive across a kernel,
// which at 64 VGPRs spills K1's stash).
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); // row_bcast:31 -> rows 2, 3
    return x;
}

// Inclusive max over the lanes of a wave, the same DPP pattern (no LDS).
__device__ __forceinline__ uint32_t wave_incl_max_dpp(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
    return x;
}

// Run marks (round 6): the flattened segment readers deal a wave's runs' groups to lanes back to back
// (slot c = 64 q + lane of row q < NG); the run owning a slot is found without ds_bpermute.  Each run
// with groups marks its first slot (lane + 1) in the wave's byte table `marks` (NG * 16 words; runs
// starting past the table mark nothing -- their slots take the caller's binary search), after the
// caller wrote the runs' bounds to its own per-wave table; a slot's run is then the max of the marks
// up to it, a DPP scan carried across the rows in order.  One wave's LDS operations run in order;
// the fences keep the compiler's.
template <int NG>
__device__ __forceinline__ void run_marks_set(uint32_t* marks, bool has_groups, uint32_t excl, uint32_t lane) {
    for (uint32_t w = lane; w < NG * 16; w += 64) marks[w] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (has_groups && excl < 64u * NG) reinterpret_cast<uint8_t*>(marks)[excl] = (uint8_t)(lane + 1);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
// 1 + the lane of the run owning slot c (rows in order, carry starting at 0); >= 1 for every slot
// below the batch's group total
__device__ __forceinline__ uint32_t run_marks_find(const uint32_t* marks, uint32_t c, uint32_t& carry) {
    const uint32_t r1 = max(wave_incl_max_dpp((uint32_t)reinterpret_cast<const uint8_t*>(marks)[c]), carry);
    carry = (uint32_t)__builtin_amdgcn_readlane((int)r1, 63);
    return r1;
}

// Exclusive scan of v[0..n) in LDS (n <= PER * blockDim.x, blockDim.x <= kPBlock).  EVEN: scan the
// counts rounded up to even (the build's even-length runs) in the same pass.  One barrier: after
// it every wave adds up the totals of the waves before it itself instead of waiting for one wave
// to scan them.  The caller synchronises before reading v[] or reusing wsum[].
template <bool EVEN = false, int PER = 4>
__device__ __forceinline__ void block_exclusive_scan(uint32_t* v, uint32_t n, uint32_t* wsum) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t loc[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t s = tid * PER + q;
        const uint32_t c = s < n ? v[s] : 0;
        loc[q] = EVEN ? (c + 1) & ~1u : c;
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
    static_assert(kPBlock / 64 <= 16, "one 16-lane group sums the wave totals");
    uint32_t before = lane < wave ? wsum[lane] : 0u;  // lanes 0..15 hold the earlier waves' totals
#pragma unroll
    for (int o = 8; o; o >>= 1) before += __shfl_xor(before, o);
    before = (uint32_t)__shfl((int)before, 0);
    uint32_t run = before + incl - sum;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t s = tid * PER + q;
        if (s < n) v[s] = run;
        run += loc[q];
    }
}

// The same over u16 counts packed two per word (count of s = half s & 1 of v[s >> 1]), in place;
// PER counts (PER / 2 words) per thread: n <= PER * blockDim.x (the 512-thread K1 shape with 4 096
// segments takes PER = 8), every start must fit 16 bits (the caller's CP <= 65535).
template <bool EVEN = false, int PER = 4>
__device__ __forceinline__ void block_exclusive_scan16(uint32_t* v, uint32_t n, uint32_t* wsum) {
    static_assert(PER % 2 == 0, "whole words per thread");
    constexpr int PW = PER / 2;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t nw = (n + 1) / 2;
    uint32_t loc[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int w = 0; w < PW; ++w) {
        const uint32_t x = tid * PW + w < nw ? v[tid * PW + w] : 0u;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t c = tid * PER + 2 * w + h < n ? (x >> (16 * h)) & 0xFFFFu : 0u;
            loc[2 * w + h] = EVEN ? (c + 1) & ~1u : c;
            sum += loc[2 * w + h];
        }
    }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= (uint32_t)o) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t before = lane < wave ? wsum[lane] : 0u;
#pragma unroll
    for (int o = 8; o; o >>= 1) before += __shfl_xor(before, o);
    before = (uint32_t)__shfl((int)before, 0);
    uint32_t run = before + incl - sum;
#pragma unroll
    for (int w = 0; w < PW; ++w) {
        const uint32_t r0 = run, r1 = r0 + loc[2 * w];
        run = r1 + loc[2 * w + 1];
        if (tid * PW + w < nw) v[tid * PW + w] = r0 | (r1 << 16);
    }
}

// Compute units of the current device, cached per device: the segment kernels run one workgroup
// per CU (128 KiB of LDS) and split a short last round of segments over the idle ones.
inline uint32_t device_cu_count() {
    static std::atomic<uint32_t> cache[64] = {};  // builds run from several host threads
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    uint32_t n = cache[dev].load(std::memory_order_relaxed);
    if (!n) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) return 0;
        n = (uint32_t)v;
        cache[dev].store(n, std::memory_order_relaxed);
    }
    return n;
}
// VBF_K3_SPLIT = 0 turns the last-round split of k_seg_or and k_probe_seg off (A/B; speed only)
inline bool tail_split_enabled() {
    static const int v = [] { const char* e = getenv("VBF_K3_SPLIT"); return e ? atoi(e) : 1; }();
    return v != 0;
}
inline bool probe_split_enabled() { return tail_split_enabled(); }

// K2 (vbf_partition.hip): ends[rows][cols] -> endsT[cols][rows], shared by build and probe.
void launch_transpose_u16(const uint16_t* in, uint16_t* out, uint32_t rows, uint32_t cols, hipStream_t s);
// The same with row strides (in: in_stride, out: out_stride elements); both multiples of 8 and
// 16-byte aligned buffers take a 16-byte-vector kernel, any other strides an element kernel.
hipError_t launch_transpose_u16_strided(const uint16_t* in, uint16_t* out, uint32_t rows, uint32_t cols,
                                  uint32_t in_stride, uint32_t out_stride, hipStream_t s);

// Partitioned probe plan (vbf_probe_part.hip): KT keys per tile, C = KT * k entries, segments of
// 2^sb filter positions, `cap` padded entries per tile in the workspace.
struct ProbePlan {
    uint32_t k, R, KT, C, nseg, nseg_pad, cap, lds1;
    uint64_t m, mu, nwords;
};
// Segments of an interleaved group of filters (vbf_multi_part.hip): 2^17 one-byte positions.
constexpr int kByteSegBits = 17;
ProbePlan make_probe_plan(uint32_t m, uint32_t k, int sb);
// Q1 (hash + sort entries by segment) for segments of 2^sb positions (kSegBits or kByteSegBits).
hipError_t launch_probe_pack(const KeyBatch& kb, const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles,
                             uint32_t* tiles, uint16_t* ends, int sb, hipStream_t s);

}  // namespace vbf
