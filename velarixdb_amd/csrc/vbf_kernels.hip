// vbf_kernels.hip -- gfx950 kernels for velarixdb's Bloom-filter path.
//
//   Build  : BloomFilter::set over a key batch (bf.rs:84-92 via build_filter_from_entries :126-128)
//   Probe  : BloomFilter::contains per key (bf.rs:95-105), one answer byte per key
//   Count  : Probe + per-wave ballot popcount, one 64-bit atomic per wave (FPR sweeps)
//   Hashes : the raw calculate_hash values (bf.rs:222-227), for parity tests
//
// Layout in HBM: keys packed back to back, either fixed stride (key j at j*stride) or
// offsets[N+1] (u64, key j = [offsets[j]-off_base, offsets[j+1]-off_base)).  Filter =
// ceil(m/32) u32 words, bit i = word[i>>5] bit (i&31) (bit-vec 0.6.3 BitVec<u32>).
//
// One lane per key: the lane absorbs the shared `LE64(len) || key` blocks once, then runs
// 5 SipRounds per seed.  Fixed 8/16/24/32-byte keys get a specialised kernel with
// 16-byte coalesced loads (the 100M x 16 B headline workload).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keyhash.hpp"
#include "sip13.hpp"
#include "vbf_kernels.hpp"

namespace vbf {

enum class Op { Build, Probe, Count, Hashes };

struct Args {
    const uint8_t* keys;
    const uint64_t* offsets;
    uint64_t off_base;
    uint64_t stride;
    uint64_t n;
    uint64_t m;
    uint64_t mu;
    uint32_t k;
    uint32_t* words;         // Build
    const uint32_t* rwords;  // Probe / Count
    uint8_t* out;            // Probe
    uint64_t* out64;         // Hashes
    uint32_t* partial;          // Count: one hit count per workgroup, summed by k_count_finish
    uint64_t part_base;
};

constexpr int kBlock = 256;

// The per-key action, given a callable hash(i) for seeds i = 0..k-1.  Returns the probe answer.
template <Op OP, bool M31, class H>
__device__ __forceinline__ bool act(const Args& a, uint64_t j, const H& hash) {
    if constexpr (OP == Op::Build) {
        for (uint32_t i = 0; i < a.k; ++i) {
            const uint32_t idx = fast_mod(hash(i), a.m, a.mu);
            atomicOr(a.words + (idx >> 5), 1u << (idx & 31));  // no-return global_atomic_or
        }
        return true;
    } else if constexpr (OP == Op::Hashes) {
        for (uint32_t i = 0; i < a.k; ++i) a.out64[j * a.k + i] = hash(i);
        return true;
    } else {
        bool hit = true;  // k == 0 -> vacuously true (bf.rs:104)
        for (uint32_t i = 0; i < a.k; ++i) {
            const uint32_t idx = mod_m<M31>(hash(i), a.m, a.mu);
            if (!((a.rwords[idx >> 5] >> (idx & 31)) & 1u)) {  // bf.rs:100-102 early exit
                hit = false;
                break;
            }
        }
        if constexpr (OP == Op::Probe) a.out[j] = hit ? 1 : 0;
        return hit;
    }
}

// Hits per workgroup go to a partial array (one plain store each), not to one global counter:
// a same-address atomic per wave serialises at the L2 (~1.6M of them for 100M keys).
template <Op OP>
__device__ __forceinline__ void finish_count(const Args& a, bool hit) {
    if constexpr (OP == Op::Count) {
        __shared__ uint32_t wsum[kBlock / 64];
        const unsigned long long mask = __ballot(hit);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = (uint32_t)__popcll(mask);
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (int w = 0; w < kBlock / 64; ++w) t += wsum[w];
            a.partial[a.part_base + blockIdx.x] = t;
        }
    }
}

// Sum of np partial counts, added to *count with one atomic.
__global__ __launch_bounds__(1024) void k_count_finish(const uint32_t* partial, uint64_t np,
                                                       unsigned long long* count) {
    __shared__ unsigned long long ws[16];
    unsigned long long t = 0;
    for (uint64_t i = threadIdx.x; i < np; i += 1024) t += partial[i];
    for (int o = 32; o > 0; o >>= 1) t += __shfl_down(t, o);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int w = 0; w < 16; ++w) s += ws[w];
        atomicAdd(count, s);
    }
}

hipError_t launch_count_finish(const uint32_t* partial, uint64_t np, unsigned long long* count, hipStream_t s) {
    hipLaunchKernelGGL(k_count_finish, dim3(1), dim3(1024), 0, s, partial, np, count);
    return hipGetLastError();
}

uint64_t count_partials(uint64_t n) { return (n + kBlock - 1) / kBlock + 2; }

// ---- one lane per key, any layout (keyhash.hpp) ----
template <Op OP, int FMT, bool LP, bool M31>
__global__ __launch_bounds__(kBlock) void k_keys(Args a) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    bool hit = false;
    if (j < a.n) {
        const DevKeys dk{a.keys, a.offsets, a.off_base, a.stride, a.n};
        const Prefix p = key_prefix<FMT, LP>(dk, j);
        hit = act<OP, M31>(a, j, [&](uint32_t i) { return prefix_hash(p, i); });
    }
    finish_count<OP>(a, hit);
}

// ---- host-side dispatch ----

template <Op OP>
static void dispatch(const Args& a, bool lp, hipStream_t s) {
    const uint64_t blocks = (a.n + kBlock - 1) / kBlock;
    with_fmt(pick_fmt(a.keys, a.offsets, a.stride), lp, [&]<int FMT, bool LP>() {
        // probes with m <= 2^31: the one-word remainder (sip13.hpp fast_mod31) on the lookup chain
        constexpr bool kProbe = OP == Op::Probe || OP == Op::Count;
        if (kProbe && a.m <= (1ull << 31))
            hipLaunchKernelGGL((k_keys<OP, FMT, LP, kProbe>), dim3((unsigned)blocks), dim3(kBlock), 0, s, a);
        else
            hipLaunchKernelGGL((k_keys<OP, FMT, LP, false>), dim3((unsigned)blocks), dim3(kBlock), 0, s, a);
    });
}

static Args make_args(const KeyBatch& kb, uint64_t m, uint32_t k) {
    Args a{};
    a.keys = kb.keys;
    a.offsets = kb.offsets;
    a.off_base = kb.off_base;
    a.stride = kb.stride;
    a.n = kb.n;
    a.m = m;
    a.mu = m ? (~0ull / m) : 0;
    a.k = k;
    return a;
}

// Largest grid one launch takes; bigger batches are split (keys never move).
static constexpr uint64_t kMaxKeysPerLaunch = (uint64_t)kBlock * 0x7fffffffull;

template <Op OP, class F>
static hipError_t for_chunks(const KeyBatch& kb, F&& f) {
    for (uint64_t lo = 0; lo < kb.n; lo += kMaxKeysPerLaunch) {
        KeyBatch c = kb;
        c.n = (kb.n - lo) < kMaxKeysPerLaunch ? (kb.n - lo) : kMaxKeysPerLaunch;
        if (kb.offsets) {
            c.offsets = kb.offsets + lo;
        } else {
            c.keys = kb.keys + lo * kb.stride;
        }
        f(c, lo);
    }
    return hipGetLastError();
}

hipError_t launch_build(const KeyBatch& kb, uint32_t m, uint32_t k, uint32_t* words, hipStream_t s) {
    if (kb.n == 0 || k == 0) return hipSuccess;
    phase_begin(kPhaseAtomicBuild, s);
    hipError_t e = for_chunks<Op::Build>(kb, [&](const KeyBatch& c, uint64_t) {
        Args a = make_args(c, m, k);
        a.words = words;
        dispatch<Op::Build>(a, c.len_prefix, s);
    });
    phase_end(kPhaseAtomicBuild, s);
    return e;
}

hipError_t launch_probe(const KeyBatch& kb, uint32_t m, uint32_t k, const uint32_t* words,
                        uint8_t* out, hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    phase_begin(kPhaseProbe, s);
    hipError_t e = for_chunks<Op::Probe>(kb, [&](const KeyBatch& c, uint64_t lo) {
        Args a = make_args(c, m, k);
        a.rwords = words;
        a.out = out + lo;
        dispatch<Op::Probe>(a, c.len_prefix, s);
    });
    phase_end(kPhaseProbe, s);
    return e;
}

hipError_t launch_count(const KeyBatch& kb, uint32_t m, uint32_t k, const uint32_t* words,
                        unsigned long long* count, uint32_t* partial, hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    phase_begin(kPhaseProbe, s);
    hipError_t e = for_chunks<Op::Count>(kb, [&](const KeyBatch& c, uint64_t lo) {
        Args a = make_args(c, m, k);
        a.rwords = words;
        a.partial = partial;
        a.part_base = lo / kBlock;  // chunks hold whole multiples of kBlock keys
        dispatch<Op::Count>(a, c.len_prefix, s);
    });
    if (e == hipSuccess) e = launch_count_finish(partial, (kb.n + kBlock - 1) / kBlock, count, s);
    phase_end(kPhaseProbe, s);
    return e;
}

hipError_t launch_hashes(const KeyBatch& kb, uint32_t k, uint64_t* out, hipStream_t s) {
    if (kb.n == 0 || k == 0) return hipSuccess;
    return for_chunks<Op::Hashes>(kb, [&](const KeyBatch& c, uint64_t lo) {
        Args a = make_args(c, 0, k);
        a.out64 = out + lo * k;
        dispatch<Op::Hashes>(a, c.len_prefix, s);
    });
}

// ---- bitwise OR of filter arrays (multi-GPU partial filters, bf.rs OR semantics) ----
__global__ __launch_bounds__(kBlock) void k_or_words(uint32_t* dst, const uint32_t* src, uint64_t nw) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock * 4;
    for (uint64_t i = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 4; i < nw; i += stride) {
        if (i + 4 <= nw) {
            uint4 d = *reinterpret_cast<const uint4*>(dst + i);
            const uint4 v = *reinterpret_cast<const uint4*>(src + i);
            d.x |= v.x; d.y |= v.y; d.z |= v.z; d.w |= v.w;
            *reinterpret_cast<uint4*>(dst + i) = d;
        } else {
            for (uint64_t t = i; t < nw; ++t) dst[t] |= src[t];
        }
    }
}

hipError_t launch_or_words(uint32_t* dst, const uint32_t* src, uint64_t nwords, hipStream_t s) {
    if (nwords == 0) return hipSuccess;
    uint64_t blocks = (nwords / 4 + kBlock - 1) / kBlock;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    const bool al = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0;
    if (!al) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_or_words, dim3((unsigned)blocks), dim3(kBlock), 0, s, dst, src, nwords);
    return hipGetLastError();
}

// dst = src[0] | src[1] | ... | src[parts - 1], the parts `pstride` words apart: the fold of the
// multi-GPU OR all-reduce (dist.or_allreduce_) in one pass -- every part read once, dst written
// once -- where parts - 1 k_or_words launches re-read and re-write the accumulator each time.
__global__ __launch_bounds__(kBlock) void k_or_fold(uint32_t* dst, const uint32_t* src, uint64_t nw, uint32_t parts,
                                                    uint64_t pstride) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock * 4;
    for (uint64_t i = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 4; i < nw; i += stride) {
        if (i + 4 <= nw) {
            uint4 d = *reinterpret_cast<const uint4*>(src + i);
            for (uint32_t p = 1; p < parts; ++p) {
                const uint4 v = *reinterpret_cast<const uint4*>(src + (uint64_t)p * pstride + i);
                d.x |= v.x; d.y |= v.y; d.z |= v.z; d.w |= v.w;
            }
            *reinterpret_cast<uint4*>(dst + i) = d;
        } else {
            for (uint64_t t = i; t < nw; ++t) {
                uint32_t d = src[t];
                for (uint32_t p = 1; p < parts; ++p) d |= src[(uint64_t)p * pstride + t];
                dst[t] = d;
            }
        }
    }
}

hipError_t launch_or_fold(uint32_t* dst, const uint32_t* src, uint64_t nwords, uint32_t parts, uint64_t pstride,
                          hipStream_t s) {
    if (nwords == 0 || parts == 0) return hipSuccess;
    uint64_t blocks = (nwords / 4 + kBlock - 1) / kBlock;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    const bool al = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0 && pstride % 4 == 0;
    if (!al) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_or_fold, dim3((unsigned)blocks), dim3(kBlock), 0, s, dst, src, nwords, parts, pstride);
    return hipGetLastError();
}

// ---- popcount of a filter (fill ratio reporting) ----
__global__ __launch_bounds__(kBlock) void k_popcount(const uint32_t* w, uint64_t nw,
                                                      unsigned long long* out) {
    unsigned long long acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nw; i += stride)
        acc += __popc(w[i]);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

hipError_t launch_popcount(const uint32_t* words, uint64_t nwords, unsigned long long* out,
                           hipStream_t s) {
    if (nwords == 0) return hipSuccess;
    uint64_t blocks = (nwords + kBlock - 1) / kBlock;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_popcount, dim3((unsigned)blocks), dim3(kBlock), 0, s, words, nwords, out);
    return hipGetLastError();
}

// ---- synthetic workloads (bench / tests; same definitions as oracle/oracle.c) ----
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ULL;

__global__ __launch_bounds__(kBlock) void k_gen_fixed(uint64_t seed, uint64_t base, uint64_t n,
                                                       uint32_t len, uint8_t* out) {
    const uint64_t jj = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (jj >= n) return;
    const uint64_t j = base + jj;
    uint8_t* o = out + jj * len;
    if (len == 16 && ((reinterpret_cast<uintptr_t>(o) & 15) == 0)) {
        *reinterpret_cast<ulonglong2*>(o) = ulonglong2{splitmix64(seed ^ j), j};
        return;
    }
    for (uint32_t c = 0; c * 8 < len; ++c) {
        const uint64_t w = c == 0 ? splitmix64(seed ^ j) : c == 1 ? j : splitmix64(seed ^ j ^ (c * kGolden));
        for (uint32_t b = 0; b < 8 && c * 8 + b < len; ++b) o[c * 8 + b] = (uint8_t)(w >> (8 * b));
    }
}

hipError_t launch_gen_fixed(uint64_t seed, uint64_t base, uint64_t n, uint32_t len, uint8_t* out,
                            hipStream_t s) {
    if (n == 0 || len == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_fixed, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       seed, base, n, len, out);
    return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void k_gen_var(uint64_t seed, uint64_t base, uint64_t n,
                                                     const uint64_t* offsets, uint8_t* out) {
    const uint64_t jj = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (jj >= n) return;
    const uint64_t j = base + jj;
    const uint64_t beg = offsets[jj];
    const uint64_t len = offsets[jj + 1] - offsets[jj];
    uint8_t* o = out + beg;
    for (uint64_t c = 0; c * 8 < len; ++c) {
        const uint64_t w = c == 0 ? ((j << 8) | (seed & 0xff)) : splitmix64(seed ^ j ^ (c * kGolden));
        for (uint32_t b = 0; b < 8 && c * 8 + b < len; ++b) o[c * 8 + b] = (uint8_t)(w >> (8 * b));
    }
}

hipError_t launch_gen_var(uint64_t seed, uint64_t base, uint64_t n, const uint64_t* offsets,
                          uint8_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_var, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       seed, base, n, offsets, out);
    return hipGetLastError();
}

}  // namespace vbf
