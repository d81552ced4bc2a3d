// Batched read-path probe across SSTs.
//
// velarixdb answers a get by walking its key ranges: an SST is a candidate when the key lies in
// [smallest_key, biggest_key] (Vec<u8> order) and its filter contains the key
// (KeyRange::filter_sstables_by_key_range, src/key_range/range.rs:91-147; filter.contains at
// :136).  Per key and per SST it re-hashes the key k times (bf.rs:95-105).  Here one lane takes
// one key against every SST: the seed-independent SipHash blocks are absorbed once, and since
// calculate_hash(key, i) does not depend on the filter, the first four seed hashes are computed
// once and reused by every SST (only `% m` and the bit test differ).
//
// Output: out[j * nsst + s] = 1 when SST s is a candidate for key j (bit-identical to the
// reference's range test && contains()).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keyhash.hpp"
#include "sip13.hpp"
#include "vbf_kernels.hpp"

namespace vbf {

template <int FMT, bool LP>
__global__ __launch_bounds__(256) void k_multi_probe(MultiArgs a) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= a.n) return;
    const DevKeys dk{a.keys, a.offsets, a.off_base, a.stride, a.n};
    const uint8_t* kp;
    uint64_t kl;
    if (a.offsets) {
        kp = a.keys + (a.offsets[j] - a.off_base);
        kl = a.offsets[j + 1] - a.offsets[j];
    } else {
        kp = a.keys + j * a.stride;
        kl = a.stride;
    }
    const Prefix p = key_prefix<FMT, LP>(dk, j);
    // Seed hashes 0..3 are formed once, on the first table whose range holds the key, and kept
    // in named registers: a memo indexed by the runtime seed number was lowered to a scratch
    // array (a scratch load per bit test).
    uint64_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    bool have = false;
    uint8_t* out = a.out + j * a.out_stride;
    for (uint32_t s = 0; s < a.nsst; ++s) {
        const MultiSst d = a.tab[s];
        bool hit = true;
        if (a.bounds) {  // range.rs:118: searched_key >= smallest_key && searched_key <= biggest_key
            hit = cmp_bytes(kp, kl, a.bounds + d.lo_beg, d.lo_end - d.lo_beg) >= 0 &&
                  cmp_bytes(kp, kl, a.bounds + d.hi_beg, d.hi_end - d.hi_beg) <= 0;
        }
        if (hit && d.k > 0 && d.m == 0) {  // bf.rs:100 `% 0`: the reference panics on this key
            atomicOr(a.err, 1u);
            hit = false;
        } else if (hit && d.k > 0) {  // bf.rs:95-105, k == 0 -> true; early exit on the first clear bit
            if (!have) {
                h0 = prefix_hash(p, 0);
                h1 = prefix_hash(p, 1);
                h2 = prefix_hash(p, 2);
                h3 = prefix_hash(p, 3);
                have = true;
            }
            auto test = [&](uint64_t h) -> bool {  // per-table m: a wave-uniform choice of remainder code
                const uint32_t idx = d.m <= (1ull << 31) ? fast_mod31(h, (uint32_t)d.m, d.mu) : fast_mod(h, d.m, d.mu);
                return (d.words[idx >> 5] >> (idx & 31)) & 1u;
            };
            hit = test(h0) && (d.k < 2 || test(h1)) && (d.k < 3 || test(h2)) && (d.k < 4 || test(h3));
            for (uint32_t i = 4; hit && i < d.k; ++i) hit = test(prefix_hash(p, i));
        }
        out[d.col] = hit ? 1 : 0;
    }
}

hipError_t launch_multi_probe(const MultiArgs& a, bool len_prefix, hipStream_t s) {
    if (a.n == 0 || a.nsst == 0) return hipSuccess;
    const uint64_t blocks = (a.n + 255) / 256;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    with_fmt(pick_fmt(a.keys, a.offsets, a.stride), len_prefix, [&]<int FMT, bool LP>() {
        hipLaunchKernelGGL((k_multi_probe<FMT, LP>), dim3((unsigned)blocks), dim3(256), 0, s, a);
    });
    return hipGetLastError();
}

}  // namespace vbf
