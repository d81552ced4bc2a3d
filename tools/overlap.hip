// overlap.hip -- can a VALU-bound hashing kernel and an LDS / L1-return-bound segment reader share
// the CUs?  (splitting k_tile_pack into an LDS-free hash kernel and an
// LDS-only sort, pipelined over chunks on two streams.)
//   hash : SipHash-1-3 of 16-byte keys with the length prefix, k seeds, Barrett remainder, XOR-folded
//          (no memory traffic; sip13.hpp's rounds), 256-thread blocks;
//   read : k_seg_or's flattened read loop (tools/rdflat.hip, g20 groups) with its 128 KiB of LDS,
//          one 1024-thread workgroup per CU, on a k = 19-shaped image;
// each alone, then both at once on two streams.  If `both` is near max(hash, read) rather than the
// sum, the two kinds of work overlap on the same CUs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -I velarixdb_amd/csrc -o tools/overlap tools/overlap.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "sip13.hpp"

using namespace vbf;

template <int K>
__global__ __launch_bounds__(256) void k_hash(uint64_t n, uint64_t m, uint64_t mu, uint32_t* out) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    Sip s = sip_init();
    sip_compress(s, 16);
    sip_compress(s, j * 0x9E3779B97F4A7C15ULL);
    sip_compress(s, j);
    Prefix p{s, 0, 0, 32};
    const SeedCtx q = seed_ctx(p);
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) acc ^= fast_mod31(seed_hash(q, (uint32_t)i), (uint32_t)m, mu);
    if (acc == 0x12345678u) out[0] = acc;
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__global__ void k_gen(uint32_t* bnd, uint32_t ntiles, uint32_t nseg, uint32_t mean, uint32_t* used) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    uint32_t e = 0;
    for (uint32_t s = 0; s < nseg; ++s) {
        const uint32_t len = mean / 2 + mix(t * 7919u + s * 104729u + 17u) % (mean + 1);
        bnd[(uint64_t)s * ntiles + t] = e | ((e + len) << 16);
        e += len;
    }
    atomicMax(used, e);
}

__global__ __launch_bounds__(1024) void k_read(const uint8_t* img, const uint32_t* bnd, uint32_t ntiles, uint32_t nseg,
                                               uint32_t tile_bytes, uint32_t* out) {
    extern __shared__ uint32_t lds[];
    const uint32_t seg = blockIdx.x;
    if (seg >= nseg) return;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t* row = bnd + (uint64_t)seg * ntiles;
    uint32_t acc = 0;
    for (uint32_t t0 = wave * 64; t0 < ntiles; t0 += 16 * 64) {
        const uint32_t t = t0 + lane;
        const uint32_t v = t < ntiles ? row[t] : 0u;
        const uint32_t st = v & 0xFFFFu, en = v >> 16;
        const uint32_t ch = en > st ? (en + 7) / 8 - st / 8 : 0u;
        uint32_t incl = ch;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= (uint32_t)o) incl += y;
        }
        const uint32_t excl = incl - ch, total = (uint32_t)__shfl((int)incl, 63);
        for (uint32_t c = lane; c < total; c += 64) {
            uint32_t r = 0;
#pragma unroll
            for (int sft = 32; sft; sft >>= 1)
                if ((uint32_t)__shfl((int)excl, (int)r + sft) <= c) r += sft;
            const uint32_t rv = (uint32_t)__shfl((int)v, (int)r), rex = (uint32_t)__shfl((int)excl, (int)r);
            const uint8_t* tile = img + (uint64_t)min(t0 + r, ntiles - 1) * tile_bytes;
            const uint32_t gi = (rv & 0xFFFFu) / 8 + (c - rex);
            uint4 l;
            uint32_t nb;
            __builtin_memcpy(&l, tile + gi * 20, 16);
            __builtin_memcpy(&nb, tile + gi * 20 + 16, 4);
            // an LDS OR per group, as k_seg_or does per entry (keeps the LDS pipe busy too)
            atomicOr(&lds[(l.x ^ nb) & 32767], 1u << (l.y & 31));
            acc ^= l.z ^ l.w;
        }
    }
    if (acc == 0x12345678u) out[1] = acc;
}

int main() {
    const uint64_t n = 100000000, m = 1900000000ull, mu = ~0ull / m;
    const uint32_t ntiles = 65105, nseg = 1812, mean = 16;  // k = 19 shape (tools/rdflat.hip)
    uint32_t *bnd, *used, *out;
    uint8_t* img;
    if (hipMalloc(&bnd, (uint64_t)ntiles * nseg * 4) != hipSuccess || hipMalloc(&used, 4) != hipSuccess ||
        hipMalloc(&out, 64) != hipSuccess)
        return 1;
    (void)hipMemset(used, 0, 4);
    hipLaunchKernelGGL(k_gen, dim3((ntiles + 255) / 256), dim3(256), 0, 0, bnd, ntiles, nseg, mean, used);
    uint32_t cap = 0;
    (void)hipMemcpy(&cap, used, 4, hipMemcpyDeviceToHost);
    const uint32_t tile_bytes = ((cap + 7) / 8 * 20 + 16 + 15) & ~15u;
    if (hipMalloc(&img, (uint64_t)ntiles * tile_bytes + 4096) != hipSuccess) return 1;
    (void)hipMemset(img, 1, (uint64_t)ntiles * tile_bytes + 4096);
    const uint32_t lds = 128 * 1024;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_read), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipStream_t s1, s2;
    (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto hash = [&](hipStream_t s) {
        hipLaunchKernelGGL(k_hash<19>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, m, mu, out);
    };
    auto read = [&](hipStream_t s) {
        hipLaunchKernelGGL(k_read, dim3(nseg), dim3(1024), lds, s, img, bnd, ntiles, nseg, tile_bytes, out);
    };
    auto timed = [&](auto&& f) {
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0, 0);
        f();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms;
    };
    hash(s1);
    read(s2);
    (void)hipDeviceSynchronize();
    for (int rep = 0; rep < 3; ++rep) {
        const float th = timed([&] { hash(s1); });
        const float tr = timed([&] { read(s2); });
        const float tb = timed([&] { read(s2); hash(s1); });
        const float tb2 = timed([&] { hash(s1); read(s2); });
        printf("hash %.3f ms  read %.3f ms  sum %.3f  max %.3f  both (read first) %.3f  both (hash first) %.3f\n", th, tr,
               th + tr, th > tr ? th : tr, tb, tb2);
    }
    return 0;
}
