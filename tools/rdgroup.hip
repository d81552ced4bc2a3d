// rdgroup.hip -- k_seg_or's read pattern on realistic tile images, two packed formats:
//   split : the current image -- u16 low halves of every entry, then 4-bit nibbles (8 per word) in a
//           separate area; runs padded to even length, a run read as 16 B of low halves + the 8 B
//           around its nibbles per lane (8 entries per lane)
//   group : 8-entry groups of 20 B (16 B of low halves, then that group's nibble word), runs not
//           padded; a run read as whole groups (group-aligned 16 B + 4 B per lane)
// Run lengths per (tile, segment): mean M, uniform +-M/2 (the real ones are ~Poisson(M)).
// Reads only (k_seg_or with its LDS ORs ablated is read-bound).  LPR = lanes
// per run (8: k_seg_or's 8-lane groups; 4: four lanes per run, 16 runs per load instruction).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/rdgroup tools/rdgroup.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// one thread per tile: run bounds (begin | end << 16, in entries) into bnd[seg][tile]; split
// format rounds every run up to even length.  cap[tile] = entries used.
__global__ void k_gen(uint32_t* bnd, uint32_t ntiles, uint32_t nseg, uint32_t mean, int split, uint32_t* used) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    uint32_t e = 0;
    for (uint32_t s = 0; s < nseg; ++s) {
        uint32_t len = mean / 2 + mix(t * 7919u + s * 104729u + 17u) % (mean + 1);
        if (split) len = (len + 1) & ~1u;
        bnd[(uint64_t)s * ntiles + t] = e | ((e + len) << 16);
        e += len;
    }
    atomicMax(used, e);
}

template <bool GROUP, int LPR, int NG>
__global__ __launch_bounds__(1024) void k_read(const uint8_t* img, const uint32_t* bnd, uint32_t ntiles,
                                               uint32_t nseg, uint32_t tile_bytes, uint32_t cp, uint32_t* out) {
    const uint32_t nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
    const uint32_t seg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
    if (seg >= nseg) return;
    constexpr uint32_t RPI = 64 / LPR;  // runs per load instruction
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, grp = lane / LPR, q = lane % LPR;
    const uint32_t* row = bnd + (uint64_t)seg * ntiles;
    uint32_t acc = 0;
    const uint32_t step = 16 * RPI * NG;
    uint32_t t0 = wave * RPI * NG;
    auto lb = [&](uint32_t tb, int g) -> uint32_t {
        const uint32_t t = tb + g * RPI + grp;
        return t < ntiles ? row[t] : 0u;
    };
    uint32_t be[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) be[g] = lb(t0, g);
    while (t0 < ntiles) {
        uint4 l[NG];
        uint32_t nb[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const uint32_t st = be[g] & 0xFFFFu, en = be[g] >> 16;
            const uint32_t t = min(t0 + g * RPI + grp, ntiles - 1);
            const uint8_t* tile = img + (uint64_t)t * tile_bytes;
            if (GROUP) {
                uint32_t gi = (st >> 3) + q;
                if (gi * 8 >= en) gi = st >> 3;
                __builtin_memcpy(&l[g], tile + gi * 20, 16);
                __builtin_memcpy(&nb[g], tile + gi * 20 + 16, 4);
            } else {
                const uint32_t e = st + q * 8 < en ? st + q * 8 : st;
                __builtin_memcpy(&l[g], tile + e * 2, 16);
                uint2 h;
                __builtin_memcpy(&h, tile + cp * 2 + (e >> 3) * 4, 8);
                nb[g] = h.x ^ h.y;
            }
        }
        const uint32_t tn = t0 + step;
#pragma unroll
        for (int g = 0; g < NG; ++g) be[g] = lb(tn, g);
#pragma unroll
        for (int g = 0; g < NG; ++g) acc ^= l[g].x ^ l[g].y ^ l[g].z ^ l[g].w ^ nb[g];
        // runs longer than LPR * 8 entries: the rest (rare at these means)
        t0 = tn;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <bool GROUP, int LPR, int NG>
static float run(const uint8_t* img, const uint32_t* bnd, uint32_t ntiles, uint32_t nseg, uint32_t tile_bytes,
                 uint32_t cp, uint32_t* out) {
    const uint32_t nwg = nseg;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_read<GROUP, LPR, NG>), dim3(nwg), dim3(1024), 0, 0, img, bnd, ntiles, nseg, tile_bytes, cp, out);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL((k_read<GROUP, LPR, NG>), dim3(nwg), dim3(1024), 0, 0, img, bnd, ntiles, nseg, tile_bytes, cp, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    struct Cfg { const char* name; uint32_t ntiles, nseg, mean; };
    // k = 10: 100M keys / 3072 per tile, m = 1e9; k = 19: 100M / 1536, m = 1.9e9
    const Cfg cfgs[] = {{"k10", 32553, 954, 32}, {"k19", 65105, 1812, 16}};
    for (const Cfg& c : cfgs) {
        uint32_t *bnd, *used, *out;
        const uint64_t nb = (uint64_t)c.ntiles * c.nseg;
        if (hipMalloc(&bnd, nb * 4) != hipSuccess || hipMalloc(&used, 4) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
        for (int split = 1; split >= 0; --split) {
            (void)hipMemset(used, 0, 4);
            hipLaunchKernelGGL(k_gen, dim3((c.ntiles + 255) / 256), dim3(256), 0, 0, bnd, c.ntiles, c.nseg, c.mean, split, used);
            uint32_t cap = 0;
            (void)hipMemcpy(&cap, used, 4, hipMemcpyDeviceToHost);
            const uint32_t cp = (cap + 15) & ~7u;
            const uint32_t tile_bytes = split ? cp * 2 + cp / 2 : (cp / 8 + 1) * 20;
            const uint64_t bytes = (uint64_t)c.ntiles * tile_bytes + 4096;
            uint8_t* img;
            if (hipMalloc(&img, bytes) != hipSuccess) return 1;
            (void)hipMemset(img, 1, bytes);
            const double entries = (double)c.ntiles * c.nseg * c.mean;
            auto show = [&](const char* v, float ms) {
                printf("%s %-6s %-10s %.3f ms  (%.1f G runs/s, %u B per tile, %.2f GB image)\n", c.name,
                       split ? "split" : "group", v, ms, (double)nb / (ms * 1e-3) / 1e9, tile_bytes,
                       (double)c.ntiles * tile_bytes / 1e9);
            };
            (void)entries;
            if (split) {
                show("lpr8 ng5", run<false, 8, 5>(img, bnd, c.ntiles, c.nseg, tile_bytes, cp, out));
                show("lpr4 ng5", run<false, 4, 5>(img, bnd, c.ntiles, c.nseg, tile_bytes, cp, out));
                show("lpr8 ng5", run<false, 8, 5>(img, bnd, c.ntiles, c.nseg, tile_bytes, cp, out));
            } else {
                show("lpr8 ng5", run<true, 8, 5>(img, bnd, c.ntiles, c.nseg, tile_bytes, cp, out));
                show("lpr4 ng5", run<true, 4, 5>(img, bnd, c.ntiles, c.nseg, tile_bytes, cp, out));
                show("lpr8 ng5", run<true, 8, 5>(img, bnd, c.ntiles, c.nseg, tile_bytes, cp, out));
            }
            (void)hipFree(img);
        }
        (void)hipFree(bnd);
        (void)hipFree(used);
        (void)hipFree(out);
    }
    return 0;
}
