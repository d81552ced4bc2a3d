// rdpair.hip -- does co-locating a run's nibbles with its low halves speed up k_seg_or's reads?
// k = 19 pattern: 1812 segments (one workgroup each) x 68K tiles, tile images TILE bytes apart,
// one ~15-entry run per (tile, segment).  8-lane groups read one run each, NG runs per group in
// flight, lanes 0..1 the 32 bytes of low halves and lane 2 the 8 bytes of nibbles:
//   split     : low halves at seg * 32 in the tile's low-half area, nibbles at LO + seg * 8
//   colocated : the run's 40 bytes contiguous at seg * 40
// Prints ms for all runs and the useful GB/s.  hipcc --offload-arch=gfx950 -O3 -o tools/rdpair tools/rdpair.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kNG = 5;
constexpr uint32_t kSeg = 1812, kTiles = 68000, kTile = 72 * 1024, kLo = kSeg * 32;

template <bool COLO>
__global__ __launch_bounds__(1024) void k_read(const uint8_t* buf, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63, grp = lane >> 3, q = lane & 7, wave = threadIdx.x >> 6;
    const uint32_t seg = (blockIdx.x % 8) * ((kSeg + 7) / 8) + blockIdx.x / 8;  // XCD-aware, as k_seg_or
    if (seg >= kSeg) return;
    uint32_t acc = 0;
    for (uint32_t t0 = wave * 8 * kNG; t0 < kTiles; t0 += 16 * 8 * kNG) {
        uint4 v[kNG];
#pragma unroll
        for (int g = 0; g < kNG; ++g) {
            const uint32_t t = min(t0 + g * 8 + grp, kTiles - 1);
            const uint8_t* tile = buf + (uint64_t)t * kTile;
            uint64_t off;
            if (COLO)
                off = (uint64_t)seg * 40 + (q < 3 ? q * 16 : 0);
            else
                off = q < 2 ? (uint64_t)seg * 32 + q * 16 : (uint64_t)kLo + seg * 8;
            if (q < 2 || (q == 2 && !COLO)) {
                v[g] = *reinterpret_cast<const uint4*>(tile + (off & ~15ull));
            } else if (q == 2) {
                const uint2 h = *reinterpret_cast<const uint2*>(tile + (off & ~7ull));
                v[g] = make_uint4(h.x, h.y, 0, 0);
            } else {
                v[g] = make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int g = 0; g < kNG; ++g) acc ^= v[g].x ^ v[g].y ^ v[g].z ^ v[g].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t bytes = (uint64_t)kTiles * kTile + 4096;
    uint8_t* buf;
    uint32_t* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    for (int rep = 0; rep < 3; ++rep)
        for (int colo = 0; colo < 2; ++colo) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            const uint32_t nwg = ((kSeg + 7) / 8) * 8;
            (void)hipEventRecord(e0);
            if (colo)
                hipLaunchKernelGGL(k_read<true>, dim3(nwg), dim3(1024), 0, 0, buf, out);
            else
                hipLaunchKernelGGL(k_read<false>, dim3(nwg), dim3(1024), 0, 0, buf, out);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("%-10s %.3f ms  useful %.2f TB/s\n", colo ? "colocated" : "split", ms,
                   (double)kSeg * kTiles * 40 / (ms * 1e-3) / 1e12);
        }
    return 0;
}
