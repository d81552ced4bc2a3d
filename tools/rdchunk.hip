// rdchunk.hip -- read rate of scattered short chunks from HBM, the access pattern of k_seg_or
// (one ~80-byte run per tile, tiles ~77 KB apart).  8-lane groups read one chunk each (16 B per
// lane, chunk bytes = 16 x live lanes), NG chunks per group in flight; chunk positions:
//   random : uniform over the buffer (16-byte aligned)
//   strided: chunk c of "segment" s at c * stride + s * 80 -- the k_seg_or pattern, segments
//            dealt to workgroups as k_seg_or deals them
// Prints useful GB/s.   hipcc --offload-arch=gfx950 -O3 -o tools/rdchunk tools/rdchunk.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kNG = 5;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// MODE 0: random 16-B-aligned chunk starts; MODE 1: k_seg_or's tile-strided pattern.
template <int MODE>
__global__ __launch_bounds__(1024) void k_read(const uint4* buf, uint64_t n16, uint32_t live, uint32_t per_wg,
                                               uint32_t stride16, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63, grp = lane >> 3, q = lane & 7, wave = threadIdx.x >> 6;
    uint32_t acc = 0;
    const uint32_t seg = blockIdx.x;
    for (uint32_t c0 = wave * 8 * kNG; c0 < per_wg; c0 += 16 * 8 * kNG) {
        uint4 v[kNG];
#pragma unroll
        for (int g = 0; g < kNG; ++g) {
            const uint32_t c = c0 + g * 8 + grp;
            uint64_t base;
            if (MODE == 0)
                base = ((uint64_t)mix(seg * 0x9E3779B9u + c) * 65536ull + mix(c ^ seg)) % (n16 - 16);
            else
                base = (uint64_t)c * stride16 + (uint64_t)seg * 5;  // 80-byte runs back to back
            base = base % (n16 - 16);
            v[g] = buf[base + (q < live ? q : 0)];
        }
#pragma unroll
        for (int g = 0; g < kNG; ++g) acc ^= v[g].x ^ v[g].y ^ v[g].z ^ v[g].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t bytes = 2600ull << 20;
    const uint64_t n16 = bytes / 16;
    uint4* buf;
    uint32_t* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    const uint32_t nwg = 954, per_wg = 32768;  // config 2: 954 segments x ~32.5K tiles
    const uint32_t stride16 = 77 * 1024 / 16;
    for (int mode = 0; mode < 2; ++mode)
        for (uint32_t live : {4u, 5u, 8u}) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            auto launch = [&] {
                if (mode == 0)
                    hipLaunchKernelGGL(k_read<0>, dim3(nwg), dim3(1024), 0, 0, buf, n16, live, per_wg, stride16, out);
                else
                    hipLaunchKernelGGL(k_read<1>, dim3(nwg), dim3(1024), 0, 0, buf, n16, live, per_wg, stride16, out);
            };
            launch();
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            ms /= 5;
            const double useful = (double)nwg * per_wg * live * 16;
            printf("%-8s chunk %3u B: %.3f ms  %7.1f GB/s useful\n", mode ? "strided" : "random", live * 16, ms,
                   useful / (ms * 1e-3) / 1e9);
        }
    return 0;
}
