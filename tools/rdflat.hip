// rdflat.hip -- k_seg_or's flattened read loop (V6) over realistic tile images, two group formats:
//   g20 : the round-3 image -- 8-entry groups of 20 B (16 B of u16 low halves + the group's nibble
//         word), read with a 16-byte and a 4-byte load per group (two load instructions);
//   g16 : 6-entry groups of 16 B (three 20-bit entries per 64-bit half), 16-byte aligned: one
//         16-byte load per group, never straddling a cache line;
//   raw20: the g20 image read as the aligned 16-byte chunks covering each run's groups, one per
//         lane (what a reader that stages raw bytes and parses groups afterwards would load).
// A wave takes the runs of 64 consecutive tiles of its segment; their groups are dealt to lanes
// back to back (exclusive prefix + binary search, as in k_seg_or).  Each workgroup asks for 128 KiB
// of LDS so one runs per CU, as k_seg_or's bitmap forces.  Reads only; the loaded words are folded
// into a checksum.  Run lengths per (tile, segment): mean M, uniform +-M/2.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/rdflat tools/rdflat.hip
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <vector>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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

// GE entries per group, GB bytes per group; LOC (g20 only): each run's lane writes its groups'
// (run, group index) into a per-wave LDS slot table and the group lanes read their slot -- one LDS
// write per group and one read instead of the 6-step binary search over the prefix (ds_bpermute)
// plus two shuffles
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// NT (g20 only, round 5): the group loads as non-temporal loads (global_load ... nt), to see
// whether the L1 then stops filling whole 128-byte lines for the ~20 useful bytes of a short run
template <int GE, int GB, bool LOC = false, bool NT = false>
__global__ __launch_bounds__(1024) void k_read(const uint8_t* img, const uint32_t* bnd, uint32_t ntiles,
                                               uint32_t nseg, uint32_t tile_bytes, uint32_t* out) {
    extern __shared__ uint32_t lds[];
    const uint32_t nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
    const uint32_t seg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
    if (seg >= nseg) return;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t* row = bnd + (uint64_t)seg * ntiles;
    uint32_t acc = 0;
    for (uint32_t t0 = wave * 64; t0 < ntiles; t0 += 16 * 64) {
        const uint32_t t = t0 + lane;
        const uint32_t v = t < ntiles ? row[t] : 0u;
        const uint32_t st = v & 0xFFFFu, en = v >> 16;
        uint32_t ch = en > st ? (en + GE - 1) / GE - st / GE : 0u;
        if (GB == 0 && en > st) ch = ((en + 7) / 8 * 20 + 15) / 16 - (st / 8 * 20) / 16;  // 16-byte chunks
        uint32_t incl = ch;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= (uint32_t)o) incl += y;
        }
        const uint32_t excl = incl - ch, total = (uint32_t)__shfl((int)incl, 63);
        uint32_t* slot = lds + 32768 + wave * 512;
        if constexpr (LOC) {
            for (uint32_t x = 0; x < ch && excl + x < 512; ++x) slot[excl + x] = lane | ((st / 8 + x) << 6);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        for (uint32_t c = lane; c < total; c += 64) {
            uint32_t r = 0, gi;
            if (LOC && c < 512) {
                const uint32_t e = slot[c];
                r = e & 63u;
                gi = e >> 6;
            } else {
#pragma unroll
                for (int sft = 32; sft; sft >>= 1)
                    if ((uint32_t)__shfl((int)excl, (int)r + sft) <= c) r += sft;
                const uint32_t rv = (uint32_t)__shfl((int)v, (int)r), rex = (uint32_t)__shfl((int)excl, (int)r);
                gi = (rv & 0xFFFFu) / (GE ? GE : 8) + (c - rex);
            }
            const uint8_t* tile = img + (uint64_t)min(t0 + r, ntiles - 1) * tile_bytes;
            uint4 l;
            if (GB == 0) {  // raw: aligned 16-byte chunks of the run's byte range (GE = 8, 20-byte groups)
                const uint32_t rv = (uint32_t)__shfl((int)v, (int)r), rex = (uint32_t)__shfl((int)excl, (int)r);
                l = *reinterpret_cast<const uint4*>(tile + ((rv & 0xFFFFu) / 8 * 20 / 16 + (c - rex)) * 16);
                acc ^= l.x ^ l.y ^ l.z ^ l.w;
            } else if (GB == 16) {
                l = *reinterpret_cast<const uint4*>(tile + gi * 16);
                acc ^= l.x ^ l.y ^ l.z ^ l.w;
            } else if (NT) {
                const u32x4 v4 = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(tile + gi * GB));
                const uint32_t nb = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(tile + gi * GB + 16));
                acc ^= v4.x ^ v4.y ^ v4.z ^ v4.w ^ nb;
            } else {
                uint32_t nb;
                __builtin_memcpy(&l, tile + gi * GB, 16);
                __builtin_memcpy(&nb, tile + gi * GB + 16, 4);
                acc ^= l.x ^ l.y ^ l.z ^ l.w ^ nb;
            }
        }
    }
    if (acc == 0x12345678u) lds[0] = acc;
    __syncthreads();
    if (threadIdx.x == 0 && lds[0] == 0x12345678u) out[0] = acc;
}

template <int GE, int GB, bool LOC = false, bool NT = false>
static float run(const uint8_t* img, const uint32_t* bnd, uint32_t ntiles, uint32_t nseg, uint32_t tile_bytes,
                 uint32_t* out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const uint32_t lds = 128 * 1024 + 16 * 512 * 4;  // bitmap + per-wave slot tables (LOC)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_read<GE, GB, LOC, NT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL((k_read<GE, GB, LOC, NT>), dim3(nseg), dim3(1024), lds, 0, img, bnd, ntiles, nseg, tile_bytes, out);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL((k_read<GE, GB, LOC, NT>), dim3(nseg), dim3(1024), lds, 0, img, bnd, ntiles, nseg, tile_bytes,
                           out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

// usage: rdflat [formats]   formats: comma-separated of 0 (g20, the shipped group image), 1 (g16),
// 2 (raw20), 3 (g20loc: slot-table locate), 4 (g20nt: non-temporal group loads); default "0"
// (profiles/r05/rdflat_nt.txt ran "0,4", profiles/r04/rdflat*.log "0,1,2" and "0,3")
int main(int argc, char** argv) {
    std::vector<int> fmts;
    for (const char* p = argc > 1 ? argv[1] : "0"; *p;) {
        fmts.push_back((int)strtol(p, (char**)&p, 10));
        if (*p == ',') ++p;
        else if (*p) return 2;
    }
    struct Cfg { const char* name; uint32_t ntiles, nseg, mean; };
    // k = 10: 100M keys / 3072 per tile, m = 1e9; k = 19: 100M / 1536, m = 1.9e9; and 19 with a
    // 3072-key tile (one k_tile_pack workgroup per CU)
    // cfg5x2: config 5 with a k_tile_pack tile twice as large (one workgroup per CU, ~14 336 keys):
    // half the tiles, ~14-entry runs
    const Cfg cfgs[] = {{"k10", 32553, 954, 32}, {"k19", 65105, 1812, 16}, {"cfg5", 69755, 4096, 7},
                        {"cfg5x2", 34878, 4096, 14}};
    for (const Cfg& c : cfgs) {
        uint32_t *bnd, *used, *out;
        const uint64_t nb = (uint64_t)c.ntiles * c.nseg;
        if (hipMalloc(&bnd, nb * 4) != hipSuccess || hipMalloc(&used, 4) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
        (void)hipMemset(used, 0, 4);
        hipLaunchKernelGGL(k_gen, dim3((c.ntiles + 255) / 256), dim3(256), 0, 0, bnd, c.ntiles, c.nseg, c.mean, used);
        uint32_t cap = 0;
        (void)hipMemcpy(&cap, used, 4, hipMemcpyDeviceToHost);
        for (int fmt : fmts) {
            const uint32_t tile_bytes = fmt != 1 ? ((cap + 7) / 8 * 20 + 16 + 15) & ~15u : ((cap + 5) / 6 * 16 + 16);
            const uint64_t bytes = (uint64_t)c.ntiles * tile_bytes + 4096;
            uint8_t* img;
            if (hipMalloc(&img, bytes) != hipSuccess) return 1;
            (void)hipMemset(img, 1, bytes);
            for (int rep = 0; rep < 2; ++rep) {
                const float ms = fmt == 0   ? run<8, 20>(img, bnd, c.ntiles, c.nseg, tile_bytes, out)
                                 : fmt == 1 ? run<6, 16>(img, bnd, c.ntiles, c.nseg, tile_bytes, out)
                                 : fmt == 3 ? run<8, 20, true>(img, bnd, c.ntiles, c.nseg, tile_bytes, out)
                                 : fmt == 4 ? run<8, 20, false, true>(img, bnd, c.ntiles, c.nseg, tile_bytes, out)
                                            : run<8, 0>(img, bnd, c.ntiles, c.nseg, tile_bytes, out);
                printf("%-6s %s %.3f ms  (%.1f G runs/s, %u B per tile, %.2f GB image)\n", c.name,
                       fmt == 0 ? "g20" : fmt == 1 ? "g16" : fmt == 3 ? "g20loc" : fmt == 4 ? "g20nt" : "raw20", ms,
                       (double)nb / (ms * 1e-3) / 1e9, tile_bytes,
                       (double)c.ntiles * tile_bytes / 1e9);
            }
            (void)hipFree(img);
        }
        (void)hipFree(bnd);
        (void)hipFree(used);
        (void)hipFree(out);
    }
    return 0;
}
