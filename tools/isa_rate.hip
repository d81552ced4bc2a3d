// isa_rate.hip -- issue rate of the VALU instructions the SipHash rounds are built from, on gfx950.
// Each kernel runs ITER iterations of 8 independent instructions of one kind per lane (inline
// asm, no dependency between the 8), with 8 waves per SIMD, and prints lane-ops per second and
// cycles per wave-instruction per SIMD (2.0 = the SIMD-32 rate of a full-rate op).
//   hipcc --offload-arch=gfx950 -O3 -o tools/isa_rate tools/isa_rate.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIter = 8192;
constexpr int kBlock = 256;

#define OPS8(INSN, C) \
    asm volatile(INSN : "+v"(a0) : C(b0)); asm volatile(INSN : "+v"(a1) : C(b1)); \
    asm volatile(INSN : "+v"(a2) : C(b2)); asm volatile(INSN : "+v"(a3) : C(b3)); \
    asm volatile(INSN : "+v"(a4) : C(b4)); asm volatile(INSN : "+v"(a5) : C(b5)); \
    asm volatile(INSN : "+v"(a6) : C(b6)); asm volatile(INSN : "+v"(a7) : C(b7));

template <int OP>
__global__ __launch_bounds__(kBlock) void k_rate(uint32_t* out) {
    const uint32_t t = threadIdx.x + blockIdx.x * kBlock;
    if constexpr (OP == 2 || OP == 4 || OP == 9) {  // 64-bit operands
        uint64_t a0 = t, a1 = t * 3, a2 = t * 5, a3 = t * 7, a4 = t * 9, a5 = t * 11, a6 = t * 13, a7 = t * 15;
        uint64_t b0 = ~a0, b1 = ~a1, b2 = ~a2, b3 = ~a3, b4 = ~a4, b5 = ~a5, b6 = ~a6, b7 = ~a7;
        for (int i = 0; i < kIter; ++i) {
            if constexpr (OP == 2) { OPS8("v_lshl_add_u64 %0, %0, 0, %1", "v") }
            if constexpr (OP == 4) { OPS8("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]", "v") }
            if constexpr (OP == 9) { OPS8("v_xor_b32 %0, %0, %1", "v") }  // placeholder, unused
        }
        const uint64_t s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0;
        if (s == 0x1234567) out[0] = (uint32_t)s;
    } else {
        uint32_t a0 = t, a1 = t * 3, a2 = t * 5, a3 = t * 7, a4 = t * 9, a5 = t * 11, a6 = t * 13, a7 = t * 15;
        uint32_t b0 = ~a0, b1 = ~a1, b2 = ~a2, b3 = ~a3, b4 = ~a4, b5 = ~a5, b6 = ~a6, b7 = ~a7;
        for (int i = 0; i < kIter; ++i) {
            if constexpr (OP == 0) { OPS8("v_xor_b32 %0, %0, %1", "v") }
            if constexpr (OP == 1) { OPS8("v_alignbit_b32 %0, %0, %1, 13", "v") }
            if constexpr (OP == 3) { OPS8("v_mov_b32 %0, %1", "v") }
            if constexpr (OP == 5) { OPS8("v_mul_hi_u32 %0, %0, %1", "v") }
            if constexpr (OP == 6) { OPS8("v_mul_lo_u32 %0, %0, %1", "v") }
            if constexpr (OP == 7) { OPS8("v_add_u32 %0, %0, %1", "v") }
            if constexpr (OP == 8) { OPS8("v_perm_b32 %0, %0, %1, %1", "v") }
            if constexpr (OP == 11) { OPS8("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96", "v") }
        }
        const uint32_t s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0;
        if (s == 0x1234567) out[0] = s;
    }
}

// v_mad_u64_u32 (64-bit accumulate) and the v_add_co/v_addc pair, as the compiler emits them.
template <int OP>
__global__ __launch_bounds__(kBlock) void k_rate64(uint32_t* out) {
    const uint32_t t = threadIdx.x + blockIdx.x * kBlock;
    uint64_t a[8];
    uint32_t b[8];
    for (int j = 0; j < 8; ++j) { a[j] = (uint64_t)t * (2 * j + 3); b[j] = t ^ (j * 0x9E37u); }
    for (int i = 0; i < kIter; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (OP == 0) {
                asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]) : "s0", "s1");
            } else {
                unsigned c, c2;
                const uint32_t lo = __builtin_addc((uint32_t)a[j], b[j], 0u, &c);
                const uint32_t hi = __builtin_addc((uint32_t)(a[j] >> 32), b[(j + 3) & 7], c, &c2);
                a[j] = ((uint64_t)hi << 32) | lo;
            }
        }
        if constexpr (OP == 1) asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]));
    }
    uint64_t s = 0;
    for (int j = 0; j < 8; ++j) s ^= a[j];
    if (s == 0x1234567) out[0] = (uint32_t)s;
}

template <class K>
static void run(K kern, const char* name, double ops_per_iter, uint32_t* d) {
    int dev = 0, cus = 0, clk = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);  // kHz
    const int blocks = cus * 8;  // 8 x 256 threads per CU = 8 waves per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(kBlock), 0, 0, d);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(kBlock), 0, 0, d);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double lane_ops = (double)blocks * kBlock * kIter * ops_per_iter;
    const double rate = lane_ops / (ms * 1e-3);
    // wave-instructions per SIMD per cycle at the nominal clock
    const double wave_insts_per_simd = lane_ops / 64.0 / (cus * 4.0);
    const double cycles = ms * 1e-3 * clk * 1e3;
    printf("%-34s %8.3f ms  %7.1f T lane-ops/s  %5.2f cycles per wave-instruction per SIMD\n", name, ms,
           rate / 1e12, cycles / wave_insts_per_simd);
}

int main() {
    uint32_t* d;
    hipMalloc(&d, 64);
    run(k_rate<0>, "v_xor_b32", 8, d);
    run(k_rate<1>, "v_alignbit_b32", 8, d);
    run(k_rate<8>, "v_perm_b32", 8, d);
    run(k_rate<3>, "v_mov_b32", 8, d);
    run(k_rate<7>, "v_add_u32", 8, d);
    run(k_rate<11>, "v_bitop3_b32", 8, d);
    run(k_rate<2>, "v_lshl_add_u64", 8, d);
    run(k_rate<4>, "v_pk_mov_b32 (swap halves)", 8, d);
    run(k_rate<5>, "v_mul_hi_u32", 8, d);
    run(k_rate<6>, "v_mul_lo_u32", 8, d);
    run(k_rate64<0>, "v_mad_u64_u32", 8, d);
    run(k_rate64<1>, "v_add_co + v_addc (per pair)", 8, d);
    hipFree(d);
    return 0;
}
