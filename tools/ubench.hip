// ubench.hip -- microbenchmarks that decide the Bloom-build kernel design on gfx950.
//   hash-*   : SipHash-1-3 prefix + k=10 seeds per lane, XOR-folded (no memory traffic):
//              variants of the 64-bit rotate / add lowering.
//   atomic   : random 32-bit atomicOr rate into arrays of several sizes.
//   gather   : random 32-bit load rate from the same arrays.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -o tools/ubench tools/ubench.hip
#include <hip/hip_runtime.h>
#include <string>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

struct S { uint64_t v0, v1, v2, v3; };

// V0: plain C rotates (compiler picks v_lshlrev_b64 + v_lshrrev + v_or)
__device__ __forceinline__ uint64_t rotl_c(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }
// V1: v_alignbit_b32 pair
template <int B>
__device__ __forceinline__ uint64_t rotl_a(uint64_t x) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - B);
    const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - B);
    return ((uint64_t)nhi << 32) | nlo;
}
__device__ __forceinline__ uint64_t swap32(uint64_t x) { return (x >> 32) | (x << 32); }
// V9: rotate as one 32-bit shift of the high word + one v_lshl_add_u64: (x << B) + (hi >> (32 - B))
// (the two parts share no bit, so + is |; LLVM turns a C + into v_lshlrev_b64 + v_or, hence asm).
// Measured round 4: WRONG (the check prints MISMATCH: the instruction's shift field is 3 bits, so a
// shift by 13..21 is not encodable as such) and slower anyway (2.93 vs 2.85 ms) -- kept as a record.
template <int B>
__device__ __forceinline__ uint64_t rotl_l(uint64_t x) {
    const uint64_t y = (uint64_t)((uint32_t)(x >> 32) >> (32 - B));
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, %2, %3" : "=v"(r) : "v"(x), "n"(B), "v"(y));
    return r;
}
// 64-bit add as add_co/addc through inline asm (defeats v_lshl_add_u64 selection)
__device__ __forceinline__ uint64_t add_cc(uint64_t a, uint64_t b) {
    uint32_t lo, hi;
    asm volatile("v_add_co_u32 %0, vcc, %2, %3\n\tv_addc_co_u32 %1, vcc, %4, %5, vcc"
                 : "=v"(lo), "=v"(hi)
                 : "v"((uint32_t)a), "v"((uint32_t)b), "v"((uint32_t)(a >> 32)), "v"((uint32_t)(b >> 32))
                 : "vcc");
    return ((uint64_t)hi << 32) | lo;
}

// 64-bit add as add_co/addc through non-volatile asm (schedulable)
__device__ __forceinline__ uint64_t add_nv(uint64_t a, uint64_t b) {
    uint32_t lo, hi;
    asm("v_add_co_u32 %0, vcc, %2, %3\n\tv_addc_co_u32 %1, vcc, %4, %5, vcc"
        : "=&v"(lo), "=v"(hi)
        : "v"((uint32_t)a), "v"((uint32_t)b), "v"((uint32_t)(a >> 32)), "v"((uint32_t)(b >> 32))
        : "vcc");
    return ((uint64_t)hi << 32) | lo;
}

// swap32(a) + b with explicit 32-bit carry ops: the halves of a are consumed crosswise, so no
// register-pair re-alignment is needed (V5).
__device__ __forceinline__ uint64_t add_sw(uint64_t a, uint64_t b) {
    unsigned c0, c1;
    const unsigned lo = __builtin_addc((unsigned)(a >> 32), (unsigned)b, 0u, &c0);
    const unsigned hi = __builtin_addc((unsigned)a, (unsigned)(b >> 32), c0, &c1);
    (void)c1;
    return ((uint64_t)hi << 32) | lo;
}

// Rotate by 32 in ONE instruction: v_pk_mov_b32 with op_sel picks the halves crosswise, so the
// result lands in an aligned pair ready for v_lshl_add_u64 (the plain form costs 2 v_mov_b32).
__device__ __forceinline__ uint64_t swap_pk(uint64_t x) {
    uint64_t r;
    asm("v_pk_mov_b32 %0, %1, %1 op_sel:[1,0]" : "=v"(r) : "v"(x));
    return r;
}

// V10: swap32(a) + b as v_mad_u64_u32(a.hi, 1, b) (64-bit: carries into the high word) plus a.lo
// added to the high word -- no v_mov pair re-aligning the swapped value
__device__ __forceinline__ uint64_t add_swm(uint64_t a, uint64_t b) {
    uint64_t r, c;
    asm("v_mad_u64_u32 %0, %1, %2, 1, %3" : "=v"(r), "=s"(c) : "v"((uint32_t)(a >> 32)), "v"(b));
    (void)c;
    uint32_t hi;  // a 32-bit add (LLVM would fold a C add back into a 64-bit one + a v_mov)
    asm("v_add_u32 %0, %1, %2" : "=v"(hi) : "v"((uint32_t)(r >> 32)), "v"((uint32_t)a));
    return ((uint64_t)hi << 32) | (uint32_t)r;
}

template <int V>
__device__ __forceinline__ void round_(S& s) {
    if constexpr (V == 10) {
        // v0 and v2 kept un-swapped where the swap feeds an add (logical v2 = swap32(stored) at exit)
        s.v0 += s.v1; s.v1 = rotl_a<13>(s.v1); s.v1 ^= s.v0;
        s.v2 = add_swm(s.v2, s.v3); s.v3 = rotl_a<16>(s.v3); s.v3 ^= s.v2;
        s.v0 = add_swm(s.v0, s.v3); s.v3 = rotl_a<21>(s.v3); s.v3 ^= s.v0;
        s.v2 += s.v1; s.v1 = rotl_a<17>(s.v1); s.v1 ^= s.v2;
    } else if constexpr (V == 9) {
        s.v0 += s.v1; s.v1 = rotl_l<13>(s.v1); s.v1 ^= s.v0; s.v0 = swap32(s.v0);
        s.v2 += s.v3; s.v3 = rotl_l<16>(s.v3); s.v3 ^= s.v2;
        s.v0 += s.v3; s.v3 = rotl_l<21>(s.v3); s.v3 ^= s.v0;
        s.v2 += s.v1; s.v1 = rotl_l<17>(s.v1); s.v1 ^= s.v2; s.v2 = swap32(s.v2);
    } else if constexpr (V == 6) {
        s.v0 += s.v1; s.v1 = rotl_a<13>(s.v1); s.v1 ^= s.v0; s.v0 = swap_pk(s.v0);
        s.v2 += s.v3; s.v3 = rotl_a<16>(s.v3); s.v3 ^= s.v2;
        s.v0 += s.v3; s.v3 = rotl_a<21>(s.v3); s.v3 ^= s.v0;
        s.v2 += s.v1; s.v1 = rotl_a<17>(s.v1); s.v1 ^= s.v2; s.v2 = swap_pk(s.v2);
    } else if constexpr (V == 0) {
        s.v0 += s.v1; s.v1 = rotl_c(s.v1, 13); s.v1 ^= s.v0; s.v0 = rotl_c(s.v0, 32);
        s.v2 += s.v3; s.v3 = rotl_c(s.v3, 16); s.v3 ^= s.v2;
        s.v0 += s.v3; s.v3 = rotl_c(s.v3, 21); s.v3 ^= s.v0;
        s.v2 += s.v1; s.v1 = rotl_c(s.v1, 17); s.v1 ^= s.v2; s.v2 = rotl_c(s.v2, 32);
    } else if constexpr (V == 1) {
        s.v0 += s.v1; s.v1 = rotl_a<13>(s.v1); s.v1 ^= s.v0; s.v0 = swap32(s.v0);
        s.v2 += s.v3; s.v3 = rotl_a<16>(s.v3); s.v3 ^= s.v2;
        s.v0 += s.v3; s.v3 = rotl_a<21>(s.v3); s.v3 ^= s.v0;
        s.v2 += s.v1; s.v1 = rotl_a<17>(s.v1); s.v1 ^= s.v2; s.v2 = swap32(s.v2);
    } else if constexpr (V == 5) {
        // v0, v2 are kept UNswapped where a swap would feed an add: add_sw folds the swap in
        s.v0 += s.v1; s.v1 = rotl_a<13>(s.v1); s.v1 ^= s.v0;
        s.v2 = add_sw(s.v2, s.v3); s.v3 = rotl_a<16>(s.v3); s.v3 ^= s.v2;
        s.v0 = add_sw(s.v0, s.v3); s.v3 = rotl_a<21>(s.v3); s.v3 ^= s.v0;
        s.v2 += s.v1; s.v1 = rotl_a<17>(s.v1); s.v1 ^= s.v2;
        // at exit v2 is logically swap32(v2): the next round's first v2 use is add_sw (swap folded)
    } else if constexpr (V == 3) {
        s.v0 = add_nv(s.v0, s.v1); s.v1 = rotl_a<13>(s.v1); s.v1 ^= s.v0; s.v0 = swap32(s.v0);
        s.v2 = add_nv(s.v2, s.v3); s.v3 = rotl_a<16>(s.v3); s.v3 ^= s.v2;
        s.v0 = add_nv(s.v0, s.v3); s.v3 = rotl_a<21>(s.v3); s.v3 ^= s.v0;
        s.v2 = add_nv(s.v2, s.v1); s.v1 = rotl_a<17>(s.v1); s.v1 ^= s.v2; s.v2 = swap32(s.v2);
    } else {
        s.v0 = add_cc(s.v0, s.v1); s.v1 = rotl_a<13>(s.v1); s.v1 ^= s.v0; s.v0 = swap32(s.v0);
        s.v2 = add_cc(s.v2, s.v3); s.v3 = rotl_a<16>(s.v3); s.v3 ^= s.v2;
        s.v0 = add_cc(s.v0, s.v3); s.v3 = rotl_a<21>(s.v3); s.v3 ^= s.v0;
        s.v2 = add_cc(s.v2, s.v1); s.v1 = rotl_a<17>(s.v1); s.v1 ^= s.v2; s.v2 = swap32(s.v2);
    }
}

template <int V>
__device__ __forceinline__ void comp(S& s, uint64_t m) { s.v3 ^= m; round_<V>(s); s.v0 ^= m; }

// V5 representation: v2 is stored un-swapped between rounds (logical v2 = swap32(stored)).
__device__ __forceinline__ uint64_t lv2(const S& s) { return swap32(s.v2); }

template <int V>
__device__ __forceinline__ uint64_t fin(S s, uint64_t b) {
    if constexpr (V == 5 || V == 10) {
        s.v3 ^= b; round_<V>(s); s.v0 ^= b;
        s.v2 ^= (0xffull << 32);  // logical v2 ^= 0xff on the stored (swapped) form
        round_<V>(s); round_<V>(s); round_<V>(s);
        return s.v0 ^ s.v1 ^ lv2(s) ^ s.v3;
    }
    s.v3 ^= b; round_<V>(s); s.v0 ^= b; s.v2 ^= 0xff; round_<V>(s); round_<V>(s); round_<V>(s);
    return s.v0 ^ s.v1 ^ s.v2 ^ s.v3;
}

template <int V>
__global__ __launch_bounds__(256) void k_hash(uint64_t n, int k, uint64_t* out) {
    uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    S s{0x736f6d6570736575ULL, 0x646f72616e646f6dULL, 0x6c7967656e657261ULL, 0x7465646279746573ULL};
    comp<V>(s, 16); comp<V>(s, j * 0x9E3779B97F4A7C15ULL); comp<V>(s, j);
    uint64_t acc = 0;
    for (int i = 0; i < k; ++i) {
        S t = s;
        comp<V>(t, (uint64_t)i);
        acc ^= fin<V>(t, 32ull << 56);
    }
    if (acc == 0x123456789ull) out[0] = acc;  // keep it live, never taken in practice
}

__device__ __forceinline__ uint32_t fmod_(uint64_t x, uint64_t m, uint64_t mu) {
    const uint64_t q = __umul64hi(x, mu);
    uint64_t r = x - q * m;
    r = r >= m ? r - m : r;
    return (uint32_t)r;
}

// Exact x % m for 2^13 <= m < 2^32 with one 32-bit multiply: an f64 estimate of the quotient
// (off by at most one), the remainder's low word in integers, and the f64 remainder estimate
// (error <= 2^10) to tell which multiple of 2^32 the low word stands for.
__device__ __forceinline__ uint32_t fmod_f64(uint64_t x, uint32_t m, double inv_m, double m_f) {
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    const double xf = __fma_rn((double)xh, 4294967296.0, (double)xl);
    const double qf = floor(xf * inv_m);
    const double qh = floor(qf * (1.0 / 4294967296.0));
    const uint32_t ql = (uint32_t)__fma_rn(-qh, 4294967296.0, qf);
    const uint32_t rl = xl - ql * m;
    const double d = __fma_rn(-qf, m_f, xf) - (double)rl;
    uint32_t r = rl;
    if (d < -2147483648.0) r = rl + m;
    else if (d > 2147483648.0 || rl >= m) r = rl - m;
    return r;
}

__global__ void k_mod_check(uint64_t n, uint64_t m, uint64_t mu, double inv_m, unsigned long long* bad) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    uint64_t x = j * 0x9E3779B97F4A7C15ULL;
    x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ULL; x ^= x >> 32;
    if ((j & 7) == 0) x = ~0ull - (j >> 3);              // near 2^64
    if ((j & 7) == 1) x = (j >> 3) * m + (j & 0xff) - 128;  // near multiples of m
    const uint32_t a = (uint32_t)(x % m);
    const uint32_t b = fmod_f64(x, (uint32_t)m, inv_m, (double)m);
    if (a != b) atomicAdd(bad, 1ull);
}

// MODE: 0 = V1 hash only; 1 = V1 + mod; 2 = V1, two seeds interleaved, + mod; 3 = V3 + mod;
// 5 = V5 (swap folded into carry adds) + mod
template <int MODE, int BS>
__global__ __launch_bounds__(BS) void k_hash2(uint64_t n, int k, uint64_t m, uint64_t mu, uint64_t* out) {
    const double inv_m = 1.0 / (double)m;
    extern __shared__ uint32_t pad[];
    uint64_t j = (uint64_t)blockIdx.x * BS + threadIdx.x;
    if (j >= n) return;
    constexpr int V = MODE == 3 ? 3 : MODE == 5 ? 5 : MODE == 6 ? 6 : MODE == 7 ? 6 : MODE == 9 ? 9 : MODE == 10 ? 10 : 1;
    S s{0x736f6d6570736575ULL, 0x646f72616e646f6dULL, 0x6c7967656e657261ULL, 0x7465646279746573ULL};
    if constexpr (V == 5 || V == 10) s.v2 = swap32(s.v2);  // stored form
    comp<V>(s, 16); comp<V>(s, j * 0x9E3779B97F4A7C15ULL); comp<V>(s, j);
    uint64_t acc = 0;
    if constexpr (MODE == 2 || MODE == 7) {
        int i = 0;
        for (; i + 1 < k; i += 2) {
            S t0 = s, t1 = s;
            comp<V>(t0, (uint32_t)i);
            comp<V>(t1, (uint32_t)(i + 1));
            const uint64_t h0 = fin<V>(t0, 32ull << 56);
            const uint64_t h1 = fin<V>(t1, 32ull << 56);
            acc += fmod_(h0, m, mu) + fmod_(h1, m, mu);
        }
        if (i < k) { S t = s; comp<V>(t, (uint32_t)i); acc += fmod_(fin<V>(t, 32ull << 56), m, mu); }
    } else {
        for (int i = 0; i < k; ++i) {
            S t = s;
            comp<V>(t, (uint32_t)i);
            const uint64_t h = fin<V>(t, 32ull << 56);
            if constexpr (MODE == 0) acc ^= h;
            else if constexpr (MODE == 8) acc += fmod_f64(h, (uint32_t)m, inv_m, (double)m);
            else acc += fmod_(h, m, mu);
        }
    }
    if (acc == 0x123456789ull) out[0] = acc + pad[0];
}

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return (uint32_t)x;
}

__global__ __launch_bounds__(256) void k_atomic(uint32_t* w, uint32_t nw, uint64_t n, int per) {
    uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    for (int i = 0; i < per; ++i) {
        uint32_t h = mix32(j * 16 + i);
        atomicOr(w + (h % nw), 1u << (h & 31));
    }
}

__global__ __launch_bounds__(256) void k_gather(const uint32_t* w, uint32_t nw, uint64_t n, int per, uint32_t* out) {
    uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    uint32_t acc = 0;
    for (int i = 0; i < per; ++i) {
        uint32_t h = mix32(j * 16 + i);
        acc += w[h % nw];
    }
    if (acc == 0xdeadbeef) out[0] = acc;
}

// LDS op throughput: every lane issues N ops at pseudo-random word addresses of a 32K-word
// (128 KiB) LDS array.  OP: 0 ds_or (atomic, no return), 1 ds_add_rtn, 2 ds_write_b32,
// 3 ds_write_b16, 4 ds_or with value 0 on odd lanes (branch-free masking).
template <int OP>
__global__ __launch_bounds__(1024) void k_lds(int n, uint32_t* out) {
    __shared__ uint32_t a[32768];
    for (int i = threadIdx.x; i < 32768; i += 1024) a[i] = 0;
    __syncthreads();
    uint32_t x = (blockIdx.x * 1024 + threadIdx.x) * 2654435761u + 1, acc = 0;
    for (int i = 0; i < n; ++i) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        const uint32_t w = x & 32767;
        if constexpr (OP == 0) atomicOr(&a[w], 1u << (x >> 27));
        else if constexpr (OP == 1) acc += atomicAdd(&a[w], 1u);
        else if constexpr (OP == 2) a[w] = x;
        else if constexpr (OP == 3) reinterpret_cast<uint16_t*>(a)[x & 65535] = (uint16_t)x;
        else atomicOr(&a[w], (threadIdx.x & 1) ? 0u : (1u << (x >> 27)));
    }
    __syncthreads();
    if (acc == 0xdeadbeef || a[threadIdx.x] == 0xdeadbeef) out[0] = acc;
}

// Segment-major reservation: each of ntiles workgroups reserves room for its runs in nseg
// per-segment cursors (one returning atomicAdd per segment per tile).
__global__ __launch_bounds__(1024) void k_reserve(uint32_t* cur, uint32_t nseg, uint32_t* out) {
    uint32_t acc = 0;
    for (uint32_t s = threadIdx.x; s < nseg; s += 1024) acc += atomicAdd(&cur[s], 32u + (s & 7));
    if (acc == 0xdeadbeef) out[0] = acc;
}

// Scatter of the tile runs to segment-major slots: 8-lane groups write 80-byte runs.
__global__ __launch_bounds__(1024) void k_scatter(uint4* dst, uint32_t nseg, uint32_t ntiles, uint32_t slot16) {
    const uint32_t t = blockIdx.x, grp = threadIdx.x >> 3, q = threadIdx.x & 7;
    for (uint32_t s = grp; s < nseg; s += 128)
        if (q < 5) dst[((uint64_t)s * ntiles + t) * slot16 + q] = make_uint4(t, s, q, 1);
}

// Stream read of n16 uint4 (one pass, grid-stride).
__global__ __launch_bounds__(256) void k_stream(const uint4* src, uint64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0xdeadbeef) out[0] = acc;
}

template <class F>
static float time_ms(F&& f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

template <int V>
__global__ void k_hash_check(uint64_t* out) {
    const uint64_t j = threadIdx.x;
    S s{0x736f6d6570736575ULL, 0x646f72616e646f6dULL, 0x6c7967656e657261ULL, 0x7465646279746573ULL};
    if constexpr (V == 5 || V == 10) s.v2 = swap32(s.v2);
    comp<V>(s, 16); comp<V>(s, j * 0x9E3779B97F4A7C15ULL); comp<V>(s, j);
    out[j] = fin<V>(s, 32ull << 56);
}

int main(int argc, char** argv) {
    const bool hash_only = argc > 1 && std::string(argv[1]) == "hash";
    const uint64_t n = 100000000;
    uint64_t* out;
    CHECK(hipMalloc(&out, 8));
    const unsigned blocks = (unsigned)((n + 255) / 256);
    {
        uint64_t *c1, *c6;
        CHECK(hipMalloc(&c1, 64 * 8)); CHECK(hipMalloc(&c6, 64 * 8));
        hipLaunchKernelGGL(k_hash_check<1>, dim3(1), dim3(64), 0, 0, c1);
        hipLaunchKernelGGL(k_hash_check<6>, dim3(1), dim3(64), 0, 0, c6);
        uint64_t h1[64], h6[64];
        CHECK(hipMemcpy(h1, c1, 512, hipMemcpyDeviceToHost)); CHECK(hipMemcpy(h6, c6, 512, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < 64; ++i) bad += h1[i] != h6[i];
        printf("V6 (v_pk_mov_b32 swap) == V1 hashes: %s\n", bad ? "MISMATCH" : "ok");
    }
    {
        uint64_t *c1, *c5;
        CHECK(hipMalloc(&c1, 64 * 8)); CHECK(hipMalloc(&c5, 64 * 8));
        hipLaunchKernelGGL(k_hash_check<1>, dim3(1), dim3(64), 0, 0, c1);
        hipLaunchKernelGGL(k_hash_check<5>, dim3(1), dim3(64), 0, 0, c5);
        uint64_t h1[64], h5[64];
        CHECK(hipMemcpy(h1, c1, 512, hipMemcpyDeviceToHost)); CHECK(hipMemcpy(h5, c5, 512, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < 64; ++i) bad += h1[i] != h5[i];
        printf("V5 == V1 hashes: %s\n", bad ? "MISMATCH" : "ok");
    }
    {
        uint64_t *c1, *c9;
        CHECK(hipMalloc(&c1, 64 * 8)); CHECK(hipMalloc(&c9, 64 * 8));
        hipLaunchKernelGGL(k_hash_check<1>, dim3(1), dim3(64), 0, 0, c1);
        hipLaunchKernelGGL(k_hash_check<9>, dim3(1), dim3(64), 0, 0, c9);
        uint64_t h1[64], h9[64];
        CHECK(hipMemcpy(h1, c1, 512, hipMemcpyDeviceToHost)); CHECK(hipMemcpy(h9, c9, 512, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < 64; ++i) bad += h1[i] != h9[i];
        printf("V9 (shift + v_lshl_add_u64 rotates) == V1 hashes: %s\n", bad ? "MISMATCH" : "ok");
    }
    {
        uint64_t *c1, *c10;
        CHECK(hipMalloc(&c1, 64 * 8)); CHECK(hipMalloc(&c10, 64 * 8));
        hipLaunchKernelGGL(k_hash_check<1>, dim3(1), dim3(64), 0, 0, c1);
        hipLaunchKernelGGL(k_hash_check<10>, dim3(1), dim3(64), 0, 0, c10);
        uint64_t h1[64], h10[64];
        CHECK(hipMemcpy(h1, c1, 512, hipMemcpyDeviceToHost)); CHECK(hipMemcpy(h10, c10, 512, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < 64; ++i) bad += h1[i] != h10[i];
        printf("V10 (swapped adds as v_mad_u64_u32 + v_add_u32) == V1 hashes: %s\n", bad ? "MISMATCH" : "ok");
    }
    float t0 = time_ms([&] { hipLaunchKernelGGL(k_hash<0>, dim3(blocks), dim3(256), 0, 0, n, 10, out); }, 5);
    float t1 = time_ms([&] { hipLaunchKernelGGL(k_hash<1>, dim3(blocks), dim3(256), 0, 0, n, 10, out); }, 5);
    float t2 = time_ms([&] { hipLaunchKernelGGL(k_hash<2>, dim3(blocks), dim3(256), 0, 0, n, 10, out); }, 5);
    printf("hash 100M keys x k=10 (53 SipRounds/key): V0 shifts %.3f ms  V1 alignbit %.3f ms  V2 alignbit+addc %.3f ms\n",
           t0, t1, t2);
    printf("  -> G SipRounds/s: V0 %.1f  V1 %.1f  V2 %.1f\n", 53e8 / t0 / 1e6, 53e8 / t1 / 1e6, 53e8 / t2 / 1e6);
    {
        const uint64_t m = 1000000000ull, mu = ~0ull / m;
        auto run = [&](auto kern, int bs, size_t lds, const char* name) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            float t = time_ms([&] { hipLaunchKernelGGL(kern, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), lds, 0, n, 10, m, mu, out); }, 5);
            printf("  %-44s %.3f ms\n", name, t);
        };
        printf("hash variants, 100M keys x k=10 (m = 1e9):\n");
        run(k_hash2<0, 256>, 256, 0, "V1 hash only, 256 thr");
        run(k_hash2<1, 256>, 256, 0, "V1 + mod, 256 thr");
        run(k_hash2<9, 256>, 256, 0, "V9 shift+lshl_add rotates + mod, 256 thr");
        run(k_hash2<1, 256>, 256, 0, "V1 + mod, 256 thr (again)");
        run(k_hash2<9, 256>, 256, 0, "V9 shift+lshl_add rotates + mod, 256 thr (again)");
        run(k_hash2<10, 256>, 256, 0, "V10 mad_u64 swapped adds + mod, 256 thr");
        run(k_hash2<1, 256>, 256, 0, "V1 + mod, 256 thr (3rd)");
        run(k_hash2<10, 256>, 256, 0, "V10 mad_u64 swapped adds + mod, 256 thr (again)");
        run(k_hash2<2, 256>, 256, 0, "V1 2-seed interleave + mod, 256 thr");
        run(k_hash2<3, 256>, 256, 0, "V3 addc + mod, 256 thr");
        run(k_hash2<5, 256>, 256, 0, "V5 swap-folded carry adds + mod, 256 thr");
        run(k_hash2<8, 256>, 256, 0, "V1 + f64-estimate mod, 256 thr");
        run(k_hash2<8, 1024>, 1024, 80 * 1024, "V1 + f64-estimate mod, 1024 thr, 2 blocks/CU");
        {
            unsigned long long* bad;
            CHECK(hipMalloc(&bad, 8));
            for (uint64_t mm : {8192ull, 8193ull, 1000000000ull, 2147483647ull, 2147483648ull, 3000000019ull,
                                4294967295ull, 4294967291ull, 123457ull, 10000000ull}) {
                CHECK(hipMemset(bad, 0, 8));
                const uint64_t nn = 1ull << 26;
                hipLaunchKernelGGL(k_mod_check, dim3((unsigned)(nn / 256)), dim3(256), 0, 0, nn, mm, ~0ull / mm,
                                   1.0 / (double)mm, bad);
                unsigned long long hb = 0;
                CHECK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
                printf("  fmod_f64 exactness m=%llu: %llu mismatches in 2^26\n", (unsigned long long)mm, hb);
            }
        }
        run(k_hash2<6, 256>, 256, 0, "V6 pk_mov swap + mod, 256 thr");
        run(k_hash2<7, 256>, 256, 0, "V6 pk_mov swap, 2-seed + mod, 256 thr");
        run(k_hash2<6, 1024>, 1024, 80 * 1024, "V6 pk_mov swap + mod, 1024 thr, 2 blocks/CU");
        run(k_hash2<1, 1024>, 1024, 80 * 1024, "V1 + mod, 1024 thr, 2 blocks/CU");
        run(k_hash2<1, 1024>, 1024, 120 * 1024, "V1 + mod, 1024 thr, 1 block/CU (LDS)");
        run(k_hash2<2, 1024>, 1024, 120 * 1024, "V1 2-seed + mod, 1024 thr, 1 block/CU");
        run(k_hash2<3, 1024>, 1024, 120 * 1024, "V3 addc + mod, 1024 thr, 1 block/CU");
    }
    if (hash_only) return 0;
    {
        uint32_t* o;
        CHECK(hipMalloc(&o, 4));
        const int nops = 4096, blocks = 256 * 4;
        auto run = [&](auto kern, const char* name) {
            float t = time_ms([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(1024), 0, 0, nops, o); }, 3);
            const double ops = (double)blocks * 1024 * nops;
            printf("  LDS %-28s %.3f ms  %.1f G lane-ops/s  (%.1f lane-ops/clk/CU at 2.2 GHz)\n", name, t,
                   ops / t / 1e6, ops / (t * 1e-3) / 256 / 2.2e9);
        };
        printf("LDS random-address throughput (1024-thread blocks, 1 per CU at a time):\n");
        run(k_lds<0>, "ds_or_b32 (atomic)");
        run(k_lds<1>, "ds_add_rtn_u32");
        run(k_lds<2>, "ds_write_b32");
        run(k_lds<3>, "ds_write_b16");
        run(k_lds<4>, "ds_or_b32, half lanes or 0");
    }
    {
        uint32_t *cur, *o;
        CHECK(hipMalloc(&cur, 4096 * 4));
        CHECK(hipMalloc(&o, 4));
        CHECK(hipMemset(cur, 0, 4096 * 4));
        const uint32_t ntiles = 33058, nseg = 954;
        float t = time_ms([&] { hipLaunchKernelGGL(k_reserve, dim3(ntiles), dim3(1024), 0, 0, cur, nseg, o); }, 3);
        printf("segment reservation: %u tiles x %u returning atomicAdds on %u cursors: %.3f ms (%.2f G atomics/s)\n",
               ntiles, nseg, nseg, t, (double)ntiles * nseg / t / 1e6);
        uint4* big;
        const uint64_t slot16 = 8;  // 128-byte slots
        const uint64_t bytes = (uint64_t)ntiles * nseg * slot16 * 16;
        CHECK(hipMalloc(&big, bytes));
        float ts = time_ms([&] { hipLaunchKernelGGL(k_scatter, dim3(ntiles), dim3(1024), 0, 0, big, nseg, ntiles, (uint32_t)slot16); }, 3);
        printf("scatter of 80-byte runs into 128-byte segment-major slots (%.2f GB written): %.3f ms (%.1f GB/s)\n",
               (double)ntiles * nseg * 80 / 1e9, ts, (double)ntiles * nseg * 80 / ts / 1e6);
        const uint64_t n16 = (2600ull << 20) / 16;
        float tr = time_ms([&] { hipLaunchKernelGGL(k_stream, dim3(256 * 16), dim3(256), 0, 0, big, n16, o); }, 3);
        printf("stream read 2.6 GiB: %.3f ms (%.1f GB/s)\n", tr, (double)n16 * 16 / tr / 1e6);
        CHECK(hipFree(big));
    }
    uint32_t* w;
    const uint64_t maxw = 1ull << 29;  // 2 GiB
    CHECK(hipMalloc(&w, maxw * 4));
    CHECK(hipMemset(w, 0, maxw * 4));
    uint32_t* o32;
    CHECK(hipMalloc(&o32, 4));
    const uint64_t na = 100000000;
    for (uint64_t mb : {1ull, 4ull, 32ull, 125ull, 512ull, 2048ull}) {
        const uint32_t nw = (uint32_t)(mb * (1ull << 20) / 4);
        float ta = time_ms([&] { hipLaunchKernelGGL(k_atomic, dim3((unsigned)((na + 255) / 256)), dim3(256), 0, 0, w, nw, na, 10); }, 3);
        float tg = time_ms([&] { hipLaunchKernelGGL(k_gather, dim3((unsigned)((na + 255) / 256)), dim3(256), 0, 0, w, nw, na, 10, o32); }, 3);
        printf("array %5llu MiB: random atomicOr %.1f G/s   random load %.1f G/s\n", (unsigned long long)mb,
               na * 10 / ta / 1e6, na * 10 / tg / 1e6);
    }
    return 0;
}
