// vbf_tile_pack_rk.hpp -- launch of the runtime-k class kernels of K1 (k_tile_pack<..., KC>), for
// k outside the compiled set {4, 9, 10, 19}.  Included by the class translation units
// (vbf_partition_rk_a.hip: classes 5, 8, 12; vbf_partition_rk_b.hip: 16, 21, 24, 32;
// vbf_partition_rk_c.hip / _d.hip: the same classes for keys hashed without the length prefix -- the
// pre-encoded integer keys of bf.rs:275-424), which the build compiles in parallel with the rest of
// the library.
#pragma once
#include <stdlib.h>

#include "vbf_tile_pack.hpp"

namespace vbf {

// The smallest compiled class holding k seeds (0: none, k > 32).
inline uint32_t tile_pack_class(uint32_t k) {
    for (uint32_t c : {5u, 8u, 12u, 16u, 21u, 24u, 32u})
        if (k <= c) return c;
    return 0;
}

// Defined in vbf_partition_rk_a.hip (pl.kc <= 12) and vbf_partition_rk_b.hip (pl.kc >= 16), both with
// the length prefix, and vbf_partition_rk_c.hip / _d.hip (the same, no length prefix).
hipError_t launch_tile_pack_class_a(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                    uint32_t* tiles, uint16_t* ends, hipStream_t s);
hipError_t launch_tile_pack_class_b(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                    uint32_t* tiles, uint16_t* ends, hipStream_t s);
hipError_t launch_tile_pack_class_c(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                    uint32_t* tiles, uint16_t* ends, hipStream_t s);
hipError_t launch_tile_pack_class_d(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                    uint32_t* tiles, uint16_t* ends, hipStream_t s);

// VBF_SAT=0 (A/B, speed only): Barrett remainders at m = 2^32 - 1 as well (vbf_partition_sat.hip)
inline bool sat_enabled() {
    static const int on = [] { const char* e = getenv("VBF_SAT"); return e ? atoi(e) : 1; }();
    return on != 0;
}

// One class kernel: the segment counters sit at LDS address 0 (no static LDS may precede them),
// the dynamic LDS request is the plan's.
template <int FMT, int KC, bool LP>
hipError_t launch_one_class(const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles, uint16_t* ends,
                            hipStream_t s) {
    // m = 2^32 - 1 (the reference's saturated size): the end-around-carry remainder (SAT)
    auto fn = pl.m <= (1ull << 31)        ? k_tile_pack<FMT, LP, 0, true, false, 1, KC>
              : pl.m == 0xFFFFFFFFull && sat_enabled() ? k_tile_pack<FMT, LP, 0, false, false, 1, KC, kSegBits, false, true>
                                                  : k_tile_pack<FMT, LP, 0, false, false, 1, KC>;
    hipFuncAttributes fa{};
    hipError_t err = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(fn));
    if (err == hipSuccess && fa.sharedSizeBytes != 0) err = hipErrorInvalidKernelFile;
    if (err == hipSuccess)
        err = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)pl.lds1);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(fn, dim3(ntiles), dim3(512), pl.lds1, s, dk, pl, tiles, ends, (uint16_t*)nullptr);
    return hipGetLastError();
}

template <bool LP, int... KCs>
hipError_t launch_class_impl(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles,
                             uint16_t* ends, hipStream_t s) {
    hipError_t err = hipErrorInvalidValue;
    auto one = [&]<int KC>() {
        if (pl.kc != (uint32_t)KC) return;
        switch (fmt) {
            case 16: err = launch_one_class<16, KC, LP>(dk, pl, ntiles, tiles, ends, s); break;
            case 32: err = launch_one_class<32, KC, LP>(dk, pl, ntiles, tiles, ends, s); break;
            case 8: err = launch_one_class<8, KC, LP>(dk, pl, ntiles, tiles, ends, s); break;
            case 24: err = launch_one_class<24, KC, LP>(dk, pl, ntiles, tiles, ends, s); break;
            case -1: err = launch_one_class<-1, KC, LP>(dk, pl, ntiles, tiles, ends, s); break;
            default: err = launch_one_class<0, KC, LP>(dk, pl, ntiles, tiles, ends, s); break;
        }
    };
    (one.template operator()<KCs>(), ...);
    return err;
}

}  // namespace vbf
