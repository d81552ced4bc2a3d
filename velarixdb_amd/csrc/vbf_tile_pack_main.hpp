// vbf_tile_pack_main.hpp -- the compiled-k K1 launch of launch_build_partitioned (k_tile_pack for
// k = 4, 9, 10, 19 and the generic runtime-k kernel, both remainders, both K1 shapes) for one key
// layout.  Included by vbf_partition_k1_{a,b,c}.hip only: each instantiates two layouts, so the
// library's largest translation unit no longer compiles every k_tile_pack variant at once.
#pragma once
#include "vbf_tile_pack.hpp"

namespace vbf {

template <int FMT, bool LP>
hipError_t launch_main_fmt(const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles, uint16_t* ends,
                           hipStream_t s) {
    const uint64_t m = pl.m;
    const uint32_t k = pl.k;
    // m <= 2^31: the one-word remainder (fast_mod31); the runtime-k kernel keeps the general one
    auto pick = [&]<bool S>() {
        if constexpr (FMT > 0 && S) {  // the 512-thread shape (make_plan: m <= 2^31)
            if (pl.k1v && k == 10) return pl.c16 ? k_tile_pack<FMT, LP, 10, true, true, 1>
                                                 : k_tile_pack<FMT, LP, 10, true, false, 1>;
            if (pl.k1v && k == 19) return pl.c16 ? k_tile_pack<FMT, LP, 19, true, true, 1>
                                                 : k_tile_pack<FMT, LP, 19, true, false, 1>;
        } else if constexpr (S) {  // runtime-length layouts: plain counters only (make_plan)
            if (pl.k1v && k == 10) return k_tile_pack<FMT, LP, 10, true, false, 1>;
            if (pl.k1v && k == 19) return k_tile_pack<FMT, LP, 19, true, false, 1>;
        }
        return k == 10 ? (pl.c16 ? k_tile_pack<FMT, LP, 10, S, true> : k_tile_pack<FMT, LP, 10, S>)
             : k == 4  ? (pl.c16 ? k_tile_pack<FMT, LP, 4, S, true> : k_tile_pack<FMT, LP, 4, S>)
             : k == 19 ? (pl.c16 ? k_tile_pack<FMT, LP, 19, S, true> : k_tile_pack<FMT, LP, 19, S>)
             : k == 9  ? k_tile_pack<FMT, LP, 9, S>
                       : k_tile_pack<FMT, LP, 0, false>;
    };
    auto fn = m <= (1u << 31) ? pick.template operator()<true>() : pick.template operator()<false>();
    // the segment counters sit at LDS address 0: no static LDS may precede them
    hipFuncAttributes fa{};
    hipError_t err = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(fn));
    if (err == hipSuccess && fa.sharedSizeBytes != 0) err = hipErrorInvalidKernelFile;
    if (err == hipSuccess)
        err = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)pl.lds1);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(fn, dim3(ntiles), dim3(pl.k1v == 1 ? 512 : kPBlock), pl.lds1, s, dk, pl, tiles, ends,
                       (uint16_t*)nullptr);
    return hipGetLastError();
}

template <int F0, int F1>
hipError_t launch_main_pair(int fmt, bool lp, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                            uint32_t* tiles, uint16_t* ends, hipStream_t s) {
    if (fmt == F0) return lp ? launch_main_fmt<F0, true>(dk, pl, ntiles, tiles, ends, s)
                             : launch_main_fmt<F0, false>(dk, pl, ntiles, tiles, ends, s);
    if (fmt == F1) return lp ? launch_main_fmt<F1, true>(dk, pl, ntiles, tiles, ends, s)
                             : launch_main_fmt<F1, false>(dk, pl, ntiles, tiles, ends, s);
    return hipErrorInvalidValue;
}

}  // namespace vbf
