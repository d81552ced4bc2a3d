// vbf_partition_sat.hip -- K1 for m == 2^32 - 1 (k_tile_pack<..., SAT = true>).
//
// velarixdb sizes every filter of more than 2^32 - 1 bits to exactly 2^32 - 1 (bf.rs:230-233: the
// f64 -> u32 cast saturates), so every large filter -- config 5, any compaction output above
// ~226M keys at p = 1e-4 -- has this m.  There 2^32 = 1 (mod m) and a bit index is hi + lo with an
// end-around carry (mod_sat, sip13.hpp) instead of the 64-bit Barrett step.  Compiled k (4, 9, 10,
// 19) with the length prefix (every byte key) on the 1 024-thread shape the plan picks above 2^31
// (k = 4 also on the 512-thread shape under VBF_K1_4, an A/B that measured slower); its own
// translation unit so the library still builds in parallel.  The runtime-k classes take the same
// remainder in their own units (vbf_tile_pack_rk.hpp).
#include <stdlib.h>

#include "vbf_tile_pack.hpp"

namespace vbf {

template <int FMT, int K, bool C16>
static hipError_t launch_sat(const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles,
                             uint16_t* ends, hipStream_t s) {
    auto fn = k_tile_pack<FMT, true, K, false, C16, 0, 0, kSegBits, false, true>;
    if constexpr (K == 4 && FMT > 0 && C16) {  // VBF_K1_4: the 512-thread shape (make_plan)
        if (pl.k1v) fn = k_tile_pack<FMT, true, 4, false, true, 1, 0, kSegBits, false, true>;
    }
    if (pl.k1v && !(K == 4 && FMT > 0 && C16)) return hipErrorNotSupported;
    // the segment counters sit at LDS address 0: no static LDS may precede them
    hipFuncAttributes fa{};
    hipError_t err = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(fn));
    if (err == hipSuccess && fa.sharedSizeBytes != 0) err = hipErrorInvalidKernelFile;
    if (err == hipSuccess)
        err = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)pl.lds1);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(fn, dim3(ntiles), dim3(pl.k1v ? 512 : kPBlock), pl.lds1, s, dk, pl, tiles, ends,
                       (uint16_t*)nullptr);
    return hipGetLastError();
}

template <int FMT>
static hipError_t launch_sat_fmt(const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles,
                                 uint16_t* ends, hipStream_t s) {
    const bool c = pl.c16 != 0;
    switch (pl.k) {
        case 4: return c ? launch_sat<FMT, 4, true>(dk, pl, ntiles, tiles, ends, s)
                         : launch_sat<FMT, 4, false>(dk, pl, ntiles, tiles, ends, s);
        case 9: return c ? hipErrorNotSupported : launch_sat<FMT, 9, false>(dk, pl, ntiles, tiles, ends, s);
        case 10: return c ? launch_sat<FMT, 10, true>(dk, pl, ntiles, tiles, ends, s)
                          : launch_sat<FMT, 10, false>(dk, pl, ntiles, tiles, ends, s);
        case 19: return c ? launch_sat<FMT, 19, true>(dk, pl, ntiles, tiles, ends, s)
                          : launch_sat<FMT, 19, false>(dk, pl, ntiles, tiles, ends, s);
        default: return hipErrorNotSupported;
    }
}

hipError_t launch_tile_pack_sat(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles,
                                uint16_t* ends, hipStream_t s) {
    // VBF_SAT=0 (A/B, speed only): the general m > 2^31 kernels with the Barrett remainder
    static const int on = [] { const char* e = getenv("VBF_SAT"); return e ? atoi(e) : 1; }();
    if (!on || pl.m != 0xFFFFFFFFull || (pl.k1v && pl.k != 4) || pl.kc) return hipErrorNotSupported;
    switch (fmt) {
        case 16: return launch_sat_fmt<16>(dk, pl, ntiles, tiles, ends, s);
        case 32: return launch_sat_fmt<32>(dk, pl, ntiles, tiles, ends, s);
        case 8: return launch_sat_fmt<8>(dk, pl, ntiles, tiles, ends, s);
        case 24: return launch_sat_fmt<24>(dk, pl, ntiles, tiles, ends, s);
        case -1: return launch_sat_fmt<-1>(dk, pl, ntiles, tiles, ends, s);
        default: return launch_sat_fmt<0>(dk, pl, ntiles, tiles, ends, s);
    }
}

}  // namespace vbf
