// vbf_probe_pu_rk_a.hip -- U1 of the round-6 probe (k_tile_pack<..., KC, POS = 2>) for the runtime-k
// classes 5, 8 and 12, every key layout (fixed and runtime lengths) hashed with the length prefix, m <= 2^31; a translation
// unit of its own so the library builds in parallel (vbf_probe_pu.hip launches it).
#include "vbf_tile_pack_rk.hpp"

namespace vbf {

template <int FMT, int KC>
static hipError_t launch_pu_one_class(const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles,
                                      uint32_t* endsT, uint32_t* posv, hipStream_t s) {
    auto fn = k_tile_pack<FMT, true, 0, true, false, 1, KC, kSegBits, 2, false>;
    hipFuncAttributes fa{};
    hipError_t err = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(fn));
    if (err == hipSuccess && fa.sharedSizeBytes != 0) err = hipErrorInvalidKernelFile;
    if (err == hipSuccess)
        err = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)pl.lds1);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(fn, dim3(ntiles), dim3(512), pl.lds1, s, dk, pl, tiles, reinterpret_cast<uint16_t*>(endsT),
                       reinterpret_cast<uint16_t*>(posv));
    return hipGetLastError();
}

hipError_t launch_pu_pack_class_a(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles, uint32_t* tiles,
                                  uint32_t* endsT, uint32_t* posv, hipStream_t s) {
    hipError_t err = hipErrorNotSupported;
    auto one = [&]<int KC>() {
        if (pl.kc != (uint32_t)KC) return;
        switch (fmt) {
            case 16: err = launch_pu_one_class<16, KC>(dk, pl, ntiles, tiles, endsT, posv, s); break;
            case 32: err = launch_pu_one_class<32, KC>(dk, pl, ntiles, tiles, endsT, posv, s); break;
            case 8: err = launch_pu_one_class<8, KC>(dk, pl, ntiles, tiles, endsT, posv, s); break;
            case 24: err = launch_pu_one_class<24, KC>(dk, pl, ntiles, tiles, endsT, posv, s); break;
            case -1: err = launch_pu_one_class<-1, KC>(dk, pl, ntiles, tiles, endsT, posv, s); break;
            default: err = launch_pu_one_class<0, KC>(dk, pl, ntiles, tiles, endsT, posv, s); break;
        }
    };
    one.template operator()<5>();
    one.template operator()<8>();
    one.template operator()<12>();
    return err;
}

}  // namespace vbf
