// vbf_partition_rk_d.hip -- K1 runtime-k classes 16, 21, 24 and 32 for keys hashed without the
// length prefix (vbf_partition_rk_c.hip's, vbf_tile_pack_rk.hpp).
#include "vbf_tile_pack_rk.hpp"

namespace vbf {
hipError_t launch_tile_pack_class_d(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                    uint32_t* tiles, uint16_t* ends, hipStream_t s) {
    return launch_class_impl<false, 16, 21, 24, 32>(fmt, dk, pl, ntiles, tiles, ends, s);
}
}  // namespace vbf
