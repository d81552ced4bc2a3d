// vbf_partition_k1_c.hip -- K1 (k_tile_pack, compiled k) for offsets and runtime strides (config 3) (vbf_tile_pack_main.hpp).
#include "vbf_tile_pack_main.hpp"

namespace vbf {
hipError_t launch_tile_pack_main_c(int fmt, bool lp, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                    uint32_t* tiles, uint16_t* ends, hipStream_t s) {
    return launch_main_pair<-1, 0>(fmt, lp, dk, pl, ntiles, tiles, ends, s);
}
}  // namespace vbf
