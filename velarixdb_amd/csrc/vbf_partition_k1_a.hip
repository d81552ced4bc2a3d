// vbf_partition_k1_a.hip -- K1 (k_tile_pack, compiled k) for the 16- and 32-byte rows (configs 2, 4, 5) (vbf_tile_pack_main.hpp).
#include "vbf_tile_pack_main.hpp"

namespace vbf {
hipError_t launch_tile_pack_main_a(int fmt, bool lp, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                    uint32_t* tiles, uint16_t* ends, hipStream_t s) {
    return launch_main_pair<16, 32>(fmt, lp, dk, pl, ntiles, tiles, ends, s);
}
}  // namespace vbf
