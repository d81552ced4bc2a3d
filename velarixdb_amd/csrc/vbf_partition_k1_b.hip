// vbf_partition_k1_b.hip -- K1 (k_tile_pack, compiled k) for the 8- and 24-byte rows (vbf_tile_pack_main.hpp).
#include "vbf_tile_pack_main.hpp"

namespace vbf {
hipError_t launch_tile_pack_main_b(int fmt, bool lp, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                    uint32_t* tiles, uint16_t* ends, hipStream_t s) {
    return launch_main_pair<8, 24>(fmt, lp, dk, pl, ntiles, tiles, ends, s);
}
}  // namespace vbf
