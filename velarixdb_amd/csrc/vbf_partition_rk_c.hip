// vbf_partition_rk_c.hip -- K1 runtime-k classes 5, 8 and 12 for keys hashed without the length
// prefix (len_prefix = 0: callers that pre-encode other Hash impls, e.g. the usize / i32 keys of
// bf.rs:275-424; vbf_tile_pack_rk.hpp).
#include "vbf_tile_pack_rk.hpp"

namespace vbf {
hipError_t launch_tile_pack_class_c(int fmt, const DevKeys& dk, const PartPlan& pl, uint32_t ntiles,
                                    uint32_t* tiles, uint16_t* ends, hipStream_t s) {
    return launch_class_impl<false, 5, 8, 12>(fmt, dk, pl, ntiles, tiles, ends, s);
}
}  // namespace vbf
