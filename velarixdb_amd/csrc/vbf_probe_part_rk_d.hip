// vbf_probe_part_rk_d.hip -- the partitioned probe's runtime-k class packs, classes 16, 21, 24, 32, keys without the length prefix
// (vbf_probe_pack.hpp).
#include "vbf_probe_pack.hpp"

namespace vbf {
hipError_t launch_probe_pack_class_d(int fmt, uint32_t kc, const DevKeys& dk, const ProbePlan& pl, uint32_t ntiles,
                                     uint32_t* tiles, uint16_t* ends, hipStream_t s) {
    return launch_probe_pack_classes<false, kSegBits, 16, 21, 24, 32>(fmt, kc, dk, pl, ntiles, tiles, ends, s);
}
}  // namespace vbf
