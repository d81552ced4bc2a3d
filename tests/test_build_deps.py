"""velarixdb_amd/build.py: an object is rebuilt when any header it reaches changed (round 6: a header
edited while an earlier build ran is still caught, objects are checked against their own includes)."""
import os
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "velarixdb_amd"))
import build  # noqa: E402


def _names(paths):
    return {os.path.basename(p) for p in paths}


def test_deps_follow_includes_transitively():
    deps = _names(build._deps(os.path.join(build.CSRC, "vbf_partition.hip")))
    # vbf_partition.hip -> vbf_tile_pack.hpp -> vbf_partition.hpp -> sip13.hpp / keyhash.hpp / vbf_kernels.hpp
    assert {"vbf_partition.hip", "vbf_tile_pack.hpp", "vbf_partition.hpp", "sip13.hpp", "keyhash.hpp",
            "vbf_kernels.hpp"} <= deps


def test_every_source_exists_and_reaches_its_headers():
    for s in build.SOURCES:
        src = os.path.join(build.CSRC, s)
        assert os.path.exists(src), s
        deps = build._deps(src)
        assert src in deps and all(os.path.exists(d) for d in deps)
