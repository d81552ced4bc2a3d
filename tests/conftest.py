import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; runs the HIP path")
    # Build the in-tree artefacts when a fresh checkout lacks them (hipcc cross-compiles
    # gfx950 without a GPU; the oracle is plain gcc).
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_vbf_build", os.path.join(ROOT, "velarixdb_amd", "build.py"))
    vbuild = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(vbuild)  # loads build.py alone: the package import needs the .so
    vbuild.build()
    import oracle  # noqa: F401  (builds liboracle.so on import when missing)


def load_golden(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def ora():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def vbf():
    """The product library on a real device: fails (not skips) without one."""
    from velarixdb_amd import build
    build.build()
    import velarixdb_amd
    n = velarixdb_amd.device_count()
    assert n > 0, "gpu-marked test needs a HIP device: " + velarixdb_amd.lib.vbf_last_error().decode()
    return velarixdb_amd
