"""seed_hash == prefix_hash on the host (sip13.hpp compiles for host and device).

The partitioned build and probe hash compile-time key lengths with seed_hash, which computes
the seed-independent half of the first per-seed SipRound once per key; prefix_hash is the
direct restatement of calculate_hash (bf.rs:222-227) that the golden vectors pin.  The GPU
parity tests check the kernels bit for bit; this checks the identity itself without a GPU.
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)


@pytest.mark.skipif(HIPCC is None, reason="hipcc not found")
def test_seed_hash_equals_prefix_hash(tmp_path):
    src = os.path.join(HERE, "host", "seed_hash_check.cpp")
    exe = str(tmp_path / "seed_hash_check")
    # the header includes hip_runtime.h; compiled as HIP for the host side only
    subprocess.check_call([HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O2", "-std=c++20", src, "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout
