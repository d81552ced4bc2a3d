"""The C ABI from a plain C host (examples/c_host.c, gcc, no Python or PyTorch in the process):
the call sequence a Rust FFI caller makes -- new, set over the entries, contains, serialize, the
bit words, and the sharded fan-in build -- checked against the oracle."""
import os
import struct
import subprocess

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_c_host_matches_oracle(vbf, ora, tmp_path):
    from velarixdb_amd import build
    from velarixdb_amd.keys import HostBatch
    exe = os.path.join(ROOT, "examples", "c_host")  # built by __graft_entry__.build()
    if not os.path.exists(exe):
        exe = build.build_examples()
    n, L, p = 300_000, 16, 0.01
    keys = np.random.default_rng(5).integers(0, 256, n * L, dtype=np.uint8)
    kf = tmp_path / "keys.bin"
    keys.tofile(kf)
    out = str(tmp_path / "f")
    env = {k: v for k, v in os.environ.items() if k != "VBF_LIB"}
    r = subprocess.run([exe, str(kf), str(n), str(L), repr(p), out], capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0, r.stderr
    m, k, hits, nn, restored, async_equal = map(int, r.stdout.split())
    assert restored == 1 and async_equal == 1
    assert (m, k) == (vbf.num_bits(n, p), vbf.num_hash_functions(vbf.num_bits(n, p), n))
    assert hits == nn == n
    want = ora.build_words(HostBatch(keys, None, L, n, 1), m, k)
    words = np.fromfile(out + ".words", np.uint32)
    assert np.array_equal(words, want)
    # filter.db metadata: u32 k | u32 n | f64 p, little endian (bf.rs:158-172)
    assert open(out + ".meta", "rb").read() == struct.pack("<IId", k, n, p)
    # filter.db with the persisted bits: the reference's 16 bytes, then the extension (layout
    # spec tests/filter_file_spec.py), the words of the recovery shape (here this filter's)
    from tests import filter_file_spec as ff
    fdb = open(out + ".filterdb", "rb").read()
    assert fdb[:16] == struct.pack("<IId", k, n, p)
    assert fdb == ff.encode(k, n, p, m, want, entries=n)
    sw = np.fromfile(out + ".shards", np.uint32).reshape(2, -1)
    h = n // 2
    assert np.array_equal(sw[0], ora.build_words(HostBatch(keys[:h * L], None, L, h, 1), m, k))
    assert np.array_equal(sw[1], ora.build_words(HostBatch(keys[h * L:], None, L, n - h, 1), m, k))
    assert np.array_equal(sw[0] | sw[1], want)  # OR of the shards == the whole build


def test_memtable_latency_tool_host_equals_device(vbf):
    """examples/memtable_latency.c: the memtable's one-key calls on a host-resident and a
    device-resident filter end with identical words (CPU SipHash rounds vs the kernels)."""
    import json
    import subprocess
    exe = os.path.join(ROOT, "examples", "memtable_latency")
    out = subprocess.run([exe, "20000", "1500", "200000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert (r["m"], r["k"]) == (9815, 19)
    assert r["host_words_equal_device_words"] is True
    assert r["device"]["n_elements"] > 0
    c = r["compaction_filter"]  # the read path on a device-resident filter (host mirror)
    assert c["false_negatives"] == 0 and c["get_us_mirror"]["gets"] > 0
