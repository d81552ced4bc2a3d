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


def test_rust_binding_call_sequence_replay(vbf, ora, tmp_path):
    """examples/rust_replay.c replays the FFI calls of INTEGRATION.md's patched bf.rs bodies (no
    rustc here): a BloomFilter with public fields only -- velarixdb's own
    `BloomFilter { file_path, ..Default::default() }` (db/recovery.rs:143-146) -- through
    compaction (new -> build_filter_from_entries -> write), a restart with persisted bits
    (Default{file_path} -> recover_meta -> build_filter_from_entries skipped -> contains), a
    memtable-born SST (per-key contains + set, 16-byte filter.db, recover + GPU rebuild at the
    recovery m) and Clone then set on the clone (bf.rs:242-254: count copied, bits shared)."""
    import json
    from velarixdb_amd import build
    from velarixdb_amd.keys import pack_offsets
    from tests import filter_file_spec as ff
    exe = os.path.join(ROOT, "examples", "rust_replay")
    if not os.path.exists(exe):
        build.build_examples()
    rng = np.random.default_rng(11)
    n, p = 40_000, 1e-4
    lens = rng.integers(1, 40, n)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    data.tofile(tmp_path / "keys.bin")
    off.tofile(tmp_path / "offs.bin")
    env = {k: v for k, v in os.environ.items() if k != "VBF_LIB"}
    r = subprocess.run([exe, str(tmp_path / "keys.bin"), str(tmp_path / "offs.bin"), str(n), repr(p), str(tmp_path)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    o = json.loads(r.stdout.strip().splitlines()[-1])
    b = pack_offsets(data, off)
    m, k = vbf.num_bits(n, p), vbf.num_hash_functions(vbf.num_bits(n, p), n)
    assert (o["m"], o["k"]) == (m, k)
    want = ora.build_words(b, m, k)
    rd = lambda name: np.fromfile(tmp_path / (name + ".words"), np.uint32)  # noqa: E731
    # 1. compaction: the GPU build, persisted after the reference's 16 bytes
    assert np.array_equal(rd("built"), want)
    assert open(tmp_path / "sst1" / "filter.db", "rb").read() == ff.encode(k, n, p, m, want, entries=n)
    # 2. restart with persisted bits: restored, rebuild skipped, stored n + entries (range.rs:121-124)
    assert o["skipped"] == [0, 1, 0]
    assert (o["rec_m"], o["rec_k"], o["rec_n"], o["hits"]) == (m, k, 2 * n, n)
    assert np.array_equal(rd("recovered"), want)
    assert o["rec_device"] >= 0  # recovered onto a GPU (VBF_DEVICE_AUTO)
    # 3. memtable-born: per-key set into the memtable's m; 16-byte filter.db; rebuilt at m(n_stored)
    m_mt = vbf.num_bits(n // 2, p)
    assert o["mt_m"] == m_mt
    assert open(tmp_path / "sst2" / "filter.db", "rb").read() == struct.pack("<IId", vbf.num_hash_functions(m_mt, n // 2),
                                                                          o["mt_n"], p)
    mt_want = np.zeros((m_mt + 31) // 32, np.uint32)
    ora.build_words(b, m_mt, vbf.num_hash_functions(m_mt, n // 2), words=mt_want)
    assert np.array_equal(rd("memtable"), mt_want)
    m_rb = vbf.num_bits(o["mt_n"], p)
    assert (o["rb_m"], o["rb_n"], o["rb_hits"]) == (m_rb, o["mt_n"] + n, n)
    assert np.array_equal(rd("rebuilt"), ora.build_words(b, m_rb, vbf.num_hash_functions(m_mt, n // 2)))
    assert o["released"] == 2  # both queued builds dropped their packed Vec
    # 4. Clone + set on the clone: count copied and diverging, bits shared
    assert (o["n_orig"], o["n_clone"]) == (o["n_before"], o["n_before"] + 1)
    assert o["fresh_in_orig"] == 1 and o["shared"] == 1
    assert o["default_ok"] == 1
