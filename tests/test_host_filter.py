"""Host-resident filters (device = HOST): the memtable's per-put path, on the CPU in libvbf.

The reference's memtable does a contains + set per put and a contains per get
(src/memtable/mem.rs:207-230); SURVEY.md 8(b) keeps those single-key calls on the host with the
identical hash.  libvbf runs them with the kernels' SipHash-1-3 rounds (csrc/sip13.hpp compiled
for the host) and Rust's `hash % m` -- not the oracle.  These tests need no GPU: they compare
that host path with the golden vectors and with the oracle, and restate the reference's filter
and memtable unit tests on it.  The same restatements run on the GPU in test_gpu_residency.py.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN
from tests_util import MemTableMirror, parse_data_db, parse_filter_db

SST = os.path.join(GOLDEN, "sst_fixtures")


def test_random_sets_match_golden(golden):
    from velarixdb_amd import HOST, BloomFilter
    from velarixdb_amd.keys import pack
    seen = 0
    for s in golden("random_sets"):
        if "words" not in s:
            continue
        f = BloomFilter.sized(s["m"], s["k"], device=HOST)
        f.set_many(pack([bytes.fromhex(x) for x in s["keys"]]))
        assert ["%08x" % x for x in f.words()] == s["words"]
        if "neg_keys" in s:
            got = f.contains_many(pack([bytes.fromhex(x) for x in s["neg_keys"]]))
            assert got.astype(int).tolist() == s["neg_hits"]
        seen += 1
    assert seen >= 3


def test_hash_indices_match_golden(golden):
    """One key, k = 1 per seed: the single bit set is calculate_hash(key, 0) % m (bf.rs:88)."""
    from velarixdb_amd import HOST, BloomFilter
    from velarixdb_amd.keys import RawMessage, pack
    for v in golden("hashes"):
        key = bytes.fromhex(v["key"])
        h0 = int(v["h"][0], 16)
        for m in (1000003, 65521, 64, 1):
            f = BloomFilter.sized(m, 1, device=HOST)
            f.set_many(pack([key] if v["len_prefix"] else [RawMessage(key)]))
            w = f.words()
            idx = h0 % m
            assert int(w[idx >> 5]) >> (idx & 31) & 1 and int(np.unpackbits(w.view(np.uint8)).sum()) == 1


def test_fpr_tests_match_golden(golden):
    """bf.rs:307-424 (n = 10 000 usize keys, 2 000 negatives) on a host-resident filter."""
    from velarixdb_amd import HOST, BloomFilter
    for v in golden("fpr_tests"):
        p = float.fromhex(v["p"])
        bf = BloomFilter(p, 10000, device=HOST)
        assert (bf.num_bits(), bf.no_of_hash_func) == (v["m"], v["k"])
        bf.set_many(range(10000))
        w = bf.words()
        assert hashlib.sha256(w.astype("<u4").tobytes()).hexdigest() == v["sha256"]
        fp = int(bf.contains_many(range(10000, 12000)).sum())
        assert fp == v["false_positives"] and fp / 2000 <= p * 1.1
        assert bf.contains_many(range(10000)).all()


def test_bf_rs_unit_tests():
    """test_set_and_contain (bf.rs:275-291), test_number_of_elements (:294-304)."""
    from velarixdb_amd import HOST, BloomFilter, I32Vec
    bf = BloomFilter(0.01, 10, device=HOST)
    assert bf.num_elements() == 0 and bf.no_of_hash_func == 9 and bf.num_bits() == 95
    bf.set(I32Vec((1, 2, 3, 4)))
    assert bf.num_elements() == 1 and bf.contains(I32Vec((1, 2, 3, 4)))
    bf = BloomFilter(0.01, 10, device=HOST)
    for i in range(10):
        bf.set(i)
    assert bf.num_elements() == 10


def test_fixture_ssts_match_golden(golden):
    """recover_meta + build_filter_from_entries (range.rs:121-124) of the reference's SSTs."""
    from velarixdb_amd import HOST, BloomFilter
    want = {s["name"]: s for s in golden("sst_fixtures")["ssts"]}
    for name in sorted(os.listdir(SST)):
        bf = BloomFilter.default(device=HOST)
        bf.file_path = os.path.join(SST, name, "filter.db")
        bf.recover_meta()
        assert bf.host_resident
        k, n, p = parse_filter_db(bf.file_path)
        assert (bf.no_of_hash_func, bf.no_of_elements, bf.num_bits()) == (k, n, want[name]["m"])
        keys = parse_data_db(os.path.join(SST, name, "data.db"))
        bf.build_filter_from_entries(keys)
        assert bf.no_of_elements == n + len(keys)
        assert hashlib.sha256(bf.words().astype("<u4").tobytes()).hexdigest() == want[name]["sha256"]
        assert int(bf.contains_many([b"zz%05d" % i for i in range(5000)]).sum()) == want[name]["neg_hits_zz5000"]
        assert all(bf.contains(x) for x in keys[:50])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_keys_match_oracle(ora, seed):
    """Every length 0..200 (several blocks, every tail), both encodings, runtime k up to 40."""
    from velarixdb_amd import HOST, BloomFilter
    from velarixdb_amd.keys import pack_offsets
    rng = np.random.default_rng(seed)
    n = 3000
    lens = rng.integers(0, 201, size=n)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    data = rng.integers(0, 256, size=int(off[-1]) + 1, dtype=np.uint8)
    for lp in (1, 0):
        m = int(rng.integers(1, 200_000))
        k = int(rng.integers(1, 41))
        b = pack_offsets(data, off, len_prefix=lp)
        f = BloomFilter.sized(m, k, device=HOST)
        f.set_many(b)
        assert np.array_equal(f.words(), ora.build_words(b, m, k))
        assert f.contains_many(b).all()
        neg = pack_offsets(data[::-1].copy(), off, len_prefix=lp)
        assert np.array_equal(f.contains_many(neg), ora.probe(neg, m, k, f.words()).astype(bool))


def _mem(p=1e-300):
    from velarixdb_amd import HOST
    return MemTableMirror(51200, p, HOST)


def test_memtable_sizing():
    """mem.rs:188-191 with the tests' buffer_size 51200 (512 entries) and the default p."""
    from velarixdb_amd import num_bits, num_hash_functions
    for p in (1e-300, 1e-10, 1e-4):
        mt = _mem(p)
        bf = mt.bloom_filter
        assert bf.num_elements() == 0  # mem.rs:349,366,384
        m = num_bits(512, p)
        assert (bf.num_bits(), bf.no_of_hash_func) == (m, num_hash_functions(m, 512))
    assert (_mem(1e-4).bloom_filter.num_bits(), _mem(1e-4).bloom_filter.no_of_hash_func) == (9815, 19)
    assert _mem(1e-300).bloom_filter.no_of_hash_func == 1437  # k = floor(m/n) (bf.rs:236-239)


def test_memtable_get_and_negative_key():
    """test_get (mem.rs:405-426): the inserted key is found, [8,2,3,4] is not."""
    mt = _mem()
    key = bytes([1, 2, 3, 4])
    mt.insert(key, 400)
    assert mt.get(key) == 400
    assert mt.get(bytes([8, 2, 3, 4])) is None
    assert mt.bloom_filter.num_elements() == 1


def test_memtable_insert_counts_sets_only():
    """test_insert (mem.rs:378-402): the same key three times -> one set (contains first)."""
    mt = _mem()
    for _ in range(3):
        mt.insert(bytes([1, 2, 3, 4]), 400)
    assert mt.bloom_filter.num_elements() == 1


def test_memtable_update_delete_unknown_key():
    """test_update / test_delete (mem.rs:502-569): an unknown key is KeyNotFoundInMemTable."""
    mt = _mem()
    mt.insert(bytes([1, 2, 3, 4]), 400)
    mt.update(bytes([1, 2, 3, 4]), 300)
    assert mt.get(bytes([1, 2, 3, 4])) == 300
    with pytest.raises(KeyError):
        mt.update(bytes([2, 2, 3, 4]), 1)
    with pytest.raises(KeyError):
        mt.delete(bytes([2, 2, 3, 4]), 1)


def test_memtable_concurrent_writes():
    """test_concurrent_write (mem.rs:431-499): five threads insert under the table's mutex."""
    import threading
    mt = _mem(1e-4)
    lock = threading.Lock()
    keys = [bytes([i, 2, 3, 4]) for i in range(1, 6)]

    def put(i):
        with lock:
            mt.insert(keys[i], i)

    th = [threading.Thread(target=put, args=(i,)) for i in range(5)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert [mt.get(k) for k in keys] == [0, 1, 2, 3, 4]


def test_handle_semantics_host():
    """Clone shares the bits and copies the count (bf.rs:242-254); clear (:180-195); words."""
    from velarixdb_amd import HOST, BloomFilter
    bf = BloomFilter(1e-4, 512, device=HOST)
    keys = [b"key%04d" % i for i in range(300)]
    bf.set_many(keys)
    c = bf.clone()
    c.set(b"extra")
    assert bf.contains(b"extra") and (bf.no_of_elements, c.no_of_elements) == (300, 301)
    w = bf.words()
    other = BloomFilter(1e-4, 512, device=HOST)
    other.load_words(w)
    assert other.contains_many(keys).all() and np.array_equal(other.words(), w)
    fresh = bf.clear()
    assert not bf.words().any() and not c.words().any() and fresh.host_resident
    assert (fresh.num_bits(), fresh.no_of_hash_func, fresh.no_of_elements) == (9815, 19, 0)
    bf.set_num_elements(7)
    assert bf.no_of_elements == 7 and bf.serialize()[4:8] == (7).to_bytes(4, "little")


def test_pristine_host_filter_holds_no_host_words():
    """BloomFilter::new on the host (bf.rs:62-81) allocates no bit array until its
    first use -- the compaction filter (sized.rs:192-193) goes new -> migrate to a GPU without
    touching host memory.  Reading a never-written filter gives zeros; the first set allocates
    the words; clear keeps them; a contains on a fresh filter answers false (m > 0, k > 0)."""
    from velarixdb_amd import HOST, BloomFilter
    bf = BloomFilter(1e-4, 2_000_000, device=HOST)  # m = 38.3M bits: 4.8 MB of words
    assert bf.host_bytes == 0
    assert bf.no_of_hash_func == 19 and bf.num_bits() == 38_340_233
    c = bf.clone()  # shares the (still unallocated) bits
    assert c.host_bytes == 0
    w = bf.words()
    assert w.shape == (bf.num_words(),) and not w.any() and bf.host_bytes == 0
    fresh = bf.clear()
    assert bf.host_bytes == 0 and fresh.host_bytes == 0
    assert not bf.contains(b"never set")
    assert bf.host_bytes == bf.num_words() * 4  # the probe needs the words: allocated, zero
    g = BloomFilter(1e-4, 1000, device=HOST)
    g.set(b"key")
    assert g.host_bytes == g.num_words() * 4 and g.contains(b"key") and c.host_bytes == bf.host_bytes


def test_host_filter_rejects_device_entry_points():
    from velarixdb_amd import HOST, BloomFilter
    from velarixdb_amd._lib import VBF_EINVAL, lib
    bf = BloomFilter(0.01, 100, device=HOST)
    assert lib.vbf_filter_set_dev(bf._h, None, None, 1, 1, 1, None) == VBF_EINVAL
    assert b"host-resident" in lib.vbf_last_error()
    assert lib.vbf_filter_contains_dev(bf._h, None, None, 1, 1, 1, None, None) == VBF_EINVAL
    assert bf.words_dev_ptr() is None
    # k == 0 (p > 1): vacuously true (bf.rs:104); m == 0 < k: the reference panics
    z = BloomFilter(2.0, 5, device=HOST)
    z.set(b"a")
    assert z.contains(b"zzz")
    with pytest.raises(ZeroDivisionError):
        BloomFilter.sized(0, 3, device=HOST).contains(b"a")


def test_memtable_latency_tool_runs_without_gpu():
    """examples/memtable_latency.c (plain C, no Python in the process): the host residency works
    with no GPU in the machine; puts of a 512-entry filter (m = 9815, k = 19, mem.rs:188-191)."""
    import json
    import subprocess
    from conftest import ROOT
    exe = os.path.join(ROOT, "examples", "memtable_latency")
    if not os.path.exists(exe):
        pytest.skip("examples not built (__graft_entry__.build())")
    out = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert (r["m"], r["k"]) == (9815, 19) and 0 < r["host"]["n_elements"] <= 20000


def test_host_residency_async_sync_mirror_calls():
    """Round-3 entry points on a host-resident filter, no GPU needed: set_host_async sets at once
    (nothing to overlap with) and calls the release callback before returning; sync / busy are
    trivially idle; the mirror mode is accepted (a host filter is its own mirror); the stream
    bracketing of external device writers is rejected like the other device entry points."""
    import ctypes
    from velarixdb_amd import HOST, BloomFilter
    from velarixdb_amd._lib import VBF_EINVAL, call, lib
    from velarixdb_amd.keys import pack
    keys = [b"as%05d" % i for i in range(2000)]
    bf = BloomFilter(1e-3, 2000, device=HOST)
    b = pack(keys)
    released = []
    CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
    cb = CB(lambda ctx: released.append(ctx))
    d, o = b.ptrs()
    call("vbf_filter_set_host_async", bf._h, d, o, b.stride, b.n, 1, ctypes.cast(cb, ctypes.c_void_p), 5)
    assert released == [5] and not bf.busy() and bf.no_of_elements == 2000
    bf.sync()
    assert bf.contains_many(keys).all()
    bf.set_many_async(keys[:10])  # library-copy form
    assert bf.no_of_elements == 2010
    for mode in ("off", "lazy", "eager"):
        bf.set_mirror(mode)
    assert lib.vbf_filter_set_mirror(bf._h, 7) == VBF_EINVAL
    assert lib.vbf_filter_stream_wait(bf._h, None) == VBF_EINVAL
    assert lib.vbf_filter_stream_record(bf._h, None) == VBF_EINVAL
    assert b"host-resident" in lib.vbf_last_error()
    # a pristine host filter migrates to host (no-op) and its words stay zero
    z = BloomFilter(1e-3, 1000, device=HOST)
    z.migrate(HOST)
    assert not z.words().any()


def test_multi_probe_host_filters_rejected_and_bounds_checked():
    """vbf_multi_probe_host takes device-resident filters (mirror or GPU path); host-resident ones
    are rejected before anything runs, as are NULL filters."""
    import ctypes
    from velarixdb_amd import HOST, BloomFilter
    from velarixdb_amd._lib import VBF_EINVAL, lib
    from velarixdb_amd.keys import pack
    f = BloomFilter(1e-3, 100, device=HOST)
    b = pack([b"x"])
    out = np.zeros(1, np.uint8)
    handles = (ctypes.c_void_p * 1)(f._h.value)
    d, o = b.ptrs()
    assert lib.vbf_multi_probe_host(d, o, b.stride, 1, 1, 1, handles, None, None, out.ctypes.data) == VBF_EINVAL
    nulls = (ctypes.c_void_p * 1)(None)
    assert lib.vbf_multi_probe_host(d, o, b.stride, 1, 1, 1, nulls, None, None, out.ctypes.data) == VBF_EINVAL
