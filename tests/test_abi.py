"""CPU-side checks of the C ABI: the library loads, exports every symbol include/vbf.h
declares, and its host-only logic (sizing, metadata, argument checks) matches the reference.
No kernel is launched here."""
import ctypes
import math
import os
import re
import struct

import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "vbf.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vbf_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import velarixdb_amd
    from velarixdb_amd._lib import SIGNATURES
    names = _declared()
    assert len(names) >= 30
    for n in names:
        assert hasattr(velarixdb_amd.lib, n), n
        assert n in SIGNATURES, "ctypes binding missing " + n
    assert set(SIGNATURES) == set(names)


def test_symbols_in_dynamic_table():
    out = os.popen("nm -D --defined-only %s" % os.path.join(ROOT, "velarixdb_amd", "libvbf.so")).read()
    for n in _declared():
        assert re.search(r"\bT %s\b" % n, out), n


def test_library_is_gfx950_code_object():
    so = os.path.join(ROOT, "velarixdb_amd", "libvbf.so")
    blob = open(so, "rb").read()
    assert b"gfx950" in blob
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob or b"amdgcn-amd-amdhsa--gfx950" in blob


def test_sizing_matches_golden(golden):
    from velarixdb_amd import num_bits, num_hash_functions
    for v in golden("sizing"):
        p = float.fromhex(v["p"])
        m = num_bits(v["n"], p)
        assert m == v["m"], v
        assert num_hash_functions(m, v["n"]) == v["k"], v


def test_size_asserts_like_reference():
    from velarixdb_amd._lib import VBF_EINVAL, lib
    m, k = ctypes.c_uint32(), ctypes.c_uint32()
    assert lib.vbf_size(-0.1, 10, ctypes.byref(m), ctypes.byref(k)) == VBF_EINVAL  # bf.rs:63-66
    assert b"False positive rate" in lib.vbf_last_error()
    assert lib.vbf_size(0.01, 0, ctypes.byref(m), ctypes.byref(k)) == VBF_EINVAL  # bf.rs:67
    assert lib.vbf_size(float("nan"), 10, ctypes.byref(m), ctypes.byref(k)) == VBF_EINVAL
    assert lib.vbf_size(0.01, 10, ctypes.byref(m), ctypes.byref(k)) == 0
    assert (m.value, k.value) == (95, 9)
    assert lib.vbf_last_error() == b""


def test_headline_config_sizes():
    from velarixdb_amd import num_bits, num_hash_functions
    from velarixdb_amd.workloads import fpr_for_bits_per_key
    p10, p15 = fpr_for_bits_per_key(10), fpr_for_bits_per_key(15)
    for n, p, m, k in [(1_000_000, p10, 10_000_000, 10), (100_000_000, p10, 1_000_000_000, 10),
                       (50_000_000, p10, 500_000_000, 10),
                       (1_000_000_000, p15, 4294967295, 4)]:  # u32 saturation, SURVEY 0.4
        assert num_bits(n, p) == m
        assert num_hash_functions(m, n) == k


def test_meta_roundtrip_and_layout():
    from velarixdb_amd._lib import lib
    buf = (ctypes.c_uint8 * 16)()
    lib.vbf_meta_serialize(19, 1791, 1e-4, buf)
    assert bytes(buf) == struct.pack("<IId", 19, 1791, 1e-4)
    k, n, p = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_double()
    raw = open(os.path.join(ROOT, "tests/golden/sst_fixtures/sstable_1720785462309/filter.db"), "rb").read()
    assert lib.vbf_meta_parse(raw, len(raw), ctypes.byref(k), ctypes.byref(n), ctypes.byref(p)) == 0
    assert (k.value, n.value, p.value) == (19, 1791, 1e-4)
    assert lib.vbf_meta_parse(raw, 12, ctypes.byref(k), ctypes.byref(n), ctypes.byref(p)) != 0


def test_key_encodings():
    from velarixdb_amd.keys import I32Vec, RawMessage, Usize, encode, pack
    assert encode(b"ab") == (b"ab", 1)
    assert encode(Usize(5)) == (struct.pack("<Q", 5), 0)
    assert encode(7) == (struct.pack("<Q", 7), 0)
    assert encode(I32Vec((1, 2, 3, 4))) == (struct.pack("<Q4i", 4, 1, 2, 3, 4), 0)
    assert encode(RawMessage(b"xyz")) == (b"xyz", 0)
    with pytest.raises(TypeError):
        encode("str")
    b = pack([b"a", b"bcd", b""])
    assert b.offsets.tolist() == [0, 1, 4, 4] and b.n == 3 and b.len_prefix == 1
    b = pack([b"abcd", b"efgh"])
    assert b.offsets is None and b.stride == 4
    with pytest.raises(ValueError):
        pack([b"a", 3])


def test_var_workload_lengths_match_oracle(ora):
    from velarixdb_amd.workloads import SEED_CFG3, var_lengths
    got = var_lengths(SEED_CFG3, 12345, 5000)
    want = ora.gen_var_lengths(SEED_CFG3, 12345, 5000)
    assert got.tolist() == want.tolist()
    assert got.min() >= 8 and got.max() <= 128
    mean = var_lengths(SEED_CFG3, 0, 200000).mean()
    assert 24.0 < mean < 28.0  # Zipf(1.1) on 8..128 -> ~25.9 B


def test_splitmix_matches_oracle(ora):
    import numpy as np
    from velarixdb_amd.workloads import splitmix64
    xs = np.array([0, 1, 2**63, 0x5EED0001, 2**64 - 1], dtype=np.uint64)
    assert [int(v) for v in splitmix64(xs)] == [ora.lib.ora_splitmix64(int(x)) for x in xs]


def test_product_never_imports_oracle():
    """The oracle is test infrastructure: the package and csrc must not reference it."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "velarixdb_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in txt and "liboracle" not in txt, f
                assert "from oracle" not in txt, f


def test_filter_file_extension_roundtrip():
    """filter.db with persisted bits (the layout spec, tests/filter_file_spec.py): the first 16
    bytes stay the reference's format."""
    import numpy as np
    from tests import filter_file_spec as ff
    w = np.arange(1, 1074, dtype=np.uint32) * np.uint32(2654435761)
    raw = ff.encode(19, 1791, 1e-4, 34333, w, entries=2844)
    assert raw[:16] == struct.pack("<IId", 19, 1791, 1e-4)
    k, n, p, m, words, ent = ff.decode(raw)
    assert (k, n, p, m, ent) == (19, 1791, 1e-4, 34333, 2844) and np.array_equal(words, w)
    with pytest.raises(ValueError):  # only the SST's writer knows the entry count
        ff.encode(19, 1791, 1e-4, 34333, w)
    # corrupted body -> ignored (caller rebuilds, as the reference does)
    bad = bytearray(raw)
    bad[-1] ^= 0xFF
    assert ff.decode(bytes(bad))[3:] == (None, None, None)
    # a version-1 extension (no entry count) is ignored too
    v1 = bytearray(raw)
    v1[20:24] = struct.pack("<I", 1)
    assert ff.decode(bytes(v1))[3:] == (None, None, None)
    # the reference's own 16-byte files decode without words
    ref = open(os.path.join(ROOT, "tests/golden/sst_fixtures/sstable_1720785462309/filter.db"), "rb").read()
    assert ff.decode(ref) == (19, 1791, 1e-4, None, None, None)
    with pytest.raises(EOFError):
        ff.decode(ref[:12])


def _recover_raw(raw, offset=0):
    """vbf_filter_recover_ext on host residency from `raw` placed at `offset` in a buffer."""
    import ctypes
    import numpy as np
    from velarixdb_amd import BloomFilter
    from velarixdb_amd._lib import VBF_DEVICE_HOST, call
    buf = np.zeros(len(raw) + offset, dtype=np.uint8)
    buf[offset:] = np.frombuffer(raw, dtype=np.uint8)
    h, restored = ctypes.c_void_p(), ctypes.c_int(-1)
    call("vbf_filter_recover_ext", buf.ctypes.data + offset, len(raw), VBF_DEVICE_HOST, ctypes.byref(h),
         ctypes.byref(restored))
    return BloomFilter(_handle=h), bool(restored.value)


def test_serialize_ext_compaction_filter(ora):
    """SURVEY 8(f) row 1 through the C ABI, host residency (no GPU): a compaction-built filter
    (sized from its table's entries, sized.rs:192-193) persists its own words; recovery restores
    them with no_of_elements = n + entries, as recover_meta + rebuild leave it (range.rs:117-128),
    and the bytes equal the layout spec's."""
    import numpy as np
    from tests import filter_file_spec as ff
    from velarixdb_amd import BloomFilter
    from velarixdb_amd.keys import pack
    keys = [b"k%06d" % i for i in range(17064)]
    bf = BloomFilter(0.01, len(keys), device="host")
    bf.build_filter_from_entries(keys)
    raw = bf.serialize_ext(sst_entries=len(keys))
    w = bf.words()
    assert raw == ff.encode(9, 17064, 0.01, 163559, w, entries=17064)
    assert raw[:16] == bf.serialize() == struct.pack("<IId", 9, 17064, 0.01)
    assert np.array_equal(w, ora.build_words(pack(keys), 163559, 9))
    assert bf.serialize_ext() == raw[:16]  # no entry count: the reference's file only
    for off in (0, 1, 3):  # unaligned bodies
        r, restored = _recover_raw(raw, off)
        assert restored and np.array_equal(r.words(), w)
        assert r.no_of_elements == 2 * 17064 and r.num_bits() == 163559 and r.no_of_hash_func == 9
    # the reference's rebuild gives the same bits and serialize() bytes
    rb, restored = _recover_raw(raw[:16])
    assert not restored and rb.no_of_elements == 17064 and not rb.words().any()
    rb.build_filter_from_entries(keys)
    assert np.array_equal(rb.words(), w) and rb.serialize() == r.serialize()
    # a damaged or foreign extension is ignored: the caller rebuilds
    for i in (16, 20, 24, 28, 40, len(raw) - 1):
        bad = bytearray(raw)
        bad[i] ^= 0x5A
        r2, restored = _recover_raw(bytes(bad))
        assert not restored and r2.no_of_elements == 17064 and not r2.words().any(), i
    r3, restored = _recover_raw(raw[:-4])
    assert not restored


def test_serialize_ext_memtable_filter(ora, tmp_path):
    """A memtable-born filter (sized from the write buffer, mem.rs:188-191: 512 entries, m = 9815)
    holding 300 keys recovers with m' = num_bits(300, p) (bf.rs:144-147): its own words cannot be
    reused, so the writer passes the SST's keys and the recovery-shaped words are built from them
    -- equal to the reference's rebuild.  Without keys only the 16 bytes are written."""
    import numpy as np
    from velarixdb_amd import BloomFilter, num_bits
    from velarixdb_amd.keys import pack
    keys = [b"mem%05d" % i for i in range(300)]
    mem = BloomFilter(1e-4, 512, device="host")
    mem.set_many(keys)
    assert mem.num_bits() == 9815 and num_bits(300, 1e-4) != 9815
    assert mem.serialize_ext(sst_entries=300) == mem.serialize()  # no keys: nothing to persist
    raw = mem.serialize_ext(sst_entries=300, sst_keys=keys)
    m2 = num_bits(300, 1e-4)
    r, restored = _recover_raw(raw)
    assert restored and r.num_bits() == m2 and r.no_of_elements == 600
    assert np.array_equal(r.words(), ora.build_words(pack(keys), m2, 19))
    # through write / recover_from_sst-style recover_meta
    mem.write(tmp_path, sst_entries=300, sst_keys=keys)
    f = BloomFilter.default(device="host")
    f.file_path = str(tmp_path / "filter.db")
    assert f.recover_meta() is True and np.array_equal(f.words(), r.words())
    g = BloomFilter.default(device="host")
    g.file_path = f.file_path
    assert g.recover_meta(load_bits=False) is False
    g.build_filter_from_entries(keys)
    assert np.array_equal(g.words(), r.words()) and g.serialize() == f.serialize()
    with pytest.raises(ValueError):
        mem.serialize_ext(sst_entries=299, sst_keys=keys)


def test_serialize_ext_size_query_and_errors():
    import ctypes
    from velarixdb_amd import BloomFilter
    from velarixdb_amd._lib import VBF_EINVAL, lib
    bf = BloomFilter(0.01, 1000, device="host")
    bf.set_many([b"a%d" % i for i in range(1000)])  # stored n = 1000: the recovery m is this m
    n = ctypes.c_uint64()
    assert lib.vbf_filter_serialize_ext(bf._h, None, None, 0, 1000, 1, None, 0, ctypes.byref(n)) == 0
    assert n.value == 16 + 32 + 4 * ((bf.num_bits() + 31) // 32)
    buf = (ctypes.c_uint8 * 8)()
    assert lib.vbf_filter_serialize_ext(bf._h, None, None, 0, 1000, 1, buf, 8, ctypes.byref(n)) == VBF_EINVAL
    # the reference's fixtures (16 bytes) recover unchanged
    raw = open(os.path.join(ROOT, "tests/golden/sst_fixtures/sstable_1720785462309/filter.db"), "rb").read()
    r, restored = _recover_raw(raw)
    assert not restored and (r.no_of_hash_func, r.no_of_elements, r.num_bits()) == (19, 1791, 34333)


def test_shard_build_argument_checks():
    """vbf_build_shards_host validates before touching a device (no kernel launched)."""
    from velarixdb_amd._lib import VBF_EINVAL, VBF_OK, lib
    from velarixdb_amd.compaction import _Shard
    assert lib.vbf_build_shards_host(None, 0, None, 0) == VBF_OK
    shards = (_Shard * 1)()
    assert lib.vbf_build_shards_host(ctypes.cast(shards, ctypes.c_void_p), 1, None, 0) == VBF_EINVAL
    assert b"no devices" in lib.vbf_last_error()
    assert lib.vbf_build_shards_host(None, 3, None, 1) == VBF_EINVAL
