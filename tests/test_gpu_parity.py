"""Parity of the gfx950 path (through the C ABI) with the oracle and the golden vectors.

Bar: bit-exact words, hashes and probe answers.  Small cases compare whole outputs with the
oracle; the headline sizes (tests/test_gpu_scale.py) add size-independent properties.
"""
import ctypes
import hashlib
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from tests_util import parse_data_db, parse_filter_db

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _dev(arr):
    t = torch.from_numpy(np.ascontiguousarray(arr)).to(DEV)
    return t


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def dev_batch(b):
    """HostBatch -> (keys_t, offs_t) on the GPU."""
    keys = _dev(b.data if b.data.size else np.zeros(1, np.uint8))
    offs = _dev(b.offsets.view(np.int64)) if b.offsets is not None else None
    return keys, offs


def gpu_hashes(vbf, b, k):
    keys, offs = dev_batch(b)
    out = torch.zeros(max(b.n * k, 1), dtype=torch.int64, device=DEV)
    vbf._lib.call("vbf_hashes_dev", _ptr(keys), _ptr(offs), b.stride, b.n, b.len_prefix, k,
                  _ptr(out), _stream())
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint64)[: b.n * k].reshape(b.n, k)


ATOMIC, PARTITIONED = 1, 2


def gpu_build(vbf, b, m, k, words=None, strategy=0):
    keys, offs = dev_batch(b)
    nw = (m + 31) // 32
    w = _dev(words.view(np.int32)) if words is not None else torch.zeros(max(nw, 1), dtype=torch.int32, device=DEV)
    vbf._lib.call("vbf_build_dev_ex", _ptr(keys), _ptr(offs), b.stride, b.n, b.len_prefix, m, k,
                  _ptr(w), strategy, _stream())
    torch.cuda.synchronize()
    return w.cpu().numpy().view(np.uint32)[:nw]


def gpu_probe(vbf, b, m, k, words):
    keys, offs = dev_batch(b)
    w = _dev(words.view(np.int32) if words.size else np.zeros(1, np.int32))
    out = torch.zeros(max(b.n, 1), dtype=torch.uint8, device=DEV)
    vbf._lib.call("vbf_probe_dev", _ptr(keys), _ptr(offs), b.stride, b.n, b.len_prefix, m, k,
                  _ptr(w), _ptr(out), _stream())
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    vbf._lib.call("vbf_probe_count_dev", _ptr(keys), _ptr(offs), b.stride, b.n, b.len_prefix, m, k,
                  _ptr(w), _ptr(cnt), _stream())
    torch.cuda.synchronize()
    res = out.cpu().numpy()[: b.n]
    assert int(cnt.item()) == int(res.sum())
    return res


# ----------------------------------------------------------------------------------------
def test_hashes_match_golden(vbf, golden):
    """calculate_hash (bf.rs:222-227) on the device == Perl-header SipHash vectors."""
    from velarixdb_amd.keys import HostBatch
    for v in golden("hashes"):
        key = bytes.fromhex(v["key"])
        arr = np.frombuffer(key, np.uint8).copy() if key else np.zeros(0, np.uint8)
        b = HostBatch(arr, np.array([0, len(key)], np.uint64), 0, 1, v["len_prefix"])
        h = gpu_hashes(vbf, b, len(v["h"]))
        assert ["%016x" % x for x in h[0]] == v["h"], len(key)


@pytest.mark.parametrize("L", [1, 5, 7, 8, 9, 15, 16, 17, 24, 31, 32, 33, 40, 64, 100])
@pytest.mark.parametrize("lp", [1, 0])
def test_hashes_fixed_stride_match_oracle(vbf, ora, L, lp):
    from velarixdb_amd.keys import HostBatch
    n, k = 3000, 7
    data = ora.gen_fixed(0xABC + L, 0, n, L)
    b = HostBatch(data, None, L, n, lp)
    assert np.array_equal(gpu_hashes(vbf, b, k), ora.hashes(b, k))


def test_hashes_variable_length_unaligned(vbf, ora):
    """Offsets path with every start alignment, empty keys and a 65536-byte key (consts:7)."""
    from velarixdb_amd.keys import pack
    rng = np.random.default_rng(7)
    keys = [bytes(rng.integers(0, 256, int(L), dtype=np.uint8)) for L in rng.integers(0, 70, 2000)]
    keys += [b"", b"", bytes(range(256)) * 256]  # 65536 B
    b = pack(keys)
    assert np.array_equal(gpu_hashes(vbf, b, 5), ora.hashes(b, 5))
    # shift the whole buffer by 1..7 bytes: same keys, every alignment
    for shift in range(1, 8):
        from velarixdb_amd.keys import HostBatch
        data = np.concatenate([np.zeros(shift, np.uint8), b.data])
        sb = HostBatch(data, b.offsets + np.uint64(shift), 0, b.n, 1)
        assert np.array_equal(gpu_hashes(vbf, sb, 3), ora.hashes(b, 3))


@pytest.mark.parametrize("strategy", [ATOMIC, PARTITIONED])
@pytest.mark.parametrize("L,lp,m,k", [(16, 1, 10_000_000, 10), (16, 1, 1, 3), (8, 0, 191701, 19),
                                      (32, 1, 4_000_003, 4), (24, 1, 777_777, 7), (12, 1, 50_000, 5),
                                      (16, 0, 65536, 32), (100, 1, 1_000_003, 2),
                                      (16, 1, 3_000_000_017, 1), (16, 1, 4294967295, 4),
                                      # m = 2^32 - 1 (saturated sizing): the SAT kernels' remainders
                                      (16, 1, 4294967295, 10), (32, 1, 4294967295, 19),
                                      (24, 1, 4294967295, 9), (8, 1, 4294967295, 4), (16, 0, 4294967295, 10),
                                      (16, 1, 4294967295, 14), (32, 1, 4294967295, 7), (16, 1, 4294967295, 29),
                                      # k = 19 (p = 1e-4): two lanes per key for fixed layouts
                                      (16, 1, 3_800_017, 19), (32, 0, 500_009, 19), (24, 1, 2_000_003, 19),
                                      (16, 1, 2_999_999_999, 19),
                                      # either side of m = 2^31, where the build switches remainder code
                                      (16, 1, 2147483648, 10), (16, 1, 2147483649, 10), (16, 1, 2147483647, 4)])
def test_build_fixed_matches_oracle(vbf, ora, L, lp, m, k, strategy):
    from velarixdb_amd.keys import HostBatch
    n = 200_000 if L <= 32 else 20_000
    data = ora.gen_fixed(0x5EED0001, 0, n, L)
    b = HostBatch(data, None, L, n, lp)
    if m > 100_000_000:  # sparse check for the huge arrays: compare set bits only
        got = gpu_build(vbf, b, m, k, strategy=strategy)
        hs = (ora.hashes(b, k) % np.uint64(m)).ravel()
        want_idx = np.unique(hs)
        nz = np.flatnonzero(got)
        bits = np.unpackbits(got[nz].view(np.uint8), bitorder="little").reshape(-1, 32)
        got_idx = np.sort((nz[:, None].astype(np.uint64) * np.uint64(32) + np.arange(32, dtype=np.uint64))[bits.astype(bool)])
        assert np.array_equal(got_idx, want_idx)
        return
    want = ora.build_words(b, m, k)
    got = gpu_build(vbf, b, m, k, strategy=strategy)
    assert np.array_equal(got, want)
    # probe: every key present, plus disjoint negatives (j >= n) agree with the oracle
    assert gpu_probe(vbf, b, m, k, got).all()
    neg = HostBatch(ora.gen_fixed(0x5EED0002, n, 50_000, L), None, L, 50_000, lp)
    assert np.array_equal(gpu_probe(vbf, neg, m, k, got), ora.probe(neg, m, k, want))


# every runtime-k class of k_tile_pack (vbf_tile_pack_rk.hpp: 5, 8, 12, 16, 21, 24, 32) at its
# smallest and largest k, on each key layout and on both sides of m = 2^31 (the class kernels'
# general remainder and 8-counter scan); cfg/config.rs:102-106 lets users pick any p
RK_CASES = [(16, 1, 2_000_003, k) for k in (1, 2, 3, 5, 6, 7, 8, 11, 12, 13, 14, 16, 17, 18, 20, 21, 22, 23, 24, 25, 32)]
RK_CASES += [(32, 1, 3_000_017, 14), (8, 1, 1_500_007, 6), (24, 1, 2_500_009, 23), (13, 1, 2_000_003, 17),
             (None, 1, 2_000_003, 14), (None, 1, 2_000_003, 7), (None, 1, 4_000_037, 23), (None, 1, 2_000_003, 32),
             (16, 0, 2_000_003, 14),  # no length prefix: the generic scratch-stash kernel
             (16, 1, 2_300_000_023, 23), (16, 1, 3_999_999_979, 32), (32, 1, 2_200_000_009, 14),
             (None, 1, 2_500_000_001, 23), (None, 1, 4_294_967_295, 6)]


@pytest.mark.parametrize("L,lp,m,k", RK_CASES)
def test_build_runtime_k_classes_match_oracle(vbf, ora, L, lp, m, k):
    from velarixdb_amd.keys import HostBatch, pack_offsets
    from velarixdb_amd.workloads import SEED_CFG3, var_offsets
    n = 60_000
    if L is None:
        off = var_offsets(SEED_CFG3, 0, n)
        b = pack_offsets(ora.gen_var(SEED_CFG3, 0, off), off, lp)
    else:
        b = HostBatch(ora.gen_fixed(0x5EED0101, 0, n, L), None, L, n, lp)
    got = gpu_build(vbf, b, m, k, strategy=PARTITIONED)
    if m > 100_000_000:  # compare the set bits
        want_idx = np.unique((ora.hashes(b, k) % np.uint64(m)).ravel())
        nz = np.flatnonzero(got)
        bits = np.unpackbits(got[nz].view(np.uint8), bitorder="little").reshape(-1, 32)
        got_idx = np.sort((nz[:, None].astype(np.uint64) * np.uint64(32) + np.arange(32, dtype=np.uint64))[bits.astype(bool)])
        assert np.array_equal(got_idx, want_idx)
        return
    assert np.array_equal(got, ora.build_words(b, m, k))


def test_config1_bit_exact(vbf, ora):
    """BASELINE config 1: 1M x 16 B, 10 bits/key -> m = 10,000,000, k = 10."""
    from velarixdb_amd import num_bits, num_hash_functions
    from velarixdb_amd.keys import HostBatch
    from velarixdb_amd.workloads import SEED_CFG2, fpr_for_bits_per_key
    n = 1_000_000
    m = num_bits(n, fpr_for_bits_per_key(10))
    k = num_hash_functions(m, n)
    assert (m, k) == (10_000_000, 10)
    b = HostBatch(ora.gen_fixed(SEED_CFG2, 0, n, 16), None, 16, n, 1)
    want = ora.build_words(b, m, k, threads=8)
    assert np.array_equal(gpu_build(vbf, b, m, k), want)


@pytest.mark.parametrize("strategy", [ATOMIC, PARTITIONED])
@pytest.mark.parametrize("k", [10, 7, 19])  # compile-time K (10, 19) and the runtime-k kernel (7)
def test_build_variable_length_matches_oracle(vbf, ora, strategy, k):
    from velarixdb_amd.keys import pack_offsets
    from velarixdb_amd.workloads import SEED_CFG3, SEED_CFG3_NEG, var_offsets
    n, m = 100_000, 1_000_003
    off = var_offsets(SEED_CFG3, 0, n)
    data = ora.gen_var(SEED_CFG3, 0, off)
    b = pack_offsets(data, off)
    want = ora.build_words(b, m, k)
    got = gpu_build(vbf, b, m, k, strategy=strategy)
    assert np.array_equal(got, want)
    noff = var_offsets(SEED_CFG3_NEG, 0, 30_000)
    nb = pack_offsets(ora.gen_var(SEED_CFG3_NEG, 0, noff), noff)
    assert np.array_equal(gpu_probe(vbf, nb, m, k, got), ora.probe(nb, m, k, want))


def test_device_generators_match_oracle(vbf, ora):
    from velarixdb_amd.workloads import SEED_CFG3, var_offsets
    for L in (16, 32, 13):
        out = torch.zeros(1000 * L, dtype=torch.uint8, device=DEV)
        vbf._lib.call("vbf_gen_fixed_dev", 0x5EED0001, 77, 1000, L, _ptr(out), _stream())
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ora.gen_fixed(0x5EED0001, 77, 1000, L))
    off = var_offsets(SEED_CFG3, 500, 3000)
    out = torch.zeros(int(off[-1]), dtype=torch.uint8, device=DEV)
    vbf._lib.call("vbf_gen_var_dev", SEED_CFG3, 500, 3000, _ptr(_dev(off.view(np.int64))), _ptr(out), _stream())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ora.gen_var(SEED_CFG3, 500, off))


def test_sst_fixture_rebuild_on_gpu(vbf, golden):
    """range.rs:117-128 on the fixtures through the BloomFilter mirror (recover_meta + build)."""
    want = {s["name"]: s for s in golden("sst_fixtures")["ssts"]}
    root = os.path.join(GOLDEN, "sst_fixtures")
    for name in sorted(os.listdir(root)):
        bf = vbf.BloomFilter.default()
        bf.file_path = os.path.join(root, name, "filter.db")
        bf.recover_meta()
        keys = parse_data_db(os.path.join(root, name, "data.db"))
        k, n, p = parse_filter_db(bf.file_path)
        assert (bf.no_of_hash_func, bf.no_of_elements, bf.false_positive_rate) == (k, n, p)
        assert bf.num_bits() == want[name]["m"]
        bf.build_filter_from_entries(keys)
        assert bf.no_of_elements == n + len(keys)
        w = bf.words()
        assert hashlib.sha256(w.astype("<u4").tobytes()).hexdigest() == want[name]["sha256"]
        assert bf.contains_many(keys).all()
        assert int(bf.contains_many([b"zz%05d" % i for i in range(5000)]).sum()) == want[name]["neg_hits_zz5000"]
        assert bf.contains(keys[0]) and bf.contains(b"head")


def test_bf_rs_unit_tests_on_gpu(vbf, golden):
    """bf.rs:275-424 restated against the device filter."""
    from velarixdb_amd import BloomFilter, I32Vec
    # test_set_and_contain (:275-291)
    bf = BloomFilter(0.01, 10)
    assert bf.num_elements() == 0 and bf.no_of_hash_func == 9 and bf.num_bits() == 95
    bf.set(I32Vec((1, 2, 3, 4)))
    assert bf.num_elements() == 1 and bf.contains(I32Vec((1, 2, 3, 4)))
    # test_number_of_elements (:294-304)
    bf = BloomFilter(0.01, 10)
    for i in range(10):
        bf.set(i)
    assert bf.num_elements() == 10
    # FPR tests (:307-424)
    for v in golden("fpr_tests"):
        p = float.fromhex(v["p"])
        bf = BloomFilter(p, 10000)
        bf.set_many(range(10000))
        w = bf.words()
        assert hashlib.sha256(w.astype("<u4").tobytes()).hexdigest() == v["sha256"]
        fp = int(bf.contains_many(range(10000, 12000)).sum())
        assert fp == v["false_positives"] and fp / 2000 <= p * 1.1


def test_random_sets_on_gpu(vbf, golden):
    from velarixdb_amd.keys import pack
    for s in golden("random_sets"):
        keys = [bytes.fromhex(x) for x in s["keys"]]
        b = pack(keys)
        if "words" in s:
            got = gpu_build(vbf, b, s["m"], s["k"])
            assert ["%08x" % x for x in got] == s["words"]
            if "neg_keys" in s:
                nb = pack([bytes.fromhex(x) for x in s["neg_keys"]])
                assert gpu_probe(vbf, nb, s["m"], s["k"], got).tolist() == s["neg_hits"]
        else:
            h = gpu_hashes(vbf, b, s["k"])
            assert (h % np.uint64(s["m"])).tolist() == s["indices"]


def test_saturated_m_config5_shape(vbf, ora):
    """m = u32::MAX (config 5 sizing): indices up to 2^32-2, 512 MiB words."""
    from velarixdb_amd.keys import HostBatch
    m, k, n = 4294967295, 4, 100_000
    b = HostBatch(ora.gen_fixed(0x5EED0005, 0, n, 32), None, 32, n, 1)
    got = gpu_build(vbf, b, m, k)
    hs = ora.hashes(b, k) % np.uint64(m)
    want = np.zeros((m + 31) // 32, np.uint32)
    np.bitwise_or.at(want, (hs >> np.uint64(5)).astype(np.int64).ravel(),
                     (np.uint32(1) << (hs & np.uint64(31)).astype(np.uint32)).ravel())
    assert np.array_equal(got, want)


@pytest.mark.parametrize("k", [4, 10, 19, 7])
def test_saturated_m_variable_length(vbf, ora, k):
    """m = 2^32 - 1 with runtime-length keys: the SAT kernels (k = 4, 10, 19: end-around-carry
    remainders, sip13.hpp mod_sat) and a runtime-k class (7) against the oracle's hashes % m."""
    from velarixdb_amd.keys import pack_offsets
    from velarixdb_amd.workloads import SEED_CFG3, var_offsets
    m, n = 4294967295, 60_000
    off = var_offsets(SEED_CFG3, 7, n)
    b = pack_offsets(ora.gen_var(SEED_CFG3, 7, off), off)
    got = gpu_build(vbf, b, m, k, strategy=PARTITIONED)
    want_idx = np.unique((ora.hashes(b, k) % np.uint64(m)).ravel())
    nz = np.flatnonzero(got)
    bits = np.unpackbits(got[nz].view(np.uint8), bitorder="little").reshape(-1, 32)
    got_idx = np.sort((nz[:, None].astype(np.uint64) * np.uint64(32) + np.arange(32, dtype=np.uint64))[bits.astype(bool)])
    assert np.array_equal(got_idx, want_idx)


def test_edge_cases(vbf, ora):
    from velarixdb_amd import BloomFilter
    from velarixdb_amd._lib import VBF_EDIVZERO, lib
    from velarixdb_amd.keys import pack
    # empty batch: no-op
    w = gpu_build(vbf, pack([]), 1000, 5)
    assert not w.any()
    # k == 0 (p > 1): contains is vacuously true (bf.rs:104)
    bf = BloomFilter(2.0, 5)
    assert bf.num_bits() == 0 and bf.no_of_hash_func == 0
    bf.set(b"a")
    assert bf.contains(b"zzz")
    # m == 0 with k > 0: the reference panics -> ZeroDivisionError / VBF_EDIVZERO
    rc = lib.vbf_build_dev(None, None, 1, 1, 1, 0, 3, None, None)
    assert rc == VBF_EDIVZERO
    # duplicates are idempotent, OR accumulates into existing bits
    b1 = pack([b"x", b"y"])
    b2 = pack([b"x", b"x", b"y", b"y"])
    assert np.array_equal(gpu_build(vbf, b1, 999, 4), gpu_build(vbf, b2, 999, 4))
    base = np.zeros(32, np.uint32)
    base[3] = 0xF0F0F0F0
    got = gpu_build(vbf, b1, 1024, 4, words=base.copy())
    assert np.array_equal(got, ora.build_words(b1, 1024, 4, words=base.copy()))


def test_filter_handle_semantics(vbf, tmp_path):
    from velarixdb_amd import BloomFilter
    bf = BloomFilter(1e-4, 512)  # memtable sizing, mem.rs:188-191
    assert (bf.num_bits(), bf.no_of_hash_func) == (9815, 19)
    keys = [b"key%04d" % i for i in range(300)]
    bf.set_many(keys)
    c = bf.clone()  # shares bits (bf.rs:249)
    c.set(b"extra")
    assert bf.contains(b"extra")
    assert bf.no_of_elements == 300 and c.no_of_elements == 301
    # write / recover_meta (bf.rs:114-150): m recomputed from stored n
    bf.write(tmp_path)
    assert open(tmp_path / "filter.db", "rb").read()[:16] == bf.serialize()  # reference bytes
    r = BloomFilter.default()
    r.file_path = str(tmp_path / "filter.db")
    r.recover_meta()
    assert r.no_of_hash_func == 19 and r.no_of_elements == 300
    assert r.num_bits() == vbf.num_bits(300, 1e-4) and not r.words().any()
    # clear (bf.rs:180-195): zeroes the shared array, fresh filter has same m, k, p
    fresh = bf.clear()
    assert not bf.words().any() and not c.words().any()
    assert (fresh.num_bits(), fresh.no_of_hash_func, fresh.no_of_elements) == (9815, 19, 0)
    # persistence of words round-trips
    fresh.set_many(keys)
    w = fresh.words()
    other = BloomFilter(1e-4, 512)
    other.load_words(w)
    assert other.contains_many(keys).all()
    # recover without a path
    with pytest.raises(FileNotFoundError):
        BloomFilter.default().recover_meta()


def test_host_pointer_api_matches_device_api(vbf, ora):
    """vbf_build_host / vbf_probe_host: chunked pinned-staging path == oracle (multi-chunk)."""
    from velarixdb_amd._lib import call
    from velarixdb_amd.workloads import SEED_CFG3, var_offsets
    n, m, k = 3_000_000, 30_000_001, 7  # 48 MB of keys -> fixed path uses one chunk per 64 MB
    data = ora.gen_fixed(0x77, 0, n, 16)
    words = np.zeros((m + 31) // 32, np.uint32)
    words[::97] = 0x1  # OR semantics with pre-set bits
    want = words.copy()
    call("vbf_build_host", data.ctypes.data, None, 16, n, 1, m, k, words.ctypes.data, words.size, 0)
    from velarixdb_amd.keys import HostBatch
    ora.build_words(HostBatch(data, None, 16, n, 1), m, k, words=want, threads=8)
    assert np.array_equal(words, want)
    out = np.zeros(n, np.uint8)
    call("vbf_probe_host", data.ctypes.data, None, 16, n, 1, m, k, words.ctypes.data, words.size,
         out.ctypes.data, 0)
    assert out.all()
    # variable length, > 64 MB of key bytes -> several chunks with rebased offsets
    nv = 3_000_000
    off = var_offsets(SEED_CFG3, 0, nv)
    vdata = ora.gen_var(SEED_CFG3, 0, off)
    assert off[-1] > 64 << 20
    w2 = np.zeros((m + 31) // 32, np.uint32)
    call("vbf_build_host", vdata.ctypes.data, off.ctypes.data, 0, nv, 1, m, k, w2.ctypes.data, w2.size, 0)
    from velarixdb_amd.keys import pack_offsets
    assert np.array_equal(w2, ora.build_words(pack_offsets(vdata, off), m, k, threads=8))


def test_filter_db_persisted_bits(vbf, tmp_path):
    """compaction-built filters (m from their own n) recover without a
    rebuild and equal the rebuild; memtable-born ones (m from capacity) still need it."""
    from velarixdb_amd import BloomFilter
    keys = [b"k%06d" % i for i in range(17064)]
    bf = BloomFilter(0.01, len(keys))  # compactors/sized.rs:192 sizing
    bf.build_filter_from_entries(keys)
    bf.write(tmp_path, sst_entries=len(keys))
    r = BloomFilter.default()
    r.file_path = bf.file_path
    assert r.recover_meta() is True
    rebuilt = BloomFilter.default()
    rebuilt.file_path = bf.file_path
    assert rebuilt.recover_meta(load_bits=False) is False
    rebuilt.build_filter_from_entries(keys)  # what range.rs:117-128 does
    assert np.array_equal(r.words(), rebuilt.words())
    # memtable-born: sized for 512 entries, holds 300 -> stored n = 300, m' != m: its own words
    # cannot be restored; with the SST's keys the writer persists the recovery-shaped words
    mem = BloomFilter(1e-4, 512)
    mem.set_many(keys[:300])
    d2 = tmp_path / "mem"
    d2.mkdir()
    mem.write(d2, sst_entries=300)
    r2 = BloomFilter.default()
    r2.file_path = mem.file_path
    assert r2.recover_meta() is False and not r2.words().any()
    mem.write(d2, sst_entries=300, sst_keys=keys[:300])
    r3 = BloomFilter.default()
    r3.file_path = mem.file_path
    assert r3.recover_meta() is True and r3.no_of_elements == 600
    r2.build_filter_from_entries(keys[:300])  # what range.rs:117-128 does
    assert np.array_equal(r3.words(), r2.words()) and r3.serialize() == r2.serialize()


def test_product_library_ignores_ablation_env(vbf, tmp_path):
    """VBF_ABLATE (timing experiments that skip phases) only acts in the separate ablation build
    (vbf_kernels.hpp); the product libvbf.so must build correct filters with it set."""
    import subprocess
    import sys
    from conftest import ROOT
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import numpy as np, oracle, velarixdb_amd as v\n"
        "from velarixdb_amd.keys import pack_fixed\n"
        "b = pack_fixed(np.random.default_rng(3).integers(0, 256, (300000, 16), dtype=np.uint8))\n"
        "m, k = 3_000_000, 10\n"
        "w = np.zeros((m + 31) // 32, np.uint32)\n"
        "v._lib.call('vbf_build_host', b.data.ctypes.data, None, 16, b.n, 1, m, k, w.ctypes.data, w.size, 0)\n"
        "assert np.array_equal(w, oracle.build_words(b, m, k)), 'ablation env changed the product build'\n"
        "print('ok')\n" % ROOT)
    env = {kk: vv for kk, vv in os.environ.items() if kk != "VBF_LIB"}
    for a in ("1", "4", "7"):
        env["VBF_ABLATE"] = a
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and "ok" in r.stdout, (a, r.stderr[-2000:])


def test_variable_length_knobs_same_words(vbf, ora, tmp_path):
    """The speed-only knobs of the variable-length partitioned build (VBF_LEN_ORDER: lanes in
    length order or key order; VBF_STAGE_KEYS: (begin, length) staged in LDS or read from the
    offsets) must give the oracle's words in every combination.  The library reads them once per
    process, so each combination builds in a child process (vbf_build_host, AUTO: partitioned at
    these sizes, >= 2^22 bit indices) and the parent checks the words against the oracle."""
    import subprocess
    import sys
    from conftest import ROOT
    from velarixdb_amd.keys import pack_offsets
    from velarixdb_amd.workloads import SEED_CFG3, var_offsets
    cases = ((2_000_003, 10), (3_800_000, 19), (900_001, 4))
    n = 1_100_000
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import numpy as np, oracle as ora, velarixdb_amd as v\n"
        "from velarixdb_amd.keys import pack_offsets\n"
        "from velarixdb_amd.workloads import SEED_CFG3, var_offsets\n"
        "off = var_offsets(SEED_CFG3, 7, %d)\n"
        "b = pack_offsets(ora.gen_var(SEED_CFG3, 7, off), off)\n"
        "for m, k in %r:\n"
        "    w = np.zeros((m + 31) // 32, np.uint32)\n"
        "    v._lib.call('vbf_build_host', b.data.ctypes.data, b.offsets.ctypes.data, 0, b.n, 1, m, k,\n"
        "                w.ctypes.data, w.size, 0)\n"
        "    np.save(sys.argv[1] + '_%%d.npy' %% k, w)\n"
        "print('ok')\n" % (ROOT, n, cases))
    off = var_offsets(SEED_CFG3, 7, n)
    b = pack_offsets(ora.gen_var(SEED_CFG3, 7, off), off)
    want = {k: ora.build_words(b, m, k, threads=8) for m, k in cases}
    for lo, st in (("0", "0"), ("1", "0"), ("0", "1"), ("1", "1")):
        env = {kk: vv for kk, vv in os.environ.items() if kk != "VBF_LIB"}
        env["VBF_LEN_ORDER"], env["VBF_STAGE_KEYS"] = lo, st
        stem = str(tmp_path / ("w%s%s" % (lo, st)))
        r = subprocess.run([sys.executable, "-c", code, stem], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0 and "ok" in r.stdout, (lo, st, r.stderr[-2000:])
        for m, k in cases:
            assert np.array_equal(np.load(stem + "_%d.npy" % k), want[k]), (lo, st, m, k)


def test_partitioned_build_knobs_same_words(vbf, ora, tmp_path):
    """The speed-only knobs of the fixed-length partitioned build -- VBF_K1 (the 1024-thread K1 with
    two lanes per key at k = 19, or the 512-thread one-lane-per-key shape), VBF_ENDS_T (K1 writes
    the run ends transposed, or the transpose kernel does), VBF_K3 (k_seg_or's tile loops: two-stage,
    three-stage with 8-lane groups and its >8-group tail, flattened groups found by binary search or,
    the default since round 6, by run marks) -- must give the
    oracle's words in every combination, on random keys and on a batch whose runs are thousands of
    entries long (three keys repeated).  Each combination builds in a child process (the library
    reads the knobs once per process)."""
    import subprocess
    import sys
    from conftest import ROOT
    from velarixdb_amd.keys import pack_fixed
    # m = 2_999_999_999 has > 2048 segments: the 512-thread shape does not apply, V = 0 runs
    cases = ((3_800_017, 19), (10_000_000, 10), (2_999_999_999, 19), (40_000_003, 10))
    rng = np.random.default_rng(77)
    rand = rng.integers(0, 256, (700_000, 16), dtype=np.uint8)
    hot = rng.integers(0, 256, (3, 16), dtype=np.uint8)
    rows = np.concatenate([rand, np.repeat(hot, 150_000, axis=0)])
    np.save(tmp_path / "rows.npy", rows)
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import numpy as np, velarixdb_amd as v\n"
        "from velarixdb_amd.keys import pack_fixed\n"
        "b = pack_fixed(np.load(sys.argv[2]))\n"
        "for m, k in %r:\n"
        "    w = np.zeros((m + 31) // 32, np.uint32)\n"
        "    v._lib.call('vbf_build_host', b.data.ctypes.data, None, 16, b.n, 1, m, k, w.ctypes.data, w.size, 0)\n"
        "    nz = np.flatnonzero(w)\n"
        "    np.save(sys.argv[1] + '_%%d_%%d.npy' %% (m, k), np.stack([nz.astype(np.uint64), w[nz].astype(np.uint64)]))\n"
        "print('ok')\n" % (ROOT, cases))
    b = pack_fixed(rows)
    want = {}
    for m, k in cases:
        if m > 100_000_000:  # compare set-bit positions only (the words array is 375 MB)
            want[(m, k)] = np.unique((ora.hashes(b, k) % np.uint64(m)).ravel())
        else:
            want[(m, k)] = ora.build_words(b, m, k, threads=8)
    # (VBF_K1, VBF_ENDS_T, VBF_K3, VBF_K3_SPLIT): the last one splits k_seg_or's last round of
    # segments over several workgroups (m = 2_999_999_999: 2 862 segments)
    combos = (("0", "0", "0", "1"), ("1", "1", "0", "0"), ("1", "0", "3", "1"), ("0", "1", "1", "1"),
              ("1", "1", "4", "1"), ("-1", "1", "12", "0"), ("0", "0", "10", "1"), ("1", "1", "13", "1"),
              ("1", "1", "16", "0"), ("0", "1", "11", "1"))
    for k1, et, k3, sp in combos:
        env = {kk: vv for kk, vv in os.environ.items() if kk != "VBF_LIB"}
        env["VBF_K1"], env["VBF_ENDS_T"], env["VBF_K3"], env["VBF_K3_SPLIT"] = k1, et, k3, sp
        stem = str(tmp_path / ("w%s%s%s%s" % (k1, et, k3, sp)))
        r = subprocess.run([sys.executable, "-c", code, stem, str(tmp_path / "rows.npy")], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and "ok" in r.stdout, (k1, et, k3, sp, r.stderr[-2000:])
        for m, k in cases:
            nz, val = np.load(stem + "_%d_%d.npy" % (m, k))  # the child's nonzero words
            if m > 100_000_000:
                bits = np.unpackbits(val.astype(np.uint32).view(np.uint8), bitorder="little").reshape(-1, 32)
                idx = np.sort((nz[:, None] * np.uint64(32) + np.arange(32, dtype=np.uint64))[bits.astype(bool)])
                assert np.array_equal(idx, want[(m, k)]), (k1, et, k3, sp, m, k)
            else:
                got = np.zeros((m + 31) // 32, np.uint32)
                got[nz.astype(np.int64)] = val.astype(np.uint32)
                assert np.array_equal(got, want[(m, k)]), (k1, et, k3, sp, m, k)


@pytest.mark.parametrize("layout,m,k", [
    ("usize", 14_377_000, 14),       # p = 1e-3 over usize keys (bf.rs:307-424's encoding): class 16
    ("usize", 4_294_967_295, 6),     # saturated m, class 8 with the end-around-carry remainder
    ("i32", 9_000_011, 7),           # 4-byte rows: the runtime-stride layout, class 8
    ("vec_i32", 23_000_003, 23),     # &Vec<i32>: LE64(len) || LE32 x len, offsets layout, class 24
    ("usize", 3_000_000_017, 31),    # m > 2^31 (Barrett), class 32
])
def test_runtime_k_classes_without_length_prefix(vbf, ora, layout, m, k):
    """Missing r04 #4: batches hashed without the length prefix (len_prefix = 0: the pre-encoded
    integer keys of bf.rs:275-424) at k outside {4, 9, 10, 19} take the runtime-k class kernels
    (vbf_partition_rk_c.hip) instead of the scratch-stash kernel: words equal the oracle's."""
    from velarixdb_amd.keys import HostBatch
    rng = np.random.default_rng(k)
    n = 400_000
    if layout == "usize":
        data = np.arange(n, dtype="<u8").view(np.uint8)
        b = HostBatch(data, None, 8, n, 0)
    elif layout == "i32":
        data = rng.integers(-2**31, 2**31 - 1, n, dtype=np.int64).astype("<i4").view(np.uint8)
        b = HostBatch(data, None, 4, n, 0)
    else:
        lens = rng.integers(0, 9, n)
        parts, off = [], [0]
        for j, c in enumerate(lens):
            msg = np.uint64(c).tobytes() + rng.integers(-2**31, 2**31 - 1, int(c), dtype=np.int64).astype("<i4").tobytes()
            parts.append(msg)
            off.append(off[-1] + len(msg))
        b = HostBatch(np.frombuffer(b"".join(parts), np.uint8).copy(), np.asarray(off, np.uint64), 0, n, 0)
    got = gpu_build(vbf, b, m, k, strategy=PARTITIONED)
    if m > 100_000_000:
        nz = np.flatnonzero(got)
        bits = np.unpackbits(got[nz].view(np.uint8), bitorder="little").reshape(-1, 32).astype(bool)
        idx = np.sort((nz.astype(np.uint64)[:, None] * np.uint64(32) + np.arange(32, dtype=np.uint64))[bits])
        assert np.array_equal(idx, np.unique((ora.hashes(b, k) % np.uint64(m)).ravel()))
    else:
        assert np.array_equal(got, ora.build_words(b, m, k, threads=8))


# (m, k, layout) the kernel-selecting knobs gate: m = 2^32 - 1 (SAT / Barrett, k = 4 / 6 / 10 / 19,
# fixed and runtime-length keys), the runtime-k classes (k = 7, 14, 23), k = 19 and 10 on the 512-
# and 1 024-thread shapes; `probe`: the partitioned probe is also run (round-3 pipeline: VBF_Q3)
KNOB_CASES = (
    (4_294_967_295, 4, "f32", True), (4_294_967_295, 4, "f16", True), (4_294_967_295, 6, "f16", True),
    (4_294_967_295, 10, "f16", False), (4_294_967_295, 19, "f16", True), (4_294_967_295, 4, "var", True),
    (4_294_967_295, 7, "var", False), (20_000_003, 7, "f16", True), (30_000_001, 14, "var", False),
    (40_000_000, 23, "f32", False), (3_800_017, 19, "f16", False), (10_000_000, 10, "var", False),
    (6_000_011, 10, "f16", True), (200_000_003, 19, "f16", True), (300_000_001, 10, "var", True),
    (150_000_007, 10, "f32", False), (100_000_007, 19, "var", False),
)
# every kernel-changing knob of DESIGN.md section 8b that VERDICT r04 found untested (one child each;
# the library reads them once per process)
KNOB_COMBOS = (
    {"VBF_SAT": "0"}, {"VBF_KCLASS": "0"}, {"VBF_K1_4": "1"}, {"VBF_C16": "0"}, {"VBF_C16": "1"},
    {"VBF_C16": "1", "VBF_K1": "0"}, {"VBF_Q3": "0"}, {},
)


def test_kernel_knobs_same_words(vbf, ora, tmp_path):
    """the speed-only knobs that select other kernels -- VBF_SAT=0 (the
    Barrett kernels at m = 2^32 - 1), VBF_KCLASS=0 (the scratch-stash runtime-k kernel), VBF_K1_4=1
    (k = 4 on the 512-thread shape: the case whose packed-counter scan was once wrong),
    VBF_C16=0/1 (plain or packed segment counters, on either K1 shape), VBF_Q3=0 (the partitioned
    probe's one-pass segment test) -- give the oracle's words (bf.rs:84-92) and probe answers
    (bf.rs:95-105) at the shapes they gate.  Round 5: the builds are explicitly partitioned
    (VBF_BUILD_PARTITIONED: at 300K keys AUTO would take the atomic kernel for k <= 13, so the K1
    knobs were not exercised at those shapes before), and four shapes of the 512-thread K1 with
    m well above one segment were added.  Each setting runs in a child process; the parent
    compares every child's words and answers with the oracle's."""
    import subprocess
    import sys
    from conftest import ROOT
    from velarixdb_amd.keys import pack_fixed, pack_offsets
    from velarixdb_amd.workloads import SEED_CFG3, var_offsets
    n = 300_000
    f16 = ora.gen_fixed(0x5EED0A16, 0, n, 16).reshape(n, 16)
    f32 = ora.gen_fixed(0x5EED0A32, 0, n, 32).reshape(n, 32)
    vo = var_offsets(SEED_CFG3, 11, n)
    vd = ora.gen_var(SEED_CFG3, 11, vo)
    # probe batches: the first half of the keys (positives) + as many negatives
    nf16 = ora.gen_fixed(0x5EED0B16, 0, n // 2, 16).reshape(-1, 16)
    nf32 = ora.gen_fixed(0x5EED0B32, 0, n // 2, 32).reshape(-1, 32)
    nvo = var_offsets(SEED_CFG3 ^ 0xFF, 5, n // 2)
    nvd = ora.gen_var(SEED_CFG3 ^ 0xFF, 5, nvo)
    h = int(vo[n // 2])
    pvd = np.concatenate([vd[:h], nvd])
    pvo = np.concatenate([vo[: n // 2 + 1], nvo[1:] + np.uint64(h)])
    arrs = dict(f16=f16, f32=f32, vd=vd, vo=vo, pf16=np.concatenate([f16[: n // 2], nf16]),
                pf32=np.concatenate([f32[: n // 2], nf32]), pvd=pvd, pvo=pvo)
    np.savez(tmp_path / "keys.npz", **arrs)
    batches = {"f16": pack_fixed(f16), "f32": pack_fixed(f32), "var": pack_offsets(vd, vo)}
    pbatches = {"f16": pack_fixed(arrs["pf16"]), "f32": pack_fixed(arrs["pf32"]), "var": pack_offsets(pvd, pvo)}
    code = (
        "import sys, ctypes; sys.path.insert(0, %r)\n"
        "import numpy as np, torch, velarixdb_amd as v\n"
        "from velarixdb_amd.keys import pack_fixed, pack_offsets\n"
        "a = np.load(sys.argv[2])\n"
        "B = {'f16': pack_fixed(a['f16']), 'f32': pack_fixed(a['f32']), 'var': pack_offsets(a['vd'], a['vo'])}\n"
        "P = {'f16': pack_fixed(a['pf16']), 'f32': pack_fixed(a['pf32']), 'var': pack_offsets(a['pvd'], a['pvo'])}\n"
        "vp = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None\n"
        "res = {}\n"
        "for i, (m, k, lay, probe) in enumerate(%r):\n"
        "    b = B[lay]\n"
        "    kd0 = torch.from_numpy(b.data).cuda()\n"
        "    od0 = torch.from_numpy(b.offsets.view(np.int64)).cuda() if b.offsets is not None else None\n"
        "    wd0 = torch.zeros((m + 31) // 32, dtype=torch.int32, device='cuda')\n"
        "    v._lib.call('vbf_build_dev_ex', vp(kd0), vp(od0), b.stride, b.n, 1, m, k, vp(wd0), 2, None)\n"
        "    torch.cuda.synchronize()\n"
        "    w = wd0.cpu().numpy().view(np.uint32)\n"
        "    del kd0, od0, wd0\n"
        "    nz = np.flatnonzero(w)\n"
        "    res['nz%%d' %% i], res['w%%d' %% i] = nz.astype(np.uint64), w[nz]\n"
        "    if probe:\n"
        "        pb = P[lay]\n"
        "        kd = torch.from_numpy(pb.data).cuda()\n"
        "        od = torch.from_numpy(pb.offsets.view(np.int64)).cuda() if pb.offsets is not None else None\n"
        "        wd = torch.from_numpy(w.view(np.int32)).cuda()\n"
        "        out = torch.zeros(pb.n, dtype=torch.uint8, device='cuda')\n"
        "        v._lib.call('vbf_probe_dev_ex', vp(kd), vp(od), pb.stride, pb.n, 1, m, k, vp(wd), vp(out), 2, None)\n"
        "        torch.cuda.synchronize()\n"
        "        res['p%%d' %% i] = out.cpu().numpy()\n"
        "        del kd, od, wd, out\n"
        "np.savez(sys.argv[1], **res)\n"
        "print('ok')\n" % (ROOT, KNOB_CASES))
    outs = []
    for j, knobs in enumerate(KNOB_COMBOS):
        env = {kk: vv for kk, vv in os.environ.items() if kk != "VBF_LIB" and not kk.startswith("VBF_")}
        env.update(knobs)
        stem = str(tmp_path / ("knob%d.npz" % j))
        r = subprocess.run([sys.executable, "-c", code, stem, str(tmp_path / "keys.npz")], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and "ok" in r.stdout, (knobs, r.stderr[-2000:])
        outs.append(stem)
    for i, (m, k, lay, probe) in enumerate(KNOB_CASES):
        want = ora.build_words(batches[lay], m, k, threads=8)
        wp = ora.probe(pbatches[lay], m, k, want, threads=8) if probe else None
        for j, knobs in enumerate(KNOB_COMBOS):
            res = np.load(outs[j])
            nz, val = res["nz%d" % i], res["w%d" % i]
            wnz = np.flatnonzero(want)
            assert np.array_equal(nz, wnz.astype(np.uint64)) and np.array_equal(val, want[wnz]), (knobs, m, k, lay)
            if probe:
                assert np.array_equal(res["p%d" % i], wp), (knobs, m, k, lay)
        if probe:
            assert wp[: n // 2].all()  # no false negative


@pytest.mark.parametrize("strategy", [1, 2])
def test_concentrated_indices(vbf, ora, strategy):
    """Adversarial skew: 3M copies of three keys put every tile's 30K bit indices into a handful of
    segments (runs of thousands, the tail loops of k_seg_or / k_probe_seg), alongside one
    ordinary key.  Words and probe answers (both probe strategies) must still be exact."""
    from velarixdb_amd.keys import pack_fixed
    rng = np.random.default_rng(21)
    base = rng.integers(0, 256, (4, 16), dtype=np.uint8)
    rows = np.repeat(base[:3], 1_000_000, axis=0)
    rows = np.concatenate([rows, base[3:]])
    b = pack_fixed(rows)
    m, k = 1_000_000_000, 10
    got = gpu_build(vbf, b, m, k, strategy=strategy)
    want = ora.build_words(pack_fixed(base), m, k)
    assert np.array_equal(got, want)
    assert int(np.unpackbits(got.view(np.uint8)).sum()) <= 40
    keys, offs = dev_batch(b)
    w = _dev(got.view(np.int32))
    for ps in (1, 2):
        cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
        vbf._lib.call("vbf_probe_count_dev_ex", _ptr(keys), _ptr(offs), b.stride, b.n, b.len_prefix, m, k,
                      _ptr(w), _ptr(cnt), ps, _stream())
        torch.cuda.synchronize()
        assert int(cnt.item()) == b.n, ps
    neg = pack_fixed(rng.integers(0, 256, (200_000, 16), dtype=np.uint8))
    assert not gpu_probe(vbf, neg, m, k, got).any()  # 40 bits of 1e9: no false positive expected


def test_or_words_kernel(vbf):
    """vbf_or_words_dev (the local OR of the multi-GPU filter merge, dist.or_words_dev): equal to
    a bitwise OR for ragged lengths; misaligned pointers are refused."""
    from velarixdb_amd.dist import or_words_dev
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    for n in (1, 3, 4, 1023, 1 << 20, (1 << 20) + 5):
        a = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=DEV, generator=g)
        b = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=DEV, generator=g)
        want = a | b
        or_words_dev(a, b)
        torch.cuda.synchronize()
        assert torch.equal(a, want), n
    a = torch.zeros(9, dtype=torch.int32, device=DEV)
    with pytest.raises(vbf.VbfError):
        vbf._lib.call("vbf_or_words_dev", _ptr(a[1:]), _ptr(a[:8]), 8, _stream())
    with pytest.raises(ValueError):
        or_words_dev(torch.zeros(4, dtype=torch.int32), torch.zeros(4, dtype=torch.int32))


def test_or_fold_kernel(vbf):
    """vbf_or_fold_dev (dist.or_fold_dev: the one-pass fold of the multi-GPU OR all-reduce, VERDICT
    r05 #7): the OR of 1..8 back-to-back parts, into a separate buffer and in place into part 0,
    ragged lengths (the words past a multiple of 4 take the scalar tail); misaligned pointers,
    an unaligned stride and overlapping parts are refused."""
    from velarixdb_amd.dist import or_fold_dev
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    for parts in (1, 2, 3, 8):
        for chunk in (4, 1024, (1 << 18) + 4):
            src = torch.randint(-2**31, 2**31 - 1, (parts * chunk,), dtype=torch.int32, device=DEV, generator=g)
            want = src[:chunk].clone()
            for p in range(1, parts):
                want |= src[p * chunk:(p + 1) * chunk]
            out = torch.full((chunk,), 0x5A5A5A5A, dtype=torch.int32, device=DEV)
            or_fold_dev(out, src, parts, chunk)
            or_fold_dev(src[:chunk], src, parts, chunk)  # in place, as or_allreduce_ runs it
            torch.cuda.synchronize()
            assert torch.equal(out, want) and torch.equal(src[:chunk], want), (parts, chunk)
    # nwords not a multiple of 4 (the tail loop), parts 8 words apart
    src = torch.randint(-2**31, 2**31 - 1, (24,), dtype=torch.int32, device=DEV, generator=g)
    out = torch.zeros(8, dtype=torch.int32, device=DEV)
    vbf._lib.call("vbf_or_fold_dev", _ptr(out), _ptr(src), 7, 3, 8, _stream())
    torch.cuda.synchronize()
    assert torch.equal(out[:7], (src[0:8] | src[8:16] | src[16:24])[:7]) and int(out[7]) == 0
    a = torch.zeros(40, dtype=torch.int32, device=DEV)
    for args in ((_ptr(a[1:]), _ptr(a[8:]), 8, 2, 8), (_ptr(a), _ptr(a[8:]), 8, 2, 10), (_ptr(a), _ptr(a[8:]), 8, 2, 4)):
        with pytest.raises(vbf.VbfError):
            vbf._lib.call("vbf_or_fold_dev", *args, _stream())


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,k,strategy", [
    (200_000, 600_000_000, 10, PARTITIONED),  # one workgroup per segment: the fused path
    (200_000, 600_000_000, 19, PARTITIONED),
    (200_000, 10_000_000, 10, PARTITIONED),   # few segments, several workgroups each: zeroed first
    (50_000, 600_000_000, 10, ATOMIC),        # zeroed first
    (0, 1_000_003, 7, 0),                     # no keys: the new filter is all zeros
])
def test_fresh_build_ignores_prior_words(vbf, ora, n, m, k, strategy):
    """VBF_BUILD_FRESH (BloomFilter::new + build_filter_from_entries, bf.rs:62-81,126-128): into
    words full of garbage, the result is exactly the oracle's filter of the keys alone."""
    from velarixdb_amd._lib import VBF_BUILD_FRESH
    from velarixdb_amd.keys import HostBatch
    L = 16
    data = ora.gen_fixed(0x5EED0001, 0, max(n, 1), L)[: n * L]
    b = HostBatch(data, None, L, n, 1)
    nw = (m + 31) // 32
    garbage = np.random.default_rng(7).integers(0, 2**32, nw, dtype=np.uint64).astype(np.uint32)
    got = gpu_build(vbf, b, m, k, words=garbage, strategy=strategy | VBF_BUILD_FRESH)
    if n == 0:
        assert not got.any()
        return
    hs = (ora.hashes(b, k) % np.uint64(m)).ravel()
    want = np.zeros(nw, np.uint32)
    np.bitwise_or.at(want, (hs >> np.uint64(5)).astype(np.int64), (np.uint32(1) << (hs & np.uint64(31)).astype(np.uint32)))
    assert np.array_equal(got, want)


def test_build_workspace_cap_halves_the_chunk(vbf):
    """a partitioned build whose one-chunk workspace cannot be allocated runs in
    smaller chunks instead of failing with VBF_ENOMEM.  VBF_WS_MAX_BYTES caps the workspace: 60M
    keys x k = 10 (6e8 bit indices, ~1.6 GB of workspace in one chunk) under a 0.9 GB cap run in
    chunks of 2^28 indices -- the same words as the one-chunk build, fresh (into garbage) and ORed
    into earlier words; a cap below the smallest chunk's workspace is VBF_ENOMEM."""
    import os
    n, L, m, k = 60_000_000, 16, 600_000_000, 10
    keys = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    vbf._lib.call("vbf_gen_fixed_dev", 0x5EED0E71, 0, n, L, _ptr(keys), _stream())
    want = torch.zeros((m + 31) // 32, dtype=torch.int32, device=DEV)
    vbf._lib.call("vbf_build_dev_ex", _ptr(keys), None, L, n, 1, m, k, _ptr(want), 2, _stream())
    torch.cuda.synchronize()
    os.environ["VBF_WS_MAX_BYTES"] = str(900_000_000)
    try:
        fresh = torch.full_like(want, -1)
        vbf._lib.call("vbf_build_dev_ex", _ptr(keys), None, L, n, 1, m, k, _ptr(fresh), 2 | 0x100, _stream())
        half = torch.zeros_like(want)
        vbf._lib.call("vbf_build_dev_ex", _ptr(keys), None, L, n // 2, 1, m, k, _ptr(half), 2, _stream())
        vbf._lib.call("vbf_build_dev_ex", _ptr(keys[n // 2 * L:]), None, L, n - n // 2, 1, m, k, _ptr(half), 2,
                      _stream())
        torch.cuda.synchronize()
        assert torch.equal(fresh, want) and torch.equal(half, want)
        os.environ["VBF_WS_MAX_BYTES"] = str(100_000_000)
        with pytest.raises(vbf.VbfError, match="VBF_WS_MAX_BYTES"):
            vbf._lib.call("vbf_build_dev_ex", _ptr(keys), None, L, n, 1, m, k, _ptr(half), 2, _stream())
    finally:
        os.environ.pop("VBF_WS_MAX_BYTES", None)
