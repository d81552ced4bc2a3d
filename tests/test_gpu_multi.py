"""GPU parity for the batched read-path probe across SSTs:
out[j, s] = smallest_s <= key_j <= biggest_s && filter_s.contains(key_j) (range.rs:118,136),
checked against the oracle's probe (bf.rs:95-105) and Python's bytes order (= Rust Ord for
Vec<u8>).  Bit-exact."""
import ctypes
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
SST = os.path.join(GOLDEN, "sst_fixtures")


def _oracle_contains(ora, keys, m, k, words):
    from velarixdb_amd.keys import pack
    return ora.probe(pack(keys), m, k, words).astype(bool)


def test_fixture_ssts_candidates(vbf, ora):
    from velarixdb_amd.key_range import SstRange, candidates, filter_sstables_many
    ranges, all_keys, orc = [], [], []
    for name in sorted(os.listdir(SST)):
        data, index = vbf.sst.read_sst_files(os.path.join(SST, name))
        ent = vbf.sst.load_entries(data, index)
        keys = ent.key_list()
        bf = vbf.BloomFilter.default()
        bf.file_path = os.path.join(SST, name, "filter.db")
        bf.recover_meta(load_bits=False)
        bf.rebuild_from_sst(data, index)
        ranges.append(SstRange(keys[0], keys[-1], bf))
        words = ora.build_words(vbf.pack(keys), bf.num_bits(), bf.no_of_hash_func)
        orc.append((keys[0], keys[-1], bf.num_bits(), bf.no_of_hash_func, words))
        all_keys += keys[::7]
    q = all_keys + [b"", b"0", b"zzzzzz", b"head", b"00", b"\xff" * 9] + \
        [r.smallest_key for r in ranges] + [r.biggest_key for r in ranges] + \
        [r.smallest_key[:-1] for r in ranges] + [r.biggest_key + b"\0" for r in ranges] + \
        [b"k%06d" % i for i in range(3000)]
    got = candidates(q, ranges)
    want = np.zeros_like(got)
    for s, (lo, hi, m, k, words) in enumerate(orc):
        inr = np.array([lo <= x <= hi for x in q])
        want[:, s] = inr & _oracle_contains(ora, q, m, k, words)
    assert np.array_equal(got, want)
    assert got[: len(all_keys)].any(axis=1).all()  # every stored key finds its SST
    lists = filter_sstables_many(q[:50], ranges)
    assert lists == [np.flatnonzero(r).tolist() for r in want[:50]]


@pytest.mark.parametrize("seed", [1, 2])
def test_random_filters_contains_all(vbf, ora, seed):
    from velarixdb_amd.key_range import contains_all
    rng = np.random.default_rng(seed)
    specs = [(0.01, 50), (0.1, 1000), (1e-4, 300), (0.5, 3), (1.0, 5), (0.3, 20000), (1e-7, 64)]
    filters, orc = [], []
    for p, n in specs:
        f = vbf.BloomFilter(p, n)
        ks = [rng.bytes(int(rng.integers(0, 40))) for _ in range(n)]
        f.set_many(ks)
        filters.append(f)
        orc.append((f.num_bits(), f.no_of_hash_func, ora.build_words(vbf.pack(ks), f.num_bits(), f.no_of_hash_func)))
    q = [rng.bytes(int(rng.integers(0, 70))) for _ in range(20000)]
    got = contains_all(q, filters)
    for s, (m, k, words) in enumerate(orc):
        assert np.array_equal(got[:, s], _oracle_contains(ora, q, m, k, words)), s
    assert got[:, 4].all()  # p = 1.0 -> m = 0, k = 0: contains() is vacuously true


def test_device_api_matches_single_probes(vbf):
    """2M device-resident fixed keys x 8 filters: vbf_multi_probe_dev equals 8 single probes."""
    import torch
    from velarixdb_amd._lib import call
    n, L, S = 2_000_000, 16, 8
    dev = torch.device("cuda:0")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    keys = torch.empty(n * L, dtype=torch.uint8, device=dev)
    call("vbf_gen_fixed_dev", 0x5EED0001, 0, n, L, P(keys), None)
    filters = []
    for s in range(S):
        f = vbf.BloomFilter(0.01 * (s + 1) / 4, n // (s + 1))
        f.set_dev(P(keys[s * 1000 * L:]), None, L, n // (s + 1) - s * 1000 if s else n // (s + 1), 1)
        filters.append(f)
    out = torch.empty(n * S, dtype=torch.uint8, device=dev)
    handles = (ctypes.c_void_p * S)(*[f._h.value for f in filters])
    call("vbf_multi_probe_dev", P(keys), None, L, n, 1, S, handles, None, None, P(out), None)
    torch.cuda.synchronize()
    got = out.view(n, S).cpu().numpy()
    for s, f in enumerate(filters):
        one = torch.empty(n, dtype=torch.uint8, device=dev)
        f.contains_dev(P(keys), None, L, n, P(one))
        torch.cuda.synchronize()
        assert np.array_equal(got[:, s], one.cpu().numpy()), s


def test_zero_bits_with_hashes_raises(vbf):
    from velarixdb_amd.key_range import contains_all
    from velarixdb_amd._lib import call
    h = ctypes.c_void_p()
    meta = (ctypes.c_uint8 * 16).from_buffer_copy(struct.pack("<IId", 3, 10, 1.0))  # m = 0, k = 3
    call("vbf_filter_recover", meta, 16, 0, ctypes.byref(h))
    bad = vbf.BloomFilter(_handle=h)
    assert bad.num_bits() == 0 and bad.no_of_hash_func == 3
    with pytest.raises(ZeroDivisionError):
        contains_all([b"a"], [vbf.BloomFilter(0.01, 10), bad])
    assert contains_all([], [bad]).shape == (0, 1)


@pytest.fixture
def multi_mode():
    """VBF_MULTI (read per call by libvbf): 1 = every filter one lane per key, 2 = interleaved
    groups of equal-(m, k) filters whenever supported; restored afterwards."""
    old = os.environ.get("VBF_MULTI")

    def set_mode(v):
        os.environ["VBF_MULTI"] = str(v)
    yield set_mode
    if old is None:
        os.environ.pop("VBF_MULTI", None)
    else:
        os.environ["VBF_MULTI"] = old


@pytest.mark.parametrize("seed", [3, 4])
def test_interleaved_groups_match_oracle(vbf, ora, multi_mode, seed):
    """Filters of one (m, k) probed as interleaved groups (vbf_multi_part.hip): groups of 3 and of
    10 (split 8 + 2), pairs at k = 14 and 7, mixed with filters of other sizes and an empty-range SST,
    with and without key ranges; bit-exact against the oracle and against the one-lane-per-key path."""
    from velarixdb_amd.key_range import SstRange, candidates, contains_all
    rng = np.random.default_rng(seed)
    # k = 9 (class 12), 19 (the group pipeline), 14 (class 16) and 7 (class 8) in groups: the interleaved
    # round-3 pack takes the runtime-k class kernels over 2^17-position segments (round 6)
    specs = ([(0.01, 4000)] * 3 + [(1e-4, 2500)] * 10 + [(0.05, 700), (0.001, 3000)] + [(1e-3, 3500)] * 2
             + [(0.03, 3000)] * 2)
    order = rng.permutation(len(specs))
    filters, orc, ranges = [], [], []
    for i in order:
        p, n = specs[i]
        f = vbf.BloomFilter(p, n)
        ks = sorted({rng.bytes(int(rng.integers(1, 24))) for _ in range(n)})
        f.set_many(ks)
        filters.append(f)
        orc.append((f.num_bits(), f.no_of_hash_func, ora.build_words(vbf.pack(ks), f.num_bits(), f.no_of_hash_func)))
        lo, hi = (ks[0], ks[-1]) if rng.random() < 0.8 else (b"\xff\xff", b"\xff\xff\x00")
        ranges.append(SstRange(lo, hi, f))
    q = [rng.bytes(int(rng.integers(0, 30))) for _ in range(30000)]
    q += [r.smallest_key for r in ranges] + [r.biggest_key for r in ranges]
    want_c = np.stack([_oracle_contains(ora, q, m, k, w) for m, k, w in orc], axis=1)
    inr = np.array([[r.smallest_key <= x <= r.biggest_key for r in ranges] for x in q])
    for mode in (2, 1):
        multi_mode(mode)
        assert np.array_equal(contains_all(q, filters), want_c), mode
        assert np.array_equal(candidates(q, ranges), want_c & inr), mode


def test_interleaved_groups_device_large(vbf, multi_mode):
    """1.5M device keys x 8 same-size filters (the AUTO path): equals 8 single probes."""
    import torch
    from velarixdb_amd._lib import call
    n, L, S = 1_500_000, 16, 8
    dev = torch.device("cuda:0")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    keys = torch.empty(n * L, dtype=torch.uint8, device=dev)
    call("vbf_gen_fixed_dev", 0x5EED0C01, 0, n, L, P(keys), None)
    filters = []
    per = n // S
    for s in range(S):
        f = vbf.BloomFilter(0.0082, per)
        f.set_dev(P(keys[s * per * L:]), None, L, per, 1)
        filters.append(f)
    handles = (ctypes.c_void_p * S)(*[f._h.value for f in filters])
    multi_mode(0)
    out = torch.empty(n * S, dtype=torch.uint8, device=dev)
    call("vbf_multi_probe_dev", P(keys), None, L, n, 1, S, handles, None, None, P(out), None)
    torch.cuda.synchronize()
    got = out.view(n, S).cpu().numpy()
    assert got.any(axis=1).all()  # every key is in one of the filters
    for s, f in enumerate(filters):
        one = torch.empty(n, dtype=torch.uint8, device=dev)
        f.contains_dev(P(keys), None, L, n, P(one))
        torch.cuda.synchronize()
        assert np.array_equal(got[:, s], one.cpu().numpy()), s


@pytest.mark.parametrize("k_bits,L,ranged", [(10, 16, False), (19, None, True), (19, 32, False), (10, None, True)])
def test_group_pipeline_matches_round3_pipeline_and_oracle(vbf, ora, multi_mode, k_bits, L, ranged):
    """The round-4 group pipeline (VBF_MULTI_GP=1: the build's tile image with 2^17-byte segments,
    per-entry result bytes, a key's results found through the pack's position table) against the
    round-3 pipeline (VBF_MULTI_GP=0) and the oracle: k = 10 and the reference default k = 19,
    fixed and variable-length keys, with and without key ranges, groups of 8 + 3 filters."""
    import torch
    from velarixdb_amd._lib import call
    from velarixdb_amd.keys import HostBatch, pack_offsets
    from velarixdb_amd.workloads import fpr_for_bits_per_key, var_offsets
    n, S, per = 1_200_000, 11, 150_000
    dev = torch.device("cuda:0")
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    if L is None:
        off_h = var_offsets(0x5EED0F01, 0, n)
        host = ora.gen_var(0x5EED0F01, 0, off_h)
        hb = pack_offsets(host, off_h)
        keys = torch.from_numpy(host).to(dev)
        offs = torch.from_numpy(off_h.view(np.int64)).to(dev)
        stride = 0
        key_list = [bytes(host[off_h[j]:off_h[j + 1]]) for j in range(n)]
    else:
        host = ora.gen_fixed(0x5EED0F01, 0, n, L)
        hb = HostBatch(host, None, L, n, 1)
        keys = torch.from_numpy(host).to(dev)
        offs, stride = None, L
        key_list = [bytes(host[j * L:(j + 1) * L]) for j in range(n)]
    p = fpr_for_bits_per_key(k_bits)
    filters, words = [], []
    for s_ in range(S):
        f = vbf.BloomFilter(p, per)
        lo = s_ * 90_000
        sub = key_list[lo:lo + per]
        f.set_many(sub)
        filters.append(f)
        words.append(f.words())
    m, k = filters[0].num_bits(), filters[0].no_of_hash_func
    assert k == k_bits and all(f.num_bits() == m for f in filters)
    handles = (ctypes.c_void_p * S)(*[f._h.value for f in filters])
    bounds = bounds_off = None
    lo_hi = []
    if ranged:
        rng = np.random.default_rng(k_bits)
        parts, bo = [], [0]
        for s_ in range(S):
            a, b = sorted(rng.choice(n, 2, replace=False))
            lo_hi.append((key_list[a], key_list[b]) if key_list[a] <= key_list[b] else (key_list[b], key_list[a]))
            for x in lo_hi[-1]:
                parts.append(x)
                bo.append(bo[-1] + len(x))
        bounds = torch.from_numpy(np.frombuffer(b"".join(parts), np.uint8).copy()).to(dev)
        bounds_off = np.asarray(bo, np.uint64)
    outs = {}
    for gp in ("1", "0"):
        os.environ["VBF_MULTI_GP"] = gp
        try:
            multi_mode(0)
            out = torch.empty(n * S, dtype=torch.uint8, device=dev)
            call("vbf_multi_probe_dev", P(keys), P(offs), stride, n, 1, S, handles, P(bounds),
                 bounds_off.ctypes.data if bounds_off is not None else None, P(out), None)
            torch.cuda.synchronize()
            outs[gp] = out.view(n, S).cpu().numpy()
        finally:
            os.environ.pop("VBF_MULTI_GP", None)
    assert np.array_equal(outs["1"], outs["0"])
    got = outs["1"]
    sl = slice(0, n, 7)  # oracle on every 7th key
    for s_ in range(S):
        want = ora.probe(hb, m, k, words[s_], threads=8)[sl].astype(bool)
        if ranged:
            lo, hi = lo_hi[s_]
            want &= np.array([lo <= x <= hi for x in key_list[sl]])
        assert np.array_equal(got[sl, s_].astype(bool), want), s_


@pytest.mark.parametrize("m,k", [(120_000_000, 10), (268_434_000, 19), (5_000, 10), (40_000_003, 10)])
def test_group_pipeline_edge_sizes(vbf, ora, multi_mode, m, k):
    """The group pipeline at its size limits: 916 segments of 2^17 with sparse filters (short and
    empty runs), m just under 2^28 at k = 19 (2 048 segments: the run-padding reserve would take
    most of the tile, so the round-3 pipeline answers -- the same answers either way), one segment
    (m = 5 000: every tile split over many workgroups), and a mid size; 8 filters of one (m, k),
    device keys; equal to the round-3 pipeline and to the oracle."""
    import torch
    from velarixdb_amd._lib import call
    from velarixdb_amd.keys import HostBatch
    n, L, S = 1_100_000, 16, 8
    dev = torch.device("cuda:0")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    host = ora.gen_fixed(0x5EED0F11, 0, n, L)
    keys = torch.from_numpy(host).to(dev)
    filters, words = [], []
    for s_ in range(S):
        f = vbf.BloomFilter.sized(m, k)
        per = 200_000
        f.set_dev(P(keys[s_ * 100_000 * L:]), None, L, per, 1)
        filters.append(f)
        words.append(f.words())
    handles = (ctypes.c_void_p * S)(*[f._h.value for f in filters])
    outs = {}
    for gp in ("1", "0"):
        os.environ["VBF_MULTI_GP"] = gp
        try:
            multi_mode(0)
            out = torch.empty(n * S, dtype=torch.uint8, device=dev)
            call("vbf_multi_probe_dev", P(keys), None, L, n, 1, S, handles, None, None, P(out), None)
            torch.cuda.synchronize()
            outs[gp] = out.view(n, S).cpu().numpy()
        finally:
            os.environ.pop("VBF_MULTI_GP", None)
    assert np.array_equal(outs["1"], outs["0"])
    sl = slice(0, n, 5)
    hb = HostBatch(host, None, L, n, 1)
    for s_ in range(S):
        want = ora.probe(hb, m, k, words[s_], threads=8)[sl].astype(bool)
        assert np.array_equal(outs["1"][sl, s_].astype(bool), want), s_


@pytest.mark.parametrize("groups", [[0, 1, 0, 2, 1, 0], [5, 4, 3, 2, 1, 0], [7, 7, 7, 7, 7, 7]])
def test_grouped_split_equals_one_device_probe(vbf, ora, groups):
    """the path vbf_multi_probe_host takes for filters on several GPUs -- split
    per device, bound bytes re-based per group, keys staged to each, answer columns scattered back
    -- run on this one GPU with the split given (vbf_multi_probe_host_grouped), ranged bounds and
    variable-length keys: equal to the single-device probe and to the oracle."""
    from velarixdb_amd._lib import call
    from velarixdb_amd.key_range import SstRange, _bounds, candidates
    from velarixdb_amd.keys import pack
    rng = np.random.default_rng(sum(groups))
    specs = [(0.01, 5000), (0.1, 800), (1e-4, 3000), (0.3, 20000), (1.0, 5), (1e-3, 7000)]
    ranges, orc = [], []
    for p, n in specs:
        f = vbf.BloomFilter(p, n)
        ks = sorted(rng.bytes(int(rng.integers(1, 30))) for _ in range(n))
        f.set_many(ks)
        lo, hi = ks[len(ks) // 5], ks[4 * len(ks) // 5]
        ranges.append(SstRange(lo, hi, f))
        orc.append((lo, hi, f.num_bits(), f.no_of_hash_func, ora.build_words(pack(ks), f.num_bits(), f.no_of_hash_func)))
    q = [rng.bytes(int(rng.integers(0, 40))) for _ in range(3000)] + [r.smallest_key for r in ranges] + \
        [r.biggest_key for r in ranges]
    b = pack(q)
    raw, offs = _bounds(ranges)
    handles = (ctypes.c_void_p * len(ranges))(*[r.filter._h.value for r in ranges])
    grp = (ctypes.c_int * len(ranges))(*groups)
    out = np.zeros((b.n, len(ranges)), np.uint8)
    d, o = b.ptrs()
    call("vbf_multi_probe_host_grouped", d, o, b.stride, b.n, b.len_prefix, len(ranges), handles, raw.ctypes.data,
         offs.ctypes.data, grp, out.ctypes.data)
    assert np.array_equal(out.astype(bool), candidates(q, ranges))
    for s, (lo, hi, m, k, words) in enumerate(orc):
        inr = np.array([lo <= x <= hi for x in q])
        assert np.array_equal(out[:, s].astype(bool), inr & _oracle_contains(ora, q, m, k, words)), s
