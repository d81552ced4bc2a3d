"""GPU parity for the compaction merge against the literal fold of
compactors/sized.rs:170-320 (oracle.compact_merge, pinned in tests/test_compaction.py).
Bit-exact: the same entry ids in the same order and the same tombstone map."""
import ctypes
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN
from test_compaction import fixture_arena

pytestmark = pytest.mark.gpu
SST = os.path.join(GOLDEN, "sst_fixtures")


def test_fixture_bucket_merge(vbf, ora, golden):
    """test_merge_ssts_in_buckets (sized_tier_test.rs:165-205) on the GPU, plus the merged
    table's filter (p = 0.01, the test's config) against the golden digest."""
    from velarixdb_amd.compaction import CompactionConfig, SizedTierMerger
    names = sorted(os.listdir(SST))[:6]
    tables = [vbf.sst.load_entries_from_dir(os.path.join(SST, n)) for n in names]
    mg = SizedTierMerger(CompactionConfig(use_ttl=False, entry_ttl_ms=60_000, tombstone_ttl_ms=120_000,
                                          filter_false_positive=0.01))
    merged, bf = mg.merge_bucket(tables)
    assert len(merged) == 2844 * 6
    keys, offs, cr, tb, ro = fixture_arena(ora, names)
    want = ora.compact_merge(keys, offs, cr, tb, ro)
    assert merged.key_list() == [keys[offs[i]:offs[i + 1]].tobytes() for i in want]
    g = golden("sst_fixtures")["compaction_union_first6"]
    assert (bf.num_bits(), bf.no_of_hash_func) == (g["m"], g["k"])
    assert hashlib.sha256(bf.words().astype("<u4").tobytes()).hexdigest() == g["sha256"]


def _random_bucket(rng, nruns, universe, per_run, tomb_p, t_range):
    uni = sorted({rng.bytes(int(rng.integers(0, 12))) for _ in range(universe)})
    runs = []
    for _ in range(nruns):
        pick = np.sort(rng.choice(len(uni), size=min(per_run, len(uni)), replace=False))
        ks = [uni[i] for i in pick]
        cr = rng.integers(t_range[0], t_range[1], size=len(ks))
        tb = (rng.random(len(ks)) < tomb_p).astype(np.uint8)
        runs.append((ks, cr, tb))
    return uni, runs


def _arena(runs):
    keys, offs, cr, tb, ro = bytearray(), [0], [], [], [0]
    for ks, c, t in runs:
        for k in ks:
            keys += k
            offs.append(len(keys))
        cr += c.tolist()
        tb += t.tolist()
        ro.append(len(cr))
    return (np.frombuffer(bytes(keys) or b"\0", np.uint8), np.asarray(offs, np.uint64), np.asarray(cr, np.int64),
            np.asarray(tb, np.uint8), np.asarray(ro, np.uint64))


def _gpu_merge(keys, offs, cr, tb, ro, tmap, use_ttl, ettl, tttl, now):
    from velarixdb_amd._lib import call
    mk = sorted(tmap)
    mkeys = np.frombuffer(b"".join(mk) or b"\0", np.uint8)
    moff = np.concatenate([[0], np.cumsum([len(k) for k in mk])]).astype(np.uint64)
    mt = np.asarray([tmap[k] for k in mk], np.int64)
    total = int(ro[-1])
    ids, ui, ut = (np.zeros(max(total, 1), d) for d in (np.uint32, np.uint32, np.int64))
    n, nu = ctypes.c_uint64(), ctypes.c_uint64()
    P = lambda a: a.ctypes.data if a.size else None
    call("vbf_compact_merge_host", P(keys), P(offs), P(cr), P(tb), ro.ctypes.data, ro.size - 1,
         P(mkeys) if mk else None, P(moff) if mk else None, P(mt), len(mk), int(use_ttl), ettl, tttl, now,
         ids.ctypes.data, ctypes.byref(n), ui.ctypes.data, ut.ctypes.data, ctypes.byref(nu), 0)
    new = dict(tmap)
    for e, t in zip(ui[:nu.value].tolist(), ut[:nu.value].tolist()):
        new[keys[offs[e]:offs[e + 1]].tobytes()] = t
    return ids[:n.value], new


@pytest.mark.parametrize("seed,nruns,universe,per_run,tomb_p,use_ttl", [
    (1, 1, 50, 30, 0.3, False),
    (2, 2, 200, 120, 0.2, False),
    (3, 3, 300, 200, 0.3, True),
    (4, 5, 400, 250, 0.25, False),
    (5, 8, 1000, 600, 0.1, True),
    (6, 17, 3000, 1500, 0.15, False),
    (7, 4, 20, 20, 0.5, True),       # every key in every table
    (8, 6, 5000, 10, 0.9, False),    # sparse, mostly tombstones
])
def test_random_buckets_match_fold(vbf, ora, seed, nruns, universe, per_run, tomb_p, use_ttl):
    rng = np.random.default_rng(seed)
    uni, runs = _random_bucket(rng, nruns, universe, per_run, tomb_p, (1000, 1030))  # many time ties
    keys, offs, cr, tb, ro = _arena(runs)
    start = {uni[i]: int(rng.integers(995, 1035)) for i in rng.choice(len(uni), size=len(uni) // 5, replace=False)}
    now, ettl, tttl = 1040, 20, 25  # some entries and tombstones expire
    m = ora.TombstoneMap(start)
    want = ora.compact_merge(keys, offs, cr, tb, ro, use_ttl, ettl, tttl, now, m)
    got, new = _gpu_merge(keys, offs, cr, tb, ro, start, use_ttl, ettl, tttl, now)
    assert got.tolist() == want.tolist()
    assert new == m.items()


def test_buckets_share_the_tombstone_map(vbf, ora):
    """Two buckets in one compaction pass: the second sees the first's tombstones (sized.rs:36)."""
    from velarixdb_amd.compaction import CompactionConfig, SizedTierMerger
    from velarixdb_amd.sst import SstEntries
    rng = np.random.default_rng(11)
    mg = SizedTierMerger(CompactionConfig(use_ttl=False, tombstone_ttl_ms=10**12))
    m = ora.TombstoneMap()
    for b in range(3):
        _, runs = _random_bucket(rng, 4, 300, 150, 0.3, (b * 10, b * 10 + 30))
        keys, offs, cr, tb, ro = _arena(runs)
        want = ora.compact_merge(keys, offs, cr, tb, ro, False, 0, 10**12, 10**6, m)
        tables = [SstEntries(np.frombuffer(b"".join(ks) or b"\0", np.uint8),
                             np.concatenate([[0], np.cumsum([len(k) for k in ks])]).astype(np.uint64),
                             np.zeros(len(ks), np.uint32), c.astype(np.uint64), t.astype(bool))
                  for ks, c, t in runs]
        (_, _, _, _, _, _), got = mg.merge_ids(tables, now_ms=10**6)
        assert got.tolist() == want.tolist()
        assert mg.tombstones == m.items()


def test_unsorted_table_rejected(vbf):
    from velarixdb_amd import VbfError
    keys, offs, cr, tb, ro = _arena([([b"b", b"a"], np.array([1, 2]), np.array([0, 0], np.uint8))] * 2)
    with pytest.raises(VbfError, match="strictly increasing"):
        _gpu_merge(keys, offs, cr, tb, ro, {}, False, 0, 0, 0)


def test_large_merge_and_device_gather(vbf, ora):
    """4 tables x 1M overlapping 16-byte keys on the device: ids equal the fold; gather + build
    equals a filter built from the oracle's merged keys."""
    import torch
    from velarixdb_amd._lib import call
    rng = np.random.default_rng(5)
    nr, per = 4, 1_000_000
    uni = np.unique(rng.integers(0, 2**62, size=3 * per, dtype=np.int64))
    runs_k, runs_c, runs_t = [], [], []
    for r in range(nr):
        sel = np.sort(rng.choice(uni.size, size=per, replace=False))
        k = uni[sel].astype(">u8").view(np.uint8).reshape(-1, 8)
        runs_k.append(np.concatenate([k, k], axis=1).reshape(-1))  # 16 B, big-endian order = sort order
        runs_c.append(rng.integers(0, 1000, size=per).astype(np.int64))
        runs_t.append((rng.random(per) < 0.05).astype(np.uint8))
    keys = np.concatenate(runs_k)
    offs = np.arange(nr * per + 1, dtype=np.uint64) * 16
    cr, tb = np.concatenate(runs_c), np.concatenate(runs_t)
    ro = np.arange(nr + 1, dtype=np.uint64) * per
    want = ora.compact_merge(keys, offs, cr, tb, ro, False, 0, 10**9, 500)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to(dev)
    dk, do, dc, dt = T(keys), T(offs), T(cr), T(tb)
    ids = torch.empty(nr * per, dtype=torch.int32, device=dev)
    n, nu = ctypes.c_uint64(), ctypes.c_uint64()
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    call("vbf_compact_merge_dev", P(dk), P(do), P(dc), P(dt), ro.ctypes.data, nr, None, None, None, 0, 0, 0,
         10**9, 500, P(ids), ctypes.byref(n), None, None, ctypes.byref(nu), None)
    assert n.value == want.size
    assert np.array_equal(ids[: n.value].cpu().numpy().view(np.uint32), want)
    ok_ = torch.empty(n.value * 16, dtype=torch.uint8, device=dev)
    oo = torch.empty(n.value + 1, dtype=torch.int64, device=dev)
    kb = ctypes.c_uint64()
    call("vbf_gather_entries_dev", P(dk), P(do), None, None, None, P(ids), n.value, P(ok_), ok_.numel(), P(oo),
         None, None, None, ctypes.byref(kb), None)
    torch.cuda.synchronize()
    assert kb.value == n.value * 16
    wk = keys.reshape(-1, 16)[want.astype(np.int64)].reshape(-1)
    assert np.array_equal(ok_.cpu().numpy(), wk)
    bf = vbf.BloomFilter(1e-4, n.value)
    bf.set_dev(P(ok_), P(oo), 0, n.value, 1)
    assert np.array_equal(bf.words(), ora.build_words(vbf.pack_fixed(wk.reshape(-1, 16)), bf.num_bits(),
                                                      bf.no_of_hash_func, threads=8))


def test_sharded_filter_builds(vbf, ora):
    """The compaction fan-in's independent per-table builds (vbf_build_shards_host): every
    shard's words equal the oracle's, whatever thread/device serves it; an unusable device fails
    that shard only and the call reports it."""
    from velarixdb_amd.compaction import _Shard, build_filters_sharded
    from velarixdb_amd.keys import pack, pack_fixed
    rng = np.random.default_rng(11)
    batches = [pack_fixed(rng.integers(0, 256, (20_000, 16), dtype=np.uint8)),
               pack([bytes(rng.integers(0, 256, int(n), dtype=np.uint8)) for n in rng.integers(0, 90, 5_000)]),
               pack_fixed(rng.integers(0, 256, (1, 32), dtype=np.uint8)),
               pack_fixed(rng.integers(0, 256, (70_000, 8), dtype=np.uint8))]
    for devices in ((0,), (0, 0, 0)):
        got = build_filters_sharded(batches, 0.01, devices)
        for b, (m, k, words) in zip(batches, got):
            assert np.array_equal(words, ora.build_words(b, m, k)), (devices, b.n)
    b = batches[0]
    words = np.zeros(100, np.uint32)
    d, o = b.ptrs()
    shards = (_Shard * 2)(_Shard(d, o, b.stride, b.n, 1, 3200, 3, words.ctypes.data, 100, 0),
                          _Shard(d, o, b.stride, b.n, 1, 3200, 3, words.ctypes.data, 100, 0))
    devs = (ctypes.c_int * 2)(0, 99)
    rc = vbf.lib.vbf_build_shards_host(ctypes.cast(shards, ctypes.c_void_p), 2, ctypes.cast(devs, ctypes.c_void_p), 2)
    assert rc == vbf._lib.VBF_ENODEV and shards[0].status == 0 and shards[1].status == vbf._lib.VBF_ENODEV
    assert b"shard 1" in vbf.lib.vbf_last_error()
    assert np.array_equal(words, ora.build_words(b, 3200, 3))
