"""GPU parity for the partitioned probe (contains(), bf.rs:95-105, for large batches): its
answers equal the per-key early-exit probe and the oracle, bit for bit, across key layouts,
filter sizes (one segment, a few, thousands, the u32-saturated config-5 size) and k values
(compile-time 4/10/19 and run-time k: the class packs with a register stash, with and without
the length prefix)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [  # (L or None for var-length, len_prefix, m, k, n)
    (16, 1, 100_000_000, 10, 2_000_000),
    (32, 1, 4_294_967_295, 4, 1_000_000),
    (8, 0, 5_000_000, 7, 500_000),        # 5 segments -> several workgroups per segment
    (None, 1, 300_000_000, 19, 400_000),  # variable-length keys, run-time k
    (24, 1, 1 << 20, 3, 300_000),         # exactly one segment
    (13, 1, 3_000_000_000, 3, 600_000),   # unaligned stride
    (16, 1, 1 << 31, 10, 1_000_000),      # the largest m of the one-word remainder (fast_mod31)
    (16, 1, (1 << 31) + 1, 10, 1_000_000),  # the smallest m past it (general remainder)
    (16, 1, (1 << 31) - 1, 19, 400_000),
    # m = 2^32 - 1 (saturated): the SAT probe packs (k = 10, 19; k = 4 above) and a runtime k
    (16, 1, 4_294_967_295, 10, 600_000),
    (24, 1, 4_294_967_295, 19, 300_000),
    (None, 1, 4_294_967_295, 10, 300_000),
    (16, 1, 4_294_967_295, 6, 400_000),
    # round 5: the runtime-k class probe packs (register stash) for every class, both remainders,
    # fixed and variable-length keys
    (None, 1, 300_000_007, 14, 400_000), (16, 1, 200_000_003, 23, 300_000), (32, 1, 50_000_017, 12, 400_000),
    (8, 1, 40_000_003, 32, 200_000), (16, 1, 100_000_007, 21, 300_000), (None, 1, 2_500_000_001, 7, 300_000),
    # ... and for keys hashed without the length prefix (pre-encoded integer keys)
    (16, 0, 100_000_007, 14, 300_000), (None, 0, 300_000_007, 23, 300_000), (8, 0, 3_000_000_017, 5, 400_000),
    # ... at the reference's saturated size m = 2^32 - 1: class 8 (rk_c) with fixed and
    # class 16 (rk_d) with variable-length keys
    (8, 0, 4_294_967_295, 6, 300_000), (None, 0, 4_294_967_295, 14, 300_000),
]


def _keys(torch, L, n, seed):
    from velarixdb_amd._lib import call
    dev = torch.device("cuda:0")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    if L is None:
        from velarixdb_amd.workloads import var_offsets
        offs = torch.from_numpy(var_offsets(seed, 0, n).view(np.int64)).to(dev)
        keys = torch.empty(int(offs[-1].item()), dtype=torch.uint8, device=dev)
        call("vbf_gen_var_dev", seed, 0, n, P(offs), P(keys), None)
        return keys, offs, 0
    keys = torch.empty(n * L, dtype=torch.uint8, device=dev)
    call("vbf_gen_fixed_dev", seed, 0, n, L, P(keys), None)
    return keys, None, L


@pytest.mark.parametrize("L,lp,m,k,n", CASES)
def test_partitioned_probe_matches_gather_probe(vbf, ora, L, lp, m, k, n):
    import torch
    from velarixdb_amd._lib import call
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    keys, offs, stride = _keys(torch, L, n, 0x5EED0101)
    words = torch.zeros((m + 31) // 32, dtype=torch.int32, device="cuda:0")
    half = n // 2  # build from the first half: probes see positives and negatives
    call("vbf_build_dev_ex", P(keys), P(offs), stride, half, lp, m, k, P(words), 0, None)
    outs = {}
    for strat in (1, 2):
        o = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        call("vbf_probe_dev_ex", P(keys), P(offs), stride, n, lp, m, k, P(words), P(o), strat, None)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
        call("vbf_probe_count_dev_ex", P(keys), P(offs), stride, n, lp, m, k, P(words), P(cnt), strat, None)
        torch.cuda.synchronize()
        outs[strat] = o.cpu().numpy()
        assert int(cnt.item()) == int(outs[strat].sum())
    assert np.array_equal(outs[1], outs[2])
    assert outs[2][:half].all()  # no false negatives
    # oracle on a slice of the negatives (and a few positives)
    sl = slice(half - 1000, half + 20000)
    if offs is None:
        hk = keys.cpu().numpy().reshape(n, L)[sl]
        batch = vbf.pack_fixed(hk, lp)
    else:
        o_h = offs.cpu().numpy().view(np.uint64)
        kb = keys.cpu().numpy()
        lo, hi = int(o_h[sl.start]), int(o_h[sl.stop])
        batch = vbf.pack_offsets(kb[lo:hi], o_h[sl.start:sl.stop + 1] - lo, lp)
    wh = words.cpu().numpy().view(np.uint32)
    assert np.array_equal(ora.probe(batch, m, k, wh).astype(np.uint8), outs[2][sl])


def test_partitioned_probe_edges(vbf):
    """n = 1, n not a multiple of the tile, k = 0 (always true), unsupported k falls back."""
    import torch
    from velarixdb_amd._lib import VbfError, call
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    keys, _, _ = _keys(torch, 16, 5000, 3)
    m = 1 << 27
    words = torch.zeros(m // 32, dtype=torch.int32, device="cuda:0")
    call("vbf_build_dev_ex", P(keys), None, 16, 2500, 1, m, 10, P(words), 0, None)
    for n in (1, 1849, 1851, 4999):
        a = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        b = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        call("vbf_probe_dev_ex", P(keys), None, 16, n, 1, m, 10, P(words), P(a), 1, None)
        call("vbf_probe_dev_ex", P(keys), None, 16, n, 1, m, 10, P(words), P(b), 2, None)
        assert torch.equal(a, b)
    o = torch.zeros(100, dtype=torch.uint8, device="cuda:0")
    call("vbf_probe_dev_ex", P(keys), None, 16, 100, 1, m, 0, P(words), P(o), 0, None)
    assert bool(o.all())
    with pytest.raises(VbfError):
        call("vbf_probe_dev_ex", P(keys), None, 16, 100, 1, m, 33, P(words), P(o), 2, None)


@pytest.mark.parametrize("L,m,k,n", [(16, 5_000, 10, 300_000), (None, 2_000_003, 19, 400_000),
                                     (32, 1 << 31, 19, 300_000), (8, 70_000_000, 10, 1_200_000),
                                     (16, 1_200_000_000, 10, 120_000_000)])  # 1.2e9 entries: 2 chunks
def test_position_table_probe_matches_round3_pipeline(vbf, ora, L, m, k, n):
    """The round-4 partitioned probe (VBF_PROBE_GP=1: the build's image, runs padded to whole
    groups, a position table) against the round-3 pipeline (VBF_PROBE_GP=0), answers and counts,
    and the oracle on a slice: one segment (m = 5 000, every tile split over many workgroups),
    variable-length keys at k = 19, the largest m of the path (2^31: 2 048 segments), and a batch of
    more than 2^30 entries (processed in chunks)."""
    import os
    import torch
    from velarixdb_amd._lib import call
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    keys, offs, stride = _keys(torch, L, n, 0x5EED0131)
    words = torch.zeros((m + 31) // 32, dtype=torch.int32, device="cuda:0")
    half = n // 2
    call("vbf_build_dev_ex", P(keys), P(offs), stride, half, 1, m, k, P(words), 0, None)
    res = {}
    os.environ["VBF_PROBE_PU"] = "0"  # the round-6 probe would take k = 10 / 19 at m <= 2^31 first
    for gp in ("1", "0"):
        os.environ["VBF_PROBE_GP"] = gp
        try:
            o = torch.empty(n, dtype=torch.uint8, device="cuda:0")
            call("vbf_probe_dev_ex", P(keys), P(offs), stride, n, 1, m, k, P(words), P(o), 2, None)
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
            call("vbf_probe_count_dev_ex", P(keys), P(offs), stride, n, 1, m, k, P(words), P(cnt), 2, None)
            torch.cuda.synchronize()
            res[gp] = (o.cpu().numpy(), int(cnt.item()))
        finally:
            os.environ.pop("VBF_PROBE_GP", None)
    os.environ.pop("VBF_PROBE_PU", None)
    assert np.array_equal(res["1"][0], res["0"][0]) and res["1"][1] == res["0"][1] == int(res["1"][0].sum())
    assert res["1"][0][:half].all()
    sl = slice(half - 500, min(n, half + 20000))
    if offs is None:
        batch = vbf.pack_fixed(keys.cpu().numpy().reshape(n, L)[sl], 1)
    else:
        o_h = offs.cpu().numpy().view(np.uint64)
        kb = keys.cpu().numpy()
        lo, hi = int(o_h[sl.start]), int(o_h[sl.stop])
        batch = vbf.pack_offsets(kb[lo:hi], o_h[sl.start:sl.stop + 1] - lo, 1)
    assert np.array_equal(ora.probe(batch, m, k, words.cpu().numpy().view(np.uint32)).astype(np.uint8), res["1"][0][sl])


def _probe_both(torch, call, P, keys, offs, stride, n, lp, m, k, words, env):
    """answers + count of the partitioned probe (strategy 2) under the given environment"""
    import os
    old = {kk: os.environ.get(kk) for kk in env}
    os.environ.update(env)
    try:
        o = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        call("vbf_probe_dev_ex", P(keys), P(offs), stride, n, lp, m, k, P(words), P(o), 2, None)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
        call("vbf_probe_count_dev_ex", P(keys), P(offs), stride, n, lp, m, k, P(words), P(cnt), 2, None)
        torch.cuda.synchronize()
        return o.cpu().numpy(), int(cnt.item())
    finally:
        for kk, v in old.items():
            if v is None:
                os.environ.pop(kk, None)
            else:
                os.environ[kk] = v


SAT = 4_294_967_295


@pytest.mark.parametrize("L,m,k,n,chunk_log2", [
    (32, SAT, 4, 1_000_000, None), (16, SAT, 4, 700_001, None), (8, SAT, 4, 300_000, None),
    (24, SAT, 4, 400_000, None), (32, SAT, 4, 1, None), (32, SAT, 4, 6_531, None), (32, SAT, 4, 6_532, None),
    (32, SAT, 4, 6_533, None), (32, SAT, 4, 13_065, None),
    (32, SAT, 4, 10_000_000, "22"),   # 2^22 indices per chunk: 160 tiles = 1 045 120 keys, ten chunks
    # k = 10 / 19 (p = 1e-4: velarixdb's default) at m <= 2^31: the build's 512-thread shape
    (16, 1_000_000_000, 10, 2_000_000, None), (16, 1_900_000_000, 19, 1_000_000, None),
    (32, 1 << 31, 19, 600_000, None), (8, 5_000, 10, 300_000, None), (24, 70_000_000, 10, 1_200_000, None),
    (16, 300_000_000, 19, 3_000_001, "22"),
    # runtime-k classes (k outside {4, 9, 10, 19}) at m <= 2^31: every class, the largest m
    (16, 300_000_007, 14, 1_000_000, None), (32, 50_000_017, 7, 600_000, None), (8, 40_000_003, 32, 200_000, None),
    (24, 100_000_007, 23, 400_000, None), (16, 1 << 31, 12, 500_000, None), (16, 200_000_003, 5, 900_000, None),
    (32, 150_000_001, 21, 300_000, "22"),
    # k = 4 and 9 below 2^32 - 1 (no compiled pack there): the classes 5 and 12
    (16, 300_000_001, 9, 3_000_000, None), (32, 200_000_011, 4, 5_000_000, None), (None, 400_000_009, 9, 800_000, None),
    # runtime key lengths: the offsets layout (keys dealt to lanes in length order; the answers go
    # back through the slot -> key map) and an odd fixed stride (13 B: the runtime-stride layout)
    (None, SAT, 4, 800_000, None), (None, 1_000_000_000, 10, 1_000_000, None), (None, 1_900_000_000, 19, 500_000, None),
    (None, 300_000_007, 14, 500_000, None), (None, 500_000_000, 10, 2_000_000, "22"), (13, 1_000_000_000, 10, 700_000, None),
    (13, SAT, 4, 500_000, None),
])
def test_round6_probe_on_build_image(vbf, ora, L, m, k, n, chunk_log2):
    """The round-6 probe (vbf_probe_pu.hip: the build's unpadded tile image, padded result bits,
    posv) against the earlier pipelines (VBF_PROBE_PU=0: round 3 at m = 2^32 - 1, the round-4
    position-table pipeline at k = 10 / 19), the gather probe and the oracle: answers and counts,
    half the batch positive.  Config 5's shape (m = 2^32 - 1, the reference's saturated size,
    bf.rs:230-233; k = 4) with single keys, tile edges (6 532 keys per tile) and several chunks;
    k = 10 / 19 with one segment (m = 5 000: every tile's runs split over many workgroups), the
    largest m of the path (2^31) and several chunks; every runtime-k class (the K1 class kernels with
    the class's slots per key, k at run time), k = 4 and 9 below 2^32 - 1 included (classes 5 and
    12); variable-length keys (the pack's length order, the
    answers mapped back to key order) and an odd fixed stride.  Anchor: contains(), bf.rs:95-105."""
    import torch
    from velarixdb_amd._lib import call
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    keys, offs, stride = _keys(torch, L, n, 0x5EED0161)
    words = torch.zeros((m + 31) // 32, dtype=torch.int32, device="cuda:0")
    half = max(1, n // 2)
    call("vbf_build_dev_ex", P(keys), P(offs), stride, half, 1, m, k, P(words), 0, None)
    env = {"VBF_PROBE_CHUNK_LOG2": chunk_log2} if chunk_log2 else {}
    pu = _probe_both(torch, call, P, keys, offs, stride, n, 1, m, k, words, env)
    r3 = _probe_both(torch, call, P, keys, offs, stride, n, 1, m, k, words, {"VBF_PROBE_PU": "0"})
    g = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    call("vbf_probe_dev_ex", P(keys), P(offs), stride, n, 1, m, k, P(words), P(g), 1, None)
    torch.cuda.synchronize()
    assert np.array_equal(pu[0], r3[0]) and np.array_equal(pu[0], g.cpu().numpy())
    assert pu[1] == r3[1] == int(pu[0].sum())
    assert pu[0][:half].all()
    sl = slice(max(0, half - 1000), min(n, half + 30000))
    if offs is None:
        batch = vbf.pack_fixed(keys.cpu().numpy().reshape(n, L)[sl], 1)
    else:
        o_h = offs.cpu().numpy().view(np.uint64)
        kb = keys.cpu().numpy()
        lo, hi = int(o_h[sl.start]), int(o_h[sl.stop])
        batch = vbf.pack_offsets(kb[lo:hi], o_h[sl.start:sl.stop + 1] - lo, 1)
    assert np.array_equal(ora.probe(batch, m, k, words.cpu().numpy().view(np.uint32)).astype(np.uint8), pu[0][sl])


def test_round6_probe_skewed_runs(vbf, ora):
    """Heavily repeated keys: every tile's entries fall in a handful of segments, so runs are
    thousands of entries long -- the segment pass's loop past 4 x 64 groups per batch and the lane
    that loads its run's next group itself.  Plus a filter with garbage bits set everywhere (mixed
    answers in every result byte)."""
    import torch
    from velarixdb_amd._lib import call
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    m, k, L, n = 4_294_967_295, 4, 32, 2_000_000
    base, _, _ = _keys(torch, L, 5, 0x5EED0171)
    idx = torch.arange(n, device="cuda:0") % 5
    keys = base.view(5, L)[idx].reshape(-1).contiguous()
    keys.view(n, L)[n // 3:, 0] ^= 0x5A  # a second and third population, 4 of 5 of them unbuilt
    for words in (torch.zeros((m + 31) // 32, dtype=torch.int32, device="cuda:0"),
                  torch.randint(-2**31, 2**31 - 1, ((m + 31) // 32,), dtype=torch.int32, device="cuda:0")
                  & torch.randint(-2**31, 2**31 - 1, ((m + 31) // 32,), dtype=torch.int32, device="cuda:0")):
        call("vbf_build_dev_ex", P(keys), None, L, n // 3, 1, m, k, P(words), 0, None)
        pu = _probe_both(torch, call, P, keys, None, L, n, 1, m, k, words, {})
        r3 = _probe_both(torch, call, P, keys, None, L, n, 1, m, k, words, {"VBF_PROBE_PU": "0"})
        assert np.array_equal(pu[0], r3[0]) and pu[1] == r3[1] == int(pu[0].sum())
        assert pu[0][:n // 3].all()
        uniq, first = np.unique(keys.cpu().numpy().reshape(n, L), axis=0, return_index=True)
        want = ora.probe(vbf.pack_fixed(uniq, 1), m, k, words.cpu().numpy().view(np.uint32)).astype(np.uint8)
        assert np.array_equal(want, pu[0][first])
