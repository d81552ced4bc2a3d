"""Headline-size checks (BASELINE configs 2, 3 and 5's sizing) on one MI355X.

Config 2 is compared bit for bit with the multi-threaded oracle (16 host threads, ~40 s);
the others through size-independent properties: the two build strategies agree, builds are
idempotent and order-independent (OR is commutative), every inserted key is found, and the
fill ratio matches 1 - exp(-k n / m).
"""
import ctypes
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
FRESH = 0x100  # VBF_BUILD_FRESH


def vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def sp():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def build(vbf, keys, offs, stride, n, m, k, strategy, words=None):
    nw = (m + 31) // 32
    if words is None:
        words = torch.zeros(nw, dtype=torch.int32, device=DEV)
    vbf._lib.call("vbf_build_dev_ex", vp(keys), vp(offs), stride, n, 1, m, k, vp(words), strategy, sp())
    return words


def count(vbf, keys, offs, stride, n, m, k, words):
    c = torch.zeros(1, dtype=torch.int64, device=DEV)
    vbf._lib.call("vbf_probe_count_dev", vp(keys), vp(offs), stride, n, 1, m, k, vp(words), vp(c), sp())
    return int(c.item())


def popcount(vbf, words):
    c = torch.zeros(1, dtype=torch.int64, device=DEV)
    vbf._lib.call("vbf_popcount_dev", vp(words), words.numel(), vp(c), sp())
    return int(c.item())


def test_config2_full_size_bit_exact(vbf, ora):
    from velarixdb_amd.keys import HostBatch
    from velarixdb_amd.workloads import SEED_CFG2, fpr_for_bits_per_key
    n, L = 100_000_000, 16
    m = vbf.num_bits(n, fpr_for_bits_per_key(10))
    k = vbf.num_hash_functions(m, n)
    assert (m, k) == (1_000_000_000, 10)
    keys = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    vbf._lib.call("vbf_gen_fixed_dev", SEED_CFG2, 0, n, L, vp(keys), sp())
    w_part = build(vbf, keys, None, L, n, m, k, 2)
    w_atom = build(vbf, keys, None, L, n, m, k, 1)
    assert torch.equal(w_part, w_atom)
    # idempotent: building the same keys again changes nothing
    w_again = build(vbf, keys, None, L, n, m, k, 2, words=w_part.clone())
    assert torch.equal(w_again, w_part)
    # order independence: second half first, then first half
    h = n // 2
    w_split = build(vbf, keys[h * L:], None, L, n - h, m, k, 2)
    build(vbf, keys, None, L, h, m, k, 2, words=w_split)
    assert torch.equal(w_split, w_part)
    assert count(vbf, keys, None, L, n, m, k, w_part) == n
    fill = popcount(vbf, w_part) / m
    assert abs(fill - (1 - math.exp(-k * n / m))) < 1e-3
    # the benchmarked step (bench.py): BloomFilter::new fused with the build (VBF_BUILD_FRESH)
    # into words holding garbage, the segment pass writing every word without reading it
    w_fresh = torch.randint(-2**31, 2**31 - 1, (m // 32,), dtype=torch.int32, device=DEV)
    build(vbf, keys, None, L, n, m, k, 2 | FRESH, words=w_fresh)
    # bit-exact against the oracle over the full 100M keys (16 host threads)
    host = keys.cpu().numpy()
    del keys, w_atom, w_again, w_split
    want = ora.build_words(HostBatch(host, None, L, n, 1), m, k, threads=16)
    assert np.array_equal(w_part.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(w_fresh.cpu().numpy().view(np.uint32), want)


def test_config4_shard0_fresh_bit_exact(vbf, ora):
    """Config 4's per-rank workload as bench.py --gpus N runs it on rank 0: SSTable shard 0,
    50M x 16 B keys (seed 0x5EED0040), m = 5e8, k = 10, one fresh build (new + build fused,
    the timed step) into garbage-filled words, bit-exact against the 16-thread oracle."""
    from velarixdb_amd.keys import HostBatch
    from velarixdb_amd.workloads import SEED_CFG4, fpr_for_bits_per_key
    n, L = 50_000_000, 16
    m = vbf.num_bits(n, fpr_for_bits_per_key(10))
    k = vbf.num_hash_functions(m, n)
    assert (m, k) == (500_000_000, 10)
    keys = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    vbf._lib.call("vbf_gen_fixed_dev", SEED_CFG4 + 0, 0, n, L, vp(keys), sp())
    words = torch.randint(-2**31, 2**31 - 1, ((m + 31) // 32,), dtype=torch.int32, device=DEV)
    build(vbf, keys, None, L, n, m, k, 2 | FRESH, words=words)
    assert count(vbf, keys, None, L, n, m, k, words) == n
    host = keys.cpu().numpy()
    del keys
    want = ora.build_words(HostBatch(host, None, L, n, 1), m, k, threads=16)
    assert np.array_equal(words.cpu().numpy().view(np.uint32), want)


def test_config5_rank_shape_fresh(vbf):
    """Config 5's per-rank shape on 8 GPUs: 125M x 32 B keys (1/8 of 1B), the saturated
    m = 2^32 - 1 and k = 4 of the whole filter, a fresh partitioned build into garbage equal to
    the per-key atomic build into zeros (the oracle would take minutes at this size; config 5's
    sizing slice and the 5M-key oracle checks pin the 32-byte hash)."""
    from velarixdb_amd.workloads import SEED_CFG5, fpr_for_bits_per_key
    N = 1_000_000_000
    m = vbf.num_bits(N, fpr_for_bits_per_key(15))
    k = vbf.num_hash_functions(m, N)
    assert (m, k) == (4294967295, 4)
    n, L = 125_000_000, 32
    keys = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    vbf._lib.call("vbf_gen_fixed_dev", SEED_CFG5, 0, n, L, vp(keys), sp())
    nw = (m + 31) // 32
    w_fresh = torch.randint(-2**31, 2**31 - 1, (nw,), dtype=torch.int32, device=DEV)
    build(vbf, keys, None, L, n, m, k, 2 | FRESH, words=w_fresh)
    w_atom = build(vbf, keys, None, L, n, m, k, 1)
    assert torch.equal(w_fresh, w_atom)
    assert count(vbf, keys, None, L, n, m, k, w_fresh) == n
    fill = popcount(vbf, w_fresh) / m
    assert abs(fill - (1 - math.exp(-k * n / m))) < 1e-3


@pytest.mark.timeout(600)
def test_k19_full_size_bit_exact(vbf, ora):
    """The reference's default p = 1e-4 gives k = 19 (consts/mod.rs:17, bf.rs:236-239): config 2's
    100M keys at 19 bits per key (m = 1.9e9), built with two lanes per key (vbf_partition.hpp
    build_spl), bit-exact against the atomic build and the 16-thread oracle over all 100M keys."""
    from velarixdb_amd.keys import HostBatch
    from velarixdb_amd.workloads import SEED_CFG2, fpr_for_bits_per_key
    n, L = 100_000_000, 16
    m = vbf.num_bits(n, fpr_for_bits_per_key(19))
    k = vbf.num_hash_functions(m, n)
    assert (m, k) == (1_900_000_000, 19)
    keys = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    vbf._lib.call("vbf_gen_fixed_dev", SEED_CFG2, 0, n, L, vp(keys), sp())
    w_part = build(vbf, keys, None, L, n, m, k, 2)
    w_atom = build(vbf, keys, None, L, n, m, k, 1)
    assert torch.equal(w_part, w_atom)
    del w_atom
    # the benchmarked form (bench.py --bits-per-key 19): fresh build into garbage
    w_fresh = torch.randint(-2**31, 2**31 - 1, ((m + 31) // 32,), dtype=torch.int32, device=DEV)
    build(vbf, keys, None, L, n, m, k, 2 | FRESH, words=w_fresh)
    assert torch.equal(w_fresh, w_part)
    del w_fresh
    assert count(vbf, keys, None, L, n, m, k, w_part) == n
    fill = popcount(vbf, w_part) / m
    assert abs(fill - (1 - math.exp(-k * n / m))) < 1e-3
    host = keys.cpu().numpy()
    del keys
    want = ora.build_words(HostBatch(host, None, L, n, 1), m, k, threads=16)
    assert np.array_equal(w_part.cpu().numpy().view(np.uint32), want)


def test_config3_full_size_properties(vbf, ora):
    from velarixdb_amd.keys import pack_offsets
    from velarixdb_amd.workloads import SEED_CFG3, SEED_CFG3_NEG, fpr_for_bits_per_key, var_offsets
    n = 100_000_000
    m = vbf.num_bits(n, fpr_for_bits_per_key(10))
    k = vbf.num_hash_functions(m, n)
    off_h = var_offsets(SEED_CFG3, 0, n)
    off = torch.from_numpy(off_h.view(np.int64)).to(DEV)
    keys = torch.empty(int(off_h[-1]), dtype=torch.uint8, device=DEV)
    vbf._lib.call("vbf_gen_var_dev", SEED_CFG3, 0, n, vp(off), vp(keys), sp())
    w_part = build(vbf, keys, off, 0, n, m, k, 2)
    w_atom = build(vbf, keys, off, 0, n, m, k, 1)
    assert torch.equal(w_part, w_atom)
    del w_atom
    # the benchmarked form (bench.py --config 3): fresh build into garbage, offsets layout
    w_fresh = torch.randint(-2**31, 2**31 - 1, ((m + 31) // 32,), dtype=torch.int32, device=DEV)
    build(vbf, keys, off, 0, n, m, k, 2 | FRESH, words=w_fresh)
    assert torch.equal(w_fresh, w_part)
    del w_fresh
    assert count(vbf, keys, off, 0, n, m, k, w_part) == n
    # 50M negatives: FPR near theory (fill^k) -- the reference's probabilistic contract
    nn = 50_000_000
    noff_h = var_offsets(SEED_CFG3_NEG, 0, nn)
    noff = torch.from_numpy(noff_h.view(np.int64)).to(DEV)
    nkeys = torch.empty(int(noff_h[-1]), dtype=torch.uint8, device=DEV)
    vbf._lib.call("vbf_gen_var_dev", SEED_CFG3_NEG, 0, nn, vp(noff), vp(nkeys), sp())
    fp = count(vbf, nkeys, noff, 0, nn, m, k, w_part)
    fill = popcount(vbf, w_part) / m
    assert abs(fp / nn - fill ** k) < 5e-4
    # bit-exact vs the oracle on the first 5M keys (a filter of its own)
    ns = 5_000_000
    sub = build(vbf, keys, off[: ns + 1], 0, ns, 50_000_000, k, 2)
    data = keys[: int(off_h[ns])].cpu().numpy()
    want = ora.build_words(pack_offsets(data, off_h[: ns + 1]), 50_000_000, k, threads=16)
    assert np.array_equal(sub.cpu().numpy().view(np.uint32), want)


def test_config5_sizing_slice(vbf, ora):
    """Config 5's saturated m (2^32-1 bits, k = 4) on 200M x 32 B keys (a 1/5 slice)."""
    from velarixdb_amd.workloads import SEED_CFG5, fpr_for_bits_per_key
    N = 1_000_000_000
    m = vbf.num_bits(N, fpr_for_bits_per_key(15))
    k = vbf.num_hash_functions(m, N)
    assert (m, k) == (4294967295, 4)
    n, L = 200_000_000, 32
    keys = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    vbf._lib.call("vbf_gen_fixed_dev", SEED_CFG5, 0, n, L, vp(keys), sp())
    w_part = build(vbf, keys, None, L, n, m, k, 2)
    w_atom = build(vbf, keys, None, L, n, m, k, 1)
    assert torch.equal(w_part, w_atom)
    assert count(vbf, keys, None, L, n, m, k, w_part) == n
    fill = popcount(vbf, w_part) / m
    assert abs(fill - (1 - math.exp(-k * n / m))) < 1e-3


def test_multi_chunk_partitioned_paths(vbf):
    """More bit indices in one call than one chunk holds (build: kBuildChunkIdx = 2^31, probe:
    kPartChunkIdx = 2^30): both partitioned paths process the batch in chunks.  The chunked
    build must equal the per-key atomic build bit for bit, and both probe strategies must find
    every key."""
    from velarixdb_amd.workloads import SEED_CFG2
    n, L, m, k = 220_000_000, 16, 2_200_000_000, 10  # 2.2e9 indices: 2 build / 3 probe chunks
    keys = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    vbf._lib.call("vbf_gen_fixed_dev", SEED_CFG2 ^ 0x77, 0, n, L, vp(keys), sp())
    w_part = build(vbf, keys, None, L, n, m, k, 2)
    w_atom = build(vbf, keys, None, L, n, m, k, 1)
    assert torch.equal(w_part, w_atom)
    for strat in (1, 2):
        c = torch.zeros(1, dtype=torch.int64, device=DEV)
        vbf._lib.call("vbf_probe_count_dev_ex", vp(keys), None, L, n, 1, m, k, vp(w_part), vp(c), strat, sp())
        assert int(c.item()) == n, strat
