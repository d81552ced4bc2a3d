"""GPU parity for the SST data.db decoder and the fused rebuild.

Oracle: oracle.sst_decode / sst_write (fs/mod.rs:275-332, table.rs:280-338), pinned by
tests/test_sst.py against the reference's fixture files.  Everything here is bit-exact."""
import ctypes
import hashlib
import os
import shutil

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
SST = os.path.join(GOLDEN, "sst_fixtures")
NAMES = sorted(os.listdir(SST))


def _same(ent, ref):
    keys, offs, val, created, tomb = ref
    n = offs.size - 1
    assert len(ent) == n
    assert np.array_equal(ent.offsets, offs)
    assert np.array_equal(ent.keys, keys)
    assert np.array_equal(ent.val_offsets, val)
    assert np.array_equal(ent.created_ms, created)
    assert np.array_equal(ent.tombstones.astype(np.uint8), tomb)


def _rand_sst(ora, seed, n, lengths):
    rng = np.random.default_rng(seed)
    L = rng.choice(lengths, size=n).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(L)]).astype(np.uint64)
    keys = rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)
    val = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    created = rng.integers(0, 2**63, size=n, dtype=np.uint64)
    tomb = rng.integers(0, 2, size=n, dtype=np.uint8)
    data, index = ora.sst_write(keys, offs, val, created, tomb)
    return data, index, (keys, offs, val, created, tomb)


def test_fixture_decode_bit_exact(vbf, ora):
    for name in NAMES:
        data, index = vbf.sst.read_sst_files(os.path.join(SST, name))
        _same(vbf.sst.load_entries(data, index), ora.sst_decode(data))


def test_fixture_rebuild_matches_golden(vbf, golden, tmp_path):
    """range.rs:117-128 on the reference's SSTs: recover_meta, then decode + build on the GPU."""
    want = {s["name"]: s for s in golden("sst_fixtures")["ssts"]}
    for name in NAMES:
        d = tmp_path / name
        shutil.copytree(os.path.join(SST, name), d)
        for f in os.listdir(d):
            os.chmod(d / f, 0o644)  # the fixtures are read-only; write() rewrites filter.db
        bf = vbf.BloomFilter.default()
        assert bf.recover_from_sst_dir(d) is False  # 16-byte filter.db: no bits to restore
        w = bf.words()
        assert bf.num_bits() == want[name]["m"]
        assert hashlib.sha256(w.astype("<u4").tobytes()).hexdigest() == want[name]["sha256"]
        assert bf.no_of_elements == want[name]["n_stored"] + want[name]["n_keys"]
        assert bf.get_sst_dir() == str(d)
        # a filter written at flush time, sized for this SST's keys: recovery restores its
        # persisted bits (filter_file.py) instead of rebuilding, and they equal a rebuild
        ent = vbf.sst.load_entries_from_dir(d)
        p = float.fromhex(want[name]["p"])
        f = vbf.BloomFilter(p, len(ent))
        f.set_many(ent.key_list())
        f.write(d, sst_entries=len(ent))
        f2 = vbf.BloomFilter.default()
        assert f2.recover_from_sst_dir(d) is True
        assert np.array_equal(f2.words(), f.words())
        f3 = vbf.BloomFilter(p, len(ent))
        f3.rebuild_from_sst(*vbf.sst.read_sst_files(d))
        assert np.array_equal(f3.words(), f.words())


@pytest.mark.parametrize("seed,n,lengths", [
    (1, 1, [0]),
    (2, 7, [5]),
    (3, 5000, list(range(0, 41))),
    (4, 3000, list(range(0, 300))),
    (5, 200, [4079, 4078, 4000, 1, 0]),   # one entry per block, blocks of exactly 4096 bytes
    (6, 20000, [0]),                       # empty keys only: 240 entries per 4080-byte block
    (7, 20000, [16]),
    (8, 4000, [1, 2, 3, 5, 8, 13, 21, 34, 55, 89, 144, 233, 377, 610, 987]),
    (9, 20000, [16] * 60 + [17]),          # near-uniform: most blocks fail the fixed-size guess late
    (10, 20000, [16] * 200 + [0]),
])
def test_random_sst_decode(vbf, ora, seed, n, lengths):
    data, index, ref = _rand_sst(ora, seed, n, lengths)
    _same(vbf.sst.load_entries(data, index), ref)
    assert vbf.sst.count_entries(data, index) == n


def test_tombstone_reads_byte_equal_one(vbf, ora):
    """fs/mod.rs:322: is_tombstone = byte == 1 (a byte of 2 is not a tombstone)."""
    data, index, ref = _rand_sst(ora, 9, 50, [3])
    data = data.copy()
    for j in range(50):  # entry j = 20 bytes; tombstone byte at 20 j + 19
        data[20 * j + 19] = (0, 1, 2, 255)[j % 4]
    ent = vbf.sst.load_entries(data, index)
    assert ent.tombstones.tolist() == [j % 4 == 1 for j in range(50)]
    _same(ent, ora.sst_decode(data))


def test_empty_and_malformed(vbf, ora):
    from velarixdb_amd import VbfError
    ent = vbf.sst.load_entries(b"", b"")
    assert len(ent) == 0 and ent.offsets.tolist() == [0]
    data, index, _ = _rand_sst(ora, 10, 1000, list(range(0, 60)))
    with pytest.raises(VbfError, match="malformed"):
        vbf.sst.load_entries(data[:-3], index)          # truncated last entry (UnexpectedEof)
    blocks = ora.sst_index_blocks(index)
    one = ora.sst_write(np.zeros(8, np.uint8), np.array([0, 8], np.uint64))[1]  # 1-block index
    # the whole file as ONE block of 1000 entries (~47 KB): load_entries reads entries sequentially
    # whatever the blocking (fs/mod.rs:275-332), and so does the decoder (dense-block path)
    assert data.size < 65536
    _same(vbf.sst.load_entries(data, one), ora.sst_decode(data))
    big, bigidx, _ = _rand_sst(ora, 11, 3000, list(range(20, 60)))
    assert big.size > 65535
    with pytest.raises(VbfError, match="larger than 65535"):
        vbf.sst.load_entries(big, one)                  # one block over the decoder's 64 KiB limit
    # an index offset pointing into the middle of an entry
    raw = bytearray(index.tobytes())
    L0 = int.from_bytes(raw[0:4], "little")
    raw[4 + L0:8 + L0] = int(blocks[0] + 1).to_bytes(4, "little")
    with pytest.raises(VbfError, match="malformed"):
        vbf.sst.load_entries(data, bytes(raw))
    with pytest.raises(VbfError):
        vbf.sst.load_entries(data, b"")                 # no block offsets for a non-empty file


def test_device_api_and_fused_rebuild(vbf, ora):
    """vbf_sst_decode_dev on torch buffers (count-only call, too-small outputs, full decode) and
    vbf_filter_rebuild_from_sst_dev == the oracle's build over the same keys."""
    import torch
    from velarixdb_amd._lib import VbfError, call
    n, L = 300_000, 16
    keys = np.ascontiguousarray(ora.gen_fixed(0x5EED0001, 0, n, L)).reshape(-1)
    offs = np.arange(n + 1, dtype=np.uint64) * L
    data, index = ora.sst_write(keys, offs)
    blocks = ora.sst_index_blocks(index)
    dev = torch.device("cuda:0")
    d = torch.from_numpy(data).to(dev)
    b = torch.from_numpy(blocks.view(np.int32)).to(dev)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cnt = ctypes.c_uint64()
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    call("vbf_sst_decode_dev", P(d), data.size, P(b), blocks.size, None, 0, None, None, None, None, 0,
         ctypes.byref(cnt), sp)
    assert cnt.value == n
    k_out = torch.empty(n * L, dtype=torch.uint8, device=dev)
    o_out = torch.empty(n + 1, dtype=torch.int64, device=dev)
    with pytest.raises(VbfError, match="offsets holds"):
        call("vbf_sst_decode_dev", P(d), data.size, P(b), blocks.size, P(k_out), n * L, P(o_out), None,
             None, None, n, ctypes.byref(cnt), sp)
    call("vbf_sst_decode_dev", P(d), data.size, P(b), blocks.size, P(k_out), n * L, P(o_out), None, None,
         None, n + 1, ctypes.byref(cnt), sp)
    torch.cuda.synchronize()
    assert np.array_equal(k_out.cpu().numpy(), keys)
    assert np.array_equal(o_out.cpu().numpy().view(np.uint64), offs)

    bf = vbf.BloomFilter(0.0081925494681790, n)
    m, k = bf.num_bits(), bf.no_of_hash_func
    assert bf.rebuild_from_sst_dev(P(d), data.size, P(b), blocks.size, sp) == n
    torch.cuda.synchronize()
    want = ora.build_words(vbf.pack_fixed(keys.reshape(n, L)), m, k, threads=8)
    assert np.array_equal(bf.words(), want)
    assert bf.num_elements() == n


@pytest.mark.parametrize("L", [16, 40, 1])
def test_gpu_sst_generator_matches_oracle_writer(vbf, ora, L):
    """vbf_gen_sst_fixed_dev writes the same data.db the oracle's Table::write_to_file does."""
    import torch
    from velarixdb_amd._lib import call
    n = 10_000
    per = 4096 // (L + 17)
    data = torch.empty(n * (L + 17), dtype=torch.uint8, device="cuda:0")
    blocks = torch.empty((n + per - 1) // per, dtype=torch.int32, device="cuda:0")
    call("vbf_gen_sst_fixed_dev", 0x5EED0001, 0, n, L, ctypes.c_void_p(data.data_ptr()),
         ctypes.c_void_p(blocks.data_ptr()), None)
    torch.cuda.synchronize()
    keys = np.ascontiguousarray(ora.gen_fixed(0x5EED0001, 0, n, L)).reshape(-1)
    j = np.arange(n, dtype=np.uint64)
    offs = np.arange(n + 1, dtype=np.uint64) * L
    want_d, want_i = ora.sst_write(keys, offs, j.astype(np.uint32), 1720785462000 + j,
                                   (j % 97 == 0).astype(np.uint8))
    assert np.array_equal(data.cpu().numpy(), want_d)
    assert blocks.cpu().numpy().view(np.uint32).tolist() == ora.sst_index_blocks(want_i).tolist()


def test_large_sst_decode_properties(vbf):
    """20M entries (660 MB data.db) decoded on the device: keys equal the generator's, offsets
    are j * L, and the fused rebuild equals a plain build over the same keys."""
    import torch
    from velarixdb_amd._lib import call
    n, L = 20_000_000, 16
    per = 4096 // (L + 17)
    nb = (n + per - 1) // per
    dev = torch.device("cuda:0")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    data = torch.empty(n * (L + 17), dtype=torch.uint8, device=dev)
    blocks = torch.empty(nb, dtype=torch.int32, device=dev)
    call("vbf_gen_sst_fixed_dev", 0x5EED0001, 0, n, L, P(data), P(blocks), None)
    keys = torch.empty(n * L, dtype=torch.uint8, device=dev)
    call("vbf_gen_fixed_dev", 0x5EED0001, 0, n, L, P(keys), None)
    out_k = torch.empty(n * L, dtype=torch.uint8, device=dev)
    out_o = torch.empty(n + 1, dtype=torch.int64, device=dev)
    out_v = torch.empty(n, dtype=torch.int32, device=dev)
    out_t = torch.empty(n, dtype=torch.uint8, device=dev)
    got = ctypes.c_uint64()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    call("vbf_sst_decode_dev", P(data), data.numel(), P(blocks), nb, P(out_k), n * L, P(out_o), P(out_v), None,
         P(out_t), n + 1, ctypes.byref(got), sp)
    torch.cuda.synchronize()
    assert got.value == n
    assert torch.equal(out_k, keys)
    assert torch.equal(out_o, torch.arange(n + 1, device=dev, dtype=torch.int64) * L)
    assert torch.equal(out_v, torch.arange(n, device=dev, dtype=torch.int32))
    assert torch.equal(out_t, (torch.arange(n, device=dev) % 97 == 0).to(torch.uint8))
    bf = vbf.BloomFilter(0.0081925494681790, n)
    assert bf.rebuild_from_sst_dev(P(data), data.numel(), P(blocks), nb, sp) == n
    ref = vbf.BloomFilter(0.0081925494681790, n)
    ref.set_dev(P(keys), None, L, n, 1, sp)
    torch.cuda.synchronize()
    assert np.array_equal(bf.words(), ref.words())


def test_uniform_guess_cannot_be_fooled(vbf, ora):
    """The walk's fixed-size fast path (entry i at i * (L0 + 17)) is verified at every predicted
    start.  Keys whose bytes spell LE32(16) everywhere, with lengths 16 and 20 mixed, put the
    first entry's length at many wrong offsets; the decode must still follow the real chain."""
    rng = np.random.default_rng(12)
    n = 30000
    L = rng.choice(np.array([16, 16, 16, 20], np.uint64), size=n)
    offs = np.concatenate([[0], np.cumsum(L)]).astype(np.uint64)
    keys = np.tile(np.frombuffer(np.uint32(16).tobytes(), np.uint8), int(offs[-1]) // 4 + 1)[: int(offs[-1])].copy()
    val = np.full(n, 16, np.uint32)
    created = np.full(n, 16, np.uint64)
    tomb = np.zeros(n, np.uint8)
    data, index = ora.sst_write(keys, offs, val, created, tomb)
    _same(vbf.sst.load_entries(data, index), (keys, offs, val, created, tomb))


def _entry(key, val, created, tomb):
    return len(key).to_bytes(4, "little") + key + val.to_bytes(4, "little") + created.to_bytes(8, "little") + bytes([tomb])


@pytest.mark.parametrize("layout", ["uniform", "mixed", "mixed_big"])
def test_dense_blocks_decode(vbf, ora, layout):
    """VERDICT r02 / ADVICE r01: DataFileNode::load_entries (fs/mod.rs:275-332) reads entries
    sequentially whatever the block size, so blocks of more than 256 entries (only hand-written
    files: the reference's 4096-byte blocks hold at most 4096 / 17 = 240) decode too: the walk
    counts on past 256 entries and the emit pass re-walks such a block.  Bit-exact against the
    oracle's sequential decode; blocks before and after it stay on the fast paths."""
    rng = np.random.default_rng({"uniform": 1, "mixed": 2, "mixed_big": 3}[layout])
    n, lens = {"uniform": (300, [0]), "mixed": (280, list(range(8))), "mixed_big": (1500, list(range(0, 40)))}[layout]
    body = b"".join(_entry(bytes(rng.integers(0, 256, size=int(rng.choice(lens)), dtype=np.uint8)),
                           int(rng.integers(0, 2**32)), int(rng.integers(0, 2**63)), int(rng.integers(0, 3)))
                    for _ in range(n))
    head = b"".join(_entry(b"k%05d" % i, i, 1720785462000 + i, 0) for i in range(100))  # ordinary block
    tail = b"".join(_entry(b"t%03d" % i, i, 7, 1) for i in range(50))
    data = head + body + tail
    blocks = [0, len(head), len(head) + len(body)]
    index = b"".join(len(b"x").to_bytes(4, "little") + b"x" + off.to_bytes(4, "little") for off in blocks)
    assert len(body) < 65536
    _same(vbf.sst.load_entries(data, index), ora.sst_decode(data))
    # the fused rebuild over the same file equals the build of the decoded keys
    from velarixdb_amd.keys import pack_offsets
    keys, offs, *_ = ora.sst_decode(data)
    f = vbf.BloomFilter.sized(200_003, 7)
    assert f.rebuild_from_sst(data, index) == offs.size - 1
    assert np.array_equal(f.words(), ora.build_words(pack_offsets(keys, offs), 200_003, 7))


def test_dense_block_crossing_its_end_is_an_error(vbf):
    from velarixdb_amd import VbfError
    data = _entry(b"", 7, 1, 0) * 300
    data = data[:-5]  # the last entry runs past the block (and file) end
    index = (0).to_bytes(4, "little") + (0).to_bytes(4, "little")
    with pytest.raises(VbfError, match="crosses the block end"):
        vbf.sst.load_entries(data, index)

