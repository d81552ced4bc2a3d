"""CPU checks for the SST data.db / index.db path: the oracle's writer and
decoder are pinned by the reference's own SST fixtures (src/tests/fixtures/.../sstable_*), and the
product's host-side index.db parser (no kernel) is checked against the oracle."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

SST = os.path.join(GOLDEN, "sst_fixtures")
NAMES = sorted(os.listdir(SST))


def _files(name):
    d = os.path.join(SST, name)
    return open(os.path.join(d, "data.db"), "rb").read(), open(os.path.join(d, "index.db"), "rb").read()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_writer_reproduces_reference_files(ora, name):
    """decode(data.db) then Table::write_to_file (table.rs:280-338) gives back the reference's
    data.db AND index.db byte for byte: pins the entry format, the 4096-byte block policy
    (block_manager.rs:112-139) and the index records (indexer.rs:151-170)."""
    data, index = _files(name)
    keys, offs, val, created, tomb = ora.sst_decode(data)
    assert offs.size - 1 in (2844, 2845)
    d2, i2 = ora.sst_write(keys, offs, val, created, tomb)
    assert d2.tobytes() == data and i2.tobytes() == index
    ks = [keys[offs[j]:offs[j + 1]].tobytes() for j in range(offs.size - 1)]
    assert ks == sorted(set(ks))  # a SkipMap flushed in order: sorted and unique


def test_oracle_decode_matches_fixture_golden(ora, golden):
    """Decoded key counts agree with the digests recorded from the fixtures."""
    want = {s["name"]: s for s in golden("sst_fixtures")["ssts"]}
    for name in NAMES:
        data, _ = _files(name)
        keys, offs, *_ = ora.sst_decode(data)
        assert offs.size - 1 == want[name]["n_keys"]


def test_oracle_writer_block_policy(ora):
    """An entry that does not fit the open block starts a new one; one over 4096 bytes fails
    the flush (set_entry returns BlockIsFull on an empty block)."""
    L = np.array([4079, 0, 4078, 1, 5], dtype=np.uint64)  # 4079 + 17 = 4096 exactly
    offs = np.concatenate([[0], np.cumsum(L)]).astype(np.uint64)
    keys = (np.arange(int(offs[-1])) % 251).astype(np.uint8)
    data, index = ora.sst_write(keys, offs)
    blocks = ora.sst_index_blocks(index)
    # block 0 = entry 0 (4096 B); entry 1 (17 B) + entry 2 (4095 B) = 4112 > 4096 -> split
    assert blocks.tolist() == [0, 4096, 4113, 4113 + 4095]
    with pytest.raises(ValueError):
        ora.sst_write(np.zeros(4080, np.uint8), np.array([0, 4080], np.uint64))


def test_product_index_parser_matches_oracle(ora):
    from velarixdb_amd import sst
    for name in NAMES:
        _, index = _files(name)
        assert sst.index_blocks(index).tolist() == ora.sst_index_blocks(index).tolist()
    assert sst.index_blocks(b"").size == 0
    from velarixdb_amd import VbfError
    with pytest.raises(VbfError):
        sst.index_blocks(_files(NAMES[0])[1][:-2])
