"""SST `data.db` decode on the GPU: the step before the build on the
recovery path.

velarixdb rebuilds a filter whose bits were lost by reading the SST's data.db entry by entry
into a SkipMap (DataFileNode::load_entries, src/fs/mod.rs:275-332) and hashing every key
(src/key_range/range.rs:117-128).  Here the file is decoded block-parallel on the device
(velarixdb_amd/csrc/vbf_sst.hip) straight into the build's key layout, using the block offsets
index.db already records (src/index/indexer.rs:151-170, src/sst/table.rs:331-338).

  load_entries(data, index)      -> SstEntries   fs/mod.rs:275-332 (file order; the SST writer
                                                  emits a SkipMap in order, so keys are sorted
                                                  and unique, as in the reference's SkipMap)
  load_entries_from_dir(sst_dir) -> SstEntries   Table::load_entries_from_file (table.rs:197-205)
  index_blocks(index)            -> u32 offsets  one per block
  BloomFilter.rebuild_from_sst(data, index)      range.rs:117-128, see filter.py
"""
import ctypes
import os

import numpy as np

from ._lib import call

DATA_FILE_NAME = "data"    # consts/mod.rs
INDEX_FILE_NAME = "index"  # consts/mod.rs


def _buf(b):
    a = np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray, memoryview)) else \
        np.ascontiguousarray(b, dtype=np.uint8)
    return a, (a.ctypes.data if a.size else None)


class SstEntries:
    """Decoded entries: key j = keys[offsets[j]:offsets[j+1]], plus value offset, creation time
    (ms since the epoch, as stored) and tombstone flag per entry."""

    def __init__(self, keys, offsets, val_offsets, created_ms, tombstones):
        self.keys, self.offsets = keys, offsets
        self.val_offsets, self.created_ms, self.tombstones = val_offsets, created_ms, tombstones

    def __len__(self):
        return self.offsets.size - 1

    def key(self, j):
        return self.keys[int(self.offsets[j]):int(self.offsets[j + 1])].tobytes()

    def key_list(self):
        return [self.key(j) for j in range(len(self))]


def index_blocks(index):
    """index.db bytes -> block start offsets (u32), one per block."""
    a, p = _buf(index)
    nb = ctypes.c_uint64()
    call("vbf_sst_index_blocks", p, a.size, None, 0, ctypes.byref(nb))
    out = np.zeros(nb.value, dtype=np.uint32)
    if nb.value:
        call("vbf_sst_index_blocks", p, a.size, out.ctypes.data, out.size, ctypes.byref(nb))
    return out


def count_entries(data, index, device=0):
    a, pa = _buf(data)
    b, pb = _buf(index)
    n = ctypes.c_uint64()
    call("vbf_sst_decode_host", pa, a.size, pb, b.size, None, 0, None, None, None, None, 0,
         ctypes.byref(n), device)
    return n.value


def load_entries(data, index, device=0):
    """DataFileNode::load_entries (fs/mod.rs:275-332), decoded on `device`."""
    a, pa = _buf(data)
    b, pb = _buf(index)
    n = count_entries(a, b, device)
    keys = np.zeros(a.size - 17 * n, dtype=np.uint8)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    val = np.zeros(n, dtype=np.uint32)
    created = np.zeros(n, dtype=np.uint64)
    tomb = np.zeros(n, dtype=np.uint8)
    got = ctypes.c_uint64()
    vp = lambda x: x.ctypes.data if x.size else None
    call("vbf_sst_decode_host", pa, a.size, pb, b.size, vp(keys), keys.size, offsets.ctypes.data,
         vp(val), vp(created), vp(tomb), n + 1, ctypes.byref(got), device)
    assert got.value == n
    return SstEntries(keys, offsets, val, created, tomb.astype(bool))


def read_sst_files(sst_dir):
    with open(os.path.join(sst_dir, DATA_FILE_NAME + ".db"), "rb") as f:
        data = f.read()
    with open(os.path.join(sst_dir, INDEX_FILE_NAME + ".db"), "rb") as f:
        index = f.read()
    return data, index


def load_entries_from_dir(sst_dir, device=0):
    """Table::load_entries_from_file (sst/table.rs:197-205) for the SST directory `sst_dir`."""
    return load_entries(*read_sst_files(sst_dir), device=device)
