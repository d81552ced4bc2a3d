"""Batched read-path probe across SSTs.

velarixdb's get walks its key ranges one key at a time: an SST is a candidate when the key lies
in [smallest_key, biggest_key] and the SST's filter contains it
(KeyRange::filter_sstables_by_key_range, src/key_range/range.rs:91-147).  Here a whole batch
of keys is tested against every SST in one launch (C ABI vbf_multi_probe_*), each key hashed
once for all filters.

  SstRange(smallest_key, biggest_key, filter)          key_range/range.rs `Range`
  candidates(keys, ranges)      -> bool [n, nsst]      range test && filter.contains (:118, :136)
  filter_sstables_many(keys, ranges) -> [[s, ...], ...] per key, in `ranges` order
  contains_all(keys, filters)   -> bool [n, nsst]      filters only, no range test
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import call
from .filter import BloomFilter, _raise
from ._lib import VbfError
from .keys import HostBatch, pack


@dataclass
class SstRange:
    smallest_key: bytes
    biggest_key: bytes
    filter: BloomFilter


def _bounds(ranges):
    parts, offs = [], [0]
    for r in ranges:
        for b in (bytes(r.smallest_key), bytes(r.biggest_key)):
            parts.append(b)
            offs.append(offs[-1] + len(b))
    raw = np.frombuffer(b"".join(parts) or b"\0", dtype=np.uint8)
    return raw, np.asarray(offs, dtype=np.uint64)


def _probe(batch: HostBatch, filters, bounds=None, bounds_off=None):
    nsst = len(filters)
    out = np.zeros((batch.n, nsst), dtype=np.uint8)
    handles = (ctypes.c_void_p * max(nsst, 1))(*[f._h.value for f in filters])
    d, o = batch.ptrs()
    try:
        call("vbf_multi_probe_host", d, o, batch.stride, batch.n, batch.len_prefix, nsst, handles,
             bounds.ctypes.data if bounds is not None else None,
             bounds_off.ctypes.data if bounds_off is not None else None,
             out.ctypes.data if out.size else None)
    except VbfError as e:
        _raise("multi_probe", e)
    return out.astype(bool)


def candidates(keys, ranges):
    """bool [n, len(ranges)]: key j in range s and filter s contains key j."""
    b = keys if isinstance(keys, HostBatch) else pack(keys)
    raw, offs = _bounds(ranges)
    return _probe(b, [r.filter for r in ranges], raw, offs)


def contains_all(keys, filters):
    """bool [n, len(filters)]: filters[s].contains(key j), each key hashed once."""
    b = keys if isinstance(keys, HostBatch) else pack(keys)
    return _probe(b, list(filters))


def filter_sstables_many(keys, ranges):
    """Per key, the indices of the candidate SSTs (range.rs:91-147 for a batch of keys)."""
    c = candidates(keys, ranges)
    return [np.flatnonzero(row).tolist() for row in c]
