"""Compaction merge on the GPU: the step before the build on the
compaction path.

Mirrors the merge half of SizedTierRunner (src/compactors/sized.rs):

  SizedTierMerger(config)                       SizedTierRunner::new (:40-50), `tombstones` map (:36)
  .merge_bucket(tables, now_ms)                 merge_ssts_in_buckets for one bucket (:170-200):
      -> (SstEntries merged, BloomFilter)          the pairwise fold of merge_sstables (:207-283)
                                                   with tombstone_check (:286-320), then
                                                   BloomFilter::new(p, n) + build (:192-193)
  .clear_tombstones()                           run_compaction's clear when nothing is left (:73-75)
  build_filters_sharded(batches, p, devices)    the fan-in's per-table filter builds (:192-193 for
                                                   every merged table), one table per device

The fold runs on the device (C ABI vbf_compact_merge_host); it returns the merged entries as
ids into the input tables -- what a Rust caller maps back onto its own Entry values -- and the
map updates.  Entry::has_expired reads the clock (memtable/mem.rs:149-153); here `now_ms` is an
argument (default: the current time), so results are reproducible.
"""
import ctypes
import time
from dataclasses import dataclass

import numpy as np

from ._lib import call
from .filter import DEFAULT_FALSE_POSITIVE_RATE, BloomFilter
from .keys import pack_offsets
from .sst import SstEntries

ENTRY_TTL_MS = 365 * 86400000            # consts/mod.rs:63
DEFAULT_TOMBSTONE_TTL_MS = 120 * 86400000  # consts/mod.rs:67
DEFAULT_ENABLE_TTL = False               # consts/mod.rs:69


@dataclass
class CompactionConfig:
    use_ttl: bool = DEFAULT_ENABLE_TTL
    entry_ttl_ms: int = ENTRY_TTL_MS
    tombstone_ttl_ms: int = DEFAULT_TOMBSTONE_TTL_MS
    filter_false_positive: float = DEFAULT_FALSE_POSITIVE_RATE


def _arena(tables):
    keys = np.concatenate([t.keys[int(t.offsets[0]):int(t.offsets[-1])] for t in tables]) if tables \
        else np.zeros(0, np.uint8)
    offs, run_off, base = [np.zeros(1, np.uint64)], [0], 0
    for t in tables:
        o = t.offsets.astype(np.uint64)
        offs.append(o[1:] - o[0] + base)
        base += int(o[-1] - o[0])
        run_off.append(run_off[-1] + len(t))
    offsets = np.concatenate(offs)
    created = np.concatenate([t.created_ms.astype(np.int64) for t in tables]) if tables else np.zeros(0, np.int64)
    tomb = np.concatenate([t.tombstones.astype(np.uint8) for t in tables]) if tables else np.zeros(0, np.uint8)
    val = np.concatenate([t.val_offsets.astype(np.uint32) for t in tables]) if tables else np.zeros(0, np.uint32)
    return keys, offsets, created, tomb, val, np.asarray(run_off, np.uint64)


def _p(a):
    return a.ctypes.data if a is not None and a.size else None


class SizedTierMerger:
    def __init__(self, config=None, device=0):
        self.config = config or CompactionConfig()
        self.device = device
        self.tombstones = {}  # key -> created_at ms of the newest tombstone seen

    def clear_tombstones(self):
        self.tombstones.clear()

    def merge_ids(self, tables, now_ms=None):
        """The fold for one bucket -> (arena, ids of the merged entries in key order)."""
        arena = _arena(tables)
        keys, offsets, created, tomb, val, run_off = arena
        total = int(run_off[-1])
        mk = sorted(self.tombstones)
        mkeys = np.frombuffer(b"".join(mk) or b"\0", np.uint8)
        moff = np.concatenate([[0], np.cumsum([len(k) for k in mk], dtype=np.uint64)]).astype(np.uint64)
        mtime = np.asarray([self.tombstones[k] for k in mk], np.int64)
        ids = np.zeros(max(total, 1), np.uint32)
        upd_ids = np.zeros(max(total, 1), np.uint32)
        upd_t = np.zeros(max(total, 1), np.int64)
        n_out, n_upd = ctypes.c_uint64(), ctypes.c_uint64()
        now = int(time.time() * 1000) if now_ms is None else int(now_ms)
        c = self.config
        call("vbf_compact_merge_host", _p(keys), _p(offsets), _p(created), _p(tomb), run_off.ctypes.data,
             len(tables), _p(mkeys) if mk else None, moff.ctypes.data if mk else None, _p(mtime), len(mk),
             int(c.use_ttl), c.entry_ttl_ms, c.tombstone_ttl_ms, now, ids.ctypes.data, ctypes.byref(n_out),
             upd_ids.ctypes.data, upd_t.ctypes.data, ctypes.byref(n_upd), self.device)
        for e, t in zip(upd_ids[:n_upd.value].tolist(), upd_t[:n_upd.value].tolist()):
            self.tombstones[keys[int(offsets[e]):int(offsets[e + 1])].tobytes()] = t
        return arena, ids[:n_out.value]

    def merge_bucket(self, tables, now_ms=None):
        """merge_ssts_in_buckets for one bucket: the merged table's entries and its filter,
        BloomFilter::new(filter_false_positive, n) built over them (sized.rs:192-193)."""
        (keys, offsets, created, tomb, val, _), ids = self.merge_ids(tables, now_ms)
        lens = (offsets[ids.astype(np.int64) + 1] - offsets[ids]).astype(np.int64)
        out_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        src = np.repeat(offsets[ids].astype(np.int64) - out_off[:-1].astype(np.int64), lens) + \
            np.arange(int(out_off[-1]), dtype=np.int64)
        merged = SstEntries(keys[src], out_off, val[ids], created[ids].astype(np.uint64), tomb[ids].astype(bool))
        # an empty merge reaches BloomFilter::new(p, 0), whose assert fires (bf.rs:67): AssertionError
        bf = BloomFilter(self.config.filter_false_positive, len(merged), device=self.device)
        bf.set_batch(pack_offsets(merged.keys, merged.offsets))
        return merged, bf


class _Shard(ctypes.Structure):
    """struct vbf_shard (include/vbf.h)."""
    _fields_ = [("keys", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("stride", ctypes.c_uint64),
                ("n", ctypes.c_uint64), ("len_prefix", ctypes.c_int), ("m", ctypes.c_uint32),
                ("k", ctypes.c_uint32), ("words", ctypes.c_void_p), ("nwords", ctypes.c_uint64),
                ("status", ctypes.c_int)]


def build_filters_sharded(batches, false_positive_rate=DEFAULT_FALSE_POSITIVE_RATE, devices=(0,)):
    """Independent filter builds for the tables a compaction produced (sized.rs:192-193, once
    per merged table), spread over `devices` with one host thread per device
    (vbf_build_shards_host).  batches: HostBatch per table.  Returns a list of
    (m, k, words) with words the host bit array (bit-vec BitVec<u32> layout)."""
    from .filter import num_bits, num_hash_functions
    out, shards, keep = [], (_Shard * max(1, len(batches)))(), []
    for i, b in enumerate(batches):
        m = num_bits(max(b.n, 1), false_positive_rate)
        k = num_hash_functions(m, max(b.n, 1))
        words = np.zeros((m + 31) // 32, np.uint32)
        d, o = b.ptrs()
        shards[i] = _Shard(d, o, b.stride, b.n, b.len_prefix, m, k, words.ctypes.data, words.size, 0)
        out.append((m, k, words))
        keep.append(b)
    devs = (ctypes.c_int * len(devices))(*devices)
    call("vbf_build_shards_host", ctypes.cast(shards, ctypes.c_void_p), len(batches), ctypes.cast(devs, ctypes.c_void_p),
         len(devices))
    return out
