"""Key batches for the C ABI: packing Python keys the way Rust's `Hash` impls feed them.

Rust (velarixdb src/filter/bf.rs:84,95 take `impl Hash`):
  * `Vec<u8>` / `&[u8]` / `&Vec<u8>` -> LE64(len) || bytes  (len_prefix = 1; all production
    call sites: memtable/mem.rs:209-210,224,239,267, key_range/range.rs:130,136,171, bf.rs:127)
  * `usize` (bf.rs tests :300,:319)      -> LE64(v)           (len_prefix = 0)
  * `&Vec<i32>` (bf.rs test :287)         -> LE64(n) || LE32 x n (len_prefix = 0)
"""
import struct
from dataclasses import dataclass

import numpy as np


class Usize(int):
    """An integer key hashed as Rust `usize` (8 little-endian bytes, no length prefix)."""


class I32Vec(tuple):
    """A key hashed as Rust `&Vec<i32>`: LE64(len) || LE32 elements, no further prefix."""


class RawMessage(bytes):
    """Bytes fed to the hasher verbatim (no length prefix) -- any other pre-encoded Hash impl."""


def encode(key):
    """-> (message_bytes, len_prefix) for one key."""
    if isinstance(key, RawMessage):
        return bytes(key), 0
    if isinstance(key, (bytes, bytearray, memoryview)):
        return bytes(key), 1
    if isinstance(key, str):
        raise TypeError("str keys are ambiguous; pass key.encode() (Rust keys are Vec<u8>)")
    if isinstance(key, I32Vec):
        return struct.pack("<Q%di" % len(key), len(key), *key), 0
    if isinstance(key, (int, np.integer)):
        return struct.pack("<Q", int(key) & 0xFFFFFFFFFFFFFFFF), 0
    raise TypeError("unsupported key type %r" % type(key))


@dataclass
class HostBatch:
    """Keys packed in host memory: data + offsets (n+1, absolute) or a fixed stride."""
    data: np.ndarray          # uint8
    offsets: np.ndarray       # uint64[n+1] or None
    stride: int
    n: int
    len_prefix: int

    def ptrs(self):
        d = self.data.ctypes.data if self.data.size else None
        o = self.offsets.ctypes.data if self.offsets is not None else None
        return d, o


def pack(keys):
    """Pack an iterable of keys (bytes, or ints as usize, ...) into one HostBatch."""
    keys = list(keys)
    if not keys:
        return HostBatch(np.zeros(0, np.uint8), None, 0, 0, 1)
    msgs, lps = zip(*(encode(k) for k in keys))
    lp = lps[0]
    if any(x != lp for x in lps):
        raise ValueError("a batch must use one key encoding")
    lens = np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=len(msgs))
    data = np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()
    if lens.size and np.all(lens == lens[0]) and lens[0] > 0:
        return HostBatch(data, None, int(lens[0]), len(msgs), lp)
    offsets = np.zeros(len(msgs) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    return HostBatch(data, offsets, 0, len(msgs), lp)


def pack_fixed(arr, len_prefix=1):
    """A 2-D uint8 array [n, L] of fixed-length keys."""
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    n, L = arr.shape
    return HostBatch(arr.reshape(-1), None, L, n, len_prefix)


def pack_offsets(data, offsets, len_prefix=1):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    return HostBatch(data, offsets, 0, len(offsets) - 1, len_prefix)
