"""CPU oracle for velarixdb's Bloom-filter path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.  It is
the checker, never the thing measured or shipped.  See oracle.c for the reference anchors
(bf.rs file:line) and tests/golden/ for the vectors that pin it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "liboracle.so")


def build():
    src = os.path.join(HERE, "oracle.c")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return SO


def _load():
    if not os.path.exists(SO):
        build()
    L = ctypes.CDLL(SO)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.ora_siphash13.restype = u64
    L.ora_siphash13.argtypes = [vp, ctypes.c_size_t]
    L.ora_hash.restype = u64
    L.ora_hash.argtypes = [vp, ctypes.c_size_t, i, u64]
    L.ora_num_bits.restype = u32
    L.ora_num_bits.argtypes = [u64, ctypes.c_double]
    L.ora_num_hash.restype = u32
    L.ora_num_hash.argtypes = [u32, u32]
    L.ora_build.restype = i
    L.ora_build.argtypes = [vp, vp, u64, u64, i, u32, u32, vp]
    L.ora_build_mt.restype = i
    L.ora_build_mt.argtypes = [vp, vp, u64, u64, i, u32, u32, vp, i]
    L.ora_probe.restype = i
    L.ora_probe.argtypes = [vp, vp, u64, u64, i, u32, u32, vp, vp]
    L.ora_probe_mt.restype = i
    L.ora_probe_mt.argtypes = [vp, vp, u64, u64, i, u32, u32, vp, vp, i]
    L.ora_hashes.restype = None
    L.ora_hashes.argtypes = [vp, vp, u64, u64, i, u32, vp]
    L.ora_splitmix64.restype = u64
    L.ora_splitmix64.argtypes = [u64]
    L.ora_gen_fixed.restype = None
    L.ora_gen_fixed.argtypes = [u64, u64, u64, u32, vp]
    L.ora_gen_var_len.restype = u32
    L.ora_gen_var_len.argtypes = [u64, u64]
    L.ora_gen_var.restype = None
    L.ora_gen_var.argtypes = [u64, u64, u64, vp, vp]
    L.ora_sst_write.restype = i
    L.ora_sst_write.argtypes = [vp, vp, u64, vp, vp, vp, vp, vp, vp, vp]
    L.ora_sst_decode.restype = ctypes.c_int64
    L.ora_sst_decode.argtypes = [vp, u64, vp, vp, vp, vp, vp]
    L.ora_sst_index_blocks.restype = ctypes.c_int64
    L.ora_sst_index_blocks.argtypes = [vp, u64, vp]
    L.ora_tmap_new.restype = vp
    L.ora_tmap_new.argtypes = []
    L.ora_tmap_free.restype = None
    L.ora_tmap_free.argtypes = [vp]
    L.ora_tmap_set.restype = None
    L.ora_tmap_set.argtypes = [vp, vp, u64, ctypes.c_int64]
    L.ora_tmap_get.restype = i
    L.ora_tmap_get.argtypes = [vp, vp, u64, vp]
    L.ora_tmap_size.restype = u64
    L.ora_tmap_size.argtypes = [vp]
    L.ora_tmap_dump.restype = u64
    L.ora_tmap_dump.argtypes = [vp, vp, vp, vp]
    L.ora_compact_merge.restype = ctypes.c_int64
    L.ora_compact_merge.argtypes = [vp, vp, vp, vp, vp, u32, i, u64, u64, u64, vp, vp]
    return L


lib = _load()


def siphash13(msg: bytes) -> int:
    return lib.ora_siphash13(msg, len(msg))


def calc_hash(key: bytes, seed: int, len_prefix: int = 1) -> int:
    return lib.ora_hash(key, len(key), len_prefix, seed)


def num_bits(n, p):
    return int(lib.ora_num_bits(n, p))


def num_hash(m, n):
    return int(lib.ora_num_hash(m, n & 0xFFFFFFFF))


def _ptrs(batch):
    d = batch.data.ctypes.data if batch.data.size else None
    o = batch.offsets.ctypes.data if batch.offsets is not None else None
    return d, o


def build_words(batch, m, k, words=None, threads=1):
    """OR the batch into `words` (new zeroed array when None); returns the words."""
    if words is None:
        words = np.zeros((m + 31) // 32, dtype=np.uint32)
    d, o = _ptrs(batch)
    wp = words.ctypes.data if words.size else None
    if threads > 1:
        rc = lib.ora_build_mt(d, o, batch.stride, batch.n, batch.len_prefix, m, k, wp, threads)
    else:
        rc = lib.ora_build(d, o, batch.stride, batch.n, batch.len_prefix, m, k, wp)
    if rc:
        raise ZeroDivisionError("m == 0 with k > 0")
    return words


def probe(batch, m, k, words, threads=1):
    out = np.zeros(batch.n, dtype=np.uint8)
    d, o = _ptrs(batch)
    args = (d, o, batch.stride, batch.n, batch.len_prefix, m, k,
            words.ctypes.data if words.size else None, out.ctypes.data if out.size else None)
    rc = lib.ora_probe_mt(*args, threads) if threads > 1 else lib.ora_probe(*args)
    if rc:
        raise ZeroDivisionError("m == 0 with k > 0")
    return out


def hashes(batch, k):
    out = np.zeros(batch.n * k, dtype=np.uint64)
    d, o = _ptrs(batch)
    lib.ora_hashes(d, o, batch.stride, batch.n, batch.len_prefix, k, out.ctypes.data if out.size else None)
    return out.reshape(batch.n, k)


def gen_fixed(seed, base, n, length):
    out = np.zeros(n * length, dtype=np.uint8)
    lib.ora_gen_fixed(seed, base, n, length, out.ctypes.data if out.size else None)
    return out


def gen_var_lengths(seed, base, n):
    return np.array([lib.ora_gen_var_len(seed, base + j) for j in range(n)], dtype=np.uint64)


def gen_var(seed, base, offsets):
    """Bytes for keys base..base+n-1 laid out at offsets (offsets[0] == 0)."""
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    out = np.zeros(int(offsets[-1]), dtype=np.uint8)
    lib.ora_gen_var(seed, base, n, offsets.ctypes.data, out.ctypes.data if out.size else None)
    return out


def _p(a):
    return a.ctypes.data if a is not None and a.size else None


def sst_write(keys, offsets, val_off=None, created_ms=None, tomb=None):
    """Table::write_to_file (table.rs:280-338) -> (data.db bytes, index.db bytes)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    arrs = [None if a is None else np.ascontiguousarray(a, dtype=t)
            for a, t in ((val_off, np.uint32), (created_ms, np.uint64), (tomb, np.uint8))]
    dl, il = ctypes.c_uint64(), ctypes.c_uint64()
    args = [_p(keys), _p(offsets), n] + [_p(a) for a in arrs]
    if lib.ora_sst_write(*args, None, ctypes.byref(dl), None, ctypes.byref(il)) != 0:
        raise ValueError("entry larger than a 4096-byte block (BlockIsFull)")
    data = np.zeros(dl.value, dtype=np.uint8)
    index = np.zeros(il.value, dtype=np.uint8)
    lib.ora_sst_write(*args, _p(data), ctypes.byref(dl), _p(index), ctypes.byref(il))
    return data, index


def sst_decode(data):
    """DataFileNode::load_entries (fs/mod.rs:275-332) -> (keys, offsets, val_off, created_ms, tomb)."""
    data = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    n = lib.ora_sst_decode(_p(data), data.size, None, None, None, None, None)
    if n < 0:
        raise EOFError("unexpected EOF in data.db")
    keys = np.zeros(data.size - 17 * n, dtype=np.uint8)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    val = np.zeros(n, dtype=np.uint32)
    created = np.zeros(n, dtype=np.uint64)
    tomb = np.zeros(n, dtype=np.uint8)
    lib.ora_sst_decode(_p(data), data.size, _p(keys), offsets.ctypes.data, _p(val), _p(created), _p(tomb))
    return keys, offsets, val, created, tomb


def sst_index_blocks(index):
    """index.db (indexer.rs:151-170) -> u32 block start offsets."""
    index = np.frombuffer(bytes(index), dtype=np.uint8) if not isinstance(index, np.ndarray) else index
    nb = lib.ora_sst_index_blocks(_p(index), index.size, None)
    if nb < 0:
        raise EOFError("unexpected EOF in index.db")
    offs = np.zeros(nb, dtype=np.uint32)
    lib.ora_sst_index_blocks(_p(index), index.size, _p(offs))
    return offs


class TombstoneMap:
    """The compactor's `tombstones: HashMap<Key, CreatedAt>` (compactors/sized.rs:36)."""

    def __init__(self, items=None):
        self.h = lib.ora_tmap_new()
        for k, t in (items or {}).items():
            self[k] = t

    def __del__(self):
        if getattr(self, "h", None):
            lib.ora_tmap_free(self.h)
            self.h = None

    def __setitem__(self, key, t):
        lib.ora_tmap_set(self.h, key, len(key), int(t))

    def get(self, key):
        t = ctypes.c_int64()
        return t.value if lib.ora_tmap_get(self.h, key, len(key), ctypes.byref(t)) else None

    def __len__(self):
        return lib.ora_tmap_size(self.h)

    def items(self):
        n = len(self)
        lens = np.zeros(n, np.uint64)
        times = np.zeros(n, np.int64)
        kb = lib.ora_tmap_dump(self.h, None, None, None)
        keys = np.zeros(max(kb, 1), np.uint8)
        lib.ora_tmap_dump(self.h, keys.ctypes.data, _p(lens), _p(times))
        out, o = {}, 0
        for L, t in zip(lens.tolist(), times.tolist()):
            out[keys[o:o + L].tobytes()] = t
            o += L
        return out


def compact_merge(keys, offsets, created, tomb, run_off, use_ttl=False, entry_ttl_ms=0,
                  tomb_ttl_ms=0, now_ms=0, tmap=None):
    """One bucket through merge_ssts_in_buckets' fold (sized.rs:170-320) -> merged entry ids."""
    keys = np.ascontiguousarray(keys, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    created = np.ascontiguousarray(created, np.int64)
    tomb = np.ascontiguousarray(tomb, np.uint8)
    run_off = np.ascontiguousarray(run_off, np.uint64)
    tmap = tmap if tmap is not None else TombstoneMap()
    out = np.zeros(max(int(run_off[-1]), 1), np.uint32)
    n = lib.ora_compact_merge(_p(keys), offsets.ctypes.data, _p(created), _p(tomb), run_off.ctypes.data,
                              run_off.size - 1, int(use_ttl), entry_ttl_ms, tomb_ttl_ms, now_ms, tmap.h,
                              out.ctypes.data)
    return out[:n]
