"""BloomFilter -- velarixdb's src/filter API on the gfx950 engine (C ABI in include/vbf.h).

Mirrors /root/reference/src/filter/bf.rs (velarixdb 0.0.17) method for method, with the bit
array resident in HBM.  Argument checks raise where the reference asserts or panics:

  BloomFilter::new(p, n)            bf.rs:62-81    -> BloomFilter(p, n)       AssertionError
  set(key)                          bf.rs:84-92    -> set(key)                ZeroDivisionError
  contains(key)                     bf.rs:95-105   -> contains(key)           (m == 0 and k > 0)
  write(dir)                        bf.rs:114-123  -> write(dir)
  build_filter_from_entries(e)      bf.rs:126-128  -> build_filter_from_entries(e)  (one batch)
  recover_meta()                    bf.rs:135-150  -> recover_meta()
  serialize()                       bf.rs:158-172  -> serialize()
  set_sstable_path / clear          bf.rs:175-195
  num_elements / num_bits / num_of_hash_functions / get_sst_dir  bf.rs:198-219
  Clone (shares the bit array)      bf.rs:242-254  -> clone() / copy.copy()
  Default                           bf.rs:256-267  -> BloomFilter.default()

Batch forms (set_many / contains_many and the *_dev variants taking device pointers) are the
accelerated entry points the compaction build (compactors/sized.rs:192-193), the lazy
recovery rebuild (key_range/range.rs:117-128) and bulk probes use.

Residency: `device` is a GPU index (bits in HBM, kernels), "auto" (the library picks a GPU,
round-robin) or HOST (bits in host memory, set / contains on the CPU inside libvbf with the
kernels' SipHash rounds) -- the memtable's filter, one contains + set per put
(memtable/mem.rs:207-221).  migrate() moves the bits in place.  A device-resident filter keeps a
host mirror of its bits, so single-key contains (the read path, range.rs:130,136,171) answer on
the CPU; set_mirror() tunes it.
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import (VBF_DEVICE_AUTO, VBF_DEVICE_HOST, VBF_EDIVZERO, VBF_EINVAL, VBF_EXT_NONE, VBF_MIRROR_EAGER,
                   VBF_MIRROR_LAZY, VBF_MIRROR_OFF, VbfError, call, lib)
from .keys import HostBatch, encode, pack

FILTER_FILE_NAME = "filter"  # consts/mod.rs:27
DEFAULT_FALSE_POSITIVE_RATE = 1e-4  # consts/mod.rs:17
HOST = VBF_DEVICE_HOST  # device= for a host-resident (memtable) filter
AUTO = VBF_DEVICE_AUTO  # device= for library placement (round-robin over the GPUs)
MIRROR_MODES = {"off": VBF_MIRROR_OFF, "lazy": VBF_MIRROR_LAZY, "eager": VBF_MIRROR_EAGER}


def _dev(device):
    if device == "host":
        return VBF_DEVICE_HOST
    if device == "auto":
        return VBF_DEVICE_AUTO
    return int(device)


def num_bits(n, p):
    """calculate_no_of_bits (bf.rs:230-233)."""
    return int(lib.vbf_num_bits(n, p))


def num_hash_functions(m, n):
    """calculate_no_of_hash_function (bf.rs:236-239); n is `as u32`."""
    return int(lib.vbf_num_hash_functions(m, n & 0xFFFFFFFF))


# zero-copy asynchronous sets: the batches the library still reads, released by its worker
_INFLIGHT = {}
_INFLIGHT_IDS = __import__("itertools").count(1)


@ctypes.CFUNCTYPE(None, ctypes.c_void_p)
def _release(ctx):
    _INFLIGHT.pop(ctx, None)


_RELEASE_PTR = ctypes.cast(_release, ctypes.c_void_p)

# A forked child inherits _INFLIGHT, but the jobs behind those entries never run there (the
# library reports them as failed, vbf.h), so nothing would ever release them: the child forgets
# them instead of waiting 60 s for them at exit.
if hasattr(os, "register_at_fork"):
    os.register_at_fork(after_in_child=_INFLIGHT.clear)


@__import__("atexit").register
def _drain_inflight():
    """At interpreter exit, wait for the zero-copy jobs still queued: the library's worker would
    otherwise call _release (Python code) after the interpreter is gone."""
    import time
    for _, f in list(_INFLIGHT.values()):
        try:
            lib.vbf_filter_sync(f._h)  # a failed job's status is of no use at exit
        except Exception:  # noqa: BLE001
            pass
    t_end = time.monotonic() + 60
    while _INFLIGHT and time.monotonic() < t_end:  # the callbacks run just after the jobs
        time.sleep(0.001)


def _raise(fn, exc):
    code = exc.code
    if code == VBF_EDIVZERO:
        raise ZeroDivisionError("attempt to calculate the remainder with a divisor of zero "
                                "(bf.rs:88): %s" % exc) from None
    if code == VBF_EINVAL:
        raise AssertionError(str(exc)) from None
    raise exc


class BloomFilter:
    """A Bloom filter whose bits live in MI355X HBM; see the module docstring."""

    def __init__(self, false_positive_rate=None, no_of_elements=None, device=0, _handle=None):
        self.sst_dir = None
        self.file_path = None
        self.bits_restored = False
        if _handle is not None:
            self._h = _handle
            return
        h = ctypes.c_void_p()
        try:
            call("vbf_filter_new", float(false_positive_rate), int(no_of_elements), _dev(device), ctypes.byref(h))
        except VbfError as e:
            _raise("new", e)
        self._h = h

    # -- constructors ------------------------------------------------------------------
    @classmethod
    def default(cls, device=0):
        h = ctypes.c_void_p()
        call("vbf_filter_default", _dev(device), ctypes.byref(h))
        return cls(_handle=h)

    @classmethod
    def sized(cls, m, k, false_positive_rate=0.0, device=0):
        """A filter of exactly m bits and k hash functions (the struct's pub fields set directly)."""
        h = ctypes.c_void_p()
        call("vbf_filter_new_sized", int(m), int(k), float(false_positive_rate), _dev(device), ctypes.byref(h))
        return cls(_handle=h)

    def clone(self):
        h = ctypes.c_void_p()
        call("vbf_filter_clone", self._h, ctypes.byref(h))
        c = BloomFilter(_handle=h)
        c.sst_dir, c.file_path = self.sst_dir, self.file_path
        return c

    __copy__ = clone

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.vbf_filter_free(h)
            self._h = None

    # -- fields (bf.rs:38-58) ------------------------------------------------------------
    @property
    def no_of_hash_func(self):
        return int(lib.vbf_filter_num_hash_functions(self._h))

    @property
    def no_of_elements(self):
        return int(lib.vbf_filter_num_elements(self._h))

    @property
    def false_positive_rate(self):
        return float(lib.vbf_filter_false_positive_rate(self._h))

    @property
    def device(self):
        return int(lib.vbf_filter_device(self._h))

    @property
    def host_resident(self):
        return self.device == VBF_DEVICE_HOST

    @property
    def host_bytes(self):
        """Host memory the bits hold (vbf_filter_host_bytes): host words are allocated on first use."""
        return int(lib.vbf_filter_host_bytes(self._h))

    def migrate(self, device):
        """Move the (shared) bit array to GPU `device` or to host memory ("host"), in place."""
        call("vbf_filter_migrate", self._h, _dev(device))
        return self

    def set_sst_entries(self, n):
        """Record the entry count of the SST this filter was built from (handle bookkeeping that
        the Rust binding's write() hands to serialize_ext; vbf_filter_set_sst_entries)."""
        call("vbf_filter_set_sst_entries", self._h, VBF_EXT_NONE if n is None else int(n))

    @property
    def sst_entries(self):
        v = int(lib.vbf_filter_sst_entries(self._h))
        return None if v == VBF_EXT_NONE else v

    def take_restored(self):
        """True once after recover_meta() loaded persisted bits (vbf_filter_take_restored)."""
        rc = lib.vbf_filter_take_restored(self._h)
        if rc < 0:
            _lib.check("vbf_filter_take_restored", rc)
        return bool(rc)

    def set_num_elements(self, n):
        """bf.rs:143: `self.no_of_elements = AtomicU32::new(n)`."""
        call("vbf_filter_set_num_elements", self._h, int(n) & 0xFFFFFFFF)

    def num_elements(self):
        return self.no_of_elements

    def num_bits(self):
        return int(lib.vbf_filter_num_bits(self._h))

    def num_of_hash_functions(self):
        return self.no_of_hash_func

    def num_words(self):
        return (self.num_bits() + 31) // 32

    def words_dev_ptr(self):
        """Device pointer for a caller that WRITES the bits (declare it with stream_record)."""
        return lib.vbf_filter_words_dev(self._h)

    def words_dev_read_ptr(self):
        """Device pointer for read-only use (the host mirror stays trusted)."""
        return lib.vbf_filter_words_dev_read(self._h)

    def get_sst_dir(self):
        if self.sst_dir is None:
            raise ValueError("called `Option::unwrap()` on a `None` value (bf.rs:218)")
        return self.sst_dir

    def set_sstable_path(self, path):
        self.sst_dir = os.fspath(path)

    # -- set / contains ----------------------------------------------------------------
    def set(self, key):
        """bf.rs:84-92 for one key (a batch of one on the GPU)."""
        self.set_many([key])

    def contains(self, key):
        """bf.rs:95-105 for one key."""
        return bool(self.contains_many([key])[0])

    def set_batch(self, b: HostBatch):
        d, o = b.ptrs()
        try:
            call("vbf_filter_set_host", self._h, d, o, b.stride, b.n, b.len_prefix)
        except VbfError as e:
            _raise("set", e)

    def contains_batch(self, b: HostBatch):
        out = np.zeros(b.n, dtype=np.uint8)
        d, o = b.ptrs()
        try:
            call("vbf_filter_contains_host", self._h, d, o, b.stride, b.n, b.len_prefix,
                 out.ctypes.data if b.n else None)
        except VbfError as e:
            _raise("contains", e)
        return out.astype(bool)

    def set_many(self, keys):
        self.set_batch(keys if isinstance(keys, HostBatch) else pack(keys))

    def set_many_async(self, keys, zero_copy=False):
        """set_many that returns before the GPU work is done (vbf_filter_set_host_async).  Later
        calls on the filter wait for it; sync() waits.  By default the library copies the keys
        first; zero_copy=True hands it the batch's own buffers instead, kept alive here until the
        library's release callback (as a Rust caller hands over its packed Vec)."""
        b = keys if isinstance(keys, HostBatch) else pack(keys)
        d, o = b.ptrs()
        rel, ctx = None, None
        if zero_copy:
            token = next(_INFLIGHT_IDS)
            _INFLIGHT[token] = (b, self)
            rel, ctx = _RELEASE_PTR, token
        try:
            call("vbf_filter_set_host_async", self._h, d, o, b.stride, b.n, b.len_prefix, rel, ctx)
        except VbfError as e:
            if zero_copy:
                _INFLIGHT.pop(ctx, None)
            _raise("set", e)

    def sync(self):
        """Wait for the filter's queued and in-flight work (raises a queued set's failure)."""
        call("vbf_filter_sync", self._h)

    def busy(self):
        rc = lib.vbf_filter_busy(self._h)
        if rc < 0:
            _lib.check("vbf_filter_busy", rc)
        return bool(rc)

    def set_mirror(self, mode):
        """Host-mirror mode of a device-resident filter: "off", "lazy" (default) or "eager"."""
        call("vbf_filter_set_mirror", self._h, MIRROR_MODES[mode] if isinstance(mode, str) else int(mode))

    def contains_many(self, keys):
        return self.contains_batch(keys if isinstance(keys, HostBatch) else pack(keys))

    def build_filter_from_entries(self, entries):
        """bf.rs:126-128: `entries` is a sorted map (keys = Vec<u8>) or any iterable of keys."""
        keys = entries.keys() if hasattr(entries, "keys") else entries
        self.set_many(keys)

    # device-resident batches (pointers from torch tensors or the C ABI)
    def set_dev(self, keys_ptr, offsets_ptr, stride, n, len_prefix=1, stream=None):
        try:
            call("vbf_filter_set_dev", self._h, keys_ptr, offsets_ptr, stride, n, len_prefix, stream)
        except VbfError as e:
            _raise("set", e)

    def contains_dev(self, keys_ptr, offsets_ptr, stride, n, out_ptr, len_prefix=1, stream=None):
        try:
            call("vbf_filter_contains_dev", self._h, keys_ptr, offsets_ptr, stride, n, len_prefix,
                 out_ptr, stream)
        except VbfError as e:
            _raise("contains", e)

    # -- SST rebuild (range.rs:117-128) ---------------------------------------------------
    def rebuild_from_sst(self, data, index):
        """load_entries_from_file + build_filter_from_entries (range.rs:124-125) in one device
        pass: decode data.db (bytes) with its index.db (bytes) and OR every key into the bits.
        Returns the number of entries (no_of_elements grows by it, as bf.rs:90 does per key)."""
        a = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else \
            np.ascontiguousarray(data, dtype=np.uint8)
        b = np.frombuffer(index, dtype=np.uint8) if isinstance(index, (bytes, bytearray)) else \
            np.ascontiguousarray(index, dtype=np.uint8)
        n = ctypes.c_uint64()
        try:
            call("vbf_filter_rebuild_from_sst_host", self._h, a.ctypes.data if a.size else None, a.size,
                 b.ctypes.data if b.size else None, b.size, ctypes.byref(n))
        except VbfError as e:
            _raise("rebuild", e)
        return n.value

    def rebuild_from_sst_dev(self, data_ptr, length, blocks_ptr, nblocks, stream=None):
        """Device-resident data.db bytes and block offsets (u32)."""
        n = ctypes.c_uint64()
        try:
            call("vbf_filter_rebuild_from_sst_dev", self._h, data_ptr, length, blocks_ptr, nblocks,
                 ctypes.byref(n), stream)
        except VbfError as e:
            _raise("rebuild", e)
        return n.value

    def recover_from_sst_dir(self, sst_dir):
        """The lazy recovery of range.rs:117-128 for one SST directory: recover_meta() from its
        filter.db, then -- unless persisted bits were restored (vbf_filter_recover_ext) --
        rebuild from data.db + index.db.  Returns True when the bits came from filter.db.  Either
        way the filter ends as the reference's recover_meta + build_filter_from_entries leaves
        it: the same bits and no_of_elements = stored n + the SST's entries."""
        from . import sst
        self.file_path = os.path.join(os.fspath(sst_dir), FILTER_FILE_NAME + ".db")
        restored = self.recover_meta()
        self.sst_dir = os.fspath(sst_dir)
        if not restored:
            self.rebuild_from_sst(*sst.read_sst_files(sst_dir))
        return restored

    # -- bits ----------------------------------------------------------------------------
    def words(self, out=None):
        """The bit array as uint32 words (bit-vec BitVec<u32> storage).  `out`: caller-owned
        storage to copy into (a uint32 array of at least num_words(); the Rust caller's BitVec
        storage), e.g. one already written once so its pages are resident."""
        n = self.num_words()
        if out is None:
            w = np.zeros(n, dtype=np.uint32)
        else:
            w = out
            if w.dtype != np.uint32 or not w.flags.c_contiguous or w.size < n:
                raise ValueError("out must be a contiguous uint32 array of >= %d words" % n)
        call("vbf_filter_words_to_host", self._h, w.ctypes.data if w.size else None, w.size)
        return w

    def load_words(self, words):
        w = np.ascontiguousarray(words, dtype=np.uint32)
        call("vbf_filter_words_from_host", self._h, w.ctypes.data if w.size else None, w.size)

    def clear(self):
        """bf.rs:180-195: zero the shared bits, return a fresh empty filter (same m, k, p)."""
        h = ctypes.c_void_p()
        call("vbf_filter_clear", self._h, ctypes.byref(h))
        return BloomFilter(_handle=h)

    # -- metadata / files --------------------------------------------------------------
    def serialize(self):
        """bf.rs:158-172: u32 k | u32 n | f64 p, little-endian."""
        buf = (ctypes.c_uint8 * 16)()
        call("vbf_filter_serialize", self._h, buf)
        return bytes(buf)

    def serialize_ext(self, sst_entries=None, sst_keys=None):
        """filter.db bytes (vbf_filter_serialize_ext): the reference's 16 bytes (bf.rs:158-172),
        then -- when `sst_entries` (the SST's data.db entry count) is given -- the bit array a
        restart's rebuild would produce (range.rs:117-128): this filter's own words when its m is
        the recovery m (a compaction-built filter), otherwise built from `sst_keys` (the SST's
        keys; a memtable-born filter).  Without them only the 16 bytes (the reference's file)."""
        entries = VBF_EXT_NONE if sst_entries is None else int(sst_entries)
        d = o = None
        stride, lp = 0, 1
        b = None
        if sst_keys is not None and sst_entries is not None:
            b = sst_keys if isinstance(sst_keys, HostBatch) else pack(sst_keys)
            if b.n != entries:
                raise ValueError("sst_keys holds %d keys, sst_entries says %d" % (b.n, entries))
            d, o = b.ptrs()
            stride, lp = b.stride, b.len_prefix
        need = ctypes.c_uint64()
        call("vbf_filter_serialize_ext", self._h, d, o, stride, entries, lp, None, 0, ctypes.byref(need))
        buf = np.zeros(need.value, dtype=np.uint8)
        call("vbf_filter_serialize_ext", self._h, d, o, stride, entries, lp, buf.ctypes.data, buf.size,
             ctypes.byref(need))
        return buf[:need.value].tobytes()

    def write(self, dir_path, persist_bits=True, sst_entries=None, sst_keys=None):
        """bf.rs:114-123: write `filter.db` and remember its path.

        The first 16 bytes are exactly the reference's.  With persist_bits and `sst_entries` the
        bit array follows (serialize_ext): invisible to the reference's reader, restored by
        recover_meta() here instead of a rebuild.  The writer that knows the SST passes its entry
        count (and, for a memtable-born filter, its keys); nothing is persisted otherwise."""
        path = os.path.join(os.fspath(dir_path), FILTER_FILE_NAME + ".db")
        raw = self.serialize_ext(sst_entries if persist_bits else None, sst_keys)
        assert raw[:16] == self.serialize()
        with open(path, "wb") as f:
            f.write(raw)
        self.file_path = path

    def recover_meta(self, load_bits=True):
        """bf.rs:135-150: k and n from filter.db, m recomputed from n, zeroed bits.

        Returns True when persisted bits were loaded (vbf_filter_recover_ext: their m equals the
        recomputed m and the checksum holds, so they equal what the reference's rebuild from
        data.db produces, and no_of_elements is n + entries as after that rebuild): the caller
        skips the rebuild.  False when the caller must rebuild, as the reference always does."""
        if self.file_path is None:
            raise FileNotFoundError("File path for filter not provided (err/mod.rs:19-20)")
        try:
            with open(self.file_path, "rb") as f:
                raw = f.read()
        except OSError:
            raise FileNotFoundError("Error opening filter file %s" % self.file_path) from None
        if len(raw) < 16:
            raise EOFError("unexpected EOF: filter metadata is %d < 16 bytes" % len(raw))
        if not load_bits:
            raw = raw[:16]
        src = np.frombuffer(raw, dtype=np.uint8)
        h = ctypes.c_void_p()
        restored = ctypes.c_int(0)
        call("vbf_filter_recover_ext", src.ctypes.data, src.size, self.device, ctypes.byref(h),
             ctypes.byref(restored))
        old = self._h
        self._h = h
        lib.vbf_filter_free(old)
        self.bits_restored = bool(restored.value)
        return self.bits_restored

    def __repr__(self):
        return "BloomFilter(m=%d, k=%d, n=%d, p=%g, device=%d)" % (
            self.num_bits(), self.no_of_hash_func, self.no_of_elements, self.false_positive_rate,
            self.device)
