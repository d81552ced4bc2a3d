"""`filter.db` with the bit array persisted after the reference's 16-byte header (SURVEY.md
8(f) row 1) -- an independent Python restatement of the layout that libvbf writes and reads
(vbf_filter_serialize_ext / vbf_filter_recover_ext, include/vbf.h); the tests check the C ABI's
bytes against it.

velarixdb writes only `u32 k | u32 n | f64 p` (src/filter/bf.rs:158-172) and rebuilds the bits
from data.db on the first read after a restart (src/key_range/range.rs:117-128), with m
recomputed from the stored n (bf.rs:144-147).  Its reader consumes exactly 16 bytes
(src/fs/mod.rs:768-796), so bytes appended after the header are invisible to it: a file written
here stays readable by the reference.

Extension layout (little-endian), after the 16-byte header:
    u32 magic 'VBFW' | u32 version (2) | u32 m | u32 nwords | u64 entries | u64 checksum(words)
    | words[nwords]
`entries` is the number of entries in the SST's data.db (what the reference's rebuild would
add to no_of_elements, bf.rs:91 once per entry).

On recovery the words are used only when the recorded m equals the m the reference would
recompute (num_bits(n_stored, p)) -- then the loaded filter is bit-identical to the rebuild
(same keys, same m, same k) and the rebuild can be skipped; the element count becomes
n_stored + entries, as recover_meta + build_filter_from_entries leave it (range.rs:121-124).
Otherwise (e.g. a memtable-born filter, sized from the write-buffer capacity) the caller rebuilds
exactly as the reference does.  Version-1 files (no entry count) are always rebuilt.
"""
import struct

import numpy as np

HEADER = struct.Struct("<IId")
EXT = struct.Struct("<IIIIQQ")
MAGIC = 0x57464256  # b"VBFW" little-endian
VERSION = 2


def fast_checksum(words):
    """Cheap order-sensitive 64-bit checksum used in the extension (vectorised)."""
    w = np.ascontiguousarray(words, dtype=np.uint32).astype(np.uint64)
    if w.size == 0:
        return 0
    idx = np.arange(1, w.size + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return int(np.bitwise_xor.reduce(w * np.uint64(0x9E3779B97F4A7C15) + idx * np.uint64(0xC2B2AE3D27D4EB4F)))


def encode(k, n, p, m=None, words=None, entries=None):
    """`entries`: the SST's data.db entry count, required with `words` (only the writer that
    knows the SST can give it: a memtable filter counts sets, not entries, mem.rs:209-211)."""
    out = HEADER.pack(k & 0xFFFFFFFF, n & 0xFFFFFFFF, p)
    if words is not None:
        if entries is None:
            raise ValueError("persisted words need the SST's entry count")
        w = np.ascontiguousarray(words, dtype="<u4")
        out += EXT.pack(MAGIC, VERSION, m, w.size, entries, fast_checksum(w)) + w.tobytes()
    return out


def decode(raw):
    """-> (k, n, p, m_or_None, words_or_None, entries_or_None); raises EOFError like
    FilterFileNode::recover."""
    if len(raw) < HEADER.size:
        raise EOFError("unexpected EOF: filter metadata is %d < 16 bytes" % len(raw))
    k, n, p = HEADER.unpack_from(raw, 0)
    m = words = entries = None
    if len(raw) >= HEADER.size + EXT.size:
        magic, ver, mm, nwords, ent, chk = EXT.unpack_from(raw, HEADER.size)
        body = raw[HEADER.size + EXT.size:]
        if magic == MAGIC and ver == VERSION and len(body) == 4 * nwords and nwords == (mm + 31) // 32:
            w = np.frombuffer(body, dtype="<u4").astype(np.uint32)
            if fast_checksum(w) == chk:
                m, words, entries = mm, w, ent
    return k, n, p, m, words, entries
