"""Helpers shared by the tests: the reference's on-disk formats."""
import struct


def parse_data_db(path):
    """src/fs/mod.rs:275-332: u32 key_len | key | u32 value_offset | u64 created_at | u8 tomb,
    inserted into a SkipMap -> sorted, unique keys."""
    buf = open(path, "rb").read()
    off, keys = 0, set()
    while off < len(buf):
        (klen,) = struct.unpack_from("<I", buf, off)
        off += 4
        keys.add(buf[off:off + klen])
        off += klen + 4 + 8 + 1
    assert off == len(buf)
    return sorted(keys)


def parse_filter_db(path):
    """src/fs/mod.rs:768-796 -> (k, n, p)."""
    return struct.unpack("<IId", open(path, "rb").read()[:16])
