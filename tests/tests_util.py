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


class MemTableMirror:
    """src/memtable/mem.rs reduced to what touches the filter, over the BloomFilter mirror.

    Sizing (:188-191): max_no_of_entries = capacity_bytes / 100, BloomFilter::new(p, that).
    insert (:207-221): contains, then set only when absent (so no_of_elements counts sets).
    get (:223-230): the filter first, then the map.  update / delete (:238-275): a key the
    filter rejects is KeyNotFoundInMemTable.  clear (:325-333): a fresh filter."""

    def __init__(self, capacity, false_positive_rate, device):
        from velarixdb_amd import BloomFilter
        assert false_positive_rate >= 0.0 and capacity > 0
        self.capacity, self.p, self.device = capacity, false_positive_rate, device
        self.bloom_filter = BloomFilter(false_positive_rate, capacity // 100, device=device)
        self.entries = {}

    def insert(self, key, val):
        if not self.bloom_filter.contains(key):
            self.bloom_filter.set(key)
        self.entries[bytes(key)] = val

    def get(self, key):
        if self.bloom_filter.contains(key):
            return self.entries.get(bytes(key))
        return None

    def update(self, key, val):
        if not self.bloom_filter.contains(key):
            raise KeyError("KeyNotFoundInMemTable")
        self.entries[bytes(key)] = val

    delete = update

    def clear(self):
        from velarixdb_amd import BloomFilter
        self.entries.clear()
        self.bloom_filter = BloomFilter(self.p, self.capacity // 100, device=self.device)
