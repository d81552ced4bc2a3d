"""velarixdb_amd -- MI355X-native Bloom-filter build/probe behind velarixdb's src/filter API.

The compute path is libvbf.so (hand-written HIP for gfx950, C ABI in include/vbf.h); this
package is its Python host mirror.  Importing it loads libvbf.so or raises -- there is no
CPU fallback: a batch never leaves the GPU path silently.  The one CPU path is an explicit
residency the caller chooses, device=HOST, for the memtable's per-put filter (include/vbf.h).
"""
from ._lib import LIB_PATH, VbfError, device_count, lib  # noqa: F401
from .filter import (DEFAULT_FALSE_POSITIVE_RATE, FILTER_FILE_NAME, HOST, BloomFilter,  # noqa: F401
                     num_bits, num_hash_functions)
from .keys import HostBatch, I32Vec, RawMessage, Usize, pack, pack_fixed, pack_offsets  # noqa: F401
from . import compaction, key_range, sst  # noqa: F401

__version__ = "0.1.0"
