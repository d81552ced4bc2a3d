#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ (run in the build container only).

Independence: nothing here imports or links oracle/.  The SipHash-1-3 used is the
implementation in the Perl core header shipped with this image
(/usr/lib/x86_64-linux-gnu/perl/5.34.0/CORE/perl_siphash.h, GPL/Artistic -- used in place,
never copied into the repo), compiled into a throw-away .so under /tmp.  Its 2-4 variant is
cross-checked here against CPython's own SipHash (PYTHONHASHSEED=0 hash of bytes) so the
harness itself is validated before it produces vectors.

The message encoding, sizing and bit layout restate velarixdb (reference /root/reference):
  calculate_hash   src/filter/bf.rs:222-227 (DefaultHasher = SipHash-1-3(0,0);
                   Hash for [u8] = LE64(len) || bytes; then write_u64(seed))
  sizing           src/filter/bf.rs:230-239
  set / contains   src/filter/bf.rs:84-105, bit-vec 0.6.3 BitVec<u32> LSB-first
  filter.db        src/filter/bf.rs:158-172, src/fs/mod.rs:768-796 (u32 k | u32 n | f64 p)
  data.db entries  src/fs/mod.rs:275-332, src/block/block_manager.rs:176-193
                   (u32 key_len | key | u32 value_offset | u64 created_at | u8 tombstone)
  FPR tests        src/filter/bf.rs:307-424 (usize keys 0..10000, negatives 10000..12000)

Outputs (JSON, small): siphash13.json, hashes.json, sizing.json, sst_fixtures.json,
fpr_tests.json, random_sets.json.
"""
import ctypes
import hashlib
import json
import math
import os
import struct
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
PERL_HDR = "/usr/lib/x86_64-linux-gnu/perl/5.34.0/CORE/perl_siphash.h"

C_SRC = r"""
#include <stdint.h>
#include <stddef.h>
#define CAN64BITHASH 1
#define STMT_START do
#define STMT_END while (0)
#define ROTL64(x, b) (uint64_t)(((x) << (b)) | ((x) >> (64 - (b))))
#define U8TO64_LE(p) (*(const uint64_t*)(p))
#define U64 uint64_t
#define U32 uint32_t
#define U8 uint8_t
#define STRLEN size_t
#define PERL_STATIC_INLINE static inline
#include "%s"
static const unsigned char ZERO_KEY[16] = {0};
uint64_t perl_sip13(const unsigned char* in, size_t n) {
    U64 st[4]; SIPHASH_SEED_STATE(ZERO_KEY, st[0], st[1], st[2], st[3]);
    return S_perl_hash_siphash_1_3_with_state_64((const unsigned char*)st, in, n);
}
uint64_t perl_sip24(const unsigned char* in, size_t n) {
    U64 st[4]; SIPHASH_SEED_STATE(ZERO_KEY, st[0], st[1], st[2], st[3]);
    return S_perl_hash_siphash_2_4_with_state_64((const unsigned char*)st, in, n);
}
""" % PERL_HDR


def load_perl_siphash():
    tmp = tempfile.mkdtemp(prefix="vbf_golden_")
    src = os.path.join(tmp, "psip.c")
    so = os.path.join(tmp, "libpsip.so")
    with open(src, "w") as f:
        f.write(C_SRC)
    subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", so, src])
    lib = ctypes.CDLL(so)
    for fn in (lib.perl_sip13, lib.perl_sip24):
        fn.restype = ctypes.c_uint64
        fn.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    return lib


LIB = load_perl_siphash()


def sip13(msg: bytes) -> int:
    return LIB.perl_sip13(msg, len(msg))


def check_harness():
    """Perl 2-4 == CPython's SipHash-2-4 (hash(bytes) with PYTHONHASHSEED=0)."""
    msgs = [b"a", b"apple", b"0123456789abcdef", bytes(range(37))]
    code = "import sys;[print(hash(bytes.fromhex(h))) for h in sys.argv[1:]]"
    env = dict(os.environ, PYTHONHASHSEED="0")
    out = subprocess.check_output([sys.executable, "-c", code] + [m.hex() for m in msgs], env=env)
    py = [int(x) for x in out.split()]
    for m, h in zip(msgs, py):
        want = LIB.perl_sip24(m, len(m))
        # CPython returns the hash as Py_hash_t (signed 64-bit); -1 is remapped to -2.
        got = h & 0xFFFFFFFFFFFFFFFF
        assert got == want, (m, hex(got), hex(want))


def msg_for(key: bytes, seed: int, len_prefix: bool) -> bytes:
    pre = struct.pack("<Q", len(key)) if len_prefix else b""
    return pre + key + struct.pack("<Q", seed)


def calc_hash(key: bytes, seed: int, len_prefix: bool = True) -> int:
    return sip13(msg_for(key, seed, len_prefix))


def f64_as_u32(x: float) -> int:
    if x != x or x <= 0.0:
        return 0
    if x >= 4294967295.0:
        return 4294967295
    return int(x)


def num_bits(n: int, p: float) -> int:
    ln2 = math.log(2.0)
    x = (float(n) * (math.log(p) if p > 0 else -math.inf)) / (ln2 * ln2)
    return f64_as_u32(-math.ceil(x) if math.isfinite(x) else -x)


def num_hash(m: int, n32: int) -> int:
    if n32 == 0:
        return f64_as_u32(math.inf if m > 0 else math.nan)
    return f64_as_u32((float(m) / float(n32)) * math.ceil(math.log(2.0)))


def build(keys, m, k, len_prefix=True):
    words = [0] * ((m + 31) // 32)
    for key in keys:
        for i in range(k):
            idx = calc_hash(key, i, len_prefix) % m
            words[idx >> 5] |= 1 << (idx & 31)
    return words


def probe(keys, m, k, words, len_prefix=True):
    out = []
    for key in keys:
        hit = 1
        for i in range(k):
            idx = calc_hash(key, i, len_prefix) % m
            if not (words[idx >> 5] >> (idx & 31)) & 1:
                hit = 0
                break
        out.append(hit)
    return out


def words_digest(words):
    raw = struct.pack("<%dI" % len(words), *words)
    return hashlib.sha256(raw).hexdigest()


def popcount(words):
    return sum(bin(w).count("1") for w in words)


def parse_data_db(path):
    """src/fs/mod.rs:275-332 -> keys inserted into a SkipMap (sorted, unique)."""
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
    k, n, p = struct.unpack("<IId", open(path, "rb").read()[:16])
    return k, n, p


def main():
    check_harness()
    out = {}

    # 1. raw SipHash-1-3 vectors over bytes(range(L)) and a few named messages
    vec = []
    for L in list(range(0, 70)) + [127, 128, 129, 1000]:
        msg = bytes((i * 7 + 3) & 0xFF for i in range(L))
        vec.append({"msg": msg.hex(), "h": "%016x" % sip13(msg)})
    out["siphash13"] = vec

    # 2. calculate_hash vectors (bf.rs:222-227), byte keys and the test-only encodings
    hv = []
    named = [b"apple", b"head", bytes([1, 2, 3, 4]), b"", b"0123456789abcdef",
             bytes(range(7)), bytes(range(8)), bytes(range(9)), bytes(range(23)),
             bytes(range(24)), bytes(range(25)), bytes((i * 31) & 0xFF for i in range(200)),
             bytes((i * 13 + 5) & 0xFF for i in range(65536))]
    for key in named:
        hv.append({"key": key.hex(), "len_prefix": 1,
                   "h": ["%016x" % calc_hash(key, s) for s in range(40)]})
    # usize keys (bf.rs:300,319): message LE64(i) || LE64(seed)
    for v in (0, 1, 9, 10000, 11999, 2**63 + 5):
        key = struct.pack("<Q", v)
        hv.append({"key": key.hex(), "len_prefix": 0,
                   "h": ["%016x" % calc_hash(key, s, False) for s in range(40)]})
    # &Vec<i32> key (bf.rs:287): LE64(4) || LE32 x 4 -> raw message prefix
    key = struct.pack("<Q4i", 4, 1, 2, 3, 4)
    hv.append({"key": key.hex(), "len_prefix": 0,
               "h": ["%016x" % calc_hash(key, s, False) for s in range(40)]})
    out["hashes"] = hv

    # 3. sizing (bf.rs:230-239), incl. BASELINE configs and the saturation edge
    sz = []
    for n, p in [(10, 0.01), (10000, 0.1), (10000, 1e-4), (10000, 1e-7),
                 (1_000_000, math.exp(-10 * math.log(2) ** 2)),
                 (100_000_000, math.exp(-10 * math.log(2) ** 2)),
                 (50_000_000, math.exp(-10 * math.log(2) ** 2)),
                 (1_000_000_000, math.exp(-15 * math.log(2) ** 2)),
                 (512, 1e-4), (1791, 1e-4), (17064, 0.01), (1, 0.5), (1, 1.0), (5, 2.0),
                 (7, 0.0), (3, 1e-300)]:
        m = num_bits(n, p)
        k = num_hash(m, n & 0xFFFFFFFF)
        sz.append({"n": n, "p": p.hex(), "m": m, "k": k})
    out["sizing"] = sz

    # 4. the reference's SST fixtures: lazy rebuild (range.rs:117-128) with recovered meta
    #    (bf.rs:135-150: k from file, m recomputed from stored n), then probes.
    sst_dir = os.path.join(HERE, "sst_fixtures")
    ssts = []
    union = set()
    names = sorted(os.listdir(sst_dir))
    for idx, name in enumerate(names):
        keys = parse_data_db(os.path.join(sst_dir, name, "data.db"))
        k, n, p = parse_filter_db(os.path.join(sst_dir, name, "filter.db"))
        m = num_bits(n, p)
        words = build(keys, m, k)
        negs = [b"zz%05d" % i for i in range(5000)]
        ssts.append({"name": name, "n_keys": len(keys), "k": k, "n_stored": n, "p": p.hex(), "m": m,
                     "popcount": popcount(words), "sha256": words_digest(words),
                     "first_words": ["%08x" % w for w in words[:8]],
                     "neg_hits_zz5000": sum(probe(negs, m, k, words)),
                     "pos_hits": sum(probe(keys, m, k, words))})
        if idx < 6:
            union.update(keys)
    ukeys = sorted(union)
    m = num_bits(len(ukeys), 0.01)
    k = num_hash(m, len(ukeys))
    words = build(ukeys, m, k)
    compaction = {"n_keys": len(ukeys), "p": (0.01).hex(), "m": m, "k": k,
                  "popcount": popcount(words), "sha256": words_digest(words)}
    out["sst_fixtures"] = {"ssts": ssts, "compaction_union_first6": compaction}

    # 5. bf.rs FPR tests (usize keys)
    fpr = []
    for p in (0.1, 1e-4, 1e-7):
        n = 10000
        m = num_bits(n, p)
        k = num_hash(m, n)
        keys = [struct.pack("<Q", i) for i in range(n)]
        words = build(keys, m, k, False)
        negs = [struct.pack("<Q", i) for i in range(n, n + 2000)]
        fp = sum(probe(negs, m, k, words, False))
        fpr.append({"p": p.hex(), "m": m, "k": k, "popcount": popcount(words),
                    "sha256": words_digest(words), "false_positives": fp})
    out["fpr_tests"] = fpr

    # 6. small mixed sets with full word dumps (fixed + variable length incl. empty & 65536-B)
    import random
    rng = random.Random(0x5EED)
    sets = []
    for (nkeys, fixed_len, m, k) in [(300, 16, 5000, 7), (257, 32, 40000, 3), (100, 8, 1, 5),
                                     (64, 24, 4294967295, 4)]:
        keys = [bytes(rng.getrandbits(8) for _ in range(fixed_len)) for _ in range(nkeys)]
        words = build(keys, m, k) if m < 10**7 else None
        entry = {"keys": [x.hex() for x in keys], "m": m, "k": k}
        if words is not None:
            entry["words"] = ["%08x" % w for w in words]
        else:  # saturated m: record raw bit indices instead of 512 MiB of words
            entry["indices"] = [[calc_hash(x, i) % m for i in range(k)] for x in keys]
        sets.append(entry)
    var_keys = [b""] + [bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 140))) for _ in range(200)]
    var_keys.append(bytes((i * 13 + 5) & 0xFF for i in range(65536)))
    for (m, k) in [(3001, 5), (20000, 10)]:
        words = build(var_keys, m, k)
        negs = [bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 60))) for _ in range(300)]
        sets.append({"keys": [x.hex() for x in var_keys], "m": m, "k": k,
                     "words": ["%08x" % w for w in words],
                     "neg_keys": [x.hex() for x in negs],
                     "neg_hits": probe(negs, m, k, words)})
    out["random_sets"] = sets

    for name, obj in out.items():
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(obj, f, indent=0 if name != "random_sets" else None)
    print("golden vectors written:", ", ".join(sorted(out)))


if __name__ == "__main__":
    main()
