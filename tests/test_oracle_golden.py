"""Pin the CPU oracle against golden vectors made WITHOUT it (tests/golden/gen_golden.py:
Perl-header SipHash-1-3 + an independent Python restatement) and the reference's own SST
fixtures (src/tests/fixtures/data/.../data.db, filter.db)."""
import hashlib
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from velarixdb_amd.keys import pack, pack_offsets


def test_siphash13_vectors(ora, golden):
    for v in golden("siphash13"):
        msg = bytes.fromhex(v["msg"])
        assert "%016x" % ora.siphash13(msg) == v["h"], len(msg)


def test_calculate_hash_vectors(ora, golden):
    # bf.rs:222-227
    for v in golden("hashes"):
        key = bytes.fromhex(v["key"])
        for seed, h in enumerate(v["h"]):
            assert "%016x" % ora.calc_hash(key, seed, v["len_prefix"]) == h


def test_survey_appendix_b1(ora):
    # SURVEY.md Appendix B.1 (computed independently during the survey)
    assert "%016x" % ora.calc_hash(b"apple", 0) == "bad81882d7f3d7f4"
    assert "%016x" % ora.calc_hash(b"head", 2) == "3ec4c018bff1e383"
    assert "%016x" % ora.calc_hash(bytes([1, 2, 3, 4]), 1) == "98f794b69cd48894"


def test_sizing(ora, golden):
    # bf.rs:230-239 incl. u32 saturation and k = floor(m/n)
    for v in golden("sizing"):
        p = float.fromhex(v["p"])
        m = ora.num_bits(v["n"], p)
        assert m == v["m"], v
        assert ora.num_hash(m, v["n"]) == v["k"], v


def _sst_batches():
    from tests_util import parse_data_db, parse_filter_db
    root = os.path.join(GOLDEN, "sst_fixtures")
    for name in sorted(os.listdir(root)):
        keys = parse_data_db(os.path.join(root, name, "data.db"))
        meta = parse_filter_db(os.path.join(root, name, "filter.db"))
        yield name, keys, meta


def _digest(words):
    return hashlib.sha256(words.astype("<u4").tobytes()).hexdigest()


def test_sst_fixture_rebuild(ora, golden):
    """key_range/range.rs:117-128: recover_meta (m from stored n) then rebuild from data.db."""
    want = {s["name"]: s for s in golden("sst_fixtures")["ssts"]}
    assert len(want) == 7
    for name, keys, (k, n, p) in _sst_batches():
        w = want[name]
        m = ora.num_bits(n, p)
        assert (m, k, len(keys)) == (w["m"], w["k"], w["n_keys"])
        b = pack(keys)
        words = ora.build_words(b, m, k)
        assert int(np.unpackbits(words.view(np.uint8)).sum()) == w["popcount"]
        assert _digest(words) == w["sha256"]
        assert ["%08x" % x for x in words[:8]] == w["first_words"]
        negs = pack([b"zz%05d" % i for i in range(5000)])
        assert int(ora.probe(negs, m, k, words).sum()) == w["neg_hits_zz5000"]
        assert int(ora.probe(b, m, k, words).sum()) == len(keys)


def test_compaction_union_filter(ora, golden):
    """compactors/sized.rs:192-193 over the union of 6 fixture SSTs at fpr 0.01."""
    g = golden("sst_fixtures")["compaction_union_first6"]
    keys = set()
    for i, (_, ks, _) in enumerate(_sst_batches()):
        if i < 6:
            keys.update(ks)
    keys = sorted(keys)
    m = ora.num_bits(len(keys), 0.01)
    k = ora.num_hash(m, len(keys))
    assert (len(keys), m, k) == (g["n_keys"], g["m"], g["k"])
    words = ora.build_words(pack(keys), m, k)
    assert _digest(words) == g["sha256"]


def test_bf_rs_fpr_tests(ora, golden):
    """bf.rs:307-424 with usize keys (LE64, no length prefix)."""
    for v in golden("fpr_tests"):
        p = float.fromhex(v["p"])
        n = 10000
        m = ora.num_bits(n, p)
        k = ora.num_hash(m, n)
        assert (m, k) == (v["m"], v["k"])
        keys = np.arange(n, dtype="<u8").view(np.uint8).reshape(n, 8)
        from velarixdb_amd.keys import pack_fixed
        words = ora.build_words(pack_fixed(keys, len_prefix=0), m, k)
        assert _digest(words) == v["sha256"]
        negs = np.arange(n, n + 2000, dtype="<u8").view(np.uint8).reshape(2000, 8)
        fp = int(ora.probe(pack_fixed(negs, len_prefix=0), m, k, words).sum())
        assert fp == v["false_positives"]
        assert fp / 2000 <= p * 1.1  # the reference's own assertion


def test_random_sets(ora, golden):
    for s in golden("random_sets"):
        keys = [bytes.fromhex(x) for x in s["keys"]]
        b = pack(keys)
        if "words" in s:
            words = ora.build_words(b, s["m"], s["k"])
            assert ["%08x" % x for x in words] == s["words"]
            if "neg_keys" in s:
                negs = pack([bytes.fromhex(x) for x in s["neg_keys"]])
                assert ora.probe(negs, s["m"], s["k"], words).tolist() == s["neg_hits"]
        else:
            hs = ora.hashes(b, s["k"])
            assert ((hs % np.uint64(s["m"])).tolist()) == s["indices"]


def test_mt_build_matches_serial(ora):
    keys = ora.gen_fixed(0x5EED0001, 0, 20000, 16)
    b = pack_offsets(keys, np.arange(0, 20001 * 16, 16, dtype=np.uint64))
    m, k = 200000, 10
    a = ora.build_words(b, m, k)
    c = ora.build_words(b, m, k, threads=4)
    assert np.array_equal(a, c)
    # the threaded probe (the checker of the full-size GPU probes) answers like the serial one,
    # on positives and negatives, fixed and variable-length keys, with and without the prefix
    negs = ora.gen_fixed(0x5EED00FF, 0, 20000, 16)
    both = pack_offsets(np.concatenate([keys, negs]), np.arange(0, 40001 * 16, 16, dtype=np.uint64))
    want = ora.probe(both, m, k, a)
    assert want[:20000].all() and 0 < want[20000:].sum() < 400
    assert np.array_equal(ora.probe(both, m, k, a, threads=7), want)
    from velarixdb_amd.workloads import var_offsets
    off = var_offsets(0x5EED0003, 0, 3000)
    vb = pack_offsets(ora.gen_var(0x5EED0003, 0, off), off, 0)
    w = ora.build_words(vb, 30011, 7, threads=3)
    assert np.array_equal(w, ora.build_words(vb, 30011, 7))
    assert np.array_equal(ora.probe(vb, 30011, 7, w, threads=5), ora.probe(vb, 30011, 7, w))


def test_m_zero_panics_like_reference(ora):
    with pytest.raises(ZeroDivisionError):
        ora.build_words(pack([b"x"]), 0, 3)
    # k == 0 -> no hashing, probe vacuously true (bf.rs:104)
    words = np.zeros(0, np.uint32)
    assert ora.probe(pack([b"x"]), 0, 0, words).tolist() == [1]


def test_meta_layout():
    """bf.rs:158-172 / fs/mod.rs:768-796: u32 k | u32 n | f64 p little-endian."""
    raw = open(os.path.join(GOLDEN, "sst_fixtures", "sstable_1720785462309", "filter.db"), "rb").read()
    assert struct.unpack("<IId", raw) == (19, 1791, 1e-4)


def test_siphash13_pinned_by_openssl(golden):
    """Second independent pin of the hash arithmetic: every SipHash-1-3 vector the golden set
    holds (from the Perl core header) recomputed by OpenSSL's SipHash MAC with c = 1, d = 3 and a
    zero key (tests/golden/gen_openssl_pin.py): 234 vectors, no mismatch."""
    pin = golden("siphash13_openssl")
    assert pin["checked"] >= 200 and pin["mismatches"] == 0
    assert "c-rounds 1, d-rounds 3" in pin["tool"]


def test_oracle_matches_openssl_live(ora):
    """The oracle against OpenSSL's SipHash-1-3 on random messages, when the openssl CLI with
    SIPHASH c-rounds / d-rounds parameters is present (OpenSSL >= 3.0; this build container)."""
    import random
    import shutil
    import subprocess
    import sys
    if not shutil.which("openssl"):
        pytest.skip("no openssl CLI")
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from gen_openssl_pin import openssl_sip13
    try:
        openssl_sip13(b"probe")
    except (subprocess.CalledProcessError, ValueError):
        pytest.skip("openssl lacks SIPHASH c-rounds / d-rounds")
    rng = random.Random(20261017)
    for _ in range(40):
        msg = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 200)))
        assert ora.siphash13(msg) == openssl_sip13(msg), msg.hex()
