"""CPU checks for the compaction-merge oracle, pinned by the reference's
own known answer: test_merge_ssts_in_buckets (src/tests/sized_tier_test.rs:165-205) merges the
first six fixture SSTs with use_ttl = false and expects 2844 * 6 = 17064 entries."""
import os

import numpy as np

from conftest import GOLDEN

SST = os.path.join(GOLDEN, "sst_fixtures")


def fixture_arena(ora, names):
    ks, offs, cr, tb, ro = [], [0], [], [], [0]
    for n in names:
        k, o, v, c, t = ora.sst_decode(open(os.path.join(SST, n, "data.db"), "rb").read())
        ks.append(k)
        offs += (o[1:] + offs[-1]).tolist()
        cr.append(c.view(np.int64))
        tb.append(t)
        ro.append(ro[-1] + o.size - 1)
    return (np.concatenate(ks), np.asarray(offs, np.uint64), np.concatenate(cr), np.concatenate(tb),
            np.asarray(ro, np.uint64))


def test_merge_known_answer(ora, golden):
    names = sorted(os.listdir(SST))[:6]
    keys, offs, cr, tb, ro = fixture_arena(ora, names)
    ids = ora.compact_merge(keys, offs, cr, tb, ro)
    assert ids.size == 2844 * 6  # sized_tier_test.rs:200-204
    got = [keys[offs[i]:offs[i + 1]].tobytes() for i in ids]
    assert got == sorted(set(keys[offs[i]:offs[i + 1]].tobytes() for i in range(ro[-1])))
    want = golden("sst_fixtures")["compaction_union_first6"]
    assert ids.size == want["n_keys"]


def test_merge_fold_semantics_by_hand(ora):
    """Small cases of sized.rs:207-320 worked out by hand (times in ms, now = 10_000)."""
    def run(tables, use_ttl=False, ettl=0, tttl=10**9, tmap=None):
        keys, offs, cr, tb, ro = b"", [0], [], [], [0]
        for t in tables:
            for k, c, d in t:
                keys += k
                offs.append(len(keys))
                cr.append(c)
                tb.append(d)
            ro.append(len(cr))
        m = ora.TombstoneMap(tmap or {})
        ids = ora.compact_merge(np.frombuffer(keys, np.uint8), np.asarray(offs, np.uint64),
                                np.asarray(cr, np.int64), np.asarray(tb, np.uint8), np.asarray(ro, np.uint64),
                                use_ttl, ettl, tttl, 10_000, m)
        return ids.tolist(), m.items()
    # newer value wins; ties take the later table
    assert run([[(b"a", 5, 0)], [(b"a", 7, 0)]])[0] == [1]
    assert run([[(b"a", 9, 0)], [(b"a", 7, 0)]])[0] == [0]
    assert run([[(b"a", 7, 0)], [(b"a", 7, 0)]])[0] == [1]
    # a newer tombstone deletes; it survives its first check and is recorded in the map
    ids, m = run([[(b"a", 5, 0)], [(b"a", 7, 1)]])
    assert ids == [1] and m == {b"a": 7}
    # ... and dies at the next pairwise merge (the map already holds its own time)
    ids, m = run([[(b"a", 5, 0)], [(b"a", 7, 1)], [(b"b", 1, 0)]])
    assert ids == [2] and m == {b"a": 7}
    # an older value than a known tombstone is dropped
    assert run([[(b"x", 1, 0)], [(b"a", 3, 0)]], tmap={b"a": 4})[0] == [0]
    # entry TTL: created + ttl < now -> expired
    assert run([[(b"a", 100, 0)], [(b"b", 9_500, 0)]], use_ttl=True, ettl=1_000)[0] == [1]
    # tables[0] is never checked on its own when there is one table
    assert run([[(b"a", 1, 1)]])[0] == [0]
