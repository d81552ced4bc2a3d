"""Round-3 boundary features on the GPU: the host mirror of device-resident filters, the
asynchronous host-key set, device placement, external writers, and residency races.

* Host mirror: the reference's read path calls contains once per in-range SST
  per get (key_range/range.rs:130,136,171).  A compaction-built or recovered filter lives in HBM;
  small contains batches answer on the CPU from a pinned host copy refreshed after device writes,
  and must give the oracle's answers even right after an asynchronous set_dev on a side stream.
* set_host_async: build_filter_from_entries for a device-resident filter
  returns before the GPU work is done, so the serial compaction loop (compactors/sized.rs:170-200)
  keeps merging while the GPUs build; later calls wait for it, and the words equal the oracle.
* a migrate racing set/contains on a clone must neither crash nor lose bits.
"""
import ctypes
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SLEEP_CYCLES = 40_000_000  # ~17 ms of a spinning kernel ahead of the set_dev


def _vp(t):
    return ctypes.c_void_p(t.data_ptr())


def _side_stream_set(vbf, bf, n, seed, L=16):
    s = torch.cuda.Stream()
    keys = torch.empty(n * L, dtype=torch.uint8, device="cuda:0")
    sp = ctypes.c_void_p(s.cuda_stream)
    with torch.cuda.stream(s):
        torch.cuda._sleep(SLEEP_CYCLES)
    vbf._lib.call("vbf_gen_fixed_dev", seed, 0, n, L, _vp(keys), sp)
    bf.set_dev(_vp(keys), None, L, n, 1, sp)
    return s, keys


def _oracle_words(ora, seed, n, m, k, L=16):
    from velarixdb_amd.keys import HostBatch
    return ora.build_words(HostBatch(ora.gen_fixed(seed, 0, n, L), None, L, n, 1), m, k, threads=8)


@pytest.mark.parametrize("mode", ["lazy", "eager"])
def test_mirror_answers_after_async_set_dev(vbf, ora, mode):
    """Single-key and small-batch contains on a device filter, issued with no synchronisation
    right after a set_dev queued behind a spinning kernel on a side stream: every answer equals
    the oracle's probe of the oracle's words (positives and negatives)."""
    from velarixdb_amd.keys import HostBatch
    n, seed = 2_000_000, 0x5EED0C01
    bf = vbf.BloomFilter(0.01, n)
    bf.set_mirror(mode)
    s, keys = _side_stream_set(vbf, bf, n, seed)
    pos = ora.gen_fixed(seed, 0, 200, 16)
    neg = ora.gen_fixed(seed ^ 0xFFFF, 0, 200, 16)
    got_single = [bf.contains(bytes(pos[i * 16:(i + 1) * 16])) for i in range(50)]
    got_pos = bf.contains_batch(HostBatch(pos, None, 16, 200, 1))
    got_neg = bf.contains_batch(HostBatch(neg, None, 16, 200, 1))
    want_w = _oracle_words(ora, seed, n, bf.num_bits(), bf.no_of_hash_func)
    assert all(got_single) and got_pos.all()
    want_neg = ora.probe(HostBatch(neg, None, 16, 200, 1), bf.num_bits(), bf.no_of_hash_func, want_w).astype(bool)
    assert np.array_equal(got_neg, want_neg)
    assert np.array_equal(bf.words(), want_w)
    # a second write invalidates the mirror: new keys are found through it too
    more = ora.gen_fixed(seed + 1, 0, 100, 16)
    bf.set_many(HostBatch(more, None, 16, 100, 1))
    assert bf.contains_batch(HostBatch(more, None, 16, 100, 1)).all()
    # mirror off: the same answers through the staged GPU probe
    bf.set_mirror("off")
    assert np.array_equal(bf.contains_batch(HostBatch(neg, None, 16, 200, 1)), got_neg)
    del keys, s


def test_mirror_after_clear_load_and_rebuild(vbf, ora, golden):
    """Every device write path refreshes or invalidates the mirror: clear, load_words, the
    data.db rebuild (range.rs:117-128) and a restore from persisted bits."""
    import os
    import hashlib
    from conftest import GOLDEN
    from velarixdb_amd.keys import pack
    keys = [b"mk%05d" % i for i in range(3000)]
    bf = vbf.BloomFilter(1e-4, 3000)
    bf.set_many(keys)
    assert bf.contains(keys[7])
    bf.clear()
    assert not bf.contains(keys[7]) and not bf.words().any()
    w = ora.build_words(pack(keys), bf.num_bits(), bf.no_of_hash_func)
    bf.load_words(w)
    assert bf.contains(keys[7]) and np.array_equal(bf.words(), w)
    # fixture SST rebuild, then the probe of its smallest key answers from the mirror
    sst = os.path.join(GOLDEN, "sst_fixtures", "sstable_1720785462309")
    want = golden("sst_fixtures")["ssts"][0]
    f = vbf.BloomFilter.default()
    f.file_path = os.path.join(sst, "filter.db")
    f.recover_meta()
    from tests_util import parse_data_db
    ks = parse_data_db(os.path.join(sst, "data.db"))
    assert not f.contains(ks[0])  # mirror of the zeroed recovered filter
    f.rebuild_from_sst(*vbf.sst.read_sst_files(sst))
    assert f.contains(ks[0]) and f.contains(ks[-1])
    assert hashlib.sha256(f.words().astype("<u4").tobytes()).hexdigest() == want["sha256"]
    negs = [b"zz%05d" % i for i in range(5000)]
    hits = sum(int(f.contains_many(negs[i:i + 250]).sum()) for i in range(0, 5000, 250))  # mirror batches
    assert hits == want["neg_hits_zz5000"]


def test_multi_probe_small_batch_from_mirrors(vbf, ora):
    """vbf_multi_probe_host with a get-sized batch answers from the filters' mirrors: equal to
    the GPU path (mirrors off) and to the range test + oracle probe, keys in and out of range."""
    from velarixdb_amd.key_range import SstRange, candidates
    from velarixdb_amd.keys import pack
    rng = np.random.default_rng(5)
    ranges = []
    for s in range(6):
        ks = sorted({bytes(rng.integers(97, 123, size=int(rng.integers(3, 12)), dtype=np.uint8)) for _ in range(2000)})
        f = vbf.BloomFilter(1e-3 if s % 2 else 1e-4, len(ks))
        f.set_many(ks)
        ranges.append((SstRange(ks[0], ks[-1], f), ks))
    probe = [ks[i] for _, ks in ranges for i in (0, 5, len(ks) - 1)]
    probe += [bytes(rng.integers(97, 123, size=6, dtype=np.uint8)) for _ in range(60)]
    rs = [r for r, _ in ranges]
    got = candidates(probe, rs)  # 78 keys: the mirror path
    for r in rs:
        r.filter.set_mirror("off")
    assert np.array_equal(candidates(probe, rs), got)  # the GPU path
    for s, (r, ks) in enumerate(ranges):
        w = r.filter.words()
        inr = np.array([r.smallest_key <= k <= r.biggest_key for k in probe])
        hit = ora.probe(pack(probe), r.filter.num_bits(), r.filter.no_of_hash_func, w).astype(bool)
        assert np.array_equal(got[:, s], inr & hit), s


def test_set_host_async_returns_before_the_build(vbf, ora):
    """set_many_async returns while the build is still running (busy), the next call waits for
    it, and the words equal the oracle's.  The library copied the keys: the caller's buffer is
    overwritten right after the call without effect."""
    from velarixdb_amd.keys import HostBatch
    n, seed = 20_000_000, 0x5EED0C02
    host = ora.gen_fixed(seed, 0, n, 16)
    bf = vbf.BloomFilter(0.01, n)
    bf.set_many_async(HostBatch(host, None, 16, n, 1))
    assert bf.busy(), "set_host_async waited for its GPU work"
    assert bf.no_of_elements == n
    saved = host.copy()
    host[:] = 0  # the library works from its own copy
    assert bf.contains(bytes(saved[:16]))  # waits for the queued set
    assert not bf.busy()
    assert np.array_equal(bf.words(), _oracle_words(ora, seed, n, bf.num_bits(), bf.no_of_hash_func))


def test_set_host_async_release_callback_and_order(vbf, ora):
    """The zero-copy form: the library reads the caller's buffer and calls release(ctx) from
    its worker when done (a Rust caller drops its packed Vec there).  Two queued batches and a
    clone's set land in submission order; sync() waits for all."""
    from velarixdb_amd._lib import call
    from velarixdb_amd.keys import HostBatch
    n, seed = 8_000_000, 0x5EED0C03
    a = ora.gen_fixed(seed, 0, n, 16)
    b = ora.gen_fixed(seed, n, n, 16)
    released = []
    done = threading.Event()
    CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p)

    def rel(ctx):
        released.append(ctx)
        if len(released) == 2:
            done.set()

    cb = CB(rel)
    bf = vbf.BloomFilter(0.01, 2 * n)
    call("vbf_filter_set_host_async", bf._h, a.ctypes.data, None, 16, n, 1, ctypes.cast(cb, ctypes.c_void_p), 11)
    c = bf.clone()
    call("vbf_filter_set_host_async", c._h, b.ctypes.data, None, 16, n, 1, ctypes.cast(cb, ctypes.c_void_p), 22)
    assert bf.busy()
    bf.sync()
    assert done.wait(5) and released == [11, 22]
    assert not c.busy()
    want = _oracle_words(ora, seed, 2 * n, bf.num_bits(), bf.no_of_hash_func)
    assert np.array_equal(c.words(), want)
    assert bf.no_of_elements == n and c.no_of_elements == 2 * n  # counters per handle (bf.rs:248)
    # host-resident filters set at once and release immediately
    h = vbf.BloomFilter(0.01, 1000, device="host")
    small = HostBatch(a[:16000], None, 16, 1000, 1)
    call("vbf_filter_set_host_async", h._h, small.data.ctypes.data, None, 16, 1000, 1,
         ctypes.cast(cb, ctypes.c_void_p), 33)
    assert released[-1] == 33 and not h.busy()


def test_auto_placement_and_fanout(vbf, ora):
    """VBF_DEVICE_AUTO: filters land round-robin on the visible GPUs (one here); several filters
    built asynchronously from one thread, as a serial compaction loop would, all bit-exact."""
    from velarixdb_amd.keys import HostBatch
    ndev = vbf.device_count()
    fs = []
    for t in range(4):
        n = 1_000_000 + 250_000 * t
        f = vbf.BloomFilter(0.001, n, device="auto")
        assert 0 <= f.device < ndev
        host = ora.gen_fixed(0x5EED0D00 + t, 0, n, 16)
        f.set_many_async(HostBatch(host, None, 16, n, 1))
        fs.append((f, n))
    devs = [f.device for f, _ in fs]
    assert devs == [(devs[0] + i) % ndev for i in range(4)]
    for t, (f, n) in enumerate(fs):
        assert np.array_equal(f.words(), _oracle_words(ora, 0x5EED0D00 + t, n, f.num_bits(), f.no_of_hash_func))


def test_external_writer_stream_record(vbf, ora):
    """A kernel writing the bits through words_dev_ptr (here the OR of a second filter) bracketed
    by stream_wait / stream_record: later host calls (mirror contains, words) see its result."""
    from velarixdb_amd._lib import call
    from velarixdb_amd.keys import pack
    ka = [b"a%05d" % i for i in range(4000)]
    kb = [b"b%05d" % i for i in range(4000)]
    fa = vbf.BloomFilter.sized(200_000, 7)
    fb = vbf.BloomFilter.sized(200_000, 7)
    fa.set_many(ka)
    fb.set_many(kb)
    assert not fa.contains_many(kb[:100]).all()
    s = torch.cuda.Stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    call("vbf_filter_stream_wait", fa._h, sp)
    call("vbf_filter_stream_wait", fb._h, sp)
    with torch.cuda.stream(s):
        torch.cuda._sleep(SLEEP_CYCLES)
    call("vbf_or_words_dev", ctypes.c_void_p(fa.words_dev_ptr()), ctypes.c_void_p(fb.words_dev_ptr()),
         fa.num_words(), sp)
    call("vbf_filter_stream_record", fa._h, sp)
    assert fa.contains_many(kb[:100]).all() and fa.contains_many(ka[:100]).all()
    assert np.array_equal(fa.words(), ora.build_words(pack(ka + kb), 200_000, 7))


def test_migrate_races_set_and_contains_on_a_clone(vbf, ora):
    """residency is read under the filter's lock.  One thread moves the
    bits between host and GPU while another sets and probes through a clone; no crash, every
    key set is found, and the final words equal the oracle's."""
    from velarixdb_amd import HOST
    from velarixdb_amd.keys import pack
    keys = [b"race%06d" % i for i in range(20000)]
    bf = vbf.BloomFilter(1e-3, len(keys), device=HOST)
    c = bf.clone()
    stop = threading.Event()
    errs = []

    def mover():
        try:
            i = 0
            while not stop.is_set():
                bf.migrate(0 if i % 2 == 0 else HOST)
                i += 1
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = threading.Thread(target=mover)
    th.start()
    try:
        for i in range(0, len(keys), 500):
            c.set_many(keys[i:i + 500])
            assert c.contains_many(keys[:i + 500]).all()
            assert c.contains(keys[i])
    finally:
        stop.set()
        th.join()
    assert not errs, errs
    assert np.array_equal(bf.words(), ora.build_words(pack(keys), bf.num_bits(), bf.no_of_hash_func))


def test_migrate_of_a_pristine_filter_moves_no_bits(vbf, ora):
    """A filter no key was set in since new / clear (BitVec::from_elem, bf.rs:71) migrates by
    allocating zeroed words on the target; one with bits copies them.  The Rust patch moves a
    fresh compaction filter to its GPU (VBF_DEVICE_AUTO) before the batch build."""
    from velarixdb_amd import HOST
    from velarixdb_amd.keys import pack
    keys = [b"pm%06d" % i for i in range(50000)]
    f = vbf.BloomFilter(0.01, 1_000_000, device=HOST)
    f.migrate("auto")
    assert not f.host_resident and not f.words().any()
    f.set_many(keys)
    f.migrate(HOST)
    want = ora.build_words(pack(keys), f.num_bits(), f.no_of_hash_func)
    assert f.host_resident and np.array_equal(f.words(), want)
    f.migrate(0)
    assert np.array_equal(f.words(), want)
    f.clear()
    f.migrate(HOST)
    assert not f.words().any()
    f.migrate(0)
    assert not f.words().any() and not f.contains(keys[0])


def test_multi_probe_does_not_deadlock_behind_queued_sets(vbf, ora):
    """a multi-probe over filters whose asynchronous sets sit in one device's
    FIFO worker in the order B, A.  The probe must not wait for A's job while holding B's lock
    (the worker runs B's job first, under B's lock).  A long job on a third filter keeps B and
    A queued while the probe takes its locks.  The answers equal the oracle's."""
    from velarixdb_amd.key_range import SstRange, candidates
    from velarixdb_amd.keys import HostBatch, pack
    n_long, n, L = 60_000_000, 4_000_000, 16
    fc = vbf.BloomFilter(0.01, n_long)
    fb = vbf.BloomFilter(0.01, n)
    fa = vbf.BloomFilter(0.01, n)
    hc = ora.gen_fixed(0x5EED0E00, 0, n_long, L)
    hb = ora.gen_fixed(0x5EED0E01, 0, n, L)
    ha = ora.gen_fixed(0x5EED0E02, 0, n, L)
    fc.set_many_async(HostBatch(hc, None, L, n_long, 1), zero_copy=True)
    fb.set_many_async(HostBatch(hb, None, L, n, 1), zero_copy=True)
    fa.set_many_async(HostBatch(ha, None, L, n, 1), zero_copy=True)
    probe = [bytes(hb[i * L:(i + 1) * L]) for i in range(20)] + [bytes(ha[i * L:(i + 1) * L]) for i in range(20)]
    probe += [b"neg%05d" % i for i in range(40)]
    rs = [SstRange(b"\x00", b"\xff" * 20, fa), SstRange(b"\x00", b"\xff" * 20, fb)]
    res, errs = [], []

    def run():
        try:
            res.append(candidates(probe, rs))
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = threading.Thread(target=run, daemon=True)
    th.start()
    th.join(120)
    assert not th.is_alive(), "multi-probe deadlocked behind the queued sets"
    assert not errs, errs
    got = res[0]
    for col, (f, h) in enumerate(((fa, ha), (fb, hb))):
        w = _oracle_words(ora, 0x5EED0E02 if f is fa else 0x5EED0E01, n, f.num_bits(), f.no_of_hash_func)
        assert np.array_equal(f.words(), w)
        want = ora.probe(pack(probe), f.num_bits(), f.no_of_hash_func, w).astype(bool)
        assert np.array_equal(got[:, col], want), col
    fc.sync()


def test_external_write_without_record_is_seen(vbf, ora):
    """bits written through words_dev_ptr and only synchronised (no
    stream_record) are still seen by the host paths -- contains from the mirror, words -- and by
    migrate, even when the filter was pristine (nothing set through the API)."""
    from velarixdb_amd import HOST
    from velarixdb_amd._lib import call
    from velarixdb_amd.keys import HostBatch, pack
    m, k, n, L = 1_000_003, 7, 50_000, 16
    ka = ora.gen_fixed(0x5EED0E10, 0, n, L)
    kb = ora.gen_fixed(0x5EED0E11, 0, n, L)
    bb = HostBatch(kb, None, L, n, 1)
    dev_b = torch.from_numpy(kb).to("cuda:0")
    for pristine in (False, True):
        f = vbf.BloomFilter.sized(m, k)
        if not pristine:
            f.set_batch(HostBatch(ka, None, L, n, 1))
            assert f.contains_batch(HostBatch(ka[:L * 100], None, L, 100, 1)).all()  # fills the mirror
            assert not f.contains_batch(HostBatch(kb[:L * 100], None, L, 100, 1)).all()
        ptr = ctypes.c_void_p(f.words_dev_ptr())
        s = torch.cuda.Stream()
        # an external writer: the raw build kernel ORs B's keys into the filter's words
        call("vbf_build_dev", _vp(dev_b), None, L, n, 1, m, k, ptr, ctypes.c_void_p(s.cuda_stream))
        s.synchronize()  # ... and no vbf_filter_stream_record
        want = ora.build_words(bb, m, k)
        if not pristine:
            ora.build_words(HostBatch(ka, None, L, n, 1), m, k, words=want)
        assert f.contains_batch(HostBatch(kb[:L * 100], None, L, 100, 1)).all()
        assert np.array_equal(f.words(), want)
        f.migrate(HOST)
        assert np.array_equal(f.words(), want)
        f.migrate(0)
        assert np.array_equal(f.words(), want)
        assert f.contains_many([bytes(kb[:L])]).all()


def test_async_set_failure_reported_by_next_call(vbf, ora):
    """a queued set that fails on the GPU side (here the staging allocation
    for one key claimed to be 2^40 bytes long: the device has no such memory) is reported by the
    next call on the filter -- vbf_filter_sync -- and only once; the release callback still runs;
    the filter keeps working and its bits are unchanged."""
    from velarixdb_amd._lib import VbfError, call
    from velarixdb_amd.keys import HostBatch
    n, L = 100_000, 16
    host = ora.gen_fixed(0x5EED0E20, 0, n, L)
    f = vbf.BloomFilter(0.01, n)
    f.set_batch(HostBatch(host, None, L, n, 1))
    before = f.words()
    released = threading.Event()
    CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
    cb = CB(lambda ctx: released.set())
    buf = np.zeros(64, np.uint8)
    offs = np.array([0, 1 << 40], dtype=np.uint64)
    call("vbf_filter_set_host_async", f._h, buf.ctypes.data, offs.ctypes.data, 0, 1, 1,
         ctypes.cast(cb, ctypes.c_void_p), 7)
    with pytest.raises(VbfError) as ei:
        call("vbf_filter_sync", f._h)
    assert "asynchronous set" in str(ei.value)
    assert released.wait(10)
    call("vbf_filter_sync", f._h)  # reported once
    assert np.array_equal(f.words(), before)
    assert f.contains_batch(HostBatch(host[:L * 1000], None, L, 1000, 1)).all()
    # the same failure reaches a contains queued behind it
    call("vbf_filter_set_host_async", f._h, buf.ctypes.data, offs.ctypes.data, 0, 1, 1,
         ctypes.cast(cb, ctypes.c_void_p), 8)
    with pytest.raises(VbfError):
        f.contains_batch(HostBatch(host[:L], None, L, 1, 1))
    # the failed allocation's error stays with that job: the next set the device's worker thread
    # runs, on another filter, succeeds (the sticky HIP error of the failed hipMalloc is cleared)
    g = vbf.BloomFilter(0.01, n, device=f.device)
    g.set_many_async(HostBatch(host, None, L, n, 1))
    g.sync()
    assert np.array_equal(g.words(), ora.build_words(HostBatch(host, None, L, n, 1), g.num_bits(), g.no_of_hash_func))
    assert f.contains_batch(HostBatch(host[:L], None, L, 1, 1)).all()


def test_fork_with_a_queued_set_fails_fast_in_the_child(vbf, ora):
    """a child forked while the parent has a set queued on a filter makes
    set_host_async its first call on that filter.  The parent's job never runs in the child, so
    the call must return VBF_EINVAL (AssertionError in the binding) at once instead of queueing
    behind it and leaving every later drain waiting forever; the child's copy of the binding's
    in-flight table is empty (no 60 s wait at exit).  The child makes no HIP call.  The parent's
    jobs are held in the device's worker by a release callback that blocks until the fork is over,
    so the set is deterministically still queued; afterwards the parent's words equal the oracle's."""
    import os
    from velarixdb_amd import filter as vf
    from velarixdb_amd._lib import call
    from velarixdb_amd.keys import HostBatch
    n, L = 200_000, 16
    gate = threading.Event()
    CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
    cb = CB(lambda ctx: gate.wait(60))
    fa = vbf.BloomFilter(0.01, n)
    fb = vbf.BloomFilter(0.01, n, device=fa.device)
    ha = ora.gen_fixed(0x5EED0E40, 0, n, L)
    hb = ora.gen_fixed(0x5EED0E41, 0, n, L)
    # fa's job runs, then the worker blocks in its release callback: fb's job stays queued
    call("vbf_filter_set_host_async", fa._h, ha.ctypes.data, None, L, n, 1, ctypes.cast(cb, ctypes.c_void_p), 1)
    fb.set_many_async(HostBatch(hb, None, L, n, 1), zero_copy=True)
    assert vf._INFLIGHT and fb.busy()
    pid = os.fork()
    if pid == 0:  # the child: no HIP call on any path below
        code = 3
        try:
            try:
                fb.set_many_async(HostBatch(hb[:L * 10], None, L, 10, 1))
                code = 1  # queued behind a job that never runs here
            except AssertionError as e:
                code = 0 if "forked" in str(e) else 2
            if vf._INFLIGHT:
                code = 4
        finally:
            os._exit(code)
    try:
        _, status = os.waitpid(pid, 0)
    finally:
        gate.set()
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status
    fb.sync()
    fa.sync()
    assert np.array_equal(fb.words(), _oracle_words(ora, 0x5EED0E41, n, fb.num_bits(), fb.no_of_hash_func))
    assert np.array_equal(fa.words(), _oracle_words(ora, 0x5EED0E40, n, fa.num_bits(), fa.no_of_hash_func))


def _wait_child(pid, limit=60.0):
    import os
    import signal
    import time
    t0 = time.time()
    while time.time() - t0 < limit:
        done, status = os.waitpid(pid, os.WNOHANG)
        if done:
            return status
        time.sleep(0.05)
    os.kill(pid, signal.SIGKILL)
    os.waitpid(pid, 0)
    raise AssertionError("the forked child hung")


def test_forked_child_device_calls_fail_fast(vbf, ora):
    """A child forked from a process that used the GPU through the library (nothing queued) gets
    VBF_EINVAL ("forked") from every device-resident filter call instead of HIP calls that can
    hang or fault: a synchronous build, a queued set (refused before it is queued or counted),
    single-key contains (the host mirror is the parent's pinned memory), a words copy, a
    new device filter and a stateless device-pointer call.  Host-resident filters keep working in
    the child.  The parent is unaffected."""
    import os
    from velarixdb_amd._lib import call
    from velarixdb_amd.filter import HOST
    from velarixdb_amd.keys import HostBatch
    n, L = 100_000, 16
    h = ora.gen_fixed(0x5EED0E60, 0, n, L)
    f = vbf.BloomFilter(0.01, n)
    f.set_batch(HostBatch(h, None, L, n, 1))
    assert f.contains(bytes(h[:L]))
    pid = os.fork()
    if pid == 0:
        code = 10
        try:
            code = 0
            probes = [
                lambda: f.set_batch(HostBatch(h[:L * 10], None, L, 10, 1)),
                # the queued set itself fails (it used to queue, count and start a worker,
                # and only the next drain reported it)
                lambda: f.set_many_async(HostBatch(h[:L * 10], None, L, 10, 1)),
                lambda: f.contains(bytes(h[:L])),
                lambda: f.words(),
                lambda: vbf.BloomFilter(0.01, 1000, device=f.device),
                lambda: call("vbf_popcount_dev", None, 0, None, None),  # a stateless device entry point
            ]
            for i, p in enumerate(probes):
                try:
                    p()
                    code = 20 + i
                    break
                except AssertionError as e:
                    if "forked" not in str(e):
                        code = 40 + i
                        break
            if code == 0 and f.num_elements() != n:  # the failed set counted nothing
                code = 70
            if code == 0:  # the host path needs no GPU
                g = vbf.BloomFilter(0.01, 1000, device=HOST)
                g.set_batch(HostBatch(h[:L * 10], None, L, 10, 1))
                if not g.contains(bytes(h[:L])):
                    code = 60
        finally:
            os._exit(code)
    status = _wait_child(pid)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, (status, os.WEXITSTATUS(status))
    f.set_batch(HostBatch(h[:L * 10], None, L, 10, 1))
    assert np.array_equal(f.words(), _oracle_words(ora, 0x5EED0E60, n, f.num_bits(), f.no_of_hash_func))


def test_words_dev_read_keeps_the_mirror(vbf, ora):
    """the read-only pointer (vbf_filter_words_dev_read, the OR source of a
    merge) does not mark the filter externally written, so single-key contains keep answering
    from the host mirror -- while vbf_filter_words_dev does mark it (every host read copies)."""
    from velarixdb_amd.keys import HostBatch
    n, L = 100_000, 16
    h = ora.gen_fixed(0x5EED0E50, 0, n, L)
    f = vbf.BloomFilter(0.01, n)
    f.set_batch(HostBatch(h, None, L, n, 1))
    assert f.contains(bytes(h[:L]))
    ro = f.words_dev_read_ptr()
    assert ro and ro == f.words_dev_read_ptr()
    # a device write behind the library's back is NOT seen through the mirror after a read-only
    # hand-out (by contract the reader does not write) ...
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    neg = ora.gen_fixed(0x5EED0E51, 0, 64, L)
    assert not f.contains_batch(HostBatch(neg, None, L, 64, 1)).all()
    vbf._lib.call("vbf_build_dev", ctypes.c_void_p(torch.from_numpy(neg).to("cuda:0").data_ptr()), None, L, 64, 1,
                  f.num_bits(), f.no_of_hash_func, ctypes.c_void_p(ro), ctypes.c_void_p(s.cuda_stream))
    s.synchronize()
    assert not f.contains_batch(HostBatch(neg, None, L, 64, 1)).all()  # the mirror was trusted
    # ... while the writable pointer makes every host read copy the words again
    f.words_dev_ptr()
    assert f.contains_batch(HostBatch(neg, None, L, 64, 1)).all()


@pytest.mark.parametrize("n", [300_000, 20_000_000])  # one staged key chunk; five (64 MiB each)
def test_compaction_path_allocates_no_host_words_and_builds_fresh(vbf, ora, n):
    """VERDICT r05 #4, the patched build_filter_from_entries: new on the
    host (bf.rs:62-81) -> migrate(AUTO) -> set_host_async -> words.  The host-side `new` allocates
    no bit array and the move to the GPU copies none (vbf_filter_host_bytes stays 0); the device
    words of the pristine filter are zeroed asynchronously and the queued build's first chunk is
    the fused fresh build, the later chunks OR in after it; the words equal the oracle's.  A
    pristine device filter read before any set is all zeros (the asynchronous zero fill is
    ordered before every use, the device pointer included)."""
    from velarixdb_amd.filter import AUTO, HOST
    from velarixdb_amd.keys import HostBatch
    L = 16
    h = ora.gen_fixed(0x5EED0E80, 0, n, L)
    f = vbf.BloomFilter(1e-4, n, device=HOST)
    assert f.host_bytes == 0
    f.migrate(AUTO)
    assert not f.host_resident and f.host_bytes == 0
    f.set_many_async(HostBatch(h, None, L, n, 1), zero_copy=True)
    f.sync()
    assert np.array_equal(f.words(), _oracle_words(ora, 0x5EED0E80, n, f.num_bits(), f.no_of_hash_func))
    assert f.no_of_elements == n
    for read in ("pointer", "words"):
        g = vbf.BloomFilter(0.01, 1_000_000, device=HOST)
        g.migrate(AUTO)
        if read == "pointer":  # the zero fill is done before the pointer is handed out
            c = torch.zeros(1, dtype=torch.int64, device="cuda:0")
            vbf._lib.call("vbf_popcount_dev", ctypes.c_void_p(g.words_dev_read_ptr()), g.num_words(),
                          ctypes.c_void_p(c.data_ptr()), None)
            assert int(c.item()) == 0
        assert not g.words().any() and not g.contains(b"never set") and g.host_bytes == g.num_words() * 4
