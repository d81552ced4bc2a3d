"""world_size-2, 3 and 8 gloo runs of the multi-GPU exchange (velarixdb_amd/dist.py) on CPU.

The partial filters here are built by the oracle (the checker) from each rank's key shard; the
property under test is the exchange: OR-all-reduce(partials) == the filter of all keys
(builds are linear in the key set under OR, bf.rs:84-92).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, m, k, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from velarixdb_amd.dist import or_allreduce_, or_fold_host, padded_words, shard_range
        from velarixdb_amd.keys import HostBatch
        lo, hi = shard_range(n, rank, world)
        keys = oracle.gen_fixed(0x5EED0005, lo, hi - lo, 32)
        partial = oracle.build_words(HostBatch(keys, None, 32, hi - lo, 1), m, k)
        nwords = (m + 31) // 32
        buf, chunk = padded_words(nwords, world, "cpu")
        buf[:nwords] = torch.from_numpy(partial.view(np.int32))
        or_allreduce_(buf, chunk, fold=or_fold_host)  # gloo: CPU tensors
        first = buf[:nwords].numpy().view(np.uint32).copy()
        # a second call reuses the receive workspace: the result must not depend on its contents
        buf[:nwords] = torch.from_numpy(partial.view(np.int32))
        buf[nwords:] = 0
        or_allreduce_(buf, chunk)  # the default fold for CPU tensors
        assert np.array_equal(first, buf[:nwords].numpy().view(np.uint32))
        q.put((rank, first, buf[nwords:].abs().sum().item()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_or_allreduce_equals_single_filter(world, ora):
    """world 8 is the target node's rank count: 31 251 words split into
    8 chunks of 3 907 with 5 padding words, as config 5's exchange does at full size."""
    from velarixdb_amd.keys import HostBatch
    m, k, n = 1_000_003, 4, 40_000  # nwords not divisible by world: exercises the padding
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, m, k, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = ora.build_words(HostBatch(ora.gen_fixed(0x5EED0005, 0, n, 32), None, 32, n, 1), m, k)
    for rank, words, pad in results:
        assert np.array_equal(words, want), rank
        assert pad == 0


def test_shard_range_covers_everything():
    from velarixdb_amd.dist import shard_range
    for n in (0, 1, 7, 1000, 10**9):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_or_words_dev_rejects_mismatched_tensors():
    """shape / dtype / contiguity mismatches are Python errors, never a kernel reading
    past a buffer (checked before anything reaches the device)."""
    from velarixdb_amd.dist import or_words_dev
    a = torch.zeros(8, dtype=torch.int32)
    with pytest.raises(ValueError, match="device tensors"):
        or_words_dev(a, a)
