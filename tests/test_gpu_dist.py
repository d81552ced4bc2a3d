"""The N > 1 exchange of config 5 (one filter over keys split across ranks) as shipped: two
ranks on the one GPU of the box (gloo group, host-staged all_to_all / all_gather, the HIP OR
kernel folding the partials), launched as a child process by torch.distributed.run.  The merged
words on every rank must equal one rank's build of all the keys, bit for bit (SURVEY 8(e);
builds are linear under OR, bf.rs:84-92).  Also bench.py --config 5 --gpus 2 in the same
rehearsal mode runs to completion and finds every key."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _env():
    env = dict(os.environ)
    env.pop("VBF_LIB", None)
    env["VBF_SHARE_DEVICE"] = "1"
    env["VBF_DIST_BACKEND"] = "gloo"
    env["MASTER_ADDR"] = "127.0.0.1"
    return env


def _port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_two_rank_or_exchange_equals_single_build(vbf, tmp_path):
    from velarixdb_amd.workloads import SEED_CFG5, fpr_for_bits_per_key
    N = 1_000_000_000
    m = vbf.num_bits(N, fpr_for_bits_per_key(15))
    k = vbf.num_hash_functions(m, N)
    assert (m, k) == (4294967295, 4)  # config 5's saturated sizing
    n, L = 40_000_001, 32  # odd: the two shards differ in size
    out = str(tmp_path / "merged")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist_or_worker.py"), str(n), str(L), str(m), str(k), hex(SEED_CFG5), out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    dev = torch.device("cuda", 0)
    sp = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    keys = torch.empty(n * L, dtype=torch.uint8, device=dev)
    vbf._lib.call("vbf_gen_fixed_dev", SEED_CFG5, 0, n, L, ctypes.c_void_p(keys.data_ptr()), sp)
    words = torch.zeros((m + 31) // 32, dtype=torch.int32, device=dev)
    vbf._lib.call("vbf_build_dev_ex", ctypes.c_void_p(keys.data_ptr()), None, L, n, 1, m, k,
                  ctypes.c_void_p(words.data_ptr()), 1, sp)  # atomic, one rank, all keys
    want = words.cpu().numpy().view(np.uint32)
    del keys, words
    for rank in range(2):
        got = np.load(out + ".rank%d.npy" % rank)
        assert np.array_equal(got, want), rank


@pytest.mark.timeout(600)
def test_bench_config5_two_rank_rehearsal(vbf):
    """bench.py --config 5 --gpus 2 (spawns its ranks; shared-device gloo rehearsal) on a
    200M-key slice of config 5: completes, every key found across the ranks' sweeps."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "5", "--gpus", "2", "--keys", "200000000",
           "--steps", "2", "--warmup", "1", "--neg-keys", "1000000", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=580, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert 0.0 < line["negatives"]["fpr"] < 0.05  # 200M keys in 2^32 bits at k = 4
