#!/usr/bin/env python3
"""Timing ablation of the data.db walk (results are wrong with VBF_ABLATE set; needs the
ablation build velarixdb_amd/libvbf_ablate.so from `python velarixdb_amd/build.py --ablation`):
0 = full, 11 = staging only (no walk), 12 = synthetic 124-step walk without staging,
13 = dependent 124-step LDS chain without staging, 14 = staging + that chain."""
import os
import subprocess
import sys

CHILD = r"""
import ctypes, json, os, sys, torch
sys.path.insert(0, os.environ["ROOT"])
import velarixdb_amd as vbf
from velarixdb_amd._lib import call, lib, profile_read
n, L = 100_000_000, 16
per = 4096 // (L + 17); nb = (n + per - 1) // per
dev = torch.device("cuda:0")
P = lambda t: ctypes.c_void_p(t.data_ptr())
data = torch.empty(n * (L + 17), dtype=torch.uint8, device=dev)
blocks = torch.empty(nb, dtype=torch.int32, device=dev)
call("vbf_gen_sst_fixed_dev", 1, 0, n, L, P(data), P(blocks), None)
got = ctypes.c_uint64()
def run():
    try:
        call("vbf_sst_decode_dev", P(data), data.numel(), P(blocks), nb, None, 0, None, None, None, None, 0,
             ctypes.byref(got), None)
    except Exception as e:
        pass
for _ in range(2): run()
torch.cuda.synchronize()
lib.vbf_profile_enable(1); profile_read()
for _ in range(5): run()
torch.cuda.synchronize()
ph = profile_read()
print(json.dumps({p: round(ms / max(c, 1), 3) for p, (ms, c) in ph.items() if c}))
"""
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for a in ("0", "11", "12", "13", "14"):
    lib = os.path.join(root, "velarixdb_amd", "libvbf_ablate.so")  # build.py --ablation
    if not os.path.exists(lib):
        sys.exit("missing %s: run `python velarixdb_amd/build.py --ablation` first" % lib)
    env = dict(os.environ, VBF_ABLATE=a, ROOT=root, VBF_LIB=lib)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    print("VBF_ABLATE=%s %s" % (a, line[0] if line else out.stderr[-500:]), flush=True)
