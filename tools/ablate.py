#!/usr/bin/env python3
"""Phase ablation of the partitioned build (timing only; results are wrong with VBF_ABLATE>0).

Needs the ablation build of the library (the product libvbf.so ignores VBF_ABLATE):
`python velarixdb_amd/build.py --ablation` writes velarixdb_amd/libvbf_ablate.so, which the
children load through VBF_LIB.

Runs the config-2 build (ABL_M / ABL_K override m and k, e.g. 1900000000 / 19) in child processes with VBF_ABLATE=0/1/2 and prints the library's
per-phase hipEvent timings: 0 = full build, 1 = hash + count + scan (no place/copy),
2 = hash only (no LDS count either), 3 = seg_or loads without ds_or, 4 = seg_or ds_or on
synthetic indices without tile loads,
5 = seg_or without its tile loop (word load + LDS init + write-back), 6 = also without the word
load, 7 = LDS init only, 8 = k_tile_pack without key loads and SipHash (bit indices from a
multiply mix of the key number and seed: the count, scan, placement and copy-out alone), 9 = 8
without the placement and copy-out (the launch's fixed cost: counters, scan, tile loop).
Round 6: modes 0 / 1 / 8 / 9 split k_tile_pack's non-hash time by cause."""
import json
import os
import subprocess
import sys

CHILD = r"""
import ctypes, json, os, sys, torch
sys.path.insert(0, os.environ["ROOT"])
import velarixdb_amd as vbf
from velarixdb_amd._lib import call, lib, profile_read
n, L = 100_000_000, 16
m, k = int(os.environ.get("ABL_M", "1000000000")), int(os.environ.get("ABL_K", "10"))
dev = torch.device("cuda:0")
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
keys = torch.empty(n * L, dtype=torch.uint8, device=dev)
call("vbf_gen_fixed_dev", 0x5EED0001, 0, n, L, ctypes.c_void_p(keys.data_ptr()), sp)
words = torch.zeros((m + 31) // 32, dtype=torch.int32, device=dev)
def run():
    call("vbf_build_dev_ex", ctypes.c_void_p(keys.data_ptr()), None, L, n, 1, m, k,
         ctypes.c_void_p(words.data_ptr()), 2, sp)
for _ in range(10): run()  # clocks up before the timed launches
torch.cuda.synchronize()
lib.vbf_profile_enable(1); profile_read()
for _ in range(30): run()
torch.cuda.synchronize()
ph = profile_read()
print(json.dumps({p: round(ms / max(c, 1), 3) for p, (ms, c) in ph.items() if c}))
"""

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for a in (sys.argv[1:] or ["0", "1", "2", "3", "4", "5", "6", "7", "8", "9"]):
    lib = os.path.join(root, "velarixdb_amd", "libvbf_ablate.so")  # build.py --ablation
    if not os.path.exists(lib):
        sys.exit("missing %s: run `python velarixdb_amd/build.py --ablation` first" % lib)
    env = dict(os.environ, VBF_ABLATE=a, ROOT=root, VBF_LIB=lib)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    print("VBF_ABLATE=%s" % a, line[-1] if line else out.stderr[-2000:], flush=True)
