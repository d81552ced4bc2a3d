#!/usr/bin/env python3
"""Per-phase timing of the partitioned probe: 100M config-2 keys against their own filter.

usage: probe_phases.py [bits_per_key (10)] [VBF_PROBE_PU values, comma-separated (1,0)]
m = 1e8 x bits, k = bits (the reference's sizing at p = exp(-bits ln^2 2)); the partitioned probe
runs once per VBF_PROBE_PU value (1: the round-6 probe on the build's image, 0: the earlier
pipelines), the gather probe once."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import velarixdb_amd  # noqa: E402,F401
from velarixdb_amd._lib import call, lib, profile_read  # noqa: E402

bits = int(sys.argv[1]) if len(sys.argv) > 1 else 10
pus = sys.argv[2].split(",") if len(sys.argv) > 2 else ["1", "0"]
n, L = 100_000_000, 16
m, k = n * bits, bits
dev = torch.device("cuda:0")
P = lambda t: ctypes.c_void_p(t.data_ptr())
keys = torch.empty(n * L, dtype=torch.uint8, device=dev)
call("vbf_gen_fixed_dev", 0x5EED0001, 0, n, L, P(keys), None)
words = torch.zeros((m + 31) // 32, dtype=torch.int32, device=dev)
call("vbf_build_dev_ex", P(keys), None, L, n, 1, m, k, P(words), 0, None)
cnt = torch.zeros(1, dtype=torch.int64, device=dev)
out = torch.empty(n, dtype=torch.uint8, device=dev)
runs = [(2, "partitioned_pu" + pu, pu) for pu in pus] + [(1, "gather", None)]
for strat, name, pu in runs:
    if pu is not None:
        os.environ["VBF_PROBE_PU"] = pu
    for fn, args in (("vbf_probe_count_dev_ex", (P(cnt),)), ("vbf_probe_dev_ex", (P(out),))):
        call(fn, P(keys), None, L, n, 1, m, k, P(words), *args, strat, None)
        torch.cuda.synchronize()
        lib.vbf_profile_enable(1)
        profile_read()
        for _ in range(3):
            call(fn, P(keys), None, L, n, 1, m, k, P(words), *args, strat, None)
        torch.cuda.synchronize()
        ph = profile_read()
        lib.vbf_profile_enable(0)
        tot = sum(ms for p, (ms, c) in ph.items() if c) / 3
        print(name, fn, "total_ms %.3f" % tot, json.dumps({p: round(ms / max(c, 1), 3) for p, (ms, c) in ph.items() if c}))
        if fn == "vbf_probe_count_dev_ex":
            cnt.zero_()
            call(fn, P(keys), None, L, n, 1, m, k, P(words), P(cnt), strat, None)
            assert int(cnt.item()) == n, (name, int(cnt.item()))
