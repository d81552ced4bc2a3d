#!/usr/bin/env python3
"""Per-phase timing of the partitioned probe: 100M config-2 keys against their own filter."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import velarixdb_amd  # noqa: E402,F401
from velarixdb_amd._lib import call, lib, profile_read  # noqa: E402

n, L, m, k = 100_000_000, 16, 1_000_000_000, 10
dev = torch.device("cuda:0")
P = lambda t: ctypes.c_void_p(t.data_ptr())
keys = torch.empty(n * L, dtype=torch.uint8, device=dev)
call("vbf_gen_fixed_dev", 0x5EED0001, 0, n, L, P(keys), None)
words = torch.zeros((m + 31) // 32, dtype=torch.int32, device=dev)
call("vbf_build_dev_ex", P(keys), None, L, n, 1, m, k, P(words), 0, None)
cnt = torch.zeros(1, dtype=torch.int64, device=dev)
out = torch.empty(n, dtype=torch.uint8, device=dev)
for strat, name in ((2, "partitioned"), (1, "gather")):
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
        print(name, fn, json.dumps({p: round(ms / max(c, 1), 3) for p, (ms, c) in ph.items() if c}))
