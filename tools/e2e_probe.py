#!/usr/bin/env python3
"""End-to-end path diagnostics: raw link rates the host build is bounded by (pinned / pageable
H2D and D2H of 1.6 GB, torch copies) next to vbf_build_host on 100M x 16 B keys."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import velarixdb_amd as vbf  # noqa: E402
from velarixdb_amd import workloads as wl  # noqa: E402

dev = torch.device("cuda:0")
nb = 1_600_000_000


def rate(f, nbytes, reps=3):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return nbytes / dt / 1e9, dt * 1e3


pin = torch.empty(nb, dtype=torch.uint8).pin_memory()
pag = torch.empty(nb, dtype=torch.uint8)
pag.fill_(1)
d = torch.empty(nb, dtype=torch.uint8, device=dev)
print("H2D pinned   %.1f GB/s (%.1f ms)" % rate(lambda: d.copy_(pin, non_blocking=True), nb))
print("H2D pageable %.1f GB/s (%.1f ms)" % rate(lambda: d.copy_(pag), nb))
print("D2H pinned   %.1f GB/s (%.1f ms)" % rate(lambda: pin.copy_(d, non_blocking=True), nb))
print("D2H pageable %.1f GB/s (%.1f ms)" % rate(lambda: pag.copy_(d), nb))
fresh = lambda: torch.empty(125_000_000, dtype=torch.uint8).copy_(d[:125_000_000])
print("D2H 125 MB into a fresh pageable tensor %.1f GB/s (%.1f ms)" % rate(fresh, 125_000_000))
a = np.ones(nb, np.uint8)
b = np.empty(nb, np.uint8)
t0 = time.perf_counter()
np.copyto(b, a)
print("host memcpy 1 thread %.1f GB/s" % (nb / (time.perf_counter() - t0) / 1e9))
del pin, pag, d, a, b
n, L = 100_000_000, 16
keys = torch.empty(n * L, dtype=torch.uint8, device=dev)
vbf._lib.call("vbf_gen_fixed_dev", wl.SEED_CFG2, 0, n, L, ctypes.c_void_p(keys.data_ptr()),
              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
host = keys.cpu().numpy()
del keys
m, k = 1_000_000_000, 10
words = np.zeros((m + 31) // 32, np.uint32)
for rep in range(3):
    t0 = time.perf_counter()
    vbf._lib.call("vbf_build_host", host.ctypes.data, None, L, n, 1, m, k, words.ctypes.data, words.size, 0)
    print("vbf_build_host 100M x 16 B (VBF_COPY_THREADS=%s): %.1f ms"
          % (os.environ.get("VBF_COPY_THREADS", "default"), (time.perf_counter() - t0) * 1e3))

# phases of bench.py --e2e's step (BloomFilter::new -> set over host keys -> words to host)
from velarixdb_amd.keys import HostBatch  # noqa: E402
hb = HostBatch(host, None, L, n, 1)
p = wl.fpr_for_bits_per_key(10)
for rep in range(4):
    t0 = time.perf_counter()
    bf = vbf.BloomFilter(p, n, device=0)
    t1 = time.perf_counter()
    bf.set_batch(hb)
    t2 = time.perf_counter()
    w = bf.words()
    t3 = time.perf_counter()
    del bf
    t4 = time.perf_counter()
    print("e2e phases: new %.2f  set_batch %.2f  words %.2f  free %.2f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3,
                                                                          (t3 - t2) * 1e3, (t4 - t3) * 1e3))
