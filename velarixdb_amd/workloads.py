"""Synthetic key sets of BASELINE.json's configs, host side.

Fixed-length keys are generated on the device (vbf_gen_fixed_dev); variable-length key
lengths/offsets are generated here with numpy and the bytes on the device (vbf_gen_var_dev).
The same definitions are restated in oracle/oracle.c for parity tests.

  fixed:    key_j = LE64(splitmix64(seed ^ j)) || LE64(j) [|| LE64(splitmix64(seed^j^c*G)) ...]
  variable: len_j = 7 + r, r ~ Zipf(s=1.1) on {1..121} (8..128 B, mean ~25.9 B);
            word 0 = (j << 8) | (seed & 0xff), word c>=1 = splitmix64(seed ^ j ^ c*G)
"""
import math

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)

SEED_CFG2 = 0x5EED0001   # 100M x 16 B positives
SEED_NEG = 0x5EED0002    # disjoint negatives (j >= N)
SEED_CFG3 = 0x5EED0003   # variable-length positives
SEED_CFG3_NEG = 0x5EED00FF  # variable-length negatives (tag byte 0xFF)
SEED_CFG4 = 0x5EED0040   # + shard index
SEED_CFG5 = 0x5EED0005   # 1B x 32 B


def fpr_for_bits_per_key(bits_per_key):
    """p such that m = n * bits_per_key under bf.rs:230-233: p = exp(-b * ln^2 2)."""
    return math.exp(-bits_per_key * math.log(2.0) ** 2)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _zipf_thresholds(s=1.1, support=121):
    w = [float(r) ** -s for r in range(1, support + 1)]
    total = 0.0
    for x in w:
        total += x
    acc, T = 0.0, []
    for r in range(1, support):
        acc += w[r - 1]
        T.append(int((acc / total) * 9007199254740992.0))
    return np.array(T, dtype=np.uint64)


_ZIPF_T = _zipf_thresholds()


def var_lengths(seed, base, n, chunk=1 << 24):
    out = np.empty(n, dtype=np.uint64)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        j = np.arange(base + lo, base + hi, dtype=np.uint64)
        u = splitmix64(j ^ np.uint64(seed) ^ np.uint64(0xD1B54A32D192ED03)) >> np.uint64(11)
        r = np.searchsorted(_ZIPF_T, u, side="right") + 1
        out[lo:hi] = 7 + r
    return out


def var_offsets(seed, base, n):
    lens = var_lengths(seed, base, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    return off
