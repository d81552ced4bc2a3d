#!/usr/bin/env python3
"""A second, independent pin of the SipHash-1-3 arithmetic (run in the build container only).

gen_golden.py produced tests/golden/siphash13.json and hashes.json with the Perl core header's
SipHash-1-3.  This script recomputes every one of those vectors with OpenSSL's SipHash MAC
(`openssl mac SIPHASH` with c-rounds 1, d-rounds 3, a 16-byte zero key, 8-byte output: the
libcrypto implementation, no code shared with Perl's) and records the comparison in
tests/golden/siphash13_openssl.json.  Rust's DefaultHasher is SipHash-1-3 with keys (0, 0)
(bf.rs:222-227); OpenSSL emits the 64-bit result as little-endian bytes.

Nothing here imports or links oracle/ or the product library.
"""
import json
import os
import struct
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


def openssl_sip13(msg: bytes) -> int:
    with tempfile.NamedTemporaryFile(delete=False) as f:
        f.write(msg)
        path = f.name
    try:
        out = subprocess.run(["openssl", "mac", "-in", path, "-macopt", "hexkey:" + "00" * 16, "-macopt", "size:8",
                              "-macopt", "c-rounds:1", "-macopt", "d-rounds:3", "SIPHASH"],
                             capture_output=True, text=True, check=True).stdout.strip()
    finally:
        os.unlink(path)
    return int.from_bytes(bytes.fromhex(out), "little")


def main():
    version = subprocess.run(["openssl", "version"], capture_output=True, text=True, check=True).stdout.strip()
    checked, bad, sample = 0, [], []
    for v in json.load(open(os.path.join(HERE, "siphash13.json"))):
        msg = bytes.fromhex(v["msg"])
        got = openssl_sip13(msg)
        checked += 1
        if got != int(v["h"], 16):
            bad.append(v["msg"][:64])
        if len(sample) < 8:
            sample.append({"msg": v["msg"], "h": "%016x" % got})
    for v in json.load(open(os.path.join(HERE, "hashes.json"))):
        key = bytes.fromhex(v["key"])
        prefix = (struct.pack("<Q", len(key)) if v["len_prefix"] else b"") + key
        for s, h in enumerate(v["h"][:8]):  # seeds 0..7 of every key (the 64 KiB key included)
            got = openssl_sip13(prefix + struct.pack("<Q", s))
            checked += 1
            if got != int(h, 16):
                bad.append("%s seed %d" % (v["key"][:32], s))
    res = {"tool": version + ": openssl mac SIPHASH, c-rounds 1, d-rounds 3, key 00*16, size 8 (LE bytes)",
           "reference": "bf.rs:222-227 DefaultHasher = SipHash-1-3(k0 = k1 = 0)",
           "checked": checked, "mismatches": len(bad), "mismatch_examples": bad[:10], "sample": sample}
    with open(os.path.join(HERE, "siphash13_openssl.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("tool", "checked", "mismatches")}))
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
