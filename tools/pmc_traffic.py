#!/usr/bin/env python3
"""HBM traffic per build launch from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE runs).

Corrections, per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): the counters are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read, so
it is doubled (both build kernels read with 16-byte loads); WRITE_SIZE is exact for 16 B/lane
stores.  Usage: pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON
"""
import collections
import csv
import re
import json
import sys

BUILD_KERNELS = ("k_tile_pack", "k_transpose_u16_v", "k_seg_or", "k_keys<(vbf::Op)0")  # k_transpose_u16 (no _v): the probe's


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(fetch_csv, write_csv, out):
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    kernels = {}
    total = 0.0
    for name in sorted(set(fetch) | set(write)):
        if not any(b in name for b in BUILD_KERNELS):
            continue
        # the probes' packs: k_tile_pack with POS = 1 (round 4) or 2 (round 6) -- POS is the template
        # argument after the segment bits (17 / 20), then SAT; round 4-5 names had POS as a bool
        if re.search(r", (17|20), (true|1|2)(, (true|false))?>", name):
            continue
        rd = fetch.get(name, 0.0) * 1024 * 2
        wr = write.get(name, 0.0) * 1024
        kernels[name.split("(")[0]] = {"read_bytes": rd, "write_bytes": wr}
        total += rd + wr
    res = {"per_launch_bytes": total, "kernels": kernels,
           "note": "FETCH_SIZE x1024 x2 (gfx950 wide-read correction) + WRITE_SIZE x1024"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
