#!/usr/bin/env python3
"""Cache-path counters of the build kernels from rocprofv3 PMC passes (scripts/gpu_round.sh steps
pmctcp10 / pmctcp19 / pmctcc / pmctcc19): per-dispatch averages per kernel, the per-CU busy
fractions of TA / TD (summed counters / 256 CUs / launch cycles, GRBM_GUI_ACTIVE / 8 XCDs), the
L2 (TCC) hit rate, and TCP->TCC read requests per (tile, segment) run of k_seg_or.

Usage: pmc_cache.py OUT_JSON LABEL:TCP_CSV:TCC_CSV:RUNS [...]
  RUNS = the launch's (tile, segment) runs, e.g. 32553*954 for config 2 at k = 10.
"""
import collections
import csv
import json
import sys

KERNELS = ("k_tile_pack", "k_seg_or")
CUS = 256


def per_kernel(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not any(k in name for k in KERNELS):
            continue
        acc[name.split("(")[0]][r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for name, disp in acc.items():
        keys = set().union(*[set(d) for d in disp.values()])
        out[name] = {c: sum(d.get(c, 0.0) for d in disp.values()) / len(disp) for c in keys}
    return out


def main(out_path, specs):
    res = {}
    for spec in specs:
        label, tcp_csv, tcc_csv, runs = spec.split(":")
        runs = eval(runs, {}, {})  # a product like 32553*954 (arguments written by hand)
        merged = per_kernel(tcp_csv)
        for name, c in per_kernel(tcc_csv).items():
            merged.setdefault(name, {}).update(c)
        for name, c in merged.items():
            cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
            if cyc:
                c["per_cu_fractions"] = {
                    "TA_busy": c.get("TA_TA_BUSY_sum", 0.0) / CUS / cyc,
                    "TD_busy": c.get("TD_TD_BUSY_sum", 0.0) / CUS / cyc,
                    "TA_stalled_by_TC": c.get("TA_ADDR_STALLED_BY_TC_CYCLES_sum", 0.0) / CUS / cyc,
                    "TD_stalled_by_TC": c.get("TD_TC_STALL_sum", 0.0) / CUS / cyc,
                }
            if c.get("TCC_REQ_sum"):
                c["tcc_hit_rate"] = c.get("TCC_HIT_sum", 0.0) / c["TCC_REQ_sum"]
            if "k_seg_or" in name and c.get("TCP_TCC_READ_REQ_sum"):
                c["runs"] = runs
                c["tcp_tcc_read_req_per_run"] = c["TCP_TCC_READ_REQ_sum"] / runs
                c["tcp_accesses_per_run"] = c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0) / runs
        res[label] = merged
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
