#!/usr/bin/env python3
"""VALU / wait fractions of the build's dominant kernel from one rocprofv3 SQ PMC pass.

Counters (one pass: 7 SQ + 1 GRBM): SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES,
SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE.
Per /opt/skills/guides/MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count
quad-cycles and WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES; GRBM_GUI_ACTIVE is
summed over the 8 XCDs (cycles of the launch = GRBM_GUI_ACTIVE / 8); a wave64 VALU instruction
issues over 2 cycles on a SIMD32, so VALU issue busy = 2 * SQ_INSTS_VALU / (1024 SIMDs * cycles).
Usage: pmc_sq.py COUNTER_CSV KERNEL_SUBSTRING OUT_JSON
"""
import collections
import csv
import json
import sys


def main(path, kernel, out):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            acc[r["Dispatch_Id"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    per = [{c: sum(v) for c, v in d.items()} for d in acc.values()]
    per = [p for p in per if "GRBM_GUI_ACTIVE" in p and "SQ_INSTS_VALU" in p]
    if not per:
        raise SystemExit("no dispatch of %s with the counters in %s" % (kernel, path))
    avg = {c: sum(p[c] for p in per) / len(per) for c in per[0]}
    cycles = avg["GRBM_GUI_ACTIVE"] / 8
    res = {
        "kernel": kernel, "dispatches": len(per), "counters_per_dispatch": avg,
        "cycles_per_dispatch": cycles,
        "valu_issue_busy": 2 * avg["SQ_INSTS_VALU"] / (1024 * cycles),
        "wave_wait_any_frac": avg.get("SQ_WAIT_ANY", 0) / avg["SQ_WAVE_CYCLES"],
        "wave_wait_inst_frac": avg.get("SQ_WAIT_INST_ANY", 0) / avg["SQ_WAVE_CYCLES"],
        "wave_active_valu_frac": avg.get("SQ_ACTIVE_INST_VALU", 0) / avg["SQ_WAVE_CYCLES"],
        "note": "valu_issue_busy = 2 cycles x SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE/8); "
                "half-rate instructions (v_alignbit, v_lshl_add_u64) take ~4.3 cycles, so the issue "
                "limit is reached below 1.0",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
