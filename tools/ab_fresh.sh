#!/bin/bash
# A/B on one box: fresh builds (VBF_BUILD_FRESH, the default) vs a separate zero-fill kernel
# before each build (--separate-zero).  Speed only; both give the same filter.
set -u
for i in 1 2 3; do
  for flag in "" "--separate-zero"; do
    out=$(timeout -k 10 300 python bench.py --no-cpu-baseline --steps 500 $flag "$@" 2>/dev/null | tail -1) || exit $?
    python3 - "$flag" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); ph = d["roofline"]["phases"]
print("%-16s %.3f G/s  %.4f ms  %s" % (sys.argv[1] or "fresh", d["value"] / 1e9, d["ms_per_step"],
      "  ".join("%s %.3f" % (k, v["ms_per_launch"]) for k, v in ph.items())))
PY
  done
done
