#!/bin/bash
# round 5: config 3's speed-only layout knobs (VBF_LEN_ORDER, VBF_STAGE_KEYS) on the round-5 kernels
set -u
for pass in 1 2; do
  for e in "VBF_LEN_ORDER=1 VBF_STAGE_KEYS=1" "VBF_LEN_ORDER=1 VBF_STAGE_KEYS=0" "VBF_LEN_ORDER=0 VBF_STAGE_KEYS=0"; do
    out=$(env $e timeout -k 10 120 python bench.py --no-cpu-baseline --steps 60 --warmup 5 --config 3 2>/dev/null | tail -1) || { echo "FAIL $e"; exit 1; }
    python3 - "$e" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); ph = d["roofline"].get("phases", {})
print("%-34s %.3f ms  %s" % (sys.argv[1], d["ms_per_step"], {k: round(v["ms_per_launch"], 3) for k, v in ph.items()}))
PY
  done
done
