#!/bin/bash
# VBF_STAGGER 0 vs 7 (the default until round 5) on configs 3 and 5 and the raw-key class kernel
set -u
for pass in 1 2; do
  for args in "--config 3 --steps 60" "--config 5 --steps 6 --warmup 2" "--raw-keys --key-bytes 8 --bits-per-key 14 --steps 60"; do
    for v in 0 7; do
      out=$(VBF_STAGGER=$v timeout -k 10 200 python bench.py --no-cpu-baseline $args 2>/dev/null | tail -1) || { echo "FAIL $v $args"; exit 1; }
      python3 - "$args" "$v" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[3]); ph = d["roofline"].get("phases", {})
print("%-50s stagger %s  %.3f ms  %s" % (sys.argv[1], sys.argv[2], d["ms_per_step"], {k: round(v["ms_per_launch"], 3) for k, v in ph.items()}))
PY
    done
  done
done
