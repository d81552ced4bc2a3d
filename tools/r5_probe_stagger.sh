#!/bin/bash
# the partitioned positive probe sweep (bench.py's positive_sweep_ms) with VBF_STAGGER 0 / 7
set -u
for pass in 1 2; do
  for a in "--bits-per-key 10" "--bits-per-key 19"; do
    for v in 0 7; do
      out=$(VBF_STAGGER=$v timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 3 $a 2>/dev/null | tail -1) || { echo "FAIL $v $a"; exit 1; }
      python3 - "$a" "$v" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[3])
print("%-18s stagger %s  build %.3f ms  positive sweep %s" % (sys.argv[1], sys.argv[2], d["ms_per_step"], d.get("positive_sweep_ms")))
PY
    done
  done
done
