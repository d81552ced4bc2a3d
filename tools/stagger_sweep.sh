#!/bin/bash
# k_tile_pack's second-workgroup stagger (VBF_STAGGER, s_sleep(127) count; speed only) at k = 10
# and 19: two alternating passes over the values.
set -u
for pass in 1 2; do
  for bpk in 10 19; do
    for v in 0 4 7 10 14; do
      out=$(VBF_STAGGER=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 5 --bits-per-key $bpk 2>/dev/null | tail -1) || { echo "FAIL $v"; exit 1; }
      python3 - "$bpk" "$v" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[3]); ph = d["roofline"]["phases"]
print("k %s stagger %s  %.3f ms  tile_sort %.3f" % (sys.argv[1], sys.argv[2], d["ms_per_step"], ph["tile_sort"]["ms_per_launch"]))
PY
    done
  done
done
