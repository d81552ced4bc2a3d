#!/bin/bash
# round 5: speed-only knobs re-swept on the round-5 kernels (VBF_K3 segment-reader variants,
# VBF_TILE_PAD workspace tile pad) at k = 10 and 19; two passes.
set -u
one() {  # $1 = env assignment, $2 = bench args
  out=$(env $1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 80 --warmup 5 $2 2>/dev/null | tail -1) || { echo "FAIL $1 $2"; exit 1; }
  python3 - "$1" "$2" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[3]); ph = d["roofline"].get("phases", {})
print("%-18s %-20s %.3f ms  %s" % (sys.argv[1], sys.argv[2], d["ms_per_step"], {k: round(v["ms_per_launch"], 3) for k, v in ph.items()}))
PY
}
for pass in 1 2; do
  for a in "--bits-per-key 10" "--bits-per-key 19"; do
    for v in 0 10 11 12 13 3 8; do one "VBF_K3=$v" "$a"; done
    for v in 0 4 8 16; do one "VBF_TILE_PAD=$v" "$a"; done
  done
done
