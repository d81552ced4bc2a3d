#!/bin/bash
# A/B of two library builds on one box: alternates `bench.py` runs with VBF_LIB unset (the product
# libvbf.so) and VBF_LIB=$AB_LIB, printing each run's value and per-phase ms.  Speed only.
# usage: AB_LIB=velarixdb_amd/libvbf_ab.so tools/ab_lib.sh [ROUNDS] [bench.py args...]
set -u
ROUNDS=${1:-3}; shift || true
for i in $(seq 1 "$ROUNDS"); do
  for lib in "" "$AB_LIB"; do
    out=$(VBF_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -1) || exit $?
    python - "$lib" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2])
ph = d.get("roofline", {}).get("phases", {})
print("%-32s %.3f G/s  %s" % (sys.argv[1] or "libvbf.so", d["value"] / 1e9,
      "  ".join("%s %.3f" % (k, v["ms_per_launch"]) for k, v in ph.items())))
PY
  done
done
