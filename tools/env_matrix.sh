#!/bin/bash
# Speed-only knob matrix: MATRIX="A=1 B=2;C=3;..." (';' separates settings, spaces the variables of
# one setting; "-" = no variables) -- bench.py phases under each setting at each BPK ("10 19").
# Stops at the first failing run.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${MATRIX}"
for bpk in ${BPK:-10 19}; do
  for e in "${SETS[@]}"; do
    vars=$e; [ "$vars" = "-" ] && vars=""
    out=$(env $vars timeout -k 10 120 python bench.py --no-cpu-baseline --steps ${STEPS:-50} --warmup 5 --bits-per-key $bpk 2>/dev/null | tail -1) || { echo "FAIL [$e] k $bpk"; exit 1; }
    python3 - "$bpk" "$e" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[3]); ph = d['roofline']['phases']
print('bpk %-3s %-36s %6.2f G/s %.3f ms' % (sys.argv[1], sys.argv[2], d['value'] / 1e9, d['ms_per_step']),
      {k: round(v['ms_per_launch'], 3) for k, v in ph.items()})
PY
  done
done
