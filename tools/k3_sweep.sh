#!/bin/bash
set -u
mkdir -p gpurun_out
for bpk in ${K3_BPK:-19 10}; do
for v in ${K3_VARIANTS:-0 1 3 4 5 6 8 10 11 12}; do
  out=$(VBF_K3=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 5 --bits-per-key $bpk 2>/dev/null | tail -1) || { echo "FAIL $v"; exit 1; }
  python3 - "$bpk" "$v" "$out" <<'PY'
import json,sys
d=json.loads(sys.argv[3]); ph=d['roofline']['phases']
print('k', sys.argv[1], 'K3', sys.argv[2], round(d['ms_per_step'],3), {k: round(v['ms_per_launch'],3) for k,v in ph.items()})
PY
done
done
