#!/bin/bash
# A/B of two library builds on the partitioned probe: bench.py's positive sweep (100M keys, all
# k lookups each) per build, alternating.  usage: AB_LIB=... tools/ab_probe.sh ROUNDS [bench args]
set -u
ROUNDS=${1:-3}; shift || true
for i in $(seq 1 "$ROUNDS"); do
  for lib in "" "$AB_LIB"; do
    out=$(VBF_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 "$@" 2>/dev/null | tail -1) || exit $?
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print('%-32s' % (sys.argv[1] or 'libvbf.so'), 'probe ms', {k: round(v, 3) for k, v in d['positive_sweep_ms'].items()})" "$lib" "$out"
  done
done
