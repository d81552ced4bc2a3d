#!/bin/bash
# two-window K1 A/B: one window (K1W=0), two windows with the 80-slot stash (K1W=1), and with a
# 64-slot stash (libvbf_var.so, the one-window tile sizes) -- separates the windows' own cost
# from the larger tile's.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/k1w
mkdir -p $O
for args in "--bits-per-key 19" ""; do
  for v in "0 " "1 " "1 velarixdb_amd/libvbf_var.so"; do
    set -- $v
    e=$1; lib=${2:-}
    VBF_LIB=$lib VBF_K1W=$e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 --warmup 5 $args > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]); print('$args', 'K1W=$e', '$lib', round(d['value']/1e9,3), 'G keys/s', {k: round(v['ms_per_launch'],3) for k,v in d['roofline'].get('phases', {}).items()})" | tee -a $O/ab2.txt
  done
done
echo done
