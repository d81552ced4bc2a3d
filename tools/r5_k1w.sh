#!/bin/bash
# round 5: the two-window K1 (VBF_K1W) -- the knob parity test (K1W = 1/2/3 among the others), the
# full-size bit-exact builds with K1W = 1, then bench A/B K1W = 0 / 1 at k = 10, k = 19, config 3.
# Each GPU step under its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/k1w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 500 --timeout-method thread -k "kernel_knobs" > $O/pytest_knobs.log 2>&1 || exit $?
echo knobs ok
VBF_K1W=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -v -m gpu --timeout 300 --timeout-method thread -k "config2_full_size or k19_full_size or config3_full_size" > $O/pytest_full.log 2>&1 || exit $?
echo full ok
for args in "" "--bits-per-key 19" "--config 3"; do
  for rep in 1 2; do
    for e in 0 1; do
      VBF_K1W=$e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 --warmup 5 $args > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
      python -c "import json,sys; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]); print('$args', 'K1W=$e', round(d['value']/1e9,3), 'G keys/s', round(d['ms_per_step'],3), 'ms', {k: round(v['ms_per_launch'],3) for k,v in d['roofline'].get('phases', {}).items()})" | tee -a $O/ab.txt
    done
  done
done
echo done
