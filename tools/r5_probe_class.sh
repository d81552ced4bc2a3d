#!/bin/bash
# round 5: runtime-k class probe packs -- probe / multi / parity tests, then the positive sweeps at
# k = 7, 14, 23 with the classes (default) and VBF_KCLASS=0 (the scratch-stash packs).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/pclass
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_probe.py tests/test_gpu_multi.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_probe.log 2>&1 || exit $?
echo tests ok
for pass in 1 2; do
  for b in 7 14 23; do
    for e in 1 0; do
      VBF_KCLASS=$e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --bits-per-key $b > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
      python3 -c "import json; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]); print('bpk $b KCLASS=$e build', round(d['ms_per_step'],3), 'ms  positive sweep', {k: round(v,3) for k,v in d['positive_sweep_ms'].items()})" | tee -a $O/sweep.txt
    done
  done
done
echo done
