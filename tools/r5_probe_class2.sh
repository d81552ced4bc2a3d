#!/bin/bash
# round 5: class probe packs without the length prefix -- probe tests, then the raw-key sweep A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/pclass2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_probe.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_probe.log 2>&1 || exit $?
echo tests ok
for pass in 1 2; do
  for e in 1 0; do
    VBF_KCLASS=$e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --raw-keys --key-bytes 8 --bits-per-key 14 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]); print('raw 8B k=14 KCLASS=$e build', round(d['ms_per_step'],3), 'ms  positive sweep', {k: round(v,3) for k,v in d['positive_sweep_ms'].items()})" | tee -a $O/sweep.txt
  done
done
echo done
