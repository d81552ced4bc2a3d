#!/bin/bash
# A/B of speed-only knobs: AB_ENVS="VAR=a VAR=b ..." -- config-2 bench phases under each setting
# (AB_PARITY=1 also runs the build parity tests under each).  Stops at the first GPU fault / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
i=0
for e in ${AB_ENVS}; do
  i=$((i+1))
  echo "== $e"
  if [ "${AB_PARITY:-0}" = 1 ]; then
    env $e timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_pytest_$i.log 2>&1
    rc=$?; tail -n 1 gpurun_out/ab_pytest_$i.log
    [ $rc -le 1 ] || exit $rc
  fi
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 ${AB_ARGS:-} > gpurun_out/ab_bench_$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_bench_$i.log; exit $rc; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_bench_$i.log') if l.startswith('{')][-1]); print(round(d['value']/1e9,2), 'G keys/s', {k: round(v['ms_per_launch'],3) for k,v in d['roofline'].get('phases', {}).items()})"
done
