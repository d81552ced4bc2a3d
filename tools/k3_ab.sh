#!/bin/bash
# A/B of the k_seg_or tile-loop variants (VBF_K3): parity tests of the build under each, then
# the config-2 bench phases.  Stops at the first GPU fault / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for v in ${K3_VARIANTS:-0 2 3 4 5}; do
  echo "== VBF_K3=$v"
  VBF_K3=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/k3_pytest_$v.log 2>&1
  rc=$?; tail -n 2 gpurun_out/k3_pytest_$v.log
  [ $rc -le 1 ] || exit $rc
  VBF_K3=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/k3_bench_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/k3_bench_$v.log; exit $rc; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/k3_bench_$v.log') if l.startswith('{')][-1]); print(round(d['value']/1e9,2), 'G keys/s', {k: round(v['ms_per_launch'],3) for k,v in d['roofline']['phases'].items()})"
done
