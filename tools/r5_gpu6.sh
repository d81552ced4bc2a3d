#!/bin/bash
# round-5 GPU session 6: the probe pack's seed fold -- probe parity, then the positive sweeps of
# config 5 (k_probe_pack, SAT) and config 2 at k = 10 / 19 against the round-start library
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_probe.py tests/test_gpu_multi.py > $O/g6_parity.log 2>&1 || exit $?
for i in 1 2; do
  for lib in "" velarixdb_amd/libvbf_base.so; do
    for a in "--config 5 --steps 3" "--steps 100" "--bits-per-key 19 --steps 50"; do
      VBF_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline $a > $O/g6_tmp.log 2>&1 || exit $?
      python - "$lib" "$a" <<'PY' >> $O/g6_probe.txt
import json, sys
d = json.loads([l for l in open("gpurun_out/g6_tmp.log") if l.startswith("{")][-1])
print("%-30s %-32s build %.3f ms  sweep %s" % (sys.argv[1] or "libvbf.so", sys.argv[2], d["ms_per_step"],
      d.get("probe_sweep_keys_per_s") and "%.2f G/s" % (d["probe_sweep_keys_per_s"] / 1e9) or d.get("positive_sweep_ms")))
PY
    done
  done
done
echo done
