set -o pipefail
K3_BPK=10 K3_VARIANTS="0 3 8 10 11 12" timeout -k 10 400 bash tools/k3_sweep.sh > gpurun_out/k3_sweep_group.log 2>&1 || exit 1
for a in 0 3; do
  out=$(VBF_LIB=velarixdb_amd/libvbf_ablate.so VBF_ABLATE=$a timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 5 2>/dev/null | tail -1) || exit 1
  echo "ablate $a $out" | cut -c1-60 >> gpurun_out/k3_sweep_group.log
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('ablate', sys.argv[2], {k: round(v['ms_per_launch'],3) for k,v in d['roofline']['phases'].items()})" "$out" $a >> gpurun_out/k3_sweep_group.log
done
