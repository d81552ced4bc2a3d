for b in 19 10; do for v in 0 4; do
  VBF_K3=$v timeout -k 10 200 python bench.py --no-cpu-baseline --bits-per-key $b --steps 10 > gpurun_out/kab_${b}_${v}.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/kab_${b}_${v}.log') if l.startswith('{')][-1]); c=d['config']; print($b, 'K3=$v', c['k'], round(d['value']/1e9,2), 'G keys/s', round(d['ms_per_step'],2), {k: round(x['ms_per_launch'],3) for k,x in d['roofline']['phases'].items()})"
done; done
