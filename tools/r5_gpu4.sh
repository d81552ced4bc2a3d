#!/bin/bash
# round-5 GPU session 4: runtime-k classes without the length prefix (parity + A/B against the
# round-start library), config-5 single build chunk (VBF_BUILD_CHUNK_LOG2=32) A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "without_length_prefix or knobs or classes or variable" > $O/g4_parity.log 2>&1 || exit $?
AB_LIB=velarixdb_amd/libvbf_base.so timeout -k 10 600 bash tools/ab_lib.sh 2 --raw-keys --key-bytes 8 --bits-per-key 14 --steps 100 > $O/g4_ab_raw14.txt 2>&1 || exit $?
for v in 31 32 31 32; do
  VBF_BUILD_CHUNK_LOG2=$v timeout -k 10 300 python -u bench.py --config 5 --steps 5 --no-cpu-baseline > $O/g4_cfg5_chunk$v.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('$O/g4_cfg5_chunk$v.log') if l.startswith('{')][-1]); print('chunk 2^$v', round(d['ms_per_step'],3), 'ms', {k: (round(x['ms_per_launch'],3), x['launches']) for k,x in d['roofline'].get('phases', {}).items()})" >> $O/g4_cfg5_chunk.txt
done
echo done
