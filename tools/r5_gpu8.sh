#!/bin/bash
# round-5 GPU session 8: config 5 with one k_tile_pack workgroup per CU
# (VBF_TILE_LDS_MIN=98304, same 7 168-key tile: what losing the second workgroup costs K1) and the
# k_seg_or reads of a twice-as-large tile (tools/rdflat cfg5x2: half the tiles, ~14-entry runs)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out
timeout -k 10 300 ./tools/rdflat > $O/g8_rdflat.txt 2>&1 || exit $?
for e in "" "VBF_TILE_LDS_MIN=98304" "" "VBF_TILE_LDS_MIN=98304"; do
  env $e timeout -k 10 300 python -u bench.py --config 5 --steps 3 --no-cpu-baseline > $O/g8_tmp.log 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/g8_tmp.log') if l.startswith('{')][-1]); print('${e:-default}', round(d['ms_per_step'],3), {k: round(x['ms_per_launch'],3) for k,x in d['roofline'].get('phases', {}).items()})" >> $O/g8_cfg5.txt
done
echo done
