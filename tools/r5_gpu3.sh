#!/bin/bash
# round-5 GPU session 3: the K1 image copy-out as non-temporal stores (VBF_IMAGE_NT), A/B against the
# round-start library on configs 2, 3 and 2 at k = 19; build parity
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "variable or fresh or concentrated or build" > $O/g3_parity.log 2>&1 || exit $?
AB_LIB=velarixdb_amd/libvbf_base.so timeout -k 10 600 bash tools/ab_lib.sh 3 --steps 300 > $O/g3_ab_cfg2.txt 2>&1 || exit $?
AB_LIB=velarixdb_amd/libvbf_base.so timeout -k 10 600 bash tools/ab_lib.sh 3 --config 3 --steps 200 > $O/g3_ab_cfg3.txt 2>&1 || exit $?
AB_LIB=velarixdb_amd/libvbf_base.so timeout -k 10 600 bash tools/ab_lib.sh 2 --bits-per-key 19 --steps 200 > $O/g3_ab_k19.txt 2>&1 || exit $?
echo done
