#!/bin/bash
# round-5 GPU session 5: the seed-slot fold in k_tile_pack and the single build chunk (2^32):
# parity, then A/B against the round-start library on configs 2, 2 at k = 19, 3
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py::test_multi_chunk_partitioned_paths tests/test_gpu_scale.py::test_config2_full_size_bit_exact > $O/g5_parity.log 2>&1 || exit $?
AB_LIB=velarixdb_amd/libvbf_base.so timeout -k 10 600 bash tools/ab_lib.sh 3 --steps 300 > $O/g5_ab_cfg2.txt 2>&1 || exit $?
AB_LIB=velarixdb_amd/libvbf_base.so timeout -k 10 600 bash tools/ab_lib.sh 2 --bits-per-key 19 --steps 200 > $O/g5_ab_k19.txt 2>&1 || exit $?
AB_LIB=velarixdb_amd/libvbf_base.so timeout -k 10 600 bash tools/ab_lib.sh 2 --config 3 --steps 200 > $O/g5_ab_cfg3.txt 2>&1 || exit $?
echo done
