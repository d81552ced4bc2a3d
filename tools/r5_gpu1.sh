#!/bin/bash
# round-5 GPU session 1: parity of the changed K1 length sort, config-3 and config-2 A/B against the
# round-start library, FETCH_SIZE calibration of the 8-byte key loads
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "variable or knob or fresh or concentrated" tests/test_gpu_scale.py::test_config3_full_size_bit_exact > $O/g1_parity.log 2>&1 || exit $?
AB_LIB=velarixdb_amd/libvbf_base.so timeout -k 10 600 bash tools/ab_lib.sh 3 --config 3 --steps 200 > $O/g1_ab_cfg3.txt 2>&1 || exit $?
AB_LIB=velarixdb_amd/libvbf_base.so timeout -k 10 600 bash tools/ab_lib.sh 2 --steps 300 > $O/g1_ab_cfg2.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $PWD/$O/fcalib -o run --output-format csv -- ./tools/fetch_calib 50000000 > $O/g1_fcalib.log 2>&1 || exit $?
echo done
