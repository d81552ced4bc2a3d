set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
AB_LIB=velarixdb_amd/libvbf_var.so timeout -k 10 600 bash tools/ab_lib.sh 3 --steps 300 > gpurun_out/g7_ab_cfg2.txt 2>&1 || exit $?
AB_LIB=velarixdb_amd/libvbf_var.so timeout -k 10 600 bash tools/ab_lib.sh 2 --bits-per-key 19 --steps 200 > gpurun_out/g7_ab_k19.txt 2>&1 || exit $?
