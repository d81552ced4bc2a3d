#!/bin/bash
# round-5 GPU session 9: class 32 at m > 2^31 with runtime-length keys (its stash left scratch
# memory with the seed-slot fold): config 3 at 30 bits per key (m = 3e9, k = 30) against the
# round-start library; and the 2-rank launch rehearsal on the box's one GPU (gloo, shared device)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out
AB_LIB=velarixdb_amd/libvbf_base.so timeout -k 10 600 bash tools/ab_lib.sh 2 --config 3 --bits-per-key 30 --keys 50000000 --neg-keys 1000000 --steps 20 > $O/g9_ab_k30.txt 2>&1 || exit $?
VBF_SHARE_DEVICE=1 VBF_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 50 --no-cpu-baseline > $O/g9_dist2.log 2>&1 || exit $?
echo done
