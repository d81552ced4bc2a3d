#!/bin/bash
# round-5 GPU session 2: k_seg_or's read loop with non-temporal group loads (tools/rdflat), and the
# config-5 build's kernel times and K1 SQ counters
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 ./tools/rdflat > $O/g2_rdflat.txt 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$O/g2_prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > $O/g2_bench5.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $PWD/$O/g2_sq5 -o run --output-format csv -- python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > $O/g2_sq5.log 2>&1 || exit $?
echo done
