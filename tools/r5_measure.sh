#!/bin/bash
# round-5 measurement refresh (profiles/r05): the default bench line, rocprofv3 kernel stats of
# configs 2 (k = 10 and 19), SQ counters of k_tile_pack (configs 2 k = 10 / 19, 3, 5) and HBM
# traffic passes (FETCH_SIZE and WRITE_SIZE in separate runs) of configs 2 (k = 10 / 19), 3, 5.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/meas
mkdir -p $O
B="python3 bench.py --no-cpu-baseline"
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -k 10 420 python3 bench.py > $O/bench_default.log 2>&1 || exit $?
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof10 -o run --output-format csv -- $B --steps 40 --warmup 5 > $O/prof10.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof19 -o run --output-format csv -- $B --steps 20 --warmup 3 --bits-per-key 19 > $O/prof19.log 2>&1 || exit $?
echo prof ok
i=0
for a in "--steps 3 --warmup 1" "--steps 3 --warmup 1 --bits-per-key 19" "--config 3 --steps 3 --warmup 1" "--config 5 --steps 2 --warmup 1"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $SQ -d $O/sq$i -o run --output-format csv -- $B $a > $O/sq$i.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch$i -o run --output-format csv -- $B $a > $O/fetch$i.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write$i -o run --output-format csv -- $B $a > $O/write$i.log 2>&1 || exit $?
  echo pmc $i ok
done
echo done
