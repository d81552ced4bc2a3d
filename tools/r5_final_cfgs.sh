#!/bin/bash
# round 5 final library: configs 5, 3 and 2 at k = 19 (bench lines + rocprofv3 kernel summaries)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/finalcfg
mkdir -p $O
timeout -k 10 300 python3 bench.py --no-cpu-baseline --config 5 --steps 8 --warmup 2 > $O/bench_cfg5.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --config 3 --steps 100 > $O/bench_cfg3.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --bits-per-key 19 --steps 100 > $O/bench_k19.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config 5 --steps 4 --warmup 1 > $O/prof5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof19 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --bits-per-key 19 --steps 20 --warmup 3 > $O/prof19.log 2>&1 || exit $?
echo done
