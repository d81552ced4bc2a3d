#!/bin/bash
# round-5 final check on the shipped build: the whole -m gpu suite, smoke(), the default bench
# line and its rocprofv3 kernel summary.  Each GPU step has its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 400 --timeout-method thread > $O/suite.log 2>&1 || exit $?
echo suite ok
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 420 python3 bench.py > $O/bench_default.log 2>&1 || exit $?
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof10 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 40 --warmup 5 > $O/prof10.log 2>&1 || exit $?
echo done
