#!/bin/bash
# the whole -m gpu suite and smoke(), as the driver runs them at round end
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 400 --timeout-method thread > $O/suite.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo done
