#!/bin/bash
# full GPU suite (what the driver runs at round end) + smoke, on the current tree
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s2_suite.log 2>&1
rc=$?
tail -6 gpurun_out/s2_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2_smoke.log 2>&1
rc=$?
tail -2 gpurun_out/s2_smoke.log
exit $rc
