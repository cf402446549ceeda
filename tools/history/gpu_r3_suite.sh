#!/bin/bash
# round 3: the whole GPU suite in one process, then smoke.  Usage: bash tools/gpu_r3_suite.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/suite_$TAG.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/suite_$TAG.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?
cat gpurun_out/smoke_$TAG.log
exit $rc
