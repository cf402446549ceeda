#!/bin/bash
# round 3: GPU tests (args: pytest selection), one process, each test bounded.  Usage: bash tools/gpu_r3_tests.sh TAG [pytest args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
shift
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -30 gpurun_out/tests_$TAG.log
exit $rc
