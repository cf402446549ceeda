#!/bin/bash
# round 3: selected GPU tests in one process, each bounded.  Usage: bash tools/gpu_r3_tests2.sh TAG pytest-args...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tests_$TAG.log | tail -30
exit $rc
