#!/bin/bash
# pool genotyping (ploidy >= 3) GPU parity tests, then the known-variant / parity suites they touch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_multisample.py tests/test_capi.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pool_tests.log 2>&1
rc=$?
tail -25 gpurun_out/pool_tests.log
exit $rc
