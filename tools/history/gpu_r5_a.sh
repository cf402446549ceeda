#!/bin/bash
# round 5: the tests touched by the ADVICE r04 fixes, then the whole GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gpu_realigner_cases.py tests/test_gpu_known.py tests/test_gpu_multisample.py tests/test_sharding.py > gpurun_out/r05a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r05a_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu -p no:cacheprovider tests \
    > gpurun_out/r05a_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r05a_suite.log
exit $rc
