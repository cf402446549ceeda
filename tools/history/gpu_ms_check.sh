#!/bin/bash
# multisample check: the population GPU tests, then the configs[4] bench with PMC traffic and kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multisample.py tests/test_sharding.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ms_tests.log 2>&1
rc=$?
tail -5 gpurun_out/ms_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ms_bench.sh ${1:-r02ms}
