#!/bin/bash
# round 4: the population read-group path (KLM + gather KPM) -- multisample GPU tests, then the configs[4] bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r04p}
timeout -k 10 600 python -u -m pytest tests/test_gpu_multisample.py tests/test_gpu_pool.py tests/test_gpu_indels.py \
    tests/test_gpu_known.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4 \
    > gpurun_out/${TAG}_ms_bench.json 2> gpurun_out/${TAG}_ms_bench.err || { tail -20 gpurun_out/${TAG}_ms_bench.err; exit 1; }
cat gpurun_out/${TAG}_ms_bench.json
