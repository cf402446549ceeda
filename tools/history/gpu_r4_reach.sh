#!/bin/bash
# round 4: realigner regions drawn from the overlapping alignments (event_reach) -- every indel-path GPU test, then
# the chr20 end to end with the indel leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r04s}
timeout -k 10 900 python -u -m pytest tests/test_gpu_indels.py tests/test_gpu_known.py tests/test_gpu_multisample.py \
    tests/test_gpu_pool.py tests/test_sharding.py -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
bash tools/gpu_r4_e2e.sh ${TAG}
