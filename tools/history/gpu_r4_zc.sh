#!/bin/bash
# round 4: zero-copy reader batches (call_bam) -- every test that reads BAM through ngsep_call_bam / region calls,
# the full-size single-sample VCFs, then the chr20 end to end with host timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r04zc}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_indels.py tests/test_gpu_known.py \
    tests/test_sharding.py tests/test_gpu_pool.py "tests/test_gpu_full_size.py::test_full_size_vcf_identical" \
    -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 \
    || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
bash tools/gpu_r4_e2e.sh ${TAG}
