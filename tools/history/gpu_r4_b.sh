#!/bin/bash
# round 4: the -knownVariants indel tests after the scan-timing fix, then the main measurement (tools/gpu_r4_main.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_known.py "tests/test_gpu_pool.py::test_pool_known_indels_vcf_identical" \
    -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04b_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_r4_main.sh r04b skip-tests
