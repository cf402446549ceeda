#!/bin/bash
# round 4: parity of the new paths (-knownVariants with the realigner, pool indels, window sharding) and the core
# suite after the KL exception-queue change, then a short default bench (KL timing)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known.py tests/test_gpu_pool.py \
    tests/test_gpu_multisample.py tests/test_gpu_indels.py tests/test_sharding.py -m gpu -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r04a_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 3 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err
echo "bench rc=$?"
