#!/bin/bash
# round 4: multisample window sizes (parity), then the N-rank rehearsal of the configs[4] bench on one card (gloo)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "tests/test_gpu_multisample.py::test_population_window_sizes" -m gpu -x -v \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_win_tests.log 2>&1 || { tail -30 gpurun_out/r04_win_tests.log; exit 1; }
tail -3 gpurun_out/r04_win_tests.log
NGSEP_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --config multisample --gpus 2 --no-cpu-baseline --no-cold --no-e2e \
    --steps 10 --warmup 2 > gpurun_out/r04_ms_gpus2.json 2> gpurun_out/r04_ms_gpus2.err || { tail -20 gpurun_out/r04_ms_gpus2.err; exit 1; }
cat gpurun_out/r04_ms_gpus2.json
