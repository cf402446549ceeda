#!/bin/bash
# round 4: PMC calibration, KL kernel stats + PMC traffic, the default bench line, then the full-size GPU tests.
# Usage: bash tools/gpu_r4_main.sh TAG [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04}
mkdir -p gpurun_out
KEY=human_chr20:30x:seed3:v3
B="python bench.py --no-cpu-baseline --no-cold --no-e2e"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/calib_$TAG -o run --output-format csv -- tools/calib/build/pmc_calib > gpurun_out/calib_$TAG.out 2>&1 || { echo calib failed; tail -5 gpurun_out/calib_$TAG.out; exit 1; }
python tools/pmc_calib.py gpurun_out/calib_$TAG gpurun_out/pmc_calibration_$TAG.json || exit 1
mkdir -p profiles && cp gpurun_out/pmc_calibration_$TAG.json profiles/pmc_calibration.json
echo "calibration done"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- $B --steps 20 --warmup 3 > gpurun_out/prof_$TAG.out 2>&1 || { tail -5 gpurun_out/prof_$TAG.out; exit 1; }
python tools/kstats.py gpurun_out/prof_$TAG gpurun_out/kernel_stats_$TAG.csv
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_$TAG -o run --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/pmcf_$TAG.out 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_$TAG -o run --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/pmcw_$TAG.out 2>&1 || exit 1
python tools/pmc_traffic.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG k_read_scan $KEY gpurun_out/pmc_traffic_$TAG.json 8
python tools/pmc_traffic.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG k_posterior kp:$KEY gpurun_out/pmc_traffic_kp_$TAG.json 4
echo "profile done"
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
echo "bench done"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_full_size.py tests/test_gpu_wgs_shard.py > gpurun_out/tests_full_$TAG.log 2>&1
  rc=$?
  tail -15 gpurun_out/tests_full_$TAG.log
  exit $rc
fi
