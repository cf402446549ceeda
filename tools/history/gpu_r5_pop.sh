#!/bin/bash
# round 5: KLM with the count bound -- population GPU tests (incl. the full-size configs[4] shard), the configs[4]
# bench line, its rocprof kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05b}
timeout -k 10 700 python -u -m pytest tests/test_gpu_multisample.py tests/test_gpu_pool.py tests/test_gpu_known.py \
    tests/test_gpu_realigner_cases.py "tests/test_gpu_full_size.py::test_full_size_population_vcf_identical" \
    -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
B="python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4"
NGSEP_TIME_POSTERIOR=1 timeout -k 10 400 $B > gpurun_out/${TAG}_ms_bench.json 2> gpurun_out/${TAG}_ms_bench.err || { tail -20 gpurun_out/${TAG}_ms_bench.err; exit 1; }
cat gpurun_out/${TAG}_ms_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_ms -o run --output-format csv -- $B > gpurun_out/prof_${TAG}_ms.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}_ms.out; exit 1; }
python tools/kstats.py gpurun_out/prof_${TAG}_ms gpurun_out/${TAG}_ms_kernel_stats.csv
head -12 gpurun_out/${TAG}_ms_kernel_stats.csv
