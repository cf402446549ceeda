#!/bin/bash
# round 4: the population read-group path -- every multisample GPU test (incl. the configs[4] full-size VCF and the
# sharded population runs), then the configs[4] bench line with rocprof kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04q}
timeout -k 10 900 python -u -m pytest tests/test_gpu_multisample.py tests/test_gpu_pool.py tests/test_gpu_indels.py \
    tests/test_gpu_known.py tests/test_sharding.py "tests/test_gpu_full_size.py::test_full_size_population_vcf_identical" \
    -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ms_$TAG -o run --output-format csv -- \
    python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4 \
    > gpurun_out/${TAG}_ms_prof.json 2> gpurun_out/${TAG}_ms_prof.err || { tail -5 gpurun_out/${TAG}_ms_prof.err; exit 1; }
python tools/kstats.py gpurun_out/prof_ms_$TAG gpurun_out/${TAG}_ms_kernel_stats.csv
timeout -k 10 600 python -u bench.py --config multisample > gpurun_out/${TAG}_ms_bench.json 2> gpurun_out/${TAG}_ms_bench.err || { tail -20 gpurun_out/${TAG}_ms_bench.err; exit 1; }
cat gpurun_out/${TAG}_ms_bench.json
