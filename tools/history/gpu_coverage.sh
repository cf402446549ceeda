# CoverageStats on the GPU: parity tests, bench, rocprof kernel stats.  Usage: bash tools/gpu_coverage.sh TAG
set -e
TAG=${1:-cov}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_coverage.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests_cov_$TAG.log 2>&1
timeout -k 10 300 python bench.py --config coverage --steps 20 --warmup 3 > gpurun_out/bench_cov_$TAG.json 2> gpurun_out/bench_cov_$TAG.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cov_$TAG -o run --output-format csv -- python bench.py --config coverage --steps 20 --warmup 3 > gpurun_out/prof_cov_$TAG.out 2>&1
NGSEP_COV_TILE=2048 timeout -k 10 300 python bench.py --config coverage --steps 20 --warmup 3 > gpurun_out/bench_cov2048_$TAG.json 2> gpurun_out/bench_cov2048_$TAG.err
echo done
