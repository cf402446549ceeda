#!/bin/bash
# round 3: KTM with per-byte LDS adds into the lane's allele sums -- multisample parity, then the configs[4] step.
# Usage: bash tools/gpu_r3_ktm3.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-ktm3}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multisample.py tests/test_gpu_pool.py "tests/test_gpu_full_size.py::test_full_size_population_vcf_identical" > gpurun_out/ktm3_tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/ktm3_tests_$TAG.log | head -20; tail -5 gpurun_out/ktm3_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/ktm3_tests_$TAG.log
B="python bench.py --config multisample --steps 20 --warmup 3 --no-cpu-baseline --no-cold --no-e2e"
for k in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/k3_$TAG.json 2> gpurun_out/k3_$TAG.err || { tail -5 gpurun_out/k3_$TAG.err; exit 1; }
  echo "run $k: $(python -c "import json; d=json.load(open('gpurun_out/k3_$TAG.json')); r=d['roofline']; print('step', round(d['ms_per_step'],4), 'KTM+KQN', round(r['kernel_avg_ms'],4), 'frac', round(r['frac'],4), 'KPM', r.get('posterior_kernel_avg_ms'))")"
done
