#!/bin/bash
# round 3: KL parity tests, then per-kernel stats of the chr20 bench under the KL ablations (diagnostics).
# Usage: bash tools/gpu_r3_kl.sh TAG [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r03}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/tests_kl_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_kl_$TAG.log; exit 1; }
  tail -3 gpurun_out/tests_kl_$TAG.log
fi
B="python bench.py --no-cpu-baseline --no-cold --no-e2e"
for AB in 0 128 256; do
  NGSEP_ABLATE=$AB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/klab_${TAG}_$AB -o run --output-format csv -- $B --steps 10 --warmup 2 > gpurun_out/klab_${TAG}_$AB.out 2>&1 || { tail -5 gpurun_out/klab_${TAG}_$AB.out; exit 1; }
  python tools/kstats.py gpurun_out/klab_${TAG}_$AB gpurun_out/kernel_stats_klab_${TAG}_$AB.csv
  echo "ablate $AB:"; head -4 gpurun_out/kernel_stats_klab_${TAG}_$AB.csv | cut -c1-60,200-
done
