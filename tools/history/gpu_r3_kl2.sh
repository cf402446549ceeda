#!/bin/bash
# round 3: KL/KG/KP parity tests then per-kernel stats of the chr20 bench (ablations given).  Usage: bash tools/gpu_r3_kl2.sh TAG AB...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/tests_kl_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_kl_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_kl_$TAG.log
B="python bench.py --no-cpu-baseline --no-cold --no-e2e"
for AB in "$@"; do
  NGSEP_ABLATE=$AB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/klab_${TAG}_$AB -o run --output-format csv -- $B --steps 10 --warmup 2 > gpurun_out/klab_${TAG}_$AB.out 2>&1 || { tail -5 gpurun_out/klab_${TAG}_$AB.out; exit 1; }
  python tools/kstats.py gpurun_out/klab_${TAG}_$AB gpurun_out/kernel_stats_klab_${TAG}_$AB.csv > /dev/null
  echo "ablate $AB:"; cut -d, -f1,2,4 gpurun_out/kernel_stats_klab_${TAG}_$AB.csv | cut -c1-30,150- | head -8
done
