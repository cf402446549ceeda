#!/bin/bash
# round 3: KL kernel time under a list of NGSEP_ABLATE values (diagnostics).  Usage: bash tools/gpu_r3_klab.sh TAG AB...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-cold --no-e2e"
for AB in "$@"; do
  NGSEP_ABLATE=$AB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/klab_${TAG}_$AB -o run --output-format csv -- $B --steps 10 --warmup 2 > gpurun_out/klab_${TAG}_$AB.out 2>&1 || { tail -5 gpurun_out/klab_${TAG}_$AB.out; exit 1; }
  python tools/kstats.py gpurun_out/klab_${TAG}_$AB gpurun_out/kernel_stats_klab_${TAG}_$AB.csv > /dev/null
  echo "ablate $AB: $(grep k_read_scan gpurun_out/kernel_stats_klab_${TAG}_$AB.csv | awk -F, '{print $(NF-4)}')"
done
