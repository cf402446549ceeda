#!/bin/bash
# round 3: KL kernel time per unroll depth (NGSEP_KL_UNROLL) and ablation (diagnostics).  Usage: bash tools/gpu_r3_klu.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-cold --no-e2e"
for U in 8 16 24; do for AB in 0 128; do
  NGSEP_KL_UNROLL=$U NGSEP_ABLATE=$AB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/klu_${TAG}_${U}_$AB -o run --output-format csv -- $B --steps 10 --warmup 2 > gpurun_out/klu_${TAG}_${U}_$AB.out 2>&1 || { tail -5 gpurun_out/klu_${TAG}_${U}_$AB.out; exit 1; }
  python tools/kstats.py gpurun_out/klu_${TAG}_${U}_$AB gpurun_out/kernel_stats_klu_${TAG}_${U}_$AB.csv > /dev/null
  echo "unroll $U ablate $AB: $(grep k_read_scan gpurun_out/kernel_stats_klu_${TAG}_${U}_$AB.csv | awk -F, '{print $(NF-4)}')"
done; done
