#!/bin/bash
# round 3 diagnostics: KL kernel time under NGSEP_ABLATE values, KTM under grid sizes / its ablation, chr20 end-to-end
# anatomy.  Usage: bash tools/gpu_r3_diag.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-diag}
mkdir -p gpurun_out
bash tools/gpu_r3_klab.sh $TAG 0 128 256 1 || exit 1
M="python bench.py --config multisample --steps 5 --warmup 2 --no-cpu-baseline --no-cold --no-e2e"
for E in "NGSEP_KTM_BPC=8" "NGSEP_KTM_BPC=6" "NGSEP_KTM_BPC=32" "NGSEP_ABLATE=32768"; do
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktm_${TAG}_${E#*=} -o run --output-format csv -- $M > gpurun_out/ktm_${TAG}_${E#*=}.out 2>&1 || { tail -5 gpurun_out/ktm_${TAG}_${E#*=}.out; exit 1; }
  echo "$E: $(python tools/kstats.py gpurun_out/ktm_${TAG}_${E#*=} | grep -E 'k_scan_multi|k_posterior_multi' | tr -s ' ' | cut -c1-80 | tr '\n' ';')"
done
bash tools/gpu_r3_e2e.sh $TAG
