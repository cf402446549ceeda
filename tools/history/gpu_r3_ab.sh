#!/bin/bash
# round 3: parity of the changed kernels, then A/B kernel times (KL sparse vs packed adds, KPM wave vs block, KTM).
# Usage: bash tools/gpu_r3_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_multisample.py tests/test_gpu_known.py tests/test_gpu_pool.py > gpurun_out/ab_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/ab_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/ab_tests_$TAG.log
bash tools/gpu_r3_klab.sh $TAG 0 4096 || exit 1
M="python bench.py --config multisample --steps 5 --warmup 2 --no-cpu-baseline --no-cold --no-e2e"
for E in "NGSEP_X=0" "NGSEP_KPM_BLOCK=1"; do
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kpm_${TAG}_${E%%=*} -o run --output-format csv -- $M > gpurun_out/kpm_${TAG}_${E%%=*}.out 2>&1 || { tail -5 gpurun_out/kpm_${TAG}_${E%%=*}.out; exit 1; }
  echo "$E: $(python tools/kstats.py gpurun_out/kpm_${TAG}_${E%%=*} | grep -E 'k_scan_multi|k_posterior_multi' | head -2 | tr -s ' ' | cut -c1-70 | tr '\n' ';')"
done
