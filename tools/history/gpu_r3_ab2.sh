#!/bin/bash
# round 3: parity after the KP/KPM/KG changes, KG sites-per-wave A/B, multisample kernel times, chr20 end to end.
# Usage: bash tools/gpu_r3_ab2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-ab2}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_multisample.py tests/test_gpu_known.py tests/test_gpu_pool.py tests/test_gpu_indels.py > gpurun_out/ab2_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/ab2_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/ab2_tests_$TAG.log
B="python bench.py --no-cpu-baseline --no-cold --no-e2e --steps 10 --warmup 2"
for K in 4 8 2; do
  NGSEP_KG_SITES=$K timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kg_${TAG}_$K -o run --output-format csv -- $B > gpurun_out/kg_${TAG}_$K.out 2>&1 || { tail -5 gpurun_out/kg_${TAG}_$K.out; exit 1; }
  echo "KG $K: $(python tools/kstats.py gpurun_out/kg_${TAG}_$K | grep -E 'k_read_scan|k_gather_kl|k_posterior' | head -3 | tr -s ' ' | cut -c1-60 | tr '\n' ';')"
done
M="python bench.py --config multisample --steps 5 --warmup 2 --no-cpu-baseline --no-cold --no-e2e"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ms_${TAG} -o run --output-format csv -- $M > gpurun_out/ms_${TAG}.out 2>&1 || { tail -5 gpurun_out/ms_${TAG}.out; exit 1; }
echo "MS: $(python tools/kstats.py gpurun_out/ms_${TAG} | grep -E 'k_scan_multi|k_posterior_multi' | head -2 | tr -s ' ' | cut -c1-60 | tr '\n' ';')"
bash tools/gpu_r3_e2e.sh $TAG > /dev/null || exit 1
grep "end-to-end" gpurun_out/e2e_${TAG}_1.log gpurun_out/e2e_${TAG}_2.log
grep "call_bam:" gpurun_out/e2e_${TAG}_2.err
