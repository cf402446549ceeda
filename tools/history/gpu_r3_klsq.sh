#!/bin/bash
# round 3: KL parity tests, KL kernel stats (ablations 0 and 128), and two SQ counter passes on KL.
# Usage: bash tools/gpu_r3_klsq.sh TAG [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r03}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/tests_kl_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_kl_$TAG.log; exit 1; }
  tail -2 gpurun_out/tests_kl_$TAG.log
fi
B="python bench.py --no-cpu-baseline --no-cold --no-e2e"
for AB in 0 128; do
  NGSEP_ABLATE=$AB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/klab_${TAG}_$AB -o run --output-format csv -- $B --steps 10 --warmup 2 > gpurun_out/klab_${TAG}_$AB.out 2>&1 || { tail -5 gpurun_out/klab_${TAG}_$AB.out; exit 1; }
  python tools/kstats.py gpurun_out/klab_${TAG}_$AB gpurun_out/kernel_stats_klab_${TAG}_$AB.csv > /dev/null
  echo "ablate $AB: $(sed -n 2p gpurun_out/kernel_stats_klab_${TAG}_$AB.csv | awk -F, '{print $(NF-4)}')"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/klsq1_$TAG -o run --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/klsq1_$TAG.out 2>&1 || exit 1
python tools/sq_counters.py gpurun_out/klsq1_$TAG k_read_scan k_gather_cols
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/klsq2_$TAG -o run --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/klsq2_$TAG.out 2>&1 || exit 1
python tools/sq_counters.py gpurun_out/klsq2_$TAG k_read_scan k_gather_cols
