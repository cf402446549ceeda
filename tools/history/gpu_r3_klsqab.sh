#!/bin/bash
# round 3: SQ/LDS counters of KL under NGSEP_ABLATE values (diagnostics).  Usage: bash tools/gpu_r3_klsqab.sh TAG AB...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-cold --no-e2e"
for AB in "$@"; do
  NGSEP_ABLATE=$AB timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/klsqab_${TAG}_$AB -o run --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/klsqab_${TAG}_$AB.out 2>&1 || exit 1
  echo "ablate $AB:"; python tools/sq_counters.py gpurun_out/klsqab_${TAG}_$AB k_read_scan
done
for AB in "$@"; do
  NGSEP_ABLATE=$AB timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_MEM_VIOLATIONS SQ_INSTS_SALU SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/klsqab2_${TAG}_$AB -o run --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/klsqab2_${TAG}_$AB.out 2>&1 || { tail -3 gpurun_out/klsqab2_${TAG}_$AB.out; exit 1; }
  echo "ablate $AB:"; python tools/sq_counters.py gpurun_out/klsqab2_${TAG}_$AB k_read_scan
done
