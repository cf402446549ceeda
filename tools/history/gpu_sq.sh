#!/bin/bash
# SQ counters of the chr20 headline kernels (one --pmc pass with --kernel-trace only)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/sq1 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold --no-e2e > gpurun_out/sq1.out 2>&1 || exit $?
python tools/sq_counters.py gpurun_out/sq1 k_tile_scan k_posterior ko_fused ko_scan
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/sq2 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold --no-e2e > gpurun_out/sq2.out 2>&1 || exit $?
python tools/sq_counters.py gpurun_out/sq2 k_tile_scan k_posterior ko_fused ko_scan
