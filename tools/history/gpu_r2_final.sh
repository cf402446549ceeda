#!/bin/bash
# round-2 closing measurements on one box: chr20 kernel stats + PMC traffic (KT, KP), multisample PMC + bench +
# kernel stats, the configs[3] shard-0 bench line, smoke.  Usage: bash tools/gpu_r2_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02d}
mkdir -p gpurun_out
bash tools/gpu_profile.sh $TAG > gpurun_out/final_prof_$TAG.log 2>&1 || { tail -5 gpurun_out/final_prof_$TAG.log; exit 1; }
echo "profile done"
bash tools/gpu_ms_bench.sh ms_$TAG > gpurun_out/final_ms_$TAG.log 2>&1 || { tail -5 gpurun_out/final_ms_$TAG.log; exit 1; }
echo "multisample done"
timeout -k 10 600 python -u bench.py --config wgs --wgs-shards 8 --wgs-shard 0 --steps 5 --warmup 1 --no-cold > gpurun_out/bench_wgs_$TAG.json 2> gpurun_out/bench_wgs_$TAG.err || { tail -5 gpurun_out/bench_wgs_$TAG.err; exit 1; }
echo "wgs done"
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
echo "smoke done"
