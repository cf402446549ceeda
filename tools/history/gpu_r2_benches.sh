#!/bin/bash
# round-2 bench lines of the current build: configs[2] chr20 (default), configs[4] multisample, configs[3] shard 0
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02e}
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
echo chr20 done
timeout -k 10 600 python -u bench.py --config multisample --steps 20 --warmup 4 > gpurun_out/bench_ms_$TAG.json 2> gpurun_out/bench_ms_$TAG.err || { tail -5 gpurun_out/bench_ms_$TAG.err; exit 1; }
echo multisample done
timeout -k 10 900 python -u bench.py --config wgs --wgs-shards 8 --wgs-shard 0 --steps 10 --warmup 3 --no-cold > gpurun_out/bench_wgs_$TAG.json 2> gpurun_out/bench_wgs_$TAG.err || { tail -5 gpurun_out/bench_wgs_$TAG.err; exit 1; }
echo wgs done
