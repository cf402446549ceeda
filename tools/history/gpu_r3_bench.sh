#!/bin/bash
# round 3: the default bench line (configs[2] chr20) and its stderr.  Usage: bash tools/gpu_r3_bench.sh TAG [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
shift
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
