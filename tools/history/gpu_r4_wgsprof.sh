#!/bin/bash
# round 4: rocprofv3 kernel stats of the configs[3] one-GPU headline (all 24 contigs, two device runs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wgs1 -o run --output-format csv -- \
    python -u bench.py --config wgs --gpus 1 --wgs-shards 1 --no-e2e --no-cpu-baseline --no-cold --steps 5 --warmup 1 \
    > gpurun_out/prof_wgs1.json 2> gpurun_out/prof_wgs1.err || { tail -5 gpurun_out/prof_wgs1.err; exit 1; }
python tools/kstats.py gpurun_out/prof_wgs1 gpurun_out/kernel_stats_wgs1.csv
cat gpurun_out/prof_wgs1.json
