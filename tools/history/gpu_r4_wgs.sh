#!/bin/bash
# round 4: the configs[3] headline on one GPU -- all 24 GRCh38-length contigs, two device runs -- with peak host RSS
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/maxrss.py python -u bench.py --config wgs --gpus 1 --wgs-shards 1 --no-e2e \
    --no-cpu-baseline --no-cold --steps 5 --warmup 1 > gpurun_out/r04_wgs1.json 2> gpurun_out/r04_wgs1.err
rc=$?
tail -4 gpurun_out/r04_wgs1.err
cat gpurun_out/r04_wgs1.json
exit $rc
