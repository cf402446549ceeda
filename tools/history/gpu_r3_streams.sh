#!/bin/bash
# round 3: the chr20 step with one stream vs a stream per result slot (pass k+1's KL beside pass k's KG/KP/KO).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-st}
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-cold --no-e2e --steps 30 --warmup 3"
for E in "NGSEP_X=0" "NGSEP_SLOT_STREAMS=1" "NGSEP_X=0" "NGSEP_SLOT_STREAMS=1"; do
  env $E timeout -k 10 300 $B > gpurun_out/st_$TAG.json 2> gpurun_out/st_$TAG.err || { tail -5 gpurun_out/st_$TAG.err; exit 1; }
  echo "$E: $(python -c "import json; d=json.load(open('gpurun_out/st_$TAG.json')); print(round(d['ms_per_step'],4), '%.4g' % d['value'], round(d['roofline']['kernel_avg_ms'],4))")"
done
