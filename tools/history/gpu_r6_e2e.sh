#!/bin/bash
# round 6: end-to-end legs (BAM -> VCF) under host settings: NGSEP_INFLATE_GATE (readers of a context inflating at once,
# 0 = no gate) for the 200-BAM population and chr20, alternated
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06e2e}
GATES=${2:-"0 2 4"}
CFGS=${3:-"multisample chr20"}
for it in 1 2; do
  for cfg in $CFGS; do
    for g in $GATES; do
      NGSEP_INFLATE_GATE=$g NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline --no-cold --steps 3 --warmup 1 \
          > gpurun_out/${TAG}_${cfg}_g${g}_$it.json 2> gpurun_out/${TAG}_${cfg}_g${g}_$it.err || { tail -20 gpurun_out/${TAG}_${cfg}_g${g}_$it.err; exit 1; }
      python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_${cfg}_g${g}_$it.json").read().strip().splitlines()[-1])
e = d.get("end_to_end") or {}
print("$cfg gate $g it $it", "e2e %.3f s" % e.get("wall_s", 0), "indels", (e.get("indels") or {}).get("wall_s"))
PY
      grep -a "population: open\|population: merge + sweep\|population: end of" gpurun_out/${TAG}_${cfg}_g${g}_$it.err | tr '\n' ' '; echo
    done
  done
done
