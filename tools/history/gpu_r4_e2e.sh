#!/bin/bash
# round 4: chr20 end to end (SNV data and the indel leg) with host timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r04e}
NGSEP_HOST_TIMING=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-cold --steps 5 --warmup 2 \
    > gpurun_out/${TAG}_e2e.json 2> gpurun_out/${TAG}_e2e.err || { tail -20 gpurun_out/${TAG}_e2e.err; exit 1; }
grep "end-to-end\|ngsep host\] \(bam\|total\|reader\|window\|sequence\|call\)" gpurun_out/${TAG}_e2e.err | grep -v "batch of" | tail -40
python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_e2e.json").read().strip().splitlines()[-1])
e = d.get("end_to_end", {})
print("e2e", e.get("wall_s"), e.get("value"), "indels", json.dumps(e.get("indels")))
PY
