#!/bin/bash
# round 6: host anatomy of the end-to-end legs (NGSEP_HOST_TIMING): chr20 BAM -> VCF (with and without indels) and the
# 200-BAM population
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06h}
NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-cold --steps 5 --warmup 1 > gpurun_out/${TAG}_e2e.json 2> gpurun_out/${TAG}_e2e.err || { tail -20 gpurun_out/${TAG}_e2e.err; exit 1; }
NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --config multisample --no-cpu-baseline --no-cold --steps 5 --warmup 1 > gpurun_out/${TAG}_pop.json 2> gpurun_out/${TAG}_pop.err || { tail -20 gpurun_out/${TAG}_pop.err; exit 1; }
python - <<PY
import json
for f in ("${TAG}_e2e", "${TAG}_pop"):
    d = json.loads(open("gpurun_out/%s.json" % f).read().strip().splitlines()[-1])
    e = d.get("end_to_end") or {}
    print(f, "e2e %s" % e.get("wall_s"), "indels %s" % (e.get("indels") or {}).get("wall_s"))
PY
grep -c "ngsep host" gpurun_out/${TAG}_e2e.err gpurun_out/${TAG}_pop.err
