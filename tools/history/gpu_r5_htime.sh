#!/bin/bash
# round 5: host timing breakdown of the population end-to-end run and of the chr20 legs (current tree)
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05ht}
NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --config multisample --no-cold --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_ms.json 2> gpurun_out/${TAG}_ms.err || { tail -20 gpurun_out/${TAG}_ms.err; exit 1; }
grep -v "bam: inflate\|projection:\|batch of" gpurun_out/${TAG}_ms.err | grep "ngsep host" | tail -40
NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --no-cold --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.err || { tail -20 gpurun_out/${TAG}_b.err; exit 1; }
python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_b.json").read().strip().splitlines()[-1])
e = d["end_to_end"]
print("chr20 snv e2e %.3f s" % e["wall_s"], "indel e2e %.3f s" % e["indels"]["wall_s"])
print(json.dumps({k: round(v, 1) for k, v in e["indels"]["phases_ms"].items() if k != "note"}))
PY
