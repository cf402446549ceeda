#!/bin/bash
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NGSEP_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 3 --warmup 1 > gpurun_out/r06cnt.json 2> gpurun_out/r06cnt.err || { tail -5 gpurun_out/r06cnt.err; exit 1; }
grep -a "population pass" gpurun_out/r06cnt.err | head -3
python -c "import json;d=json.loads(open('gpurun_out/r06cnt.json').read().strip().splitlines()[-1]);print(d['config'])"
