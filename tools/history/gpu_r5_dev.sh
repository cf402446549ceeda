#!/bin/bash
# round 5: units built on the device (k_build_units) for streamed windows and population layouts -- the whole GPU
# suite, then the chr20 end-to-end legs twice and the configs[4] population end-to-end leg
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05l}
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests \
    > gpurun_out/${TAG}_suite.log 2>&1 || { tail -30 gpurun_out/${TAG}_suite.log; exit 1; }
tail -2 gpurun_out/${TAG}_suite.log
for k in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cold --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_bench$k.json 2> gpurun_out/${TAG}_bench$k.err || { tail -20 gpurun_out/${TAG}_bench$k.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_bench$k.json").read().strip().splitlines()[-1])
e = d["end_to_end"]
print("snv e2e %.3f s" % e["wall_s"], "indel e2e %.3f s" % e["indels"]["wall_s"], "ratio %.2f" % (e["indels"]["wall_s"] / e["wall_s"]))
print("  snv phases", json.dumps({k: round(v, 1) for k, v in e["phases_ms"].items() if k != "note"}))
print("  indel phases", json.dumps({k: round(v, 1) for k, v in e["indels"]["phases_ms"].items() if k != "note"}))
PY
done
NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --config multisample --no-cold --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/${TAG}_ms.json 2> gpurun_out/${TAG}_ms.err || { tail -20 gpurun_out/${TAG}_ms.err; exit 1; }
python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_ms.json").read().strip().splitlines()[-1])
print("ms step %.3f ms" % d["ms_per_step"], "population e2e", json.dumps(d.get("end_to_end"))[:600])
PY
grep "population layout" gpurun_out/${TAG}_ms.err | tail -12
