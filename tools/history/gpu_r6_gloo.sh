#!/bin/bash
# round 6: the N = 2 rehearsal on the final kernels (gloo for the rank barrier, both ranks on the one card) and the
# N = 1 line beside it
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06g2}
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_n1.json 2> gpurun_out/${TAG}_n1.err || { tail -20 gpurun_out/${TAG}_n1.err; exit 1; }
NGSEP_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 > gpurun_out/${TAG}_gloo2.json 2> gpurun_out/${TAG}_gloo2.err || { tail -20 gpurun_out/${TAG}_gloo2.err; exit 1; }
python - <<PY
import json
for f in ("${TAG}_n1", "${TAG}_gloo2"):
    d = json.loads(open("gpurun_out/%s.json" % f).read().strip().splitlines()[-1])
    r = d["roofline"]; e = d.get("end_to_end") or {}
    print(f, "n", d["n_gpus"], "value %.4g" % d["value"], "step %.4f ms" % d["ms_per_step"], "kernel %.4f ms frac %.3f" % (r["kernel_avg_ms"], r["frac"]),
          "e2e", e.get("wall_s"), e.get("value"), "cpu", (d.get("cpu_baseline") or {}).get("value"), "scaling", d.get("scaling"))
PY
