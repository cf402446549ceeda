#!/bin/bash
# round 4: population path after the KPM record stores / biallelic genotype path and the huge-page pinned arena:
# multisample parity, then the configs[4] bench with host timing (staged layout and end to end)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r04r}
timeout -k 10 600 python -u -m pytest tests/test_gpu_multisample.py tests/test_gpu_pool.py tests/test_gpu_known.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -20 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
NGSEP_HOST_TIMING=1 NGSEP_TIME_POSTERIOR=1 timeout -k 10 500 python -u bench.py --config multisample --no-cpu-baseline --no-cold \
    --steps 20 --warmup 4 > gpurun_out/${TAG}_ms.json 2> gpurun_out/${TAG}_ms.err || { tail -20 gpurun_out/${TAG}_ms.err; exit 1; }
grep -v "batch of\|projection:\|bam: inflate" gpurun_out/${TAG}_ms.err | head -40
python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_ms.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("step %.3f ms" % d["ms_per_step"], "scan %.3f ms" % r["kernel_avg_ms"], "kpm", r["posterior_kernel_avg_ms"], "frac %.3f" % r["frac"], "e2e", d.get("end_to_end", {}).get("wall_s"))
PY
