#!/bin/bash
# round 5 (diagnostic build): KPM stage A's grid (NGSEP_STA_GRID; 16384 one-wavefront workgroups by default, ~4.9 K
# positions queued on configs[4]) -- configs[4] step and KPM time per setting
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05sg}
D=$PWD/ngsepcore_amd/lib_diag/libngsep_amd.so
for g in 16384 5120 2048 8192 16384 5120; do
  NGSEP_STA_GRID=$g NGSEP_TIME_POSTERIOR=1 NGSEP_LIB_PATH=$D timeout -k 10 300 python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 40 --warmup 5 \
      > gpurun_out/${TAG}_$g.json 2> gpurun_out/${TAG}_$g.err || { tail -5 gpurun_out/${TAG}_$g.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$g.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("grid $g step %.4f ms" % d["ms_per_step"], "klm %.4f" % r["kernel_avg_ms"], "kpm", r["posterior_kernel_avg_ms"])
PY
done
