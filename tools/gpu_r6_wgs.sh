#!/bin/bash
# round 6: the configs[3] 30x WGS line on ONE GPU with the round's kernels (kernel path and CPU baseline; the
# end-to-end leg, every contig's BAM written and read, is round 5's profiles/r05w2_wgs_1gpu_e2e_bench.json), peak host RSS
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06wgs}
timeout -k 10 1100 python -u tools/maxrss.py python -u bench.py --config wgs --gpus 1 --wgs-shards 1 --no-cold --no-e2e \
    --steps 5 --warmup 1 > gpurun_out/${TAG}_wgs1.json 2> gpurun_out/${TAG}_wgs1.err
rc=$?
tail -6 gpurun_out/${TAG}_wgs1.err
python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_wgs1.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("wgs value %.4g" % d["value"], "step %.3f ms" % d["ms_per_step"], "kernel %.3f ms frac %.3f" % (r["kernel_avg_ms"], r["frac"]),
      "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
exit $rc
