#!/bin/bash
# round 4: A/B of a KL variant library (ab/libB.so, NGSEP_LIB_PATH) against the release build on the same box:
# parity of the variant, then alternating default-config bench lines (no CPU baseline, no end-to-end leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NGSEP_LIB_PATH=$PWD/ab/libB.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_parity.log 2>&1 || { tail -20 gpurun_out/ab_parity.log; exit 1; }
tail -2 gpurun_out/ab_parity.log
B="python -u bench.py --no-cpu-baseline --no-cold --no-e2e --steps 30 --warmup 3"
for r in 1 2; do
  timeout -k 10 300 $B > gpurun_out/ab_A$r.json 2> gpurun_out/ab_A$r.err || { tail -5 gpurun_out/ab_A$r.err; exit 1; }
  NGSEP_LIB_PATH=$PWD/ab/libB.so timeout -k 10 300 $B > gpurun_out/ab_B$r.json 2> gpurun_out/ab_B$r.err || { tail -5 gpurun_out/ab_B$r.err; exit 1; }
  python - <<PY
import json
for t in ("A$r", "B$r"):
    d = json.loads(open("gpurun_out/ab_%s.json" % t).read().strip().splitlines()[-1])
    print(t, d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["roofline"]["frac"])
PY
done
