#!/bin/bash
# round 4: KPM gather A/B (ab/prev = the previous build) on the configs[4] bench, parity of the release build first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multisample.py tests/test_gpu_pool.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/kpm_parity.log 2>&1 || { tail -20 gpurun_out/kpm_parity.log; exit 1; }
tail -2 gpurun_out/kpm_parity.log
B="python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4"
for v in A P A P; do
  if [ $v = A ]; then L=$PWD/ngsepcore_amd/lib/libngsep_amd.so; else L=$PWD/ab/prev/libngsep_amd.so; fi
  NGSEP_TIME_POSTERIOR=1 NGSEP_LIB_PATH=$L timeout -k 10 300 $B > gpurun_out/kpm_$v.json 2> gpurun_out/kpm_$v.err || { tail -5 gpurun_out/kpm_$v.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/kpm_$v.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("$v", "step %.3f ms" % d["ms_per_step"], "scan %.3f ms" % r["kernel_avg_ms"], "kpm", r["posterior_kernel_avg_ms"], "frac %.3f" % r["frac"], "exact", d["config"]["exact_sites_per_gpu"])
PY
done
