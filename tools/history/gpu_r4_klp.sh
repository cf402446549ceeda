#!/bin/bash
# round 4: KL with a persistent grid (NGSEP_KL_PERSIST workgroups per CU walking the tiles) against one workgroup per
# tile: parity of each build, then alternating default-config bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in p8 p4; do
  NGSEP_LIB_PATH=$PWD/ab/$v/libngsep_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
      --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/klp_parity_$v.log 2>&1 || { tail -20 gpurun_out/klp_parity_$v.log; exit 1; }
  tail -1 gpurun_out/klp_parity_$v.log
done
B="python -u bench.py --no-cpu-baseline --no-cold --no-e2e --steps 30 --warmup 3"
for v in A p8 p4 A p8 p4; do
  if [ $v = A ]; then L=$PWD/ngsepcore_amd/lib/libngsep_amd.so; else L=$PWD/ab/$v/libngsep_amd.so; fi
  NGSEP_LIB_PATH=$L timeout -k 10 300 $B > gpurun_out/klp_$v.json 2> gpurun_out/klp_$v.err || { tail -5 gpurun_out/klp_$v.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/klp_$v.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("$v", "step %.3f ms" % d["ms_per_step"], "KL %.4f ms" % r["kernel_avg_ms"], "frac %.3f" % r["frac"])
PY
done
