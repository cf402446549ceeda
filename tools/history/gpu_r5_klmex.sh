#!/bin/bash
# round 5: KLM's exception byte counters as one add per exception (ab/klm1, NGSEP_KLM_EXLOOP=1) against the unit's
# 2-3 shifted adds (lib/) -- population parity through the A/B build, then configs[4] bench lines in turn
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05kx}
N=$PWD/ab/klm1/libngsep_amd.so
O=$PWD/ngsepcore_amd/lib/libngsep_amd.so
NGSEP_LIB_PATH=$N timeout -k 10 600 python -u -m pytest tests/test_gpu_multisample.py "tests/test_gpu_full_size.py::test_full_size_population_vcf_identical" \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
run() {   # name lib
  NGSEP_LIB_PATH=$2 timeout -k 10 300 python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 40 --warmup 5 \
      > gpurun_out/${TAG}_$1.json 2> gpurun_out/${TAG}_$1.err || { tail -5 gpurun_out/${TAG}_$1.err; return 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$1.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("$1 value %.4g" % d["value"], "step %.4f ms" % d["ms_per_step"], "klm %.4f ms" % r["kernel_avg_ms"], "frac %.3f" % r["frac"])
PY
}
run new1 $N && run old1 $O && run new2 $N && run old2 $O && run new3 $N && run old3 $O
