#!/bin/bash
# round 5: KL's !DEEP counter adds as one halfword add per exception (NGSEP_KL_EXLOOP=1, lib/) against the byte-pair adds
# (ab/kl0) -- single-sample parity first, then configs[2] bench lines in turn
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05ex}
NGSEP_LIB_PATH=$PWD/ab/kl1/libngsep_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -k "not population" \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
run() {   # name lib
  NGSEP_LIB_PATH=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cold --no-e2e --steps 40 --warmup 5 \
      > gpurun_out/${TAG}_$1.json 2> gpurun_out/${TAG}_$1.err || { tail -5 gpurun_out/${TAG}_$1.err; return 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$1.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("$1 value %.4g" % d["value"], "step %.4f ms" % d["ms_per_step"], "kl %.4f ms" % r["kernel_avg_ms"], "frac %.3f" % r["frac"])
PY
}
N=$PWD/ab/kl1/libngsep_amd.so
O=$PWD/ngsepcore_amd/lib/libngsep_amd.so
run new1 $N && run old1 $O && run new2 $N && run old2 $O && run new3 $N && run old3 $O
