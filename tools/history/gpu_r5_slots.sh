#!/bin/bash
# round 5: a stream per result slot (NGSEP_SLOT_STREAMS=1, DIAG build: the next pass's KL overlapping this pass's
# KG / KP / KO) against the one device stream, configs[2] and configs[4] lines twice each
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05sl}
D=$PWD/ngsepcore_amd/lib_diag/libngsep_amd.so
run() {   # name config [env]
  a=""; [ $2 = ms ] && a="--config multisample"
  env $3 NGSEP_LIB_PATH=$D timeout -k 10 300 python -u bench.py $a --no-cpu-baseline --no-cold --no-e2e --steps 40 --warmup 5 > gpurun_out/${TAG}_$1.json 2> gpurun_out/${TAG}_$1.err || { tail -5 gpurun_out/${TAG}_$1.err; return 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$1.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("$1", "value %.4g" % d["value"], "step %.4f ms" % d["ms_per_step"], "kernel %.4f ms" % r["kernel_avg_ms"])
PY
}
run kl1 kl && run kl2 kl NGSEP_SLOT_STREAMS=1 && run ms1 ms && run ms2 ms NGSEP_SLOT_STREAMS=1 && \
run kl1b kl && run kl2b kl NGSEP_SLOT_STREAMS=1 && run ms1b ms && run ms2b ms NGSEP_SLOT_STREAMS=1
