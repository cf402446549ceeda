#!/bin/bash
# round 5 (diagnostic build): the population end-to-end run with and without transparent huge pages on the host arrays
# (NGSEP_NO_THP) -- where the 200 file opens' time goes
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05th}
D=$PWD/ngsepcore_amd/lib_diag/libngsep_amd.so
for mode in thp nothp thp nothp; do
  if [ $mode = nothp ]; then export NGSEP_NO_THP=1; else unset NGSEP_NO_THP; fi
  NGSEP_LIB_PATH=$D NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --config multisample --no-cold --no-cpu-baseline --steps 3 --warmup 1 \
      > gpurun_out/${TAG}_$mode.json 2> gpurun_out/${TAG}_$mode.err || { tail -20 gpurun_out/${TAG}_$mode.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$mode.json").read().strip().splitlines()[-1])
print("$mode population e2e %.3f s" % d["end_to_end"]["wall_s"])
PY
  grep -E "population: open |merge \+ sweep|end of alignments" gpurun_out/${TAG}_$mode.err | tail -3
done
for mode in thp nothp; do
  if [ $mode = nothp ]; then export NGSEP_NO_THP=1; else unset NGSEP_NO_THP; fi
  NGSEP_LIB_PATH=$D timeout -k 10 400 python -u bench.py --no-cold --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_c$mode.json 2> gpurun_out/${TAG}_c$mode.err || { tail -20 gpurun_out/${TAG}_c$mode.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_c$mode.json").read().strip().splitlines()[-1])
e = d["end_to_end"]
print("$mode chr20 e2e %.3f s" % e["wall_s"], "indel %.3f s" % e["indels"]["wall_s"])
PY
done
