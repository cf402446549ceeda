#!/bin/bash
# round 6: end-to-end (BAM -> VCF) A/B of two builds of the library, alternated: ngsepcore_amd/lib_base (HEAD) and
# the in-tree build; host phase laps under NGSEP_HOST_TIMING
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06e2eab}
CFGS=${2:-"multisample"}
ITS=${3:-"1 2 3"}
for it in $ITS; do
  for cfg in $CFGS; do
    for lib in base new; do
      if [ $lib = base ]; then export NGSEP_LIB_PATH=$PWD/ngsepcore_amd/lib_base/libngsep_amd.so; else unset NGSEP_LIB_PATH; fi
      o=gpurun_out/${TAG}_${cfg}_${lib}_$it
      NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline --no-cold --steps 3 --warmup 1 \
          > $o.json 2> $o.err || { tail -20 $o.err; exit 1; }
      python - <<PY
import json
d = json.loads(open("$o.json").read().strip().splitlines()[-1])
e = d.get("end_to_end") or {}
print("$cfg $lib it $it", "e2e %.3f s" % e.get("wall_s", 0), "indels", (e.get("indels") or {}).get("wall_s"))
PY
      grep -a "population: open \|population: merge + sweep\|population: end of\|population: VCF" $o.err | tr '\n' ' '; echo
    done
  done
done
