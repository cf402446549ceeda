#!/bin/bash
# round 5: where the chr20 BAM -> VCF time goes -- the end-to-end leg with host timing on a level-6 BAM (as the
# bench writes it) and on a stored-block (level-0) BAM of the same reads: the inflate-free floor
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05lv}
for lv in 6 0 6 0; do
  NGSEP_HOST_TIMING=1 NGS_SYNTH_LEVEL=$lv timeout -k 10 400 python -u bench.py --no-cold --no-cpu-baseline --steps 5 --warmup 2 \
      > gpurun_out/${TAG}_l$lv.json 2> gpurun_out/${TAG}_l$lv.err || { tail -20 gpurun_out/${TAG}_l$lv.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_l$lv.json").read().strip().splitlines()[-1])
e = d["end_to_end"]
print("level $lv bam %.2f GB" % (e["bam_bytes"] / 1e9), "snv e2e %.3f s" % e["wall_s"], "indel e2e %.3f s" % e["indels"]["wall_s"])
PY
  grep -E "bam:|call_bam:" gpurun_out/${TAG}_l$lv.err | head -4
done
