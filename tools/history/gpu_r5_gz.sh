#!/bin/bash
# round 5: BGZF inflate on the device -- its tests, then the chr20 end-to-end leg with the device inflate (host timing)
# against the host inflate, then a kernel trace of one device-inflate run
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05gz}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gpu_inflate.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
for mode in gpu host gpu; do
  if [ $mode = gpu ]; then export NGSEP_GPU_INFLATE=1; else unset NGSEP_GPU_INFLATE; fi
  NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --no-cold --no-cpu-baseline --steps 5 --warmup 2 \
      > gpurun_out/${TAG}_$mode.json 2> gpurun_out/${TAG}_$mode.err || { tail -20 gpurun_out/${TAG}_$mode.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$mode.json").read().strip().splitlines()[-1])
e = d["end_to_end"]
print("$mode snv e2e %.3f s" % e["wall_s"], "indel e2e %.3f s" % e["indels"]["wall_s"], "records", e["vcf_records"], e["indels"]["vcf_records"])
PY
  grep -E "bam:|call_bam:" gpurun_out/${TAG}_$mode.err > gpurun_out/${TAG}_$mode.timing || true
  head -4 gpurun_out/${TAG}_$mode.timing
done
export NGSEP_GPU_INFLATE=1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- \
    python -u $GRAFT_REPO_ROOT/bench.py --no-cold --no-cpu-baseline --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1 \
    || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(ls gpurun_out/${TAG}_prof/*/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && grep -E "Name|k_inflate" "$f"
