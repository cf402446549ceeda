#!/bin/bash
# round 5: the indel path's host work -- indel / realigner / known-variant GPU tests, then the chr20 end-to-end legs
# (SNV and indels, phases) three times on one box: the box-to-box spread of these host-bound numbers is large
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05j}
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gpu_indels.py tests/test_gpu_realigner_cases.py tests/test_gpu_known.py tests/test_gpu_multi.py \
    tests/test_gpu_pool.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for k in 1 2 3; do
  timeout -k 10 400 python -u bench.py --no-cold --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_bench$k.json 2> gpurun_out/${TAG}_bench$k.err || { tail -20 gpurun_out/${TAG}_bench$k.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_bench$k.json").read().strip().splitlines()[-1])
e = d["end_to_end"]
print("snv e2e %.3f s" % e["wall_s"], "indel e2e %.3f s" % e["indels"]["wall_s"], "ratio %.2f" % (e["indels"]["wall_s"] / e["wall_s"]))
print("  indel phases", json.dumps({k: round(v, 1) for k, v in e["indels"]["phases_ms"].items() if k != "note"}))
PY
done
