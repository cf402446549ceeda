#!/bin/bash
# round 5: MultisampleVariantsDetector's merged batches admitted on all threads (admit_middle) -- population parity,
# then the population end-to-end run with host timing
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05pa}
timeout -k 10 700 python -u -m pytest tests/test_gpu_multisample.py tests/test_gpu_kpm_stages.py tests/test_gpu_multi.py \
    tests/test_gpu_realigner_cases.py "tests/test_gpu_full_size.py::test_full_size_population_vcf_identical" tests/test_gpu_known.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for k in 1 2; do
  NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --config multisample --no-cold --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_ms$k.json 2> gpurun_out/${TAG}_ms$k.err || { tail -20 gpurun_out/${TAG}_ms$k.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_ms$k.json").read().strip().splitlines()[-1])
print("population e2e %.3f s" % d["end_to_end"]["wall_s"])
PY
  grep -E "population: open |population merge: sweep|merge \+ sweep|end of alignments" gpurun_out/${TAG}_ms$k.err | tail -4
done
