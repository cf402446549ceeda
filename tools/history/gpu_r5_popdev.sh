#!/bin/bash
# round 5: population layouts from the projection chunks as uploaded -- population / known / indel GPU tests, the
# configs[4] population end-to-end leg twice with host timings
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05q}
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_multisample.py \
    "tests/test_gpu_full_size.py::test_full_size_population_vcf_identical" tests/test_gpu_kpm_stages.py tests/test_gpu_known.py \
    tests/test_gpu_pool.py tests/test_gpu_multi.py tests/test_sharding.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for k in 1 2; do
NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --config multisample --no-cold --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/${TAG}_ms$k.json 2> gpurun_out/${TAG}_ms$k.err || { tail -20 gpurun_out/${TAG}_ms$k.err; exit 1; }
python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_ms$k.json").read().strip().splitlines()[-1])
print("ms step %.3f ms" % d["ms_per_step"], "population e2e %.3f s" % d["end_to_end"]["wall_s"])
PY
grep -E "population layout|layout [0-9.]+ ms, device upload|population: " gpurun_out/${TAG}_ms$k.err | tail -12
done
