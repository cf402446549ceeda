#!/bin/bash
# round 5: the population pass without its per-pass fills (k_stage_a clears the open-position bits, the big-call count
# rides on the pass's counter memset) -- population parity, then configs[4] bench lines and a kernel summary
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05fl}
timeout -k 10 600 python -u -m pytest tests/test_gpu_multisample.py tests/test_gpu_kpm_stages.py tests/test_gpu_multi.py \
    "tests/test_gpu_full_size.py::test_full_size_population_vcf_identical" \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 40 --warmup 5 \
      > gpurun_out/${TAG}_ms$k.json 2> gpurun_out/${TAG}_ms$k.err || { tail -5 gpurun_out/${TAG}_ms$k.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_ms$k.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("ms$k value %.4g" % d["value"], "step %.4f ms" % d["ms_per_step"], "klm %.4f ms" % r["kernel_avg_ms"], "frac %.3f" % r["frac"])
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o ms -- python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4 > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || { tail -5 gpurun_out/${TAG}_prof.err; exit 1; }
f=$(ls gpurun_out/${TAG}_prof/*/*kernel_stats.csv gpurun_out/${TAG}_prof/*kernel_stats.csv 2>/dev/null | head -1)
python - "$f" <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print(x["Name"][:48], x["Calls"], "%.1f us" % (float(x["AverageNs"]) / 1e3))
PY
