#!/bin/bash
# round 5: KPM's first stage as one wavefront per position (k_stage_a) over KLM's exact-pass pairs --
# parity on the population tests (incl. the full-size configs[4] shard), then configs[4] bench lines: main (two
# stages), main1 (one stage), repeats; a rocprofv3 kernel
# summary of the main line
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05d}
timeout -k 10 500 python -u -m pytest tests/test_gpu_multisample.py "tests/test_gpu_full_size.py::test_full_size_population_vcf_identical" \
    tests/test_gpu_realigner_cases.py -k "population or multisample or Population" \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
B="python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4"
run() {   # name lib [extra env]
  env $3 NGSEP_TIME_POSTERIOR=1 NGSEP_LIB_PATH=$2 timeout -k 10 300 $B > gpurun_out/${TAG}_$1.json 2> gpurun_out/${TAG}_$1.err || { tail -5 gpurun_out/${TAG}_$1.err; return 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$1.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("$1", "step %.3f ms" % d["ms_per_step"], "klm %.3f ms" % r["kernel_avg_ms"], "kpm", r["posterior_kernel_avg_ms"], "frac %.3f" % r["frac"], "exact", d["config"]["exact_sites_per_gpu"])
PY
}
M=$PWD/ngsepcore_amd/lib/libngsep_amd.so
run main $M && run main1 $M NGSEP_KPM_ONE_STAGE=1 && run main2 $M && run main12 $M NGSEP_KPM_ONE_STAGE=1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o ms -- python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4 > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err && \
python - <<PY
import csv, glob
f = glob.glob("gpurun_out/${TAG}_prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-40s %8s calls avg %.4f ms" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
