#!/bin/bash
# round 5: KLM changes against the previous build (ab/prev) on one box -- population parity tests, configs[4] lines
# (last: the count bound's survivors to KX, k_exact_cols, instead of KLM's own exact pass)
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05s}
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_multisample.py \
    "tests/test_gpu_full_size.py::test_full_size_population_vcf_identical" tests/test_gpu_kpm_stages.py tests/test_gpu_known.py \
    tests/test_gpu_pool.py tests/test_gpu_realigner_cases.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
B="python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4"
run() {   # name lib
  NGSEP_TIME_POSTERIOR=1 NGSEP_LIB_PATH=$2 timeout -k 10 300 $B > gpurun_out/${TAG}_$1.json 2> gpurun_out/${TAG}_$1.err || { tail -5 gpurun_out/${TAG}_$1.err; return 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$1.json").read().strip().splitlines()[-1])
r = d["roofline"]; c = d["config"]
print("$1", "step %.3f ms" % d["ms_per_step"], "klm %.4f ms" % r["kernel_avg_ms"], "kpm %.4f" % r["posterior_kernel_avg_ms"], "frac %.3f" % r["frac"], "cand", c["candidates_per_gpu"], "queued", c["exact_sites_per_gpu"])
PY
}
M=$PWD/ngsepcore_amd/lib/libngsep_amd.so
P=$PWD/ab/prev/libngsep_amd.so
run new $M && run prev $P && run new2 $M && run prev2 $P && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_ms -o run --output-format csv -- $B \
    > gpurun_out/prof_${TAG}_ms.out 2>&1 && python tools/kstats.py gpurun_out/prof_${TAG}_ms gpurun_out/${TAG}_ms_kernel_stats.csv > gpurun_out/${TAG}_ms_kstats.txt && head -6 gpurun_out/${TAG}_ms_kstats.txt
