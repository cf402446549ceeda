#!/bin/bash
# round 5: KLM variants and KPM's two stages on one box -- parity of the main build on the population tests (incl. the
# full-size configs[4] shard), then configs[4] bench lines: main (compact rounds + two-stage KPM), main with one-stage
# KPM, group-aligned KLM (ab/klmA), 8 waves (ab/klmW), then the DIAG build's KLM ablations
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05c}
timeout -k 10 500 python -u -m pytest tests/test_gpu_multisample.py "tests/test_gpu_full_size.py::test_full_size_population_vcf_identical" \
    tests/test_gpu_realigner_cases.py -k "population or multisample or Population" \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
B="python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4"
run() {   # name lib ablate [extra env]
  env $4 NGSEP_ABLATE=$3 NGSEP_TIME_POSTERIOR=1 NGSEP_LIB_PATH=$2 timeout -k 10 300 $B > gpurun_out/${TAG}_$1.json 2> gpurun_out/${TAG}_$1.err || { tail -5 gpurun_out/${TAG}_$1.err; return 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$1.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("$1", "step %.3f ms" % d["ms_per_step"], "klm %.3f ms" % r["kernel_avg_ms"], "kpm", r["posterior_kernel_avg_ms"], "frac %.3f" % r["frac"], "exact", d["config"]["exact_sites_per_gpu"])
PY
}
M=$PWD/ngsepcore_amd/lib/libngsep_amd.so
D=$PWD/ngsepcore_amd/lib_diag/libngsep_amd.so
run main $M 0 && run main1 $M 0 NGSEP_KPM_ONE_STAGE=1 && run A $PWD/ab/klmA/libngsep_amd.so 0 && run W $PWD/ab/klmW/libngsep_amd.so 0 && \
run main2 $M 0 && run A2 $PWD/ab/klmA/libngsep_amd.so 0 && \
run d0 $D 0 && run dnocnt $D 65536 && run dnomark $D 131072 && run dnoexact $D 262144 && run dloads $D 524288 && run dnodif $D 1048576
