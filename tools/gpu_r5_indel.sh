#!/bin/bash
# round 5: kept alignments as views into shared blocks (keep_raw) -- the indel / realigner GPU tests, KPM's two stages
# against one stage, the default bench line (chr20 end-to-end legs with the indel phases), then KPM grid sizes (DIAG)
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05g}
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gpu_indels.py tests/test_gpu_realigner_cases.py tests/test_gpu_known.py tests/test_gpu_multi.py \
    tests/test_gpu_multisample.py tests/test_gpu_pool.py tests/test_gpu_kpm_stages.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u bench.py --no-cold > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_bench.json").read().strip().splitlines()[-1])
e = d["end_to_end"]
print("snv e2e %.3f s" % e["wall_s"], json.dumps(e["phases_ms"]))
print("indel e2e %.3f s" % e["indels"]["wall_s"], json.dumps(e["indels"]["phases_ms"]))
PY
B="python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4"
D=$PWD/ngsepcore_amd/lib_diag/libngsep_amd.so
run() {   # name [extra env]
  env $2 NGSEP_TIME_POSTERIOR=1 NGSEP_LIB_PATH=$D timeout -k 10 300 $B > gpurun_out/${TAG}_$1.json 2> gpurun_out/${TAG}_$1.err || { tail -5 gpurun_out/${TAG}_$1.err; return 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$1.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("$1", "step %.3f ms" % d["ms_per_step"], "klm %.3f ms" % r["kernel_avg_ms"], "kpm", r["posterior_kernel_avg_ms"])
PY
}
run kg256 NGSEP_KPM_GRID=256 && run kg512 NGSEP_KPM_GRID=512 && run kg768 NGSEP_KPM_GRID=768 && run kg1024 NGSEP_KPM_GRID=1024 && \
run kg768s1024 "NGSEP_KPM_GRID=768 NGSEP_STA_GRID=1024" && run kg768s2048 "NGSEP_KPM_GRID=768 NGSEP_STA_GRID=2048" && run kg5122 NGSEP_KPM_GRID=512 && run kg7682 NGSEP_KPM_GRID=768
