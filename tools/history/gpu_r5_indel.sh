#!/bin/bash
# round 5: the indel path's host work (kept alignments as views into shared blocks, the replay's fused sweep) -- the
# indel / realigner / population GPU tests, the default bench line (chr20 end-to-end legs with the indel phases), the
# configs[4] line and its rocprof kernel summary
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
timeout -k 10 300 python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4 > gpurun_out/${TAG}_ms.json 2> gpurun_out/${TAG}_ms.err || { tail -20 gpurun_out/${TAG}_ms.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_ms -o run --output-format csv -- python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4 \
    > gpurun_out/prof_${TAG}_ms.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}_ms.out; exit 1; }
python tools/kstats.py gpurun_out/prof_${TAG}_ms gpurun_out/${TAG}_ms_kernel_stats.csv > gpurun_out/${TAG}_ms_kstats.txt && head -8 gpurun_out/${TAG}_ms_kstats.txt
