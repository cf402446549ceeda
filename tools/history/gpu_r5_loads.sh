#!/bin/bash
# round 5: KL's and KLM's next-batch loads unconditional (no lane condition: the compiler no longer drains every
# outstanding load before the current batch), population groups sized on all threads -- the whole GPU suite, the
# configs[2] and configs[4] bench lines with their rocprof kernel summaries
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05r}
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests \
    > gpurun_out/${TAG}_suite.log 2>&1 || { tail -30 gpurun_out/${TAG}_suite.log; exit 1; }
tail -2 gpurun_out/${TAG}_suite.log
timeout -k 10 400 python -u bench.py --no-cold > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_bench.json").read().strip().splitlines()[-1])
r = d["roofline"]; e = d["end_to_end"]
print("chr20 step %.4f ms KL %.4f ms frac %.3f" % (d["ms_per_step"], r["kernel_avg_ms"], r["frac"]), "e2e %.3f s indel %.3f s" % (e["wall_s"], e["indels"]["wall_s"]))
PY
timeout -k 10 400 python -u bench.py --config multisample --no-cold --no-cpu-baseline > gpurun_out/${TAG}_ms.json 2> gpurun_out/${TAG}_ms.err || { tail -20 gpurun_out/${TAG}_ms.err; exit 1; }
python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_ms.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("ms step %.4f ms KLM %.4f ms frac %.3f" % (d["ms_per_step"], r["kernel_avg_ms"], r["frac"]), "population e2e %.3f s" % d["end_to_end"]["wall_s"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python -u bench.py --no-cpu-baseline --no-cold --no-e2e \
    > gpurun_out/prof_${TAG}.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}.out; exit 1; }
python tools/kstats.py gpurun_out/prof_${TAG} gpurun_out/${TAG}_kernel_stats.csv > gpurun_out/${TAG}_kstats.txt && head -5 gpurun_out/${TAG}_kstats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_ms -o run --output-format csv -- python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e \
    > gpurun_out/prof_${TAG}_ms.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}_ms.out; exit 1; }
python tools/kstats.py gpurun_out/prof_${TAG}_ms gpurun_out/${TAG}_ms_kernel_stats.csv > gpurun_out/${TAG}_ms_kstats.txt && head -6 gpurun_out/${TAG}_ms_kstats.txt
