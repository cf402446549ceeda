#!/bin/bash
# round 5: the whole GPU suite, then the default bench line (configs[2] chr20, end-to-end legs with the indel phases,
# CPU baseline), its rocprof kernel summary, and the 2-rank gloo rehearsal of the sharded end-to-end leg
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05f}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests \
    > gpurun_out/${TAG}_suite.log 2>&1 || { tail -30 gpurun_out/${TAG}_suite.log; exit 1; }
tail -2 gpurun_out/${TAG}_suite.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python -u bench.py --no-cpu-baseline --no-cold --no-e2e \
    > gpurun_out/prof_${TAG}.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}.out; exit 1; }
python tools/kstats.py gpurun_out/prof_${TAG} gpurun_out/${TAG}_kernel_stats.csv
head -8 gpurun_out/${TAG}_kernel_stats.csv
NGSEP_DIST_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --no-cpu-baseline --no-cold > gpurun_out/${TAG}_gloo2.json 2> gpurun_out/${TAG}_gloo2.err || { tail -20 gpurun_out/${TAG}_gloo2.err; exit 1; }
cat gpurun_out/${TAG}_gloo2.json
# KPM / first-stage grid sizes (DIAG build): 16384 workgroups looping over the queue vs one or two per slot
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
run g16k && run kg768 NGSEP_KPM_GRID=768 && run kg1536 NGSEP_KPM_GRID=1536 && run sg4096 NGSEP_STA_GRID=4096 && \
run sg8192 NGSEP_STA_GRID=8192 && run g16k2 && run kg1536s4096 "NGSEP_KPM_GRID=1536 NGSEP_STA_GRID=4096"
