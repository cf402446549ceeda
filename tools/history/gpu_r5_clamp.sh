#!/bin/bash
# round 5: KL's / KLM's next-batch loads clamped to the read's last unit (cache hits instead of other rows) against the
# unclamped build (ab/prev): configs[2] and configs[4] lines twice each, then the clamped build's FETCH_SIZE passes
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05c2}
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_parity.py \
    tests/test_gpu_multisample.py "tests/test_gpu_full_size.py" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
run() {   # name lib config
  a=""; [ $3 = ms ] && a="--config multisample"
  NGSEP_LIB_PATH=$2 timeout -k 10 300 python -u bench.py $a --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4 > gpurun_out/${TAG}_$1.json 2> gpurun_out/${TAG}_$1.err || { tail -5 gpurun_out/${TAG}_$1.err; return 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$1.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("$1", "step %.4f ms" % d["ms_per_step"], "kernel %.4f ms" % r["kernel_avg_ms"], "frac %.3f" % r["frac"])
PY
}
M=$PWD/ngsepcore_amd/lib/libngsep_amd.so
P=$PWD/ab/prev/libngsep_amd.so
run kl_new $M kl && run kl_prev $P kl && run ms_new $M ms && run ms_prev $P ms && run kl_new2 $M kl && run kl_prev2 $P kl && \
run ms_new2 $M ms && run ms_prev2 $P ms || exit 1
for cfg in default multisample; do
  a=""; [ $cfg = multisample ] && a="--config multisample"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "k_read_scan|k_scan_pop" -d gpurun_out/pmc_${TAG}_${cfg} -o run --output-format csv \
      -- python -u bench.py $a --no-cpu-baseline --no-cold --no-e2e --steps 3 --warmup 1 > gpurun_out/pmc_${TAG}_${cfg}.out 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_${cfg}.out; exit 1; }
  python - <<PY
import csv, glob
f = glob.glob("gpurun_out/pmc_${TAG}_${cfg}/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))]
print("$cfg FETCH_SIZE per launch (raw, KB units)", sum(v) / len(v), "launches", len(v))
PY
done
