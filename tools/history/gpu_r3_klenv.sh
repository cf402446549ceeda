#!/bin/bash
# round 3: per-kernel stats of the chr20 bench under several environments (tuning).  Usage:
#   bash tools/gpu_r3_klenv.sh TAG [--tests] "VAR=a VAR2=b" "VAR=c" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
if [ "$1" == "--tests" ]; then
  shift
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/tests_kl_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_kl_$TAG.log; exit 1; }
  tail -1 gpurun_out/tests_kl_$TAG.log
fi
B="python bench.py --no-cpu-baseline --no-cold --no-e2e"
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/klenv_${TAG}_$i -o run --output-format csv -- $B --steps 10 --warmup 2 > gpurun_out/klenv_${TAG}_$i.out 2>&1 || { tail -5 gpurun_out/klenv_${TAG}_$i.out; exit 1; }
  python tools/kstats.py gpurun_out/klenv_${TAG}_$i gpurun_out/kernel_stats_klenv_${TAG}_$i.csv > /dev/null
  echo "== $E"
  python - gpurun_out/kernel_stats_klenv_${TAG}_$i.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r['Name'].startswith('__amd'): continue
    print("  %-34s avg %8.1f min %8.1f" % (r['Name'][:34], float(r['AverageNs'])/1000, float(r['MinNs'])/1000))
PY
done
