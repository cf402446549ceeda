#!/bin/bash
# round 4: A/B/... of KL variant libraries (ab/<name>/libngsep_amd.so via NGSEP_LIB_PATH) against the release build
# on one box: parity of each variant, then alternating default-config bench lines (no CPU baseline, no e2e leg)
# usage: tools/gpu_r4_abn.sh name1 name2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  NGSEP_LIB_PATH=$PWD/ab/$v/libngsep_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
      --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/abn_parity_$v.log 2>&1 || { echo "parity $v failed"; tail -20 gpurun_out/abn_parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/abn_parity_$v.log)"
done
B="python -u bench.py --no-cpu-baseline --no-cold --no-e2e --steps 30 --warmup 3"
for r in 1 2; do
  for v in release "$@"; do
    if [ "$v" = release ]; then L=""; else L=$PWD/ab/$v/libngsep_amd.so; fi
    NGSEP_LIB_PATH=$L timeout -k 10 300 $B > gpurun_out/abn_${v}_$r.json 2> gpurun_out/abn_${v}_$r.err || { tail -5 gpurun_out/abn_${v}_$r.err; exit 1; }
    python -c "
import json
d = json.loads(open('gpurun_out/abn_${v}_$r.json').read().strip().splitlines()[-1])
print('$v', $r, d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
  done
done
