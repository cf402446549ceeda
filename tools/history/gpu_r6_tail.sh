#!/bin/bash
# round 6 experiment: the single-sample pass's tail (KG, KP, KO) on CU-masked streams beside the next pass's KL
# (NGSEP_TAIL_CUS / NGSEP_TAIL_SPREAD) -- parity first, then the configs[2] step at several splits, alternated
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06g}
NGSEP_TAIL_CUS=32 NGSEP_TAIL_SPREAD=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_full_size.py -k "not population and not chr1" > gpurun_out/${TAG}_parity.log 2>&1 || { tail -30 gpurun_out/${TAG}_parity.log; exit 1; }
tail -1 gpurun_out/${TAG}_parity.log
one() {   # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cold --no-e2e --steps 40 > gpurun_out/${TAG}_$lab.json 2> gpurun_out/${TAG}_$lab.err || { tail -5 gpurun_out/${TAG}_$lab.err; return 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_$lab.json").read().strip().splitlines()[-1])
print("$lab", "step %.4f ms" % d["ms_per_step"], "KL %.4f ms" % d["roofline"]["kernel_avg_ms"], "value %.4g" % d["value"])
PY
}
for rep in 1 2; do
  one base$rep NGSEP_X=0 && one s32_$rep NGSEP_TAIL_CUS=32 NGSEP_TAIL_SPREAD=1 && one b32_$rep NGSEP_TAIL_CUS=32 && \
  one s16_$rep NGSEP_TAIL_CUS=16 NGSEP_TAIL_SPREAD=1 && one s64_$rep NGSEP_TAIL_CUS=64 NGSEP_TAIL_SPREAD=1 || exit 1
done
NGSEP_TAIL_CUS=32 NGSEP_TAIL_SPREAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_s32 -o run --output-format csv -- python -u bench.py --no-cpu-baseline --no-cold --no-e2e \
    > gpurun_out/prof_${TAG}_s32.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}_s32.out; exit 1; }
python tools/kstats.py gpurun_out/prof_${TAG}_s32 gpurun_out/${TAG}_s32_kernel_stats.csv > gpurun_out/${TAG}_s32_kstats.txt; cat gpurun_out/${TAG}_s32_kstats.txt
