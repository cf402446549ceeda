#!/bin/bash
# round 6: chr20 step-tail kernels per build (rocprof kernel summaries, alternated)
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06tk}
shift
for it in 1 2; do
  for v in "$@"; do
    if [ $v = new ]; then L=ngsepcore_amd/lib/libngsep_amd.so; else L=ngsepcore_amd/lib_$v/libngsep_amd.so; fi
    NGSEP_LIB_PATH=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_${v}_$it -o run --output-format csv -- \
        python -u bench.py --no-cpu-baseline --no-cold --no-e2e --steps 30 --warmup 3 > gpurun_out/prof_${TAG}_${v}_$it.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}_${v}_$it.out; exit 1; }
    echo "== $v $it $(grep -a -o '"ms_per_step": [0-9.]*' gpurun_out/prof_${TAG}_${v}_$it.out)"
    python tools/kstats.py gpurun_out/prof_${TAG}_${v}_$it gpurun_out/${TAG}_${v}_${it}_kernel_stats.csv | head -6
  done
done
