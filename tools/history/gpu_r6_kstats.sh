#!/bin/bash
# round 6: a rocprofv3 kernel summary of one bench configuration per build (ngsepcore_amd/lib_<name>, "new" = lib/)
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06ks}
CFG=${2:-multisample}
shift 2
for v in "$@"; do
  if [ $v = new ]; then L=ngsepcore_amd/lib/libngsep_amd.so; else L=ngsepcore_amd/lib_$v/libngsep_amd.so; fi
  NGSEP_LIB_PATH=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$v -o run --output-format csv -- \
      python -u bench.py --config $CFG --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 3 > gpurun_out/prof_${TAG}_$v.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}_$v.out; exit 1; }
  echo "== $v"; python tools/kstats.py gpurun_out/prof_${TAG}_$v gpurun_out/${TAG}_${v}_kernel_stats.csv | head -12
done
