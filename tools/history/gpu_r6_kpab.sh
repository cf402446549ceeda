#!/bin/bash
# round 6: KP's cost split on chr20 (DIAG build ngsepcore_amd/lib_dg): full, without the posterior and emit
# (NGSEP_ABLATE=8), and KP's grid (NGSEP_KP_GRID)
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06kp}
L=$PWD/ngsepcore_amd/lib_dg/libngsep_amd.so
run() {   # name env...
  local name=$1; shift
  env "$@" NGSEP_LIB_PATH=$L NGSEP_TIME_POSTERIOR=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold --no-e2e \
      > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { tail -5 gpurun_out/${TAG}_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));r=d['roofline'];print('$name','KL',round(r['kernel_avg_ms'],4),'KP',round(r['posterior_kernel_avg_ms'] or 0,4),'step',round(d['ms_per_step'],4))"
}
for it in 1 2; do
  run full_$it NGSEP_ABLATE=0 && run noposterior_$it NGSEP_ABLATE=8 && run grid1024_$it NGSEP_KP_GRID=1024 && run grid4096_$it NGSEP_KP_GRID=4096 || exit 1
done
