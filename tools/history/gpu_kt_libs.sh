#!/bin/bash
# KT A/B over tuning builds of the library (ngsepcore_amd/lib_<name>/, NGSEP_LIB_PATH): two short chr20 benches each
# Usage: KT_LIBS="base d1 d2w3" bash tools/gpu_kt_libs.sh
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${KT_LIBS}; do
    NGSEP_LIB_PATH=$PWD/ngsepcore_amd/lib_$v/libngsep_amd.so timeout -k 10 240 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cold --no-e2e > gpurun_out/ktlib_${v}_$rep.json 2> gpurun_out/ktlib_${v}_$rep.err || { tail -5 gpurun_out/ktlib_${v}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ktlib_${v}_$rep.json'));r=d['roofline'];print('$v',$rep,'KT',round(r['kernel_avg_ms'],4),'frac',round(r['frac'],3),'step',round(d['ms_per_step'],4))"
  done
done
