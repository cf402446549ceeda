#!/bin/bash
# KT cost split on chr20: full (0), no candidate loop (1), count bound without the exact tally (128),
# plane loads + OR only (257)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for a in ${KT_ABLATE:-0 1 128 257}; do
  NGSEP_ABLATE=$a timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold --no-e2e > gpurun_out/ktab_$a.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ktab_$a.json'));r=d['roofline'];print('ablate $a','KT',round(r['kernel_avg_ms'],4),'step',round(d['ms_per_step'],4))"
done
