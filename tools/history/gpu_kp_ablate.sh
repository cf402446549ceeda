#!/bin/bash
# KP cost split: full, without the posterior (NGSEP_ABLATE=8), without the segment walk (16), both (24)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for a in 0 8 16 24; do
  NGSEP_ABLATE=$a NGSEP_TIME_POSTERIOR=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold --no-e2e > gpurun_out/kpab_$a.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/kpab_$a.json'));r=d['roofline'];print('ablate $a','KT',round(r['kernel_avg_ms'],4),'KP',round(r['posterior_kernel_avg_ms'] or 0,4),'step',round(d['ms_per_step'],4))"
done
for g in 1024 4096 8192; do
  NGSEP_KP_GRID=$g NGSEP_TIME_POSTERIOR=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold --no-e2e > gpurun_out/kpg_$g.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/kpg_$g.json'));r=d['roofline'];print('grid $g','KT',round(r['kernel_avg_ms'],4),'KP',round(r['posterior_kernel_avg_ms'] or 0,4),'step',round(d['ms_per_step'],4))"
done
