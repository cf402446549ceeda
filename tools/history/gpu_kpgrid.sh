export NGSEP_TIME_POSTERIOR=1
for g in ${KP_GRIDS:-256 512 1024 2048 4096}; do
  NGSEP_KP_GRID=$g timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold --no-e2e > gpurun_out/kpg_$g.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/kpg_$g.json'));r=d['roofline'];print('grid',$g,'post_ms',r['posterior_kernel_avg_ms'],'step_ms',round(d['ms_per_step'],4))"
done
