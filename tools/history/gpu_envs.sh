# bench lines under several environment settings.  Usage: bash tools/gpu_envs.sh "A=1 B=2" "C=3" ...
set -e
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/env_$i.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/env_$i.json'));r=d['roofline'];print('$e'.ljust(40),'value',round(d['value']/1e9,2),'kernel_ms',round(r['kernel_avg_ms'],4),'step_ms',round(d['ms_per_step'],4),'T',d['config']['tile_positions'])"
done
