# A/B of an environment switch on the default bench.  Usage: bash tools/gpu_ab.sh "ENV=1" [extra bench args]
set -e
mkdir -p gpurun_out
SW=${1:-NGSEP_ONE_STREAM=1}
shift || true
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/ab_base_$rep.json 2>/dev/null
  env $SW timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/ab_sw_$rep.json 2>/dev/null
  for t in base sw; do
    python -c "import json;d=json.load(open('gpurun_out/ab_${t}_$rep.json'));r=d['roofline'];print('$t',$rep,'value',round(d['value']/1e9,2),'kernel_ms',round(r['kernel_avg_ms'],4),'step_ms',round(d['ms_per_step'],4))"
  done
done
