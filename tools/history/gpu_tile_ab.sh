# yeast 30x (configs[1]) tile width A/B, two repeats each (diagnostics).
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for T in 256 512; do
    NGSEP_TILE_T=$T timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/ab_y_${T}_$rep.json 2> gpurun_out/ab_y_${T}_$rep.err
    python -c "import json;d=json.load(open('gpurun_out/ab_y_${T}_$rep.json'));print('T',$T,'rep',$rep,'value',round(d['value']/1e9,1),'step',round(d['ms_per_step'],4),'KT',round(d['roofline']['kernel_avg_ms'],4))"
  done
done
