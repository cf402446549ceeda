# multisample tile-size tuning (diagnostics): NGSEP_MS_BLOCK_COST values
set -e
mkdir -p gpurun_out
for c in ${1:-256 1024 2048 8192}; do
  NGSEP_MS_BLOCK_COST=$c timeout -k 10 300 python bench.py --config multisample --contig-first ${2:-0} --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/mstile_$c.json 2>gpurun_out/mstile_$c.err
  python -c "import json;d=json.load(open('gpurun_out/mstile_$c.json'));print('cost',$c,'T',d['config']['tile_positions'],'pile',d['config']['pile_bytes_per_gpu'],'ktm_ms',round(d['roofline']['kernel_avg_ms'],4),'kpm_ms',round(d['roofline']['posterior_kernel_avg_ms'],4),'step_ms',round(d['ms_per_step'],4))"
done
