# multisample kernel-phase ablation (diagnostics): 0 full, 32 gather only, 64 gather + tallies
set -e
mkdir -p gpurun_out
for a in ${1:-0 32 64}; do
  NGSEP_ABLATE=$a timeout -k 10 300 python bench.py --config multisample --contig-first 0 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/msab_$a.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/msab_$a.json'));print('ablate',$a,'ktm_ms',round(d['roofline']['kernel_avg_ms'],4),'kpm_ms',round(d['roofline']['posterior_kernel_avg_ms'],4),'step_ms',round(d['ms_per_step'],4))"
done
