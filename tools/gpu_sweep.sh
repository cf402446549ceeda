# tile-kernel tuning sweep (diagnostics): blocks per CU x ablation.  Usage: bash tools/gpu_sweep.sh "2 4 8" "0 1"
set -e
mkdir -p gpurun_out
for bpc in ${1:-4}; do
  for a in ${2:-0 1}; do
    NGSEP_BLOCKS_PER_CU=$bpc NGSEP_ABLATE=$a timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sweep_${bpc}_$a.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/sweep_${bpc}_$a.json'));print('bpc',$bpc,'ablate',$a,'kernel_ms',round(d['roofline']['kernel_avg_ms'],4),'post_ms',round(d['roofline']['posterior_kernel_avg_ms'],4),'step_ms',round(d['ms_per_step'],4))"
  done
done
