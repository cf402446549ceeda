# tile-kernel tuning sweep (diagnostics): blocks per CU x ablation.  Usage: bash tools/gpu_sweep.sh "auto 2 4" "0 1"
# ("auto" = the occupancy-derived default)
set -e
mkdir -p gpurun_out
for bpc in ${1:-auto}; do
  for a in ${2:-0 1}; do
    if [ "$bpc" = auto ]; then unset NGSEP_BLOCKS_PER_CU; else export NGSEP_BLOCKS_PER_CU=$bpc; fi
    NGSEP_ABLATE=$a timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sweep_${bpc}_$a.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/sweep_${bpc}_$a.json'));print('bpc','$bpc','ablate',$a,'kernel_ms',round(d['roofline']['kernel_avg_ms'],4),'post_ms',round(d['roofline']['posterior_kernel_avg_ms'],4),'step_ms',round(d['ms_per_step'],4))"
  done
done
unset NGSEP_BLOCKS_PER_CU
