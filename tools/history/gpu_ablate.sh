# kernel-phase ablation (diagnostics): NGSEP_ABLATE=1 no genotyping, 2 tally only
set -e
mkdir -p gpurun_out
for a in 0 1 2; do
  NGSEP_ABLATE=$a timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ablate_$a.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/ablate_$a.json'));print('ablate',$a,'kernel_ms',d['roofline']['kernel_avg_ms'],'step_ms',d['ms_per_step'])"
done
