# KT (512-position plane tiles) occupancy A/B (diagnostics): builds with NGSEP_KT16_WAVES_PER_EU 3 (lib), 4, 5.
set -e
mkdir -p gpurun_out
for v in lib lib_w4 lib_w5; do
  for g in yeast human_chr20; do
    NGSEP_LIB_PATH=$PWD/ngsepcore_amd/$v/libngsep_amd.so timeout -k 10 240 python bench.py --genome $g --steps 20 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/kw_${v}_$g.json 2> gpurun_out/kw_${v}_$g.err
    python -c "import json;d=json.load(open('gpurun_out/kw_${v}_$g.json'));print('$v','$g','value',round(d['value']/1e9,1),'step',round(d['ms_per_step'],4),'KT',round(d['roofline']['kernel_avg_ms'],4))"
  done
done
