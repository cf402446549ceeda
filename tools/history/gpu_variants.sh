# compare build variants of libngsep_amd.so (diagnostics).  Usage: bash tools/gpu_variants.sh "default exp/w6 exp/w8" "0 1"
set -e
mkdir -p gpurun_out
export NGSEP_TIME_POSTERIOR=1
for v in ${1:-default}; do
  for a in ${2:-0}; do
    tag=$(echo $v | tr '/' '_')
    if [ "$v" = default ]; then unset NGSEP_LIB_PATH; else export NGSEP_LIB_PATH=$PWD/$v/libngsep_amd.so; fi
    NGSEP_ABLATE=$a timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/var_${tag}_$a.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/var_${tag}_$a.json'));r=d['roofline'];print('$v','ablate',$a,'kernel_ms',round(r['kernel_avg_ms'],4),'post_ms',r['posterior_kernel_avg_ms'],'step_ms',round(d['ms_per_step'],4))"
  done
done
unset NGSEP_LIB_PATH
