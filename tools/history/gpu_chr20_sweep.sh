# chr20 (configs[2], HBM-bound planes) tuning sweep, diagnostics: tile width x KT workgroups per CU x KP grid.
# Usage: bash tools/gpu_chr20_sweep.sh TAG
set -e
TAG=${1:-sw}
mkdir -p gpurun_out
run() {   # name, env...
  local name=$1; shift
  env "$@" NGSEP_TIME_POSTERIOR=1 timeout -k 10 240 python bench.py --genome human_chr20 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/sw_${TAG}_$name.json 2> gpurun_out/sw_${TAG}_$name.err
  python -c "import json;d=json.load(open('gpurun_out/sw_${TAG}_$name.json'));r=d['roofline'];print('$name','KT',round(r['kernel_avg_ms'],4),'KP',round(r['posterior_kernel_avg_ms'] or 0,4),'step',round(d['ms_per_step'],4),'T',d['config']['tile_positions'])"
}
run base
run t512 NGSEP_TILE_T=512
run t128 NGSEP_TILE_T=128
run bpc2 NGSEP_BLOCKS_PER_CU=2
run bpc6 NGSEP_BLOCKS_PER_CU=6
run kp4096 NGSEP_KP_GRID=4096
run kp1024 NGSEP_KP_GRID=1024
echo done
