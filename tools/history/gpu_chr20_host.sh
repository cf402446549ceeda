# chr20 pass anatomy (diagnostics): host costs per pass and the kernel timeline at T=256 and T=512.
set -e
TAG=${1:-h}
mkdir -p gpurun_out
for T in 256 512; do
  NGSEP_TILE_T=$T NGSEP_HOST_TIMING=1 NGSEP_PROBE_HOST=1 timeout -k 10 240 python bench.py --genome human_chr20 --steps 20 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/host_${TAG}_$T.json 2> gpurun_out/host_${TAG}_$T.err
done
NGSEP_TILE_T=512 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof512_$TAG -o run --output-format csv -- python bench.py --genome human_chr20 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/prof512_$TAG.out 2>&1
echo done
