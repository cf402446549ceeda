# configs[4] multisample: PMC traffic of KTM, bench, rocprof kernel stats.  Usage: bash tools/gpu_ms_bench.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ms}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcfms_$TAG -o run --output-format csv -- python bench.py --config multisample --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/pmcfms_$TAG.out 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcwms_$TAG -o run --output-format csv -- python bench.py --config multisample --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/pmcwms_$TAG.out 2>&1
python tools/pmc_traffic.py gpurun_out/pmcfms_$TAG gpurun_out/pmcwms_$TAG k_scan_multi multisample200:10x:contig3:v2 gpurun_out/pmc_traffic_ms_$TAG.json
python tools/pmc_traffic.py gpurun_out/pmcfms_$TAG gpurun_out/pmcwms_$TAG k_posterior_multi kpm:multisample200:10x:contig3:v2 gpurun_out/pmc_traffic_kpm_$TAG.json
timeout -k 10 600 python bench.py --config multisample --steps 20 --warmup 4 > gpurun_out/bench_ms_$TAG.json 2> gpurun_out/bench_ms_$TAG.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ms_$TAG -o run --output-format csv -- python bench.py --config multisample --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/prof_ms_$TAG.out 2>&1
echo done
