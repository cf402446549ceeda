#!/bin/bash
# rocprofv3 kernel stats + PMC HBM traffic of the default bench workload.  Usage: bash tools/gpu_profile.sh TAG [bench args]
# PMC passes run separately (FETCH_SIZE, WRITE_SIZE), each with --kernel-trace only, as MI355X_MICROARCH.md prescribes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}
shift
ARGS="$@"
mkdir -p gpurun_out
KEY=$(python -c "print('human_chr20:30x:seed3:v3')")
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold --no-e2e $ARGS > gpurun_out/prof_$TAG.out 2>&1 || exit $?
python tools/kstats.py gpurun_out/prof_$TAG gpurun_out/kernel_stats_$TAG.csv
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_$TAG -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold --no-e2e $ARGS > gpurun_out/pmcf_$TAG.out 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_$TAG -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold --no-e2e $ARGS > gpurun_out/pmcw_$TAG.out 2>&1 || exit $?
python tools/pmc_traffic.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG k_tile_scan $KEY gpurun_out/pmc_traffic_$TAG.json
python tools/pmc_traffic.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG k_posterior kp:$KEY gpurun_out/pmc_traffic_kp_$TAG.json
echo done
