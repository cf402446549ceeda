#!/bin/bash
# round 4: configs[4] kernel stats and PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes) of KLM and KPM
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04m}
KEY=multisample200:10x:contig3:v3
B="python bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ms_$TAG -o run --output-format csv -- $B --steps 20 --warmup 4 \
    > gpurun_out/${TAG}_ms_prof.json 2> gpurun_out/${TAG}_ms_prof.err || { tail -5 gpurun_out/${TAG}_ms_prof.err; exit 1; }
python tools/kstats.py gpurun_out/prof_ms_$TAG gpurun_out/${TAG}_ms_kernel_stats.csv
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_ms_$TAG -o run --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/pmcf_ms_$TAG.out 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_ms_$TAG -o run --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/pmcw_ms_$TAG.out 2>&1 || exit 1
python tools/pmc_traffic.py gpurun_out/pmcf_ms_$TAG gpurun_out/pmcw_ms_$TAG k_scan_pop $KEY gpurun_out/pmc_traffic_klm_ms_$TAG.json 8
python tools/pmc_traffic.py gpurun_out/pmcf_ms_$TAG gpurun_out/pmcw_ms_$TAG k_posterior_multi kpm:$KEY gpurun_out/pmc_traffic_kpm_ms_$TAG.json 4
cat gpurun_out/pmc_traffic_klm_ms_$TAG.json gpurun_out/pmc_traffic_kpm_ms_$TAG.json
timeout -k 10 600 python -u bench.py --config multisample > gpurun_out/${TAG}_ms_bench.json 2> gpurun_out/${TAG}_ms_bench.err || { tail -20 gpurun_out/${TAG}_ms_bench.err; exit 1; }
tail -c 400 gpurun_out/${TAG}_ms_bench.json
