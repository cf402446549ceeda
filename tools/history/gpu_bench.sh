# One GPU session: parity tests, PMC traffic passes, bench, rocprof kernel stats.  Usage: bash tools/gpu_bench.sh TAG
# The PMC passes run first so the bench line carries this build's traffic (profiles/pmc_traffic.json).
set -e
TAG=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1
fi
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_$TAG -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/pmcf_$TAG.out 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_$TAG -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/pmcw_$TAG.out 2>&1
python tools/pmc_traffic.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG k_tile_p yeast:30x:seed2 gpurun_out/pmc_traffic_$TAG.json
cp gpurun_out/pmc_traffic_$TAG.json profiles/pmc_traffic.json
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/prof_$TAG.out 2>&1
if [ -n "$WITH_MS" ]; then
timeout -k 10 600 python bench.py --config multisample --steps 5 --warmup 2 > gpurun_out/bench_ms_$TAG.json 2> gpurun_out/bench_ms_$TAG.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ms_$TAG -o run --output-format csv -- python bench.py --config multisample --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/prof_ms_$TAG.out 2>&1
fi
if [ -n "$WITH_CHR20" ]; then
# BASELINE.json configs[2]: human chr20 30x, planes (~0.7 GB) larger than the Infinity Cache -> HBM-bound scan
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf20_$TAG -o run --output-format csv -- python bench.py --genome human_chr20 --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/pmcf20_$TAG.out 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw20_$TAG -o run --output-format csv -- python bench.py --genome human_chr20 --steps 3 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/pmcw20_$TAG.out 2>&1
python tools/pmc_traffic.py gpurun_out/pmcf20_$TAG gpurun_out/pmcw20_$TAG k_tile_p human_chr20:30x:seed2 gpurun_out/pmc_traffic_chr20_$TAG.json
cp gpurun_out/pmc_traffic_chr20_$TAG.json profiles/pmc_traffic_chr20.json
timeout -k 10 400 python bench.py --genome human_chr20 --steps 10 --warmup 2 > gpurun_out/bench_chr20_$TAG.json 2> gpurun_out/bench_chr20_$TAG.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_chr20_$TAG -o run --output-format csv -- python bench.py --genome human_chr20 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/prof_chr20_$TAG.out 2>&1
fi
echo done
