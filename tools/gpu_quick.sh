# quick GPU iteration: parity tests, one bench line, kernel trace summary.  Usage: bash tools/gpu_quick.sh TAG
set -e
TAG=${1:-q}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('value',round(d['value']/1e9,2),'G/s kernel_ms',round(d['roofline']['kernel_avg_ms'],4),'post_ms',d['roofline']['posterior_kernel_avg_ms'],'step_ms',round(d['ms_per_step'],4))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/prof_$TAG.out 2>&1
python tools/kstats.py gpurun_out/prof_$TAG
