#!/bin/bash
# quick GPU check: the -m gpu suite, then a short chr20 bench with KP timed (no CPU baseline / cold / e2e)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
NGSEP_TIME_POSTERIOR=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold --no-e2e ${BENCH_ARGS} > gpurun_out/quick.json 2> gpurun_out/quick.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/quick.json'));r=d['roofline'];print('KT',round(r['kernel_avg_ms'],4),'KP',round(r['posterior_kernel_avg_ms'] or 0,4),'step',round(d['ms_per_step'],4),'sites',d['config'].get('sites_called_per_gpu'))"
