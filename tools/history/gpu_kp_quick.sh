#!/bin/bash
# KP change check: parity, known variants, full-size goldens; then the chr20 bench with KP timed
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/kpq_tests.log 2>&1 || { tail -30 gpurun_out/kpq_tests.log; exit 1; }
tail -1 gpurun_out/kpq_tests.log
for k in 1 2; do
  NGSEP_TIME_POSTERIOR=1 timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cold --no-e2e > gpurun_out/kpq_$k.json 2> gpurun_out/kpq_$k.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/kpq_$k.json'));r=d['roofline'];print('KT',round(r['kernel_avg_ms'],4),'KP',round(r['posterior_kernel_avg_ms'],4),'step',round(d['ms_per_step'],4),'value',d['value'])"
done
