#!/bin/bash
# KT change check: parity + full-size goldens, then two short chr20 benches (KT average, frac, step)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ktq_tests.log 2>&1 || { tail -20 gpurun_out/ktq_tests.log; exit 1; }
tail -1 gpurun_out/ktq_tests.log
for k in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cold --no-e2e ${BENCH_ARGS} > gpurun_out/ktq_$k.json 2> gpurun_out/ktq_$k.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ktq_$k.json'));r=d['roofline'];print('KT',round(r['kernel_avg_ms'],4),'frac',round(r['frac'],3),'step',round(d['ms_per_step'],4),'value',d['value'])"
done
