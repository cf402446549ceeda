#!/bin/bash
# round 3: KTM byte-parallel bound -- multisample parity, then the configs[4] step and kernel times.
# (historical: the NGSEP_KPM_WPE / NGSEP_KPM_GRID knobs and the byte-parallel KTM were removed once measured)
# Usage: bash tools/gpu_r3_ktm.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-ktm}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multisample.py tests/test_gpu_pool.py "tests/test_gpu_full_size.py" -k "multisample or pool or population or Multisample" > gpurun_out/ktm_tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/ktm_tests_$TAG.log | head -20; tail -5 gpurun_out/ktm_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/ktm_tests_$TAG.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ktmprof_$TAG -o run --output-format csv -- python bench.py --config multisample --steps 10 --warmup 2 --no-cpu-baseline --no-cold --no-e2e > gpurun_out/ktmprof_$TAG.out 2>&1 || { tail -5 gpurun_out/ktmprof_$TAG.out; exit 1; }
python tools/kstats.py gpurun_out/ktmprof_$TAG | head -6
timeout -k 10 400 python bench.py --config multisample --steps 20 --warmup 3 --no-cpu-baseline --no-cold --no-e2e > gpurun_out/ktmb_$TAG.json 2> gpurun_out/ktmb_$TAG.err || { tail -5 gpurun_out/ktmb_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/ktmb_$TAG.json')); print('step', d['ms_per_step'], 'value %.4g' % d['value'], 'roofline', d['roofline']['kernel'], round(d['roofline']['kernel_avg_ms'],4), round(d['roofline']['frac'],4))"
# KPM: register cap (4 waves per SIMD) and grid size
NGSEP_KPM_WPE=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_multisample.py tests/test_gpu_pool.py > gpurun_out/kpm_tests_$TAG.log 2>&1 || { tail -20 gpurun_out/kpm_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/kpm_tests_$TAG.log
B="python bench.py --config multisample --steps 20 --warmup 3 --no-cpu-baseline --no-cold --no-e2e"
for E in "NGSEP_X=0" "NGSEP_KPM_WPE=4" "NGSEP_KPM_GRID=768" "NGSEP_KPM_WPE=4 NGSEP_KPM_GRID=1024" "NGSEP_KPM_GRID=4096" "NGSEP_KPM_WPE=4 NGSEP_KPM_GRID=8192"; do
  env $E NGSEP_TIMING=1 timeout -k 10 300 $B > gpurun_out/kpm_$TAG.json 2> gpurun_out/kpm_$TAG.err || { tail -5 gpurun_out/kpm_$TAG.err; exit 1; }
  echo "$E: $(python -c "import json; d=json.load(open('gpurun_out/kpm_$TAG.json')); print(round(d['ms_per_step'],4), d['roofline'].get('posterior_kernel_avg_ms'))")"
done
