#!/bin/bash
# round 6: MultisampleVariantsDetector at any depth (deep tiles -> k_scan_pop<false>, KPM / stage A columns in the
# device scratch) and the real-data read shapes, then the population suites and the smoke test
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06a}
run() {   # name, timeout, pytest args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider "$@" \
      > gpurun_out/${TAG}_$n.log 2>&1 || { tail -40 gpurun_out/${TAG}_$n.log; exit 1; }
  tail -1 gpurun_out/${TAG}_$n.log
}
run deep 500 tests/test_gpu_deep_population.py
run shapes 500 tests/test_gpu_read_shapes.py -s
run fullpop 400 tests/test_gpu_full_size.py -k deep_repeat
run pop 700 tests/test_gpu_multisample.py tests/test_gpu_kpm_stages.py tests/test_gpu_pool.py
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
