#!/bin/bash
# round 3: KL with the fused survivor gather (NGSEP_KL_FUSE=1): parity, then kernel times beside the default; the
# multisample bench (host layout after the in-place read bytes).  Usage: bash tools/gpu_r3_fuse.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-fuse}
mkdir -p gpurun_out
NGSEP_KL_FUSE=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_indels.py "tests/test_gpu_full_size.py::test_full_size_vcf_identical" > gpurun_out/fuse_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/fuse_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/fuse_tests_$TAG.log
B="python bench.py --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 3"
for E in "NGSEP_X=0" "NGSEP_KL_FUSE=1" "NGSEP_X=0" "NGSEP_KL_FUSE=1"; do
  env $E timeout -k 10 300 $B > gpurun_out/fu_$TAG.json 2> gpurun_out/fu_$TAG.err || { tail -5 gpurun_out/fu_$TAG.err; exit 1; }
  echo "$E: $(python -c "import json; d=json.load(open('gpurun_out/fu_$TAG.json')); print(round(d['ms_per_step'],4), '%.4g' % d['value'], round(d['roofline']['kernel_avg_ms'],4))")"
done
NGSEP_KL_FUSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fuprof_$TAG -o run --output-format csv -- $B > gpurun_out/fuprof_$TAG.out 2>&1 || exit 1
python tools/kstats.py gpurun_out/fuprof_$TAG | head -6
NGSEP_HOST_TIMING=1 timeout -k 10 600 python bench.py --config multisample --steps 10 --warmup 2 --no-cpu-baseline --no-cold > gpurun_out/msfu_$TAG.json 2> gpurun_out/msfu_$TAG.err || { tail -5 gpurun_out/msfu_$TAG.err; exit 1; }
grep "population layout\|layout .* ms, device upload" gpurun_out/msfu_$TAG.err | head -8
python -c "import json; d=json.load(open('gpurun_out/msfu_$TAG.json')); print('ms step', d['ms_per_step'], 'layout', d['config']['host_layout_ms'], 'upload', d['config']['h2d_upload_ms'], 'e2e', d.get('end_to_end', {}).get('wall_s'))"
