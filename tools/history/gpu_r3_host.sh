#!/bin/bash
# round 3: host-path changes -- parity tests that load FASTA files, then the chr20 end-to-end anatomy and the bench's
# end-to-end figure.  Usage: bash tools/gpu_r3_host.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-host}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_indels.py > gpurun_out/host_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/host_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/host_tests_$TAG.log
bash tools/gpu_r3_e2e.sh $TAG || exit 1
grep "batch of" gpurun_out/e2e_${TAG}_2.err | sed 's/.*admission \([0-9.]*\) ms, projection \([0-9.]*\) ms, stream \([0-9.]*\) ms, carry \([0-9.]*\) ms/\1 \2 \3 \4/' | awk '{a+=$1; p+=$2; s+=$3; c+=$4; n++} END {print n, "batches: admission", a, "projection", p, "stream", s, "carry", c, "ms"}'
grep "call_bam:" gpurun_out/e2e_${TAG}_2.err
bash tools/gpu_r3_klab.sh $TAG 0 65536 || exit 1
NGSEP_TIMING=1 timeout -k 10 300 python -u bench.py --config multisample --steps 2 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/ms_timing_$TAG.json 2> gpurun_out/ms_timing_$TAG.err || { tail -5 gpurun_out/ms_timing_$TAG.err; exit 1; }
grep "ngsep timing" gpurun_out/ms_timing_$TAG.err | head -5
