#!/bin/bash
# round 3: chr20 end-to-end anatomy on the box -- decode alone, then BAM -> VCF with the host-timing breakdown
# (NGSEP_HOST_TIMING: per-batch admission / projection, per-window layout / upload / run).  Usage: bash tools/gpu_r3_e2e.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-e2e}
mkdir -p gpurun_out /tmp/hp
timeout -k 10 300 python -u tools/host_profile.py --dir /tmp/hp --decode-only > gpurun_out/e2e_dec_$TAG.log 2>&1 || { tail -5 gpurun_out/e2e_dec_$TAG.log; exit 1; }
cat gpurun_out/e2e_dec_$TAG.log
for k in 1 2; do
  NGSEP_HOST_TIMING=1 timeout -k 10 200 python -u tools/host_profile.py --dir /tmp/hp --e2e-only > gpurun_out/e2e_${TAG}_$k.log 2> gpurun_out/e2e_${TAG}_$k.err || { tail -5 gpurun_out/e2e_${TAG}_$k.err; exit 1; }
  cat gpurun_out/e2e_${TAG}_$k.log
done
grep -v "window\|batch" gpurun_out/e2e_${TAG}_2.err | tail -20
