#!/bin/bash
# round 5: the configs[3] headline on ONE GPU with its end-to-end leg (every GRCh38-length contig's BAM -> VCF through
# ngsep_call_bam, BAMs written untimed) and the CPU baseline, peak host RSS recorded
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05w2}
timeout -k 10 1120 python -u tools/maxrss.py python -u bench.py --config wgs --gpus 1 --wgs-shards 1 --no-cold \
    --steps 5 --warmup 1 > gpurun_out/${TAG}_wgs1.json 2> gpurun_out/${TAG}_wgs1.err
rc=$?
tail -8 gpurun_out/${TAG}_wgs1.err
cat gpurun_out/${TAG}_wgs1.json
exit $rc
