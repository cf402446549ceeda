#!/bin/bash
# round 5: KZ (device BGZF inflate) microbenchmark on a synthetic BAM: batch, per-block latency, zlib check
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05zb}
timeout -k 10 300 python -u - <<'PY' > gpurun_out/${TAG}_synth.log 2>&1 || { tail -5 gpurun_out/${TAG}_synth.log; exit 1; }
import sys
sys.path.insert(0, "tools/synth")
import pysynth
s = pysynth.Synth(genome=pysynth.YEAST, n_contigs=4, contig_first=0, depth=30, seed=3)
print(s.write("/tmp/zb"))
PY
ls -la /tmp/zb*
timeout -k 10 120 tools/inflate_bench/build/inflate_bench /tmp/zb.bam 32 > gpurun_out/${TAG}.log 2>&1 || { cat gpurun_out/${TAG}.log; exit 1; }
cat gpurun_out/${TAG}.log
