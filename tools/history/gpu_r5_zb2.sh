#!/bin/bash
# round 5: KZ with a 16 KB LDS ring (8 wavefronts a CU, far copies from HBM) -- inflate tests, microbenchmark
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05zc}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gpu_inflate.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u - <<'PY' > gpurun_out/${TAG}_synth.log 2>&1 || { tail -5 gpurun_out/${TAG}_synth.log; exit 1; }
import sys
sys.path.insert(0, "tools/synth")
import pysynth
s = pysynth.Synth(genome=pysynth.YEAST, n_contigs=4, contig_first=0, depth=30, seed=3)
print(s.write("/tmp/zb"))
PY
timeout -k 10 120 tools/inflate_bench/build/inflate_bench /tmp/zb.bam 32 > gpurun_out/${TAG}.log 2>&1 || { cat gpurun_out/${TAG}.log; exit 1; }
cat gpurun_out/${TAG}.log
