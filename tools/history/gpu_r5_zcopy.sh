#!/bin/bash
# round 5: packed batches read in place from the decoded chunks (no per-record base / quality copies) -- BAM-path GPU
# tests, then the chr20 end-to-end legs with host timing, twice, and the population end-to-end run
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05zy}
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_indels.py tests/test_gpu_realigner_cases.py \
    tests/test_gpu_inflate.py tests/test_gpu_multi.py tests/test_gpu_full_size.py tests/test_gpu_known.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for k in 1 2; do
  NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --no-cold --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_b$k.json 2> gpurun_out/${TAG}_b$k.err || { tail -20 gpurun_out/${TAG}_b$k.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_b$k.json").read().strip().splitlines()[-1])
e = d["end_to_end"]
print("chr20 snv e2e %.3f s" % e["wall_s"], "indel e2e %.3f s" % e["indels"]["wall_s"], "records", e["vcf_records"], e["indels"]["vcf_records"])
PY
  grep -E "bam:|call_bam:" gpurun_out/${TAG}_b$k.err | head -4
done
timeout -k 10 400 python -u bench.py --config multisample --no-cold --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_ms.json 2> gpurun_out/${TAG}_ms.err || { tail -20 gpurun_out/${TAG}_ms.err; exit 1; }
python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_ms.json").read().strip().splitlines()[-1])
print("population e2e %.3f s" % d["end_to_end"]["wall_s"])
PY
