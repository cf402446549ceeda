#!/bin/bash
# host staging profile on the box (16 host threads): tools/host_profile.py with the per-batch breakdown summed
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NGSEP_HOST_TIMING=1 timeout -k 10 500 python tools/host_profile.py --dir /tmp/hp "$@" > gpurun_out/hp.log 2>&1
grep -v "projection: [0-9]" gpurun_out/hp.log | grep -v "batch of"
python3 - <<'PY'
import re
adm = proj = 0; n = 0
for l in open("gpurun_out/hp.log"):
    m = re.search(r"admission ([\d.]+) ms, projection ([\d.]+)", l)
    if m: adm += float(m.group(1)); proj += float(m.group(2)); n += 1
print("batches", n, "admission ms", round(adm), "projection ms", round(proj))
PY
NGSEP_HOST_TIMING=1 timeout -k 10 300 python tools/host_profile.py --dir /tmp/hp --e2e-only 2>&1 | grep -v "projection: [0-9]" | grep -v "batch of"
