#!/bin/bash
# round 4: where the population path's time goes -- host layout phases (NGSEP_HOST_TIMING) on the staged bench and the
# end-to-end run, KPM's phase stamps (NGSEP_TIMING, the diagnostics build in ab/diag)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NGSEP_HOST_TIMING=1 timeout -k 10 500 python -u bench.py --config multisample --no-cpu-baseline --no-cold --steps 3 --warmup 1 \
    > gpurun_out/popdiag_host.json 2> gpurun_out/popdiag_host.err || { tail -20 gpurun_out/popdiag_host.err; exit 1; }
grep "ngsep host\|end-to-end" gpurun_out/popdiag_host.err | head -60
NGSEP_TIMING=1 NGSEP_LIB_PATH=$PWD/ab/diag/libngsep_amd.so timeout -k 10 300 python -u bench.py --config multisample --no-cpu-baseline \
    --no-cold --steps 3 --warmup 1 > gpurun_out/popdiag_kpm.json 2> gpurun_out/popdiag_kpm.err || { tail -20 gpurun_out/popdiag_kpm.err; exit 1; }
grep "timing" gpurun_out/popdiag_kpm.err | head -10
