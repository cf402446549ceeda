#!/bin/bash
# round-2 extra checks: configs[3] chr21 full-size golden, multisample bench with its end-to-end leg, and a
# 2-rank rehearsal of bench.py --gpus 2 on one GPU (gloo for the barrier and the timing reductions)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_full_size.py -m gpu -x -q -k configs3 --timeout 450 --timeout-method thread > gpurun_out/x_full3.log 2>&1; rc=$?
tail -2 gpurun_out/x_full3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config multisample --steps 5 --warmup 2 > gpurun_out/x_ms.json 2> gpurun_out/x_ms.err || { tail -5 gpurun_out/x_ms.err; exit 1; }
tail -3 gpurun_out/x_ms.err; python -c "import json;d=json.load(open('gpurun_out/x_ms.json'));print(d['value'],d['ms_per_step'],d.get('end_to_end'))"
NGSEP_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/x_g2.json 2> gpurun_out/x_g2.err || { tail -5 gpurun_out/x_g2.err; exit 1; }
cat gpurun_out/x_g2.json
