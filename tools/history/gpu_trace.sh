# kernel trace of a short bench run + per-pass timeline.  Usage: bash tools/gpu_trace.sh TAG [env...]
set -e
TAG=${1:-t}
shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.out 2>&1
python tools/kstats.py gpurun_out/prof_$TAG
