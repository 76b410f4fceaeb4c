#!/bin/bash
# The BASELINE.json GPU configs through bench.py (c2 classic B=8, c3 graph B=8, c5 32ch 128^2 r=5
# K=16) plus a rocprofv3 kernel-trace of each; outputs under gpurun_out/ (copy to profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
for c in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err \
    || { echo "bench $c failed"; tail -5 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  cat gpurun_out/bench_${TAG}_$c.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$c -o run --output-format csv \
    -- python3 bench.py --config $c --steps 24 --warmup 4 --no-cpu > gpurun_out/prof_${TAG}_$c.log 2>&1 \
    || { echo "rocprof $c failed"; tail -5 gpurun_out/prof_${TAG}_$c.log; exit 1; }
done
