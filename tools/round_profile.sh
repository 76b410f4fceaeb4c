#!/bin/bash
# Round-end measurement on the GPU box, in this order (each step under its own time limit):
#   1. PMC passes (tools/pmc.sh) -> per-launch HBM traffic json (read by bench.py's roofline)
#   2. rocprofv3 --kernel-trace --stats over a bench run -> kernel stats csv
#   3. the full bench.py line (with the CPU baseline)
# The rocprof pass runs bench.py's default workload (the bench line's own command minus the CPU
# leg), so its per-kernel averages agree with the line's roofline k1_ms / k2_ms.
# usage: tools/round_profile.sh <round-tag>     (outputs under gpurun_out/, copy to profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_OUT=gpurun_out/pmc_$TAG bash tools/pmc.sh > gpurun_out/pmc_$TAG.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_$TAG.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc_$TAG gpurun_out/${TAG}_pmc_traffic.json || exit 1
python tools/pmc_summary.py gpurun_out/pmc_$TAG > gpurun_out/${TAG}_pmc_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -5 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
