#!/bin/bash
# One GPU call that validates and measures a working tree: GPU tests, the four bench configs, then
# A/B benches and backward timings against alternative builds (build_ab/*.so, GNCA_LIB_PATH).
# usage: tools/gpu_check.sh "<ab env sets for the headline, ';'-separated>" "<alt lib for bwd A/B>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/quick.sh || exit $?
if [ -n "${1:-}" ]; then bash tools/ab_env.sh "$1" || exit $?; fi
for lib in "" ${2:-}; do
  for spec in "--sizes 1024x72,16x40" "--sizes 16x128 --channels 32 --radius 5 --k 16"; do
    GNCA_LIB_PATH=$lib timeout -k 10 200 python tools/time_bwd.py $spec --iters 10 > gpurun_out/tb.log 2>&1 || { echo "time_bwd failed"; tail -5 gpurun_out/tb.log; exit 1; }
    sed "s|^|[${lib:-current}] |" gpurun_out/tb.log | grep "fwd"
  done
done
