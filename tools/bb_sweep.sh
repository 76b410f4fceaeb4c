#!/bin/bash
# Per-kernel backward times at one size for a list of BB tiles (GNCA_BB_TILE measurement knob).
# usage: tools/bb_sweep.sh SIZE TILE [TILE ...]    e.g. tools/bb_sweep.sh 16x40 auto 4x16 8x8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
size=$1; shift
mkdir -p gpurun_out/bbsweep
for t in "$@"; do
  if [ "$t" = auto ]; then unset GNCA_BB_TILE; else export GNCA_BB_TILE=$t; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bbsweep/$t -o run --output-format csv \
    -- python3 tools/time_bwd.py --sizes $size --iters 20 > gpurun_out/bbsweep/$t.log 2>&1 || exit $?
  echo "== $t: $(grep 'B=' gpurun_out/bbsweep/$t.log)"
  python3 tools/kstats.py gpurun_out/bbsweep/$t/run_kernel_stats.csv gnca_
done
