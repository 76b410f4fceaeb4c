#!/bin/bash
# K2 band sweep on the compact field at a config (measurement builds: GNCA_AB_KNOBS library).
# usage: tools/k2_band_c5.sh <knobs lib> "<bands>" <config> <rounds>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=$1; BANDS=${2:-"6 8 12 16 24"}; CFG=${3:-c5}; ROUNDS=${4:-2}
for r in $(seq $ROUNDS); do
  for bnd in $BANDS; do
    GNCA_LIB_PATH=$LIB GNCA_K2_BAND=$bnd timeout -k 10 200 python bench.py --config $CFG --no-cpu > gpurun_out/k2band.json 2> gpurun_out/k2band.err || { echo "bench failed: $bnd"; tail -5 gpurun_out/k2band.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/k2band.json')); print('$CFG band $bnd', 'ms/step %.4f'%d['ms_per_step'], 'k1 %.4f'%d['roofline']['k1_ms'], 'k2 %.4f'%d['roofline_k2']['k2_ms'])"
  done
done
