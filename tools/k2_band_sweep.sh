#!/bin/bash
# K2 band-height sweep (measurement only): GNCA_K2_BAND rows per K2 workgroup, headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in ${BANDS:-2 3 4 6 12}; do
  GNCA_K2_BAND=$b timeout -k 10 120 python bench.py --steps 48 --warmup 4 --no-cpu > gpurun_out/k2b.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/k2b.json')); print($b, d['roofline_k2']['k2_ms'], d['ms_per_step'])"
done
