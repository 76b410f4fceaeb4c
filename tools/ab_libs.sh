#!/bin/bash
# A/B of several libgnca builds (GNCA_LIB_PATH) on one bench config, interleaved rounds, one GPU call.
# usage: tools/ab_libs.sh "<lib1> <lib2> ..." <config> <rounds> [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS=$1; CONFIG=${2:-headline}; ROUNDS=${3:-3}; shift 3; EXTRA="$*"
for r in $(seq $ROUNDS); do
  for lib in $LIBS; do
    GNCA_LIB_PATH=$lib timeout -k 10 200 python bench.py --config $CONFIG --no-cpu --steps 40 --warmup 5 $EXTRA > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed: $lib"; tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); t=d['device_timeline']; print('$CONFIG', '$(basename $lib)', 'ms/step %.4f'%d['ms_per_step'], 'subs %d k1 %.4f k2 %.4f span %.4f'%(t.get('sub_batches',1), t['k1_ms'], t['k2_ms'], t['first_k1_start_to_last_k2_end_ms_per_step']), '%.3e'%d['value'], 'live %.3f'%d['roofline']['live_fraction'], 'tail %.3f'%(t.get('k1_tail_frac') or 0))"
  done
done
