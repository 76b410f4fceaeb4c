#!/bin/bash
# A/B/C of the current libgnca against alternative builds (GNCA_LIB_PATH) on bench configs,
# interleaved rounds in one GPU call.   usage: tools/ab_libs3.sh "<alt libs>" "<configs>" <rounds>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ALTS=$1; CONFIGS=${2:-"headline"}; ROUNDS=${3:-3}
for r in $(seq $ROUNDS); do
  for c in $CONFIGS; do
    for lib in "" $ALTS; do
      GNCA_LIB_PATH=$lib timeout -k 10 200 python bench.py --config $c --no-cpu > gpurun_out/ablib.json 2> gpurun_out/ablib.err || { echo "bench failed: $c $lib"; tail -5 gpurun_out/ablib.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/ablib.json')); r=d['roofline']; print('$c', '${lib:-current}', 'ms/step %.4f'%d['ms_per_step'], 'k1 %.4f'%r['k1_ms'], 'k2 %.4f'%d['roofline_k2']['k2_ms'])"
    done
  done
done
