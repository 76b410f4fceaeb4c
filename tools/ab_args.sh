#!/bin/bash
# A/B of the current libgnca against alternative builds (GNCA_LIB_PATH) on bench argument sets,
# interleaved rounds in one GPU call.
# usage: tools/ab_args.sh "<alt libs>" "<bench args>;<bench args>;..." <rounds>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ALTS=$1; ARGSETS=$2; ROUNDS=${3:-3}
IFS=';' read -ra SETS <<< "$ARGSETS"
for r in $(seq $ROUNDS); do
  for a in "${SETS[@]}"; do
    for lib in "" $ALTS; do
      GNCA_LIB_PATH=$lib timeout -k 10 200 python bench.py $a --no-cpu > gpurun_out/abargs.json 2> gpurun_out/abargs.err || { echo "bench failed: $a $lib"; tail -5 gpurun_out/abargs.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/abargs.json')); r=d.get('roofline',{}); print('[$a]', '${lib:-current}', 'ms/step %.4f'%d['ms_per_step'], 'G/s %.3f'%(d['value']/1e9))"
    done
  done
done
