#!/bin/bash
# A/B of the K1 variants on the headline workload (bench.py --no-cpu), each under its own limit.
# usage: tools/ab_env.sh "ENV=.. ENV2=..;ENV=..;..."   (one bench per ';'-separated env set)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "${1:-GNCA_K2_ZIGZAG=1;GNCA_K2_ZIGZAG=0}"
i=0
for envs in "${SETS[@]}"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { echo "bench failed: $envs"; tail -5 gpurun_out/ab_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$i.json')); r=d['roofline']; print('$envs', '%.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], r['kernel'], 'k1 %.4f'%r['k1_ms'], 'frac %.3f'%r['frac'], 'k2 %.4f'%d['roofline_k2']['k2_ms'])"
done
