#!/bin/bash
# Quick GPU check: GPU tests, then the headline bench and the other configs without the CPU leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
for c in ${CONFIGS:-headline c2 c3 c5}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/q_$c.json 2> gpurun_out/q_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/q_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/q_$c.json')); r=d['roofline']; print('$c', '%.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], r['kernel'], 'k1 %.4f'%r['k1_ms'], 'frac %.3f'%r['frac'], 'busy %.3f'%r['mfma_busy_frac'], 'k2 %.4f'%d['roofline_k2']['k2_ms'], 'k2frac %.3f'%d['roofline_k2']['frac'])"
done
