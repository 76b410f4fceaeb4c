#!/bin/bash
# Round-3 measurement pass: headline bench (driver's command), the other configs, and a rocprofv3
# kernel trace of the headline command (agreement with the bench's stamped K1/K2 durations).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03}
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
for c in ${CONFIGS:-c2 c3 c5}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/${TAG}_$c.err; exit 1; }
done
for f in gpurun_out/${TAG}_bench.json gpurun_out/${TAG}_c*.json; do
  python -c "import json; d=json.load(open('$f')); r=d['roofline']; t=d['device_timeline']; print('$f', '%.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'stamped %.4f span %.4f subs %d k1 %.4f k2 %.4f'%(t['stamped_rollout_ms_per_step'], t['first_k1_start_to_last_k2_end_ms_per_step'], t.get('sub_batches',1), t['k1_ms'], t['k2_ms']), 'frac %.3f'%r['frac'])"
done
if [ -n "${PROF:-1}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { echo "prof failed"; tail -5 gpurun_out/${TAG}_prof.err; exit 1; }
  find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/${TAG}_rocprof_kernel_stats.csv
  head -5 gpurun_out/${TAG}_rocprof_kernel_stats.csv | cut -c1-160
fi
