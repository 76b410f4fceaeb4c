#!/bin/bash
# Round-end evidence in one GPU call: tools/round_profile.sh <tag> (PMC traffic, rocprof stats, the
# headline bench line), then the other BASELINE configs' bench lines and the two training benches.
# Outputs under gpurun_out/ (copy to profiles/).   usage: tools/round_all.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/round_profile.sh $TAG || exit $?
python tools/prof_agree.py gpurun_out/prof_$TAG/run_kernel_trace.csv gpurun_out/bench_$TAG.json 8 > gpurun_out/${TAG}_rocprof_agreement.txt
for c in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "bench $c failed"; exit 1; }
done
timeout -k 10 400 python bench.py --mode train --steps 10 --warmup 2 > gpurun_out/bench_${TAG}_train.json 2> gpurun_out/bench_${TAG}_train.err || { echo "train failed"; exit 1; }
timeout -k 10 400 python bench.py --mode train --config c5 --steps 4 --warmup 1 > gpurun_out/bench_${TAG}_train_c5.json 2> gpurun_out/bench_${TAG}_train_c5.err || { echo "train c5 failed"; exit 1; }
for f in gpurun_out/bench_${TAG}*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', '%.4e'%d['value'], 'ms/step %.4f'%d['ms_per_step'])"; done
