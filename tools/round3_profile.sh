#!/bin/bash
# Round-3 evidence in one GPU call (each GPU step under its own time limit, stop at the first failure):
#   GPU tests; PMC passes (HBM traffic, MFMA busy, LDS conflicts) -> <tag>_pmc_traffic.json and
#   summary; rocprofv3 kernel trace of the driver's bench command; the driver's bench command itself
#   (with the CPU baseline); the other BASELINE configs.   usage: tools/round3_profile.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest_gpu.log
fi
PMC_CMD="python3 bench.py --steps 4 --warmup 1 --no-cpu --gpu-warmup-ms 0" PMC_OUT=gpurun_out/pmc_$TAG bash tools/pmc.sh > gpurun_out/pmc_$TAG.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_$TAG.log; exit 1; }
PMC_LAUNCHES_PER_STEP=${SUBS:-2} python tools/pmc_traffic.py gpurun_out/pmc_$TAG gpurun_out/${TAG}_pmc_traffic.json || exit 1
python tools/pmc_summary.py gpurun_out/pmc_$TAG > gpurun_out/${TAG}_pmc_summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { echo "rocprof failed"; tail -5 gpurun_out/${TAG}_prof.err; exit 1; }
cp gpurun_out/prof_$TAG/run_kernel_stats.csv gpurun_out/${TAG}_rocprof_kernel_stats.csv 2>/dev/null || find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_rocprof_kernel_stats.csv \;
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/${TAG}_bench96.json 2> gpurun_out/${TAG}_bench96.err || { echo "bench96 failed"; exit 1; }
for c in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/${TAG}_$c.err; exit 1; }
done
for f in gpurun_out/${TAG}_bench.json gpurun_out/${TAG}_bench96.json gpurun_out/${TAG}_c2.json gpurun_out/${TAG}_c3.json gpurun_out/${TAG}_c5.json; do
  python -c "import json; d=json.load(open('$f')); r=d['roofline']; t=d['device_timeline']; print('$f', '%.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'span %.4f subs %d k1 %.4f k2 %.4f'%(t['first_k1_start_to_last_k2_end_ms_per_step'], t['sub_batches'], t['k1_ms'], t['k2_ms']), 'frac %.3f'%r['frac'])"
done
head -6 gpurun_out/${TAG}_rocprof_kernel_stats.csv | cut -c1-150
