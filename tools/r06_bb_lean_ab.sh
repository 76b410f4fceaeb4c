# round 6: backward A/B of the lean-layout 24x24 BB instances (B >= 96 at 72^2) against the 8x24 plans
# (-DGNCA_BB_NO_LEAN): gradient tests first, then tools/time_bwd.py and the B=128 trainer iteration
# with each library, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06g_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06g_pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for lib in build_ab/lib_nolean.so graph_neural_cellular_automata_amd/libgnca.so; do
    echo "== $lib"
    GNCA_LIB_PATH=$lib timeout -k 10 200 python tools/time_bwd.py --sizes 1024x72,128x72,16x40 --iters 10 2>&1 | grep "B=" || exit 1
  done
done
for r in 1 2; do
  for lib in build_ab/lib_nolean.so graph_neural_cellular_automata_amd/libgnca.so; do
    GNCA_LIB_PATH=$lib timeout -k 10 300 python bench.py --mode train --train-batch 128 --train-size 72 --steps 4 --warmup 1 > gpurun_out/r06g_train.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r06g_train.json')); print('train128', '$lib'.split('/')[-1], 'ms/iter %.2f'%d['ms_per_step'], '%.3e'%d['value'])"
  done
done
# BB's own time at B=1024 72^2: kernel trace of tools/time_bwd.py with each library
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lib in build_ab/lib_nolean.so graph_neural_cellular_automata_amd/libgnca.so; do
  tag=$(basename $lib .so)
  GNCA_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r06g_$tag -o run -- python3 tools/time_bwd.py --sizes 1024x72 --iters 10 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/prof_r06g_$tag -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/r06g_bwd1024_kernel_stats_$tag.csv
  python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/r06g_bwd1024_kernel_stats_$tag.csv')))
for r in rows[:6]: print('$tag', r['Name'][:70], r['Calls'], '%.1f us'%(float(r['AverageNs'])/1e3))"
done
