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
bash tools/r06_bb_lean_prof.sh
