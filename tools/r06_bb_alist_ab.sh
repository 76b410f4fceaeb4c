# round 6: masked-step BB walking only the active samples' tiles (gnca_b_actlist) against the full batch's
# tile ranges (build_ab/lib_noalist.so, -DGNCA_BB_NO_ALIST): gradient + fuzz tests first, then the B=128 and
# C5 trainer iterations with each library, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06i_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06i_pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for lib in build_ab/lib_noalist.so graph_neural_cellular_automata_amd/libgnca.so; do
    for cfg in "--train-batch 128 --train-size 72" "--config c5"; do
      GNCA_LIB_PATH=$lib timeout -k 10 300 python bench.py --mode train $cfg --steps 4 --warmup 1 > gpurun_out/r06i_train.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r06i_train.json')); print('train', '$cfg', '$lib'.split('/')[-1], 'ms/iter %.2f'%d['ms_per_step'], '%.3e'%d['value'])"
    done
  done
done
