# round 6: the 24x36 classic split K1 (the trainers' message-off steps, large classic batches): GPU
# tests first, then the B=128 trainer iteration and a classic B=128 rollout with each library
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06e_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06e_pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for lib in build_ab/lib_head.so graph_neural_cellular_automata_amd/libgnca.so; do
    GNCA_LIB_PATH=$lib timeout -k 10 300 python bench.py --mode train --train-batch 128 --train-size 72 --steps 4 --warmup 1 > gpurun_out/r06e_train.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r06e_train.json')); print('train128', '$lib'.split('/')[-1], 'ms/iter %.2f'%d['ms_per_step'], '%.3e'%d['value'])"
    GNCA_LIB_PATH=$lib timeout -k 10 300 python bench.py --config c2 --batch 128 --no-cpu --steps 40 --warmup 5 > gpurun_out/r06e_c2b128.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r06e_c2b128.json')); print('classic B=128', '$lib'.split('/')[-1], 'ms/step %.4f'%d['ms_per_step'], '%.3e'%d['value'], d['roofline']['kernel'])"
  done
done
