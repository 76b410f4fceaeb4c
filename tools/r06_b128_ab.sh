# round 6: C4's 128-sample shard (one stream) with the compact fold (one K1 launch per step, K2 once
# per rollout) against the product's K1 + K2 per step
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for lib in graph_neural_cellular_automata_amd/libgnca.so build_ab/lib_foldc.so; do
    for b in 128 256; do
      GNCA_LIB_PATH=$lib timeout -k 10 200 python bench.py --batch $b --no-cpu --steps 40 --warmup 5 > gpurun_out/r06f.json 2>gpurun_out/r06f.err || { tail -3 gpurun_out/r06f.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/r06f.json')); t=d['device_timeline']; print('B=$b', '$lib'.split('/')[-1], 'ms/step %.4f'%d['ms_per_step'], '%.3e'%d['value'], 'k1 %.4f'%t['k1_ms'], d['roofline']['kernel'])"
    done
  done
done
