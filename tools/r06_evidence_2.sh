# round-6 evidence, part 2: the other BASELINE configs' lines, C4's 128-sample shard, the strong-scaling
# form at N=1, the regeneration loop, and PMC passes of the 128-sample shard and c5
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r06z}
export GNCA_LIB_SHA16=$(python3 -c "import hashlib;print(hashlib.sha256(open('graph_neural_cellular_automata_amd/libgnca.so','rb').read()).hexdigest()[:16])")
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 $to "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err; local rc=$?
  tail -c 300 gpurun_out/${T}_$name.json; echo
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${T}_$name.err; echo "STOP"; exit $rc; fi
}
step c2 300 python bench.py --config c2
step c3 300 python bench.py --config c3
step c5 300 python bench.py --config c5
step zeropad 300 python bench.py --config zeropad
step b128 300 python bench.py --batch 128
step strong1 300 python bench.py --scaling strong --no-cpu
step regen 300 python bench.py --mode regen --steps 300 --warmup 1
for c in b128 c5; do
  args="--batch 128"; lps=1; [ $c = c5 ] && args="--config c5"
  PMC_CMD="python3 bench.py --steps 4 --warmup 1 --no-cpu --gpu-warmup-ms 0 $args" PMC_OUT=gpurun_out/pmc_${T}_$c \
    timeout -k 10 900 bash tools/pmc.sh > gpurun_out/pmc_${T}_$c.log 2>&1; rc=$?
  echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_${T}_$c.log; exit $rc; }
  PMC_LAUNCHES_PER_STEP=$lps python3 tools/pmc_traffic.py gpurun_out/pmc_${T}_$c gpurun_out/${T}_pmc_traffic_$c.json
  python3 tools/pmc_summary.py gpurun_out/pmc_${T}_$c > gpurun_out/${T}_pmc_summary_$c.txt
done
