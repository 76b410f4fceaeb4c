# round-6 evidence, part 1: GPU tests, smoke, the driver's command twice, its rocprofv3 kernel trace
# (timed launches), and the headline's PMC passes tagged with the library's sha256
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r06z}
export GNCA_LIB_SHA16=$(python3 -c "import hashlib;print(hashlib.sha256(open('graph_neural_cellular_automata_amd/libgnca.so','rb').read()).hexdigest()[:16])")
echo "lib sha16 $GNCA_LIB_SHA16"
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 $to "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?
  grep -v amdgpu.ids gpurun_out/${T}_$name.log | tail -n 3 | cut -c1-300
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP"; exit $rc; fi
}
rm -f gpurun_out/drift_log.jsonl
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
cp gpurun_out/drift_log.jsonl gpurun_out/${T}_drift_log.jsonl
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step driver1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step driver2 300 python bench.py --gpus 1 --steps 20 --warmup 5
TAG=$T bash tools/r04_profile.sh prof pmc > gpurun_out/${T}_profile.log 2>&1; rc=$?; tail -12 gpurun_out/${T}_profile.log; exit $rc
