#!/bin/bash
# Run GPU steps in order; each under its own time limit.  Test failures (rc 1) continue to the
# next step; a crash, abort, fault or timeout (any other non-zero rc) ends the session.
# usage: tools/gpu_session.sh STEP [STEP ...]   STEP in: tests smoke bench ... (below)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    testsall) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    drift) run pytest_drift 400 python -u -m pytest tests/test_gpu_drift.py -m gpu -v -s -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    grad) run pytest_grad 600 python -m pytest tests/test_gpu_grad.py -m gpu -q -p no:cacheprovider ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 96 --warmup 8 ;;
    driver) run bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    benchq) run bench 600 python bench.py --steps 24 --warmup 4 --no-cpu ;;
    gpus2) run bench_gpus2 600 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu ;;
    train) run bench_train 600 python bench.py --mode train --steps 10 --warmup 2 ;;
    train2) run bench_train2 600 python bench.py --mode train --gpus 2 --steps 6 --warmup 2 --dist-backend gloo ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
