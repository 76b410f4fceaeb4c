#!/bin/bash
# Round-4 evidence for the bench line, each GPU step under its own limit, stopping at the first
# failure: (1) rocprofv3 kernel trace + stats of exactly the driver's command, summarised over the
# timed rollout's own launches (tools/timed_kernels.py); (2) the PMC passes (tools/pmc.sh) ->
# per-launch HBM traffic and MFMA busy of K1 (two sub-batch launches per step) (tools/pmc_traffic.py).
#   TAG=r04a bash tools/r04_profile.sh [prof] [pmc]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04a}
mkdir -p gpurun_out
for s in "$@"; do
  case $s in
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
        -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err
      rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_prof.err; exit $rc; }
      tr=$(find gpurun_out/prof_$TAG -name "*kernel_trace.csv" | head -1)
      st=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
      cp "$st" gpurun_out/${TAG}_rocprof_kernel_stats.csv
      python3 tools/timed_kernels.py "$tr" gpurun_out/${TAG}_prof_bench.json gpurun_out/${TAG}_timed_kernels.json | tail -30 ;;
    pmc)
      PMC_CMD="python3 bench.py --steps 4 --warmup 1 --no-cpu --gpu-warmup-ms 0" PMC_OUT=gpurun_out/pmc_$TAG \
        bash tools/pmc.sh > gpurun_out/pmc_$TAG.log 2>&1
      rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/pmc_$TAG.log; exit $rc; }
      PMC_LAUNCHES_PER_STEP=2 python3 tools/pmc_traffic.py gpurun_out/pmc_$TAG gpurun_out/${TAG}_pmc_traffic.json
      python3 tools/pmc_summary.py gpurun_out/pmc_$TAG > gpurun_out/${TAG}_pmc_summary.txt
      head -60 gpurun_out/${TAG}_pmc_summary.txt ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
