#!/bin/bash
# K1 ablation + phase timers, then clean single-stream PMC passes (no co-resident K2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ABLATE_ONLY="full,prof,no_mfma,no_gather,no_perceive,no_stage,lds_linear,no_store,mfma_only" ABLATE_PROF_SETS=w03 \
  timeout -k 10 300 python tools/ablate.py run > gpurun_out/r03d_ablate.txt 2>&1 || { echo "ablate failed"; tail -20 gpurun_out/r03d_ablate.txt; exit 1; }
cat gpurun_out/r03d_ablate.txt
GNCA_LIB_PATH=build_ab/lib_nosub.so PMC_CMD="python3 bench.py --steps 4 --warmup 1 --no-cpu --gpu-warmup-ms 0" PMC_OUT=gpurun_out/pmc_r03d bash tools/pmc.sh > gpurun_out/pmc_r03d.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_r03d.log; exit 1; }
PMC_LAUNCHES_PER_STEP=1 python tools/pmc_traffic.py gpurun_out/pmc_r03d gpurun_out/r03d_pmc_traffic.json || exit 1
python tools/pmc_summary.py gpurun_out/pmc_r03d > gpurun_out/r03d_pmc_summary.txt
head -40 gpurun_out/r03d_pmc_summary.txt
