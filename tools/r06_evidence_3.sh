# round-6 evidence, part 3: the trainer lines with their phase split and kernel trace
# (tools/r06_train_phases.sh) and the backward's timing at three sizes with a kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r06z}
T=$T bash tools/r06_train_phases.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_bwdprof -o run \
  -- python3 tools/time_bwd.py --sizes 1024x72,128x72,16x40 --iters 5 > gpurun_out/${T}_bwd.txt 2>&1; rc=$?
echo "bwd rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${T}_bwd.txt; exit $rc; }
f=$(find gpurun_out/${T}_bwdprof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_bwd_kernel_stats.csv
timeout -k 10 300 python3 tools/time_bwd.py --sizes 1024x72,128x72,16x40 --iters 10 > gpurun_out/${T}_bwd_timing.txt 2>&1
grep "B=" gpurun_out/${T}_bwd_timing.txt
