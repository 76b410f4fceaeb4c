# round-6 evidence, part 3: the trainer lines with their phase split and kernel trace
# (tools/r06_train_phases.sh) and the backward's timing at three sizes with a kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r06z}
export GNCA_LIB_SHA16=$(python3 -c "import hashlib;print(hashlib.sha256(open('graph_neural_cellular_automata_amd/libgnca.so','rb').read()).hexdigest()[:16])")
# the driver's command once more, now that profiles/ holds this build's PMC passes (pmc_build_match)
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_driver3.json 2> gpurun_out/${T}_driver3.err || exit 1
tail -c 400 gpurun_out/${T}_driver3.json; echo
# PMC passes of the small configs and the zero-padded shift on this build
for c in c2 c3 zeropad; do
  PMC_CMD="python3 bench.py --steps 4 --warmup 1 --no-cpu --gpu-warmup-ms 0 --config $c" PMC_OUT=gpurun_out/pmc_${T}_$c \
    timeout -k 10 900 bash tools/pmc.sh > gpurun_out/pmc_${T}_$c.log 2>&1; rc=$?
  echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_${T}_$c.log; exit $rc; }
  lps=1; [ $c = zeropad ] && lps=2
  PMC_LAUNCHES_PER_STEP=$lps python3 tools/pmc_traffic.py gpurun_out/pmc_${T}_$c gpurun_out/${T}_pmc_traffic_$c.json
  python3 tools/pmc_summary.py gpurun_out/pmc_${T}_$c > gpurun_out/${T}_pmc_summary_$c.txt
done
T=$T bash tools/r06_train_phases.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_bwdprof -o run \
  -- python3 tools/time_bwd.py --sizes 1024x72,128x72,16x40 --iters 5 > gpurun_out/${T}_bwd.txt 2>&1; rc=$?
echo "bwd rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${T}_bwd.txt; exit $rc; }
f=$(find gpurun_out/${T}_bwdprof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_bwd_kernel_stats.csv
timeout -k 10 300 python3 tools/time_bwd.py --sizes 1024x72,128x72,16x40 --iters 10 > gpurun_out/${T}_bwd_timing.txt 2>&1
grep "B=" gpurun_out/${T}_bwd_timing.txt
