# round-6 training measurements: phase split (GNCA_TRAIN_PHASES, synchronising) + plain timed lines +
# a rocprofv3 kernel trace of the B=128 iteration (kernel time vs wall)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r06b}
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err; local rc=$?; echo "$name rc=$rc"; tail -2 gpurun_out/${T}_$name.err | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc; return 0; }
run train128 300 python bench.py --mode train --train-batch 128 --train-size 72 --steps 4 --warmup 1
GNCA_TRAIN_PHASES=1 run train128_phases 300 python bench.py --mode train --train-batch 128 --train-size 72 --steps 4 --warmup 1
run train_c5 400 python bench.py --mode train --config c5 --steps 4 --warmup 1
GNCA_TRAIN_PHASES=1 run train_c5_phases 400 python bench.py --mode train --config c5 --steps 4 --warmup 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_train128 -o run --output-format csv \
  -- python3 bench.py --mode train --train-batch 128 --train-size 72 --steps 2 --warmup 1 > gpurun_out/${T}_train128_prof.json 2> gpurun_out/${T}_train128_prof.err
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${T}_train128_prof.err; exit $rc; }
st=$(find gpurun_out/prof_${T}_train128 -name "*kernel_stats.csv" | head -1); cp "$st" gpurun_out/${T}_train128_kernel_stats.csv
for f in train128 train128_phases train_c5 train_c5_phases train128_prof; do python3 -c "import json,sys; d=json.load(open('gpurun_out/${T}_$f.json')); print('$f', 'ms/iter %.2f'%d['ms_per_step'], '%.3e'%d['value'], d['iteration_stats'])"; done
