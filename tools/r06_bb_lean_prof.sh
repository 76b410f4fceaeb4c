# round 6: kernel trace of tools/time_bwd.py at B=1024 72^2 with the 8x24 (lib_nolean) and the lean 24x24 BB
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
# BB's own time at B=1024 72^2: kernel trace of tools/time_bwd.py with each library
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lib in build_ab/lib_nolean.so graph_neural_cellular_automata_amd/libgnca.so; do
  tag=$(basename $lib .so)
  GNCA_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r06g_$tag -o run -- python3 tools/time_bwd.py --sizes 1024x72 --iters 10 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/prof_r06g_$tag -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/r06g_bwd1024_kernel_stats_$tag.csv
  python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/r06g_bwd1024_kernel_stats_$tag.csv')))
for r in rows[:6]: print('$tag', r['Name'][:70], r['Calls'], '%.1f us'%(float(r['AverageNs'])/1e3))"
done
