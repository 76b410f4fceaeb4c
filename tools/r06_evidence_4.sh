# round-6 evidence, part 4: the BASELINE config lines once more, after parts 2 and 3 put this build's PMC
# passes of every config under profiles/ (each line's pmc_provenance then names a pass of the library it ran)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r06z}
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 $to "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err; local rc=$?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${T}_$name.json')); print('$name', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('pmc_provenance',{}).get('pmc_build_match'))" 2>/dev/null
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${T}_$name.err; echo "STOP"; exit $rc; fi
}
step c2 300 python bench.py --config c2
step c3 300 python bench.py --config c3
step c5 300 python bench.py --config c5
step zeropad 300 python bench.py --config zeropad
step b128 300 python bench.py --batch 128
step strong1 300 python bench.py --scaling strong --no-cpu
