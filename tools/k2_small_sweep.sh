# K2 band-height sweep at the small batches (c2, c3): GNCA_K2_BAND unset (the planner: 2 rows), 1..4.
# Measured r02: the planner's 2 rows are at the optimum (c2 0.0187-0.0190, c3 0.0251-0.0254 ms/step).
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for c in c2 c3; do
for b in 0 1 2 3 4; do
  if [ $b = 0 ]; then e=""; else e="GNCA_K2_BAND=$b"; fi
  env $e timeout -k 10 200 python bench.py --config $c --no-cpu > /tmp/o.json 2>/dev/null || { echo fail; exit 1; }
  python -c "import json; d=json.load(open('/tmp/o.json')); print('$c band=$b', '%.3e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'k2 %.4f'%d['roofline_k2']['k2_ms'])"
done
done
