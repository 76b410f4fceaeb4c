#!/bin/bash
# PMC passes over a short bench run, one counter group per rocprofv3 invocation (no tracing
# domains mixed with --pmc).  Output: gpurun_out/pmc/<pass>/...counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS="${PMC_CMD:-python3 bench.py --steps 4 --warmup 1 --no-cpu ${BENCH_ARGS:-}}"
REGEX="${PMC_REGEX:-gnca_k}"
OUT="${PMC_OUT:-gpurun_out/pmc}"
mkdir -p "$OUT"
# PMC_PASSES: the pass numbers to run (default every pass), e.g. "1 2 4"
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  if [ -n "${PMC_PASSES:-}" ] && ! [[ " $PMC_PASSES " == *" $i "* ]]; then continue; fi
  echo "=== pass $i: $counters"
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-include-regex "$REGEX" -d $OUT/p$i -o run --output-format csv -- $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; exit $rc; fi
done <<'LIST'
FETCH_SIZE
WRITE_SIZE
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU
SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SMEM
SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_UNALIGNED_STALL SQ_WAVES
TCC_HIT_sum TCC_MISS_sum
LIST
echo done
