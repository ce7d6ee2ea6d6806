#!/bin/bash
# Round 4: chunk-pass grid x EH knobs for the exact update (config 4).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/knobs7; mkdir -p $OUT
for r in 1 2; do for v in "ET_EH=1 ET_SGD_GRID=512" "ET_EH=1 ET_SGD_GRID=256" "ET_EH=1 ET_SGD_GRID=384" "ET_EH=1 ET_SGD_GRID=768" "ET_EH=0 ET_SGD_GRID=512" "ET_EH=1 ET_SGD_GRID=512 ET_EH_WG=48" "ET_EH=1 ET_SGD_GRID=512 ET_EC_WG=48" "ET_EH=1 ET_SGD_GRID=512 ET_CHAIN_WG=96" "ET_EH=1 ET_SGD_GRID=512 ET_EH_MIN=16384" "ET_EH=1 ET_SGD_GRID=512 ET_PLAN_SIDE=0"; do
  env $v timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4.txt; exit 1; }
  echo "$v $(tail -1 $OUT/cfg4.txt)"
done; done
for v in "ET_SGD_GRID=512" "ET_SGD_GRID=0"; do
  env $v timeout -k 10 200 python3 tools/exact_cfg4.py split > $OUT/cfg4s.txt 2>&1 || { echo CFG4S_FAIL $v; tail -5 $OUT/cfg4s.txt; exit 1; }
  echo "split $v $(tail -1 $OUT/cfg4s.txt)"
done
ET_EH=1 ET_SGD_GRID=512 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 tools/exact_cfg4.py exact > $OUT/exact_traced.txt 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/exact_traced.txt; exit 1; }
f=$(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/upd_timeline.py "$f" > $OUT/exact_timeline.txt && echo "timeline grid512" && grep -E "chains|sgd_exact|chain_emit|total" $OUT/exact_timeline.txt
