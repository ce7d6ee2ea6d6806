#!/bin/bash
# Round 4: the fed walk for the early hot columns (EH) and the regular chains only.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/fed6; mkdir -p $OUT
ET_CHAIN_FED=6 ET_EH_MIN=300 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_early_chains.py tests/test_gpu_update.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_fed6.log 2>&1 || { echo FED_TEST_FAIL; tail -30 $OUT/pytest_fed6.log; exit 1; }
echo "fed6 $(tail -1 $OUT/pytest_fed6.log)"
for r in 1 2; do for v in "ET_X=0" "ET_CHAIN_FED=4" "ET_CHAIN_FED=4 ET_EH_WG=64" "ET_CHAIN_FED=4 ET_EH_WG=96" "ET_CHAIN_FED=6" "ET_CHAIN_FED=2"; do
  env $v timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4.txt; exit 1; }
  echo "$v $(tail -1 $OUT/cfg4.txt)"
done; done
ET_CHAIN_FED=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 tools/exact_cfg4.py exact > $OUT/exact_traced.txt 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/exact_traced.txt; exit 1; }
f=$(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/upd_timeline.py "$f" > $OUT/exact_timeline.txt && echo "timeline fed4" && grep -E "chains|sgd_exact|chain_emit|total" $OUT/exact_timeline.txt
