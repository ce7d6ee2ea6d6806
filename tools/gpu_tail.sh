#!/bin/bash
# Round 4: tail chain workgroups on the caller's stream after the chunk pass (ET_TAIL_*).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/tail; mkdir -p $OUT
ET_TAIL_EC=32 ET_TAIL_EH=64 ET_TAIL_REG=128 ET_EH_MIN=300 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_early_chains.py tests/test_gpu_update.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_tail.log 2>&1 || { echo TAIL_TEST_FAIL; tail -30 $OUT/pytest_tail.log; exit 1; }
echo "tail $(tail -1 $OUT/pytest_tail.log)"
for r in 1 2; do for v in "ET_X=0" "ET_TAIL_REG=128" "ET_TAIL_EH=32" "ET_TAIL_EH=64" "ET_TAIL_EH=32 ET_TAIL_REG=128" "ET_TAIL_EH=64 ET_TAIL_REG=96 ET_TAIL_EC=32"; do
  env $v timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4.txt; exit 1; }
  echo "$v $(tail -1 $OUT/cfg4.txt)"
done; done
ET_TAIL_EH=32 ET_TAIL_REG=128 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 tools/exact_cfg4.py exact > $OUT/exact_traced.txt 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/exact_traced.txt; exit 1; }
f=$(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/upd_timeline.py "$f" > $OUT/exact_timeline.txt && echo "timeline tail" && grep -E "chains|sgd_exact|total" $OUT/exact_timeline.txt
