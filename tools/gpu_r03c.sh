#!/bin/bash
# Round 3: exact-update timeline on the current defaults + the exact/early-chain GPU tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r03c}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_early_chains.py tests/test_gpu_update.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_exact -o run --output-format csv \
  -- python3 tools/exact_cfg4.py exact > $OUT/exact_traced.txt 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/exact_traced.txt; exit 1; }
f=$(ls $OUT/prof_exact/*/run_kernel_trace.csv $OUT/prof_exact/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/upd_timeline.py "$f" > $OUT/exact_timeline.txt && grep -E "chains|sgd_exact|total" $OUT/exact_timeline.txt
