#!/bin/bash
# Round 4: the 64-deep ring chain loop (ET_CHAIN_RING=1) against the 32-deep loop: exact GPU
# tests with the ring loop, A/B of the config-4 update, kernel trace of one exact update.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ring; mkdir -p $OUT
ET_CHAIN_RING=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_early_chains.py tests/test_gpu_fullsize.py tests/test_gpu_update.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_ring.log 2>&1 || { echo TEST_FAIL; tail -30 $OUT/pytest_ring.log; exit 1; }
tail -1 $OUT/pytest_ring.log
bash tools/ab_env.sh ring ET_CHAIN_RING 2 || exit 1
ET_CHAIN_RING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 tools/exact_cfg4.py exact > $OUT/exact_traced.txt 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/exact_traced.txt; exit 1; }
f=$(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/upd_timeline.py "$f" > $OUT/exact_timeline.txt && grep -E "chains|sgd_exact|total" $OUT/exact_timeline.txt
cat $OUT/exact_traced.txt | tail -1
