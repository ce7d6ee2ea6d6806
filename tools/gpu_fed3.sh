#!/bin/bash
# Round 4: fed chains with the asm gatherer (7 gatherer waves): parity, timings, timeline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/fed3; mkdir -p $OUT
ET_CHAIN_FED=2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_early_chains.py tests/test_gpu_update.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_fed.log 2>&1 || { echo FED_TEST_FAIL; tail -30 $OUT/pytest_fed.log; exit 1; }
tail -1 $OUT/pytest_fed.log
for r in 1 2; do for v in 0 1 2; do
  ET_CHAIN_FED=$v timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4_${v}_$r.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4_${v}_$r.txt; exit 1; }
  echo "fed=$v $(tail -1 $OUT/cfg4_${v}_$r.txt)"
done; done
ET_CHAIN_FED=2 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fullsize.py -x -q -m gpu -k exact --timeout 300 --timeout-method thread > $OUT/pytest_fed_full.log 2>&1 || { echo FED_FULL_FAIL; tail -30 $OUT/pytest_fed_full.log; exit 1; }
tail -1 $OUT/pytest_fed_full.log
for v in 1 2; do
ET_CHAIN_FED=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$v -o run --output-format csv \
  -- python3 tools/exact_cfg4.py exact > $OUT/exact_traced$v.txt 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/exact_traced$v.txt; exit 1; }
f=$(ls $OUT/prof$v/*/run_kernel_trace.csv $OUT/prof$v/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/upd_timeline.py "$f" > $OUT/exact_timeline$v.txt && echo "timeline fed=$v" && grep -E "chains|sgd_exact|total" $OUT/exact_timeline$v.txt
done
for v in "ET_PLAN_SIDE=0" "ET_PLAN_SIDE=0 ET_CHAIN_FED=2" "ET_PLAN_SIDE=0 ET_CHAIN_FED=1"; do
  env $v timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4_ps.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4_ps.txt; exit 1; }
  echo "$v $(tail -1 $OUT/cfg4_ps.txt)"
done
