#!/bin/bash
# Round 4: diagnose the fed chain walk, then EH settings.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/fed4; mkdir -p $OUT
for v in 0 1; do
  ET_CHAIN_FED=$v timeout -k 10 200 python3 tools/fed_diag.py > $OUT/diag_$v.txt 2>&1 || { echo DIAG_FAIL $v; tail -20 $OUT/diag_$v.txt; exit 1; }
  cat $OUT/diag_$v.txt
done
ET_EH=1 ET_EH_MIN=300 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_early_chains.py tests/test_gpu_update.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_eh.log 2>&1 || { echo EH_TEST_FAIL; tail -30 $OUT/pytest_eh.log; exit 1; }
echo "eh $(tail -1 $OUT/pytest_eh.log)"
for r in 1 2; do for v in "ET_EH=0" "ET_EH=1" "ET_EH=1 ET_EH_MIN=16384" "ET_EH=1 ET_EH_MIN=65536" "ET_EH=1 ET_EH_WG=64"; do
  env $v timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4.txt; exit 1; }
  echo "$v $(tail -1 $OUT/cfg4.txt)"
done; done
ET_EH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 tools/exact_cfg4.py exact > $OUT/exact_traced.txt 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/exact_traced.txt; exit 1; }
f=$(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/upd_timeline.py "$f" > $OUT/exact_timeline.txt && echo "timeline eh" && grep -E "chains|sgd_exact|eh_pick|ec_emit|ec_count|chain_tiles|total" $OUT/exact_timeline.txt
# per-XCD work queues for the headline lookup (ET_SCHED=queue): parity, then A/B twice
ET_SCHED=queue timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fullsize.py -x -q -m gpu -k config3 --timeout 300 --timeout-method thread > $OUT/pytest_queue.log 2>&1 || { echo QUEUE_TEST_FAIL; tail -30 $OUT/pytest_queue.log; exit 1; }
echo "queue $(tail -1 $OUT/pytest_queue.log)"
for r in 1 2; do for v in "ET_SCHED=stripe" "ET_SCHED=queue"; do
  env $v timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-extra --cpu-seconds 2 > $OUT/bench_q.txt 2>&1 || { echo BENCH_FAIL $v; tail -5 $OUT/bench_q.txt; exit 1; }
  echo "$v $(tail -1 $OUT/bench_q.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["frac"], d["roofline"].get("achieved"))')"
done; done
