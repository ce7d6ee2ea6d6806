#!/bin/bash
# Round-4 GPU check on one MI355X: GPU suite, smoke, bench, traced bench (headline kernel
# durations), PMC traffic of the headline kernel, kernel trace of one exact config-4 update.
# Usage: tools/gpu_final_r04.sh TAG [tests|notests]
set -o pipefail
TAG=${1:-r04}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { echo GPUTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bench_traced.json 2> $OUT/bench_traced.err || { echo TRACE_FAIL; tail -5 $OUT/bench_traced.err; exit 1; }
echo trace ok
bash tools/pmc_traffic.sh $OUT/pmc --steps 5 --warmup 1 --cpu-seconds 0 --no-extra || { echo PMC_FAIL; exit 1; }
python3 tools/traffic.py $OUT/pmc k_pooled_vec criteo26_b65536 $OUT/pmc/traffic.json | tail -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_exact -o run --output-format csv \
  -- python3 tools/exact_cfg4.py exact > $OUT/exact_traced.txt 2>&1 || { echo TRACE2_FAIL; tail -5 $OUT/exact_traced.txt; exit 1; }
f=$(ls $OUT/prof_exact/*/run_kernel_trace.csv $OUT/prof_exact/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/upd_timeline.py "$f" > $OUT/exact_timeline.txt && grep -E "chains|sgd_exact|total" $OUT/exact_timeline.txt
