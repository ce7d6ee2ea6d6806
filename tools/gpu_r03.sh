#!/bin/bash
# Round-3 GPU pass: GPU test suite, bench, kernel trace of the exact config-4 update.
# Usage: tools/gpu_r03.sh TAG [tests|notests]
set -o pipefail
TAG=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/gputest.log 2>&1 || { echo GPUTEST_FAIL; tail -30 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
fi
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_exact -o run --output-format csv \
  -- python3 tools/exact_cfg4.py exact > $OUT/exact_traced.txt 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/exact_traced.txt; exit 1; }
echo trace ok
f=$(ls $OUT/prof_exact/*/run_kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] || f=$(ls $OUT/prof_exact/run_kernel_trace.csv)
python3 tools/upd_timeline.py "$f" > $OUT/exact_timeline.txt && tail -3 $OUT/exact_timeline.txt
