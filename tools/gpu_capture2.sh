#!/bin/bash
# VERDICT r04 item 4, second step: does the slowdown follow the number of hardware queues
# the process opened before the library's side streams (queue id -> CP pipe)?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-capture2}
mkdir -p $OUT
for m in dummy1 dummy2 dummy3 dummy4 hidummy1 capture+dummy3 capture; do
  timeout -k 10 240 python3 tools/capture_effect.py $m 10 >> $OUT/modes.jsonl 2> $OUT/$m.err || { echo FAIL $m; tail -5 $OUT/$m.err; exit 1; }
  tail -1 $OUT/modes.jsonl
done
m=dummy4
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_$m -o run --output-format csv \
  -- python3 tools/capture_effect.py $m 3 > $OUT/traced_$m.txt 2>&1 || { echo TRACE_FAIL $m; tail -5 $OUT/traced_$m.txt; exit 1; }
f=$(ls $OUT/prof_$m/*/run_kernel_trace.csv $OUT/prof_$m/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/queue_map.py "$f" > $OUT/queue_map_$m.txt && echo "traced $m"
