#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ix4; mkdir -p $OUT
for v in "BENCH_NO_GRAPH=1" "GPU_MAX_HW_QUEUES=8" "ET_X=0"; do
env $v timeout -k 10 300 python3 tools/cfg4_only.py config2 > $OUT/c4.txt 2>&1 || { echo C4_FAIL; tail -5 $OUT/c4.txt; exit 1; }
echo "$v $(tail -1 $OUT/c4.txt)"
done
