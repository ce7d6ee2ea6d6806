#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ix3; mkdir -p $OUT
for v in "fp16" "config2"; do
timeout -k 10 300 python3 tools/cfg4_only.py $v > $OUT/c4.txt 2>&1 || { echo C4_FAIL; tail -5 $OUT/c4.txt; exit 1; }
echo "$v $(tail -1 $OUT/c4.txt)"
done
