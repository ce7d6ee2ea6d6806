#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ix; mkdir -p $OUT
for v in "ET_X=0" "ET_EH=0" "ET_EXACT_GRID=16384" "ET_X=0"; do
  env $v timeout -k 10 200 python3 tools/upd_ix.py > $OUT/ix.txt 2>&1 || { echo IX_FAIL $v; tail -5 $OUT/ix.txt; exit 1; }
  echo "$v $(tail -1 $OUT/ix.txt)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 tools/upd_ix.py 3 1 > $OUT/traced.txt 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/traced.txt; exit 1; }
echo traced
