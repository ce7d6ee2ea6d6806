#!/bin/bash
# Round 4: per-entry latency term in the chains' S choice (ET_LAT_EH / _REG / _EC).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/knobs9; mkdir -p $OUT
for r in 1 2; do for v in "ET_X=0" "ET_LAT_EH=8" "ET_LAT_EH=16" "ET_LAT_EH=32" "ET_LAT_REG=8" "ET_LAT_REG=16" "ET_LAT_REG=32" "ET_LAT_EC=8" "ET_LAT_EH=16 ET_LAT_REG=16"; do
  env $v timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4.txt; exit 1; }
  echo "$v $(tail -1 $OUT/cfg4.txt)"
done; done
