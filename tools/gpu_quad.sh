#!/bin/bash
# Round 4: the quad walk's threshold (ET_QUAD_MIN, 64-entry groups) at the round-4 defaults.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/quad; mkdir -p $OUT
for r in 1 2; do for v in "ET_X=0" "ET_QUAD_MIN=256" "ET_QUAD_MIN=384" "ET_QUAD_MIN=512" "ET_QUAD_MIN=768" "ET_QUAD_MIN=512 ET_EH_MIN=24576"; do
  env $v timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/cfg4.txt 2>&1 || { echo CFG4_FAIL $v; tail -5 $OUT/cfg4.txt; exit 1; }
  echo "$v $(tail -1 $OUT/cfg4.txt)"
done; done
