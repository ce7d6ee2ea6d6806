#!/bin/bash
# Exact config-4 update time under several environment settings, on one box.
# Usage: tools/ab_exact.sh TAG "ENV1" "ENV2" ...   (each ENV a space-separated VAR=value list,
# "-" for none); two rounds, alternating.
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/abx_$TAG
mkdir -p $OUT
for r in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    e=""; [ "$cfg" != "-" ] && e="$cfg"
    env $e timeout -k 10 200 python3 tools/exact_cfg4.py exact > $OUT/run_${i}_$r.txt 2>&1 || { echo FAIL "$cfg"; tail -5 $OUT/run_${i}_$r.txt; exit 1; }
    echo "[$cfg] $(tail -1 $OUT/run_${i}_$r.txt)"
  done
done
